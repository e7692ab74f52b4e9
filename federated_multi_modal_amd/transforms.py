"""Device-side image transforms: the data step in front of the federated MaPLe path.

The reference's loaders run per-image CPU transforms built from its config
(configs/trainers/MaPLeFederated/*.yaml:8-13 -> Dassl build_transform -> torchvision on Pillow
images, trainers/client_datamanager.py:21-103), then cast the batch to fp16 at the model entry
(trainers/maple.py:336):

  train: RandomResizedCrop(224, scale=(0.08, 1), ratio=(3/4, 4/3), bicubic) -> RandomHorizontalFlip
         -> ToTensor -> Normalize(PIXEL_MEAN, PIXEL_STD)
  test:  Resize(224, bicubic) -> CenterCrop(224) -> ToTensor -> Normalize

Here the host only draws the random parameters (torchvision's draw order, on a torch.Generator:
RandomResizedCrop.get_params, then the flip coin) and packs an 11-int geometry row per image; the
pixels never leave HBM: one `mf_augment` call crops, resamples Pillow-exactly (22-bit fixed-point
taps, uint8 intermediate -- bit-identical to PIL.Image.resize), flips, normalises and writes the
[B,3,224,224] batch (fp16, or fp32 for the engine's img_in).  Images are decoded 8-bit RGB (HxWx3 uint8) of any size,
packed back to back in one device byte buffer (`pack_images`).
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Sequence, Tuple

import numpy as np
import torch

from ._lib import call

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)  # configs/trainers/MaPLeFederated/*.yaml PIXEL_MEAN
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)  # PIXEL_STD
INTERP = {"bicubic": 0, "bilinear": 1}


class PackedImages:
    """Decoded HxWx3 uint8 images back to back in one device buffer, with host + device offsets."""

    def __init__(self, data: torch.Tensor, offsets: Sequence[int], shapes: Sequence[Tuple[int, int]]):
        self.data = data
        self.offsets_host = np.asarray(offsets, np.int64)
        self.offsets = torch.from_numpy(self.offsets_host).to(data.device)
        self.shapes = [tuple(int(v) for v in s) for s in shapes]

    def __len__(self):
        return len(self.shapes)


def pack_images(images: Sequence[np.ndarray], device) -> PackedImages:
    offs, shapes, total = [], [], 0
    for im in images:
        if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 3:
            raise ValueError("images must be HxWx3 uint8 (decoded RGB)")
        offs.append(total)
        shapes.append(im.shape[:2])
        total += im.size
    buf = np.concatenate([np.ascontiguousarray(im).reshape(-1) for im in images]) if images else np.zeros(0, np.uint8)
    return PackedImages(torch.from_numpy(buf).to(device), offs, shapes)


def rrc_get_params(height: int, width: int, gen: torch.Generator, scale=(0.08, 1.0),
                   ratio=(3.0 / 4.0, 4.0 / 3.0)) -> Tuple[int, int, int, int]:
    """torchvision RandomResizedCrop.get_params (top, left, h, w): ten area/aspect draws, then the
    central-crop fallback."""
    area = height * width
    lr = torch.log(torch.tensor(ratio))  # float32 bounds, as torchvision draws them
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=gen).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(float(lr[0]), float(lr[1]), generator=gen)).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = int(torch.randint(0, height - h + 1, size=(1,), generator=gen).item())
            j = int(torch.randint(0, width - w + 1, size=(1,), generator=gen).item())
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def resize_short_side(height: int, width: int, size: int) -> Tuple[int, int]:
    """torchvision Resize(int): shorter side -> size, longer side int(size * long / short)."""
    short, long = (width, height) if width <= height else (height, width)
    new_short, new_long = size, int(size * long / short)
    return (new_long, new_short) if width <= height else (new_short, new_long)


class DeviceTransform:
    """Batched train / test transform on the GPU through libmapfed.so (`mf_augment`).

    train=True : RandomResizedCrop + RandomHorizontalFlip (p=0.5) + Normalize
    train=False: Resize(shorter side) + CenterCrop + Normalize
    Output: [B,3,size,size] fp16 (the model's entry dtype) or fp32 (`out_dtype`)."""

    def __init__(self, train: bool, size: int = 224, interpolation: str = "bicubic", mean=CLIP_MEAN,
                 std=CLIP_STD, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), flip_p: float = 0.5,
                 out_dtype=torch.float16, generator: torch.Generator = None):
        if interpolation not in INTERP:
            raise ValueError(f"interpolation must be one of {sorted(INTERP)}")
        self.train, self.size, self.interp = train, int(size), INTERP[interpolation]
        self.mean, self.std = tuple(float(m) for m in mean), tuple(float(s) for s in std)
        self.scale, self.ratio, self.flip_p = scale, ratio, flip_p
        self.out_dtype = out_dtype
        self.gen = generator if generator is not None else torch.Generator().manual_seed(0)
        self._ws = None

    def geometry(self, shapes: Sequence[Tuple[int, int]]) -> np.ndarray:
        """The 11-int geometry rows {H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip}, drawing the random
        parameters image by image in torchvision's order (crop params, then the flip coin)."""
        S = self.size
        rows: List[List[int]] = []
        for H, W in shapes:
            if self.train:
                i, j, h, w = rrc_get_params(H, W, self.gen, self.scale, self.ratio)
                flip = int(torch.rand(1, generator=self.gen).item() < self.flip_p)
                rows.append([H, W, i, j, h, w, S, S, 0, 0, flip])
            else:
                rh, rw = resize_short_side(H, W, S)
                oy, ox = int(round((rh - S) / 2.0)), int(round((rw - S) / 2.0))
                rows.append([H, W, 0, 0, H, W, rh, rw, oy, ox, 0])
        return np.asarray(rows, np.int32).reshape(-1, 11)

    def __call__(self, packed: PackedImages, geom: np.ndarray = None, out: torch.Tensor = None) -> torch.Tensor:
        B = len(packed)
        S = self.size
        if B == 0:
            return torch.empty(0, 3, S, S, device=packed.data.device, dtype=self.out_dtype)
        if geom is None:
            geom = self.geometry(packed.shapes)
        geom = np.ascontiguousarray(geom, np.int32)
        if geom.shape != (B, 11):
            raise ValueError("geometry must be [B, 11]")
        dev = packed.data.device
        if out is None:
            out = torch.empty(B, 3, S, S, device=dev, dtype=self.out_dtype)
        if out.shape != (B, 3, S, S) or not out.is_contiguous() or out.dtype not in (torch.float16, torch.float32):
            raise ValueError("out must be a contiguous [B,3,S,S] fp16/fp32 tensor")
        max_rows = int(geom[:, 4].max())
        need = call("mf_augment_ws_bytes", B, S, S, max_rows)
        if need < 0:
            raise ValueError("bad transform sizes")
        if self._ws is None or self._ws.numel() < need or self._ws.device != dev:
            self._ws = torch.empty(need, dtype=torch.uint8, device=dev)
        m, s = self.mean, self.std
        call("mf_augment", ctypes.c_void_p(packed.data.data_ptr()), packed.data.numel(),
             packed.offsets_host.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(packed.offsets.data_ptr()),
             geom.ctypes.data_as(ctypes.c_void_p), B, S, S, self.interp, m[0], m[1], m[2], s[0], s[1], s[2],
             ctypes.c_void_p(out.data_ptr()), int(out.dtype == torch.float16), ctypes.c_void_p(self._ws.data_ptr()),
             self._ws.numel(), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        return out


def build_transform(cfg, is_train: bool, generator: torch.Generator = None,
                    out_dtype=torch.float16) -> DeviceTransform:
    """Dassl build_transform(cfg, is_train) for the keys the reference's configs set (INPUT.SIZE,
    INPUT.INTERPOLATION, INPUT.PIXEL_MEAN / PIXEL_STD, INPUT.TRANSFORMS)."""
    inp = cfg.INPUT
    choices = list(getattr(inp, "TRANSFORMS", ["random_resized_crop", "random_flip", "normalize"]))
    supported = {"random_resized_crop", "random_flip", "normalize"}
    if not set(choices) <= supported:
        raise NotImplementedError(f"device transforms cover {sorted(supported)}, got {choices}")
    size = max(tuple(getattr(inp, "SIZE", (224, 224))))
    mean = tuple(getattr(inp, "PIXEL_MEAN", CLIP_MEAN)) if "normalize" in choices else (0.0, 0.0, 0.0)
    std = tuple(getattr(inp, "PIXEL_STD", CLIP_STD)) if "normalize" in choices else (1.0, 1.0, 1.0)
    interp = str(getattr(inp, "INTERPOLATION", "bicubic"))
    if is_train and "random_resized_crop" not in choices:
        raise NotImplementedError("train transforms without random_resized_crop")
    return DeviceTransform(is_train, size, interp, mean, std, scale=tuple(getattr(inp, "RRCROP_SCALE", (0.08, 1.0))),
                           flip_p=0.5 if (is_train and "random_flip" in choices) else 0.0, out_dtype=out_dtype,
                           generator=generator)
