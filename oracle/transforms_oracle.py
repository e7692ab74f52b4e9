"""ORACLE (test infrastructure only) — CPU restatement of the reference's image transforms.

NOT PRODUCT CODE.  Only `tests/` may import this module, and only as the checker.  The product
path (`federated_multi_modal_amd.transforms`) runs the HIP kernels of libmapfed.so and never
imports it.

The reference builds its image pipeline from its config (configs/trainers/MaPLeFederated/*.yaml:8-13:
SIZE (224, 224), INTERPOLATION "bicubic", CLIP PIXEL_MEAN / PIXEL_STD, TRANSFORMS
["random_resized_crop", "random_flip", "normalize"]) through Dassl's `build_transform`, which is
un-vendored (Dassl.pytorch master, unpinned — docs/INSTALL.md:23) and delegates to torchvision and
Pillow (both third-party; torchvision is absent here, Pillow 12.2 is importable):

  train: RandomResizedCrop(224, scale=(0.08, 1), ratio=(3/4, 4/3), bicubic) -> RandomHorizontalFlip
         -> ToTensor (u8 / 255) -> Normalize(mean, std)
  test:  Resize(224, bicubic) (shorter side) -> CenterCrop(224) -> ToTensor -> Normalize

What is restated here, from the published algorithms:
  * Pillow's two-pass separable resampling (libImaging/Resample.c: precompute_coeffs,
    normalize_coeffs_8bpc with PRECISION_BITS = 22, ImagingResampleHorizontal/Vertical_8bpc,
    ImagingResampleInner's ybox_first/ybox_last intermediate) for the bicubic (a = -0.5) and
    bilinear filters, 8-bit RGB.
  * torchvision's RandomResizedCrop.get_params, hflip, resize-output-size and center-crop offsets.

Pinning: the Pillow restatement is checked bit-for-bit against Pillow itself (`Image.resize`) in
tests/test_transforms.py; the torchvision pieces have no importable counterpart here and are
restated from the published source ("parity unpinned" for the crop-parameter sampler, whose draws
follow torchvision's order on a torch.Generator).
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def _bilinear(x: float) -> float:
    if x < 0.0:
        x = -x
    if x < 1.0:
        return 1.0 - x
    return 0.0


FILTERS = {"bicubic": (_bicubic, 2.0), "bilinear": (_bilinear, 1.0)}


def precompute_coeffs(in_size: int, out_size: int, interp: str = "bicubic") -> Tuple[List[Tuple[int, int]], List[List[int]]]:
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc for box [0, in_size): per output index the
    first source index, the tap count and the fixed-point taps."""
    filt, fsupport = FILTERS[interp]
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = fsupport * filterscale
    bounds, kk = [], []
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = []
        for x in range(xmax):
            w = filt((x + xmin - center + 0.5) * ss)
            k.append(w)
            ww += w
        if ww != 0.0:
            k = [w / ww for w in k]
        fixed = [int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS)) for w in k]
        bounds.append((xmin, xmax))
        kk.append(fixed)
    return bounds, kk


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize(img: np.ndarray, out_h: int, out_w: int, interp: str = "bicubic") -> np.ndarray:
    """PIL `Image.resize((out_w, out_h), BICUBIC|BILINEAR)` of an HxWx3 uint8 image (two passes,
    uint8 intermediate, rows ybox_first..ybox_last only)."""
    H, W, _ = img.shape
    hb, hk = precompute_coeffs(W, out_w, interp)
    vb, vk = precompute_coeffs(H, out_h, interp)
    y_first = vb[0][0]
    y_last = vb[-1][0] + vb[-1][1]
    src = img.astype(np.int64)
    tmp = np.empty((y_last - y_first, out_w, 3), np.uint8)
    for xx, ((xmin, n), k) in enumerate(zip(hb, hk)):
        acc = np.full((y_last - y_first, 3), 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += src[y_first:y_last, xmin + t, :] * k[t]
        tmp[:, xx, :] = _clip8(acc)
    t64 = tmp.astype(np.int64)
    out = np.empty((out_h, out_w, 3), np.uint8)
    for yy, ((ymin, n), k) in enumerate(zip(vb, vk)):
        acc = np.full((out_w, 3), 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += t64[ymin - y_first + t, :, :] * k[t]
        out[yy] = _clip8(acc)
    return out


# ---- torchvision (restated from its published transforms; absent here) -----------------------------

def rrc_get_params(height: int, width: int, gen, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0)):
    """torchvision RandomResizedCrop.get_params: (top, left, h, w)."""
    import torch
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=gen).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(float(log_ratio[0]), float(log_ratio[1]), generator=gen)).item()
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
    """torchvision Resize(int) output size (h, w)."""
    short, long = (width, height) if width <= height else (height, width)
    new_short, new_long = size, int(size * long / short)
    return (new_long, new_short) if width <= height else (new_short, new_long)


def center_crop_offsets(height: int, width: int, ch: int, cw: int) -> Tuple[int, int]:
    return int(round((height - ch) / 2.0)), int(round((width - cw) / 2.0))


def to_tensor_normalize(img: np.ndarray, mean, std) -> np.ndarray:
    """ToTensor (u8 -> fp32 / 255, CHW) then Normalize, in fp32 as torchvision does."""
    import torch
    t = torch.from_numpy(np.array(img, copy=True)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
    return t.sub_(m).div_(s).numpy()


def train_transform(img: np.ndarray, top: int, left: int, h: int, w: int, flip: bool, mean, std, size=224,
                    interp="bicubic") -> np.ndarray:
    crop = img[top:top + h, left:left + w]
    out = resize(crop, size, size, interp) if (h, w) != (size, size) else crop.copy()
    if flip:
        out = out[:, ::-1]
    return to_tensor_normalize(out, mean, std)


def test_transform(img: np.ndarray, mean, std, size=224, interp="bicubic") -> np.ndarray:
    H, W, _ = img.shape
    rh, rw = resize_short_side(H, W, size)
    r = resize(img, rh, rw, interp) if (rh, rw) != (H, W) else img
    oy, ox = center_crop_offsets(rh, rw, size, size)
    return to_tensor_normalize(r[oy:oy + size, ox:ox + size], mean, std)
