"""Per-client data feeding for the federated MaPLe path (the role of trainers/client_datamanager.py
and the class-union logic of trainers/maple_fed.py:48-159).

The reference reads PatternNet / UcMerced / EuroSAT images from disk through Dassl loaders with
PIL transforms (random_resized_crop, flip, CLIP normalisation).  Real datasets are out of scope
here; each client instead owns a seeded synthetic split of the same shape
-- normalised 224x224x3 images and labels over the unified class list -- generated once by the
portable PRNG (federated_multi_modal_amd.synthetic) and kept resident in HBM, so a training step
reads its batch from device memory (no host->device copy on the hot path).

Loaders yield the reference's batch dicts: {"img": [B,3,224,224] fp32, "label": [B] int64,
"caption": list[str]} (trainers/maple.py:537-545).  The train loader reshuffles every epoch with the
client's own generator (RandomSampler semantics, drop_last as Dassl's train loader:
len(train_x) >= batch).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterator, List, Sequence

import zlib

import numpy as np
import torch

from . import synthetic as syn

# Dataset shapes of the reference's clients (number of classes) and the shapes BASELINE.json names
DATASET_CLASSES = {"PatternNet": 38, "Ucmerced": 21, "EuroSAT": 10, "ImageNet": 1000}


def unified_classnames(datasets: Sequence[str], seed: int = 0) -> List[str]:
    """Sorted union of the clients' class names (trainers/maple_fed.py:98-107).  Synthetic names stand
    in for the dataset folders; the union of distinct synthetic lists is their concatenation."""
    names = []
    for i, ds in enumerate(datasets):
        names += [f"{ds.lower()}_{c}" for c in syn.synthetic_classnames(DATASET_CLASSES[ds], seed + 17 * i)]
    return sorted(set(names))


@dataclass
class _Split:
    images: torch.Tensor  # [N,3,R,R] fp32, device
    labels: torch.Tensor  # [N] int64, device
    captions: List[str] = None  # one per image (synthetic BLIP-style strings) or None


class _Loader:
    def __init__(self, split: _Split, batch: int, shuffle: bool, drop_last: bool, gen: torch.Generator):
        self.s, self.batch, self.shuffle, self.drop_last, self.gen = split, batch, shuffle, drop_last, gen

    def captions(self, idx):
        return [self.s.captions[k] for k in idx.tolist()]

    def __len__(self):
        n = self.s.labels.numel()
        return n // self.batch if self.drop_last else (n + self.batch - 1) // self.batch

    def __iter__(self) -> Iterator[Dict[str, object]]:
        n = self.s.labels.numel()
        order = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
        order = order.to(self.s.labels.device)
        for i in range(len(self)):
            idx = order[i * self.batch:(i + 1) * self.batch]
            yield {"img": self.s.images.index_select(0, idx), "label": self.s.labels.index_select(0, idx),
                   "caption": self.captions(idx) if self.s.captions is not None else None, "index": idx}


class SyntheticClientDataManager:
    """ClientDataManager stand-in: .train_loader / .test_loader / .num_classes / .lab2cname."""

    def __init__(self, client_id: int, classnames: List[str], n_train: int, n_test: int, train_batch: int,
                 test_batch: int, device, seed: int = 0, image_resolution: int = 224, captions: bool = False,
                 unique_images: int = 0):
        """captions: batches carry one synthetic caption string per image (the caption-fork datasets' Datum
        captions), which turns on the caption-conditioned prompts; off, "caption" is None (BASELINE's
        synthetic configs carry no captions).  unique_images > 0: each split generates min(size, unique_images)
        images (with their labels and, with captions, their captions) and repeats them in the same order to its
        size -- the device work per batch is the same, and the host PRNG (~25 ms per image) stays out of long
        timing runs (bench.py's round wall-time)."""
        self.client_id = client_id
        self._classnames = list(classnames)
        K = len(classnames)
        self.device = torch.device(device)

        def make(tag: str, n: int) -> _Split:
            imgs, labs = [], []
            n_gen = n if unique_images <= 0 else min(n, unique_images)
            for s0 in range(0, n_gen, 64):  # generate in chunks (host memory)
                b = syn.client_batch(seed, client_id, zlib.crc32(tag.encode()) + s0, min(64, n_gen - s0), K,
                                     image_resolution)
                imgs.append(torch.from_numpy(b.images).to(self.device))
                labs.append(torch.from_numpy(b.labels).to(self.device))
            img, lab = torch.cat(imgs), torch.cat(labs)
            caps = syn.synthetic_captions(seed, client_id, zlib.crc32(tag.encode()), n_gen) if captions else None
            if n_gen < n:  # repeat images, labels and captions alike, so image i keeps its own caption
                reps = (n + n_gen - 1) // n_gen
                img, lab = img.repeat(reps, 1, 1, 1)[:n].contiguous(), lab.repeat(reps)[:n].contiguous()
                caps = (list(caps) * reps)[:n] if caps is not None else None
            return _Split(img, lab, caps)

        self.train = make("train", n_train)
        self.test = make("test", n_test)
        g = torch.Generator().manual_seed(seed * 1000 + client_id)
        self.train_loader = _Loader(self.train, train_batch, shuffle=True, drop_last=n_train >= train_batch, gen=g)
        self.test_loader = _Loader(self.test, test_batch, shuffle=False, drop_last=False, gen=g)

    @property
    def num_classes(self) -> int:
        return len(self._classnames)

    @property
    def lab2cname(self) -> Dict[int, str]:
        return {i: c for i, c in enumerate(self._classnames)}

    @property
    def classnames(self) -> List[str]:
        return self._classnames


class _DecodedLoader:
    """Batches of decoded images run through the device transform (transforms.py): the reference's
    Dassl loader + per-image CPU transform workers (trainers/client_datamanager.py:21-103)."""

    def __init__(self, packed, labels: torch.Tensor, batch: int, shuffle: bool, drop_last: bool,
                 gen: torch.Generator, tfm, captions=None):
        self.p, self.labels, self.batch, self.shuffle, self.drop_last, self.gen, self.tfm = (
            packed, labels, batch, shuffle, drop_last, gen, tfm)
        self.captions = list(captions) if captions is not None else None

    def __len__(self):
        n = self.labels.numel()
        return n // self.batch if self.drop_last else (n + self.batch - 1) // self.batch

    def __iter__(self) -> Iterator[Dict[str, object]]:
        from .transforms import PackedImages
        n = self.labels.numel()
        order = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
        for i in range(len(self)):
            idx = order[i * self.batch:(i + 1) * self.batch]
            sel = idx.tolist()
            sub = PackedImages(self.p.data, self.p.offsets_host[sel], [self.p.shapes[k] for k in sel])
            geom = self.tfm.geometry(sub.shapes)
            img = self.tfm(sub, geom)
            idx_d = idx.to(self.labels.device)
            caps = [self.captions[k] for k in sel] if self.captions is not None else None
            yield {"img": img, "label": self.labels.index_select(0, idx_d), "caption": caps,
                   "index": idx_d, "geom": geom}


class DecodedClientDataManager:
    """ClientDataManager over decoded 8-bit RGB images of any sizes (HxWx3 uint8), kept resident in HBM
    in one packed buffer per split.  Train batches run RandomResizedCrop + flip + Normalize and test
    batches Resize + CenterCrop + Normalize on the device, bit-identical to the reference's Pillow /
    torchvision workers (tests/test_transforms.py).  `cfg` supplies INPUT.* (transforms.build_transform);
    batches are fp32 [B,3,224,224] as the reference's loaders yield them."""

    def __init__(self, client_id: int, classnames: List[str], train_images, train_labels, test_images,
                 test_labels, train_batch: int, test_batch: int, device, cfg=None, seed: int = 0,
                 train_captions=None, test_captions=None):
        from types import SimpleNamespace

        from . import transforms as T
        self.client_id = client_id
        self._classnames = list(classnames)
        self.device = torch.device(device)
        if cfg is None:
            cfg = SimpleNamespace(INPUT=SimpleNamespace(SIZE=(224, 224), INTERPOLATION="bicubic",
                                                        PIXEL_MEAN=list(T.CLIP_MEAN), PIXEL_STD=list(T.CLIP_STD),
                                                        TRANSFORMS=["random_resized_crop", "random_flip",
                                                                    "normalize"]))
        g = torch.Generator().manual_seed(seed * 1000 + client_id)
        self.train_tfm = T.build_transform(cfg, True, generator=g, out_dtype=torch.float32)
        self.test_tfm = T.build_transform(cfg, False, out_dtype=torch.float32)
        tr = T.pack_images(list(train_images), self.device)
        te = T.pack_images(list(test_images), self.device)
        ytr = torch.as_tensor(np.asarray(train_labels, np.int64), device=self.device)
        yte = torch.as_tensor(np.asarray(test_labels, np.int64), device=self.device)
        if ytr.numel() != len(tr) or yte.numel() != len(te):
            raise ValueError("one label per image")
        if ytr.numel() and (int(ytr.min()) < 0 or int(ytr.max()) >= len(classnames)):
            raise ValueError("train labels outside [0, num_classes)")
        # captions (Datum.caption of the reference's caption-fork datasets): batches carry them as a list of
        # str, which turns the caption-conditioned prompts on (trainers/maple.py:307-322)
        self.train_loader = _DecodedLoader(tr, ytr, train_batch, True, len(tr) >= train_batch, g, self.train_tfm,
                                           train_captions)
        self.test_loader = _DecodedLoader(te, yte, test_batch, False, False, g, self.test_tfm, test_captions)

    @property
    def num_classes(self) -> int:
        return len(self._classnames)

    @property
    def lab2cname(self) -> Dict[int, str]:
        return {i: c for i, c in enumerate(self._classnames)}

    @property
    def classnames(self) -> List[str]:
        return self._classnames
