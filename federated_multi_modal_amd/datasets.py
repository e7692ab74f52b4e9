"""The federated clients' datasets on disk and the class-union remap.

Reference:
  * datasets/patternnet.py, datasets/ucmerced.py: images/<class>/<file>, captions <Captions>/<class>/<file>.txt,
    split JSON (patternnet.json / Ucmerced.json) or, when absent, read_and_split_data: categories sorted,
    files in directory order, NOT shuffled, the first 50 % train, next 20 % val, rest test;
  * datasets/eurosat.py: 2750/<class>/<file>, split_zhou_EuroSAT.json (OxfordPets.read_split) or
    DTD.read_and_split_data (per-class random.shuffle, round(50 %) / round(20 %) / rest), NEW_CNAMES renames,
    captions from captions/<class>/<file>.txt;
  * Dassl DatasetBase.generate_fewshot_dataset (cfg.DATASET.NUM_SHOTS): per label in first-seen order,
    random.sample(items, shots) when there are enough items, else all of them;
  * trainers/maple_fed.py:48-159: UcMerced names renamed to PatternNet's spelling, the sorted union of the
    three datasets' class names, local labels remapped to the union index; client 0 = PatternNet,
    client 1 = UcMerced (EuroSAT only contributes class names).
Images are decoded on the host with Pillow (as the reference's Dassl loaders do, RGB) and handed to
DecodedClientDataManager, which runs the train / test transforms on the device (transforms.py).

Deviations: the reference's few-shot cache pickles are not read or written (the selection is recomputed
from a random.Random(cfg.SEED), where the reference draws from the global `random` seeded by
set_random_seed and shared with everything else); PatternNet / UcMerced split files written by their own
save_split hold 4-tuples that their read_split cannot unpack -- both 3- and 4-tuples are read here."""
from __future__ import annotations

import json
import os
import os.path as osp
import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

EUROSAT_NEW_CNAMES = {  # datasets/eurosat.py:8-19
    "AnnualCrop": "Annual Crop Land", "Forest": "Forest", "HerbaceousVegetation": "Herbaceous Vegetation Land",
    "Highway": "Highway or Road", "Industrial": "Industrial Buildings", "Pasture": "Pasture Land",
    "PermanentCrop": "Permanent Crop Land", "Residential": "Residential Buildings", "River": "River",
    "SeaLake": "Sea or Lake",
}
UCMERCED_RENAME = {  # trainers/maple_fed.py:84-93
    "tenniscourt": "tennis_court", "golfcourse": "golf_course", "parkinglot": "parking_lot",
    "storagetanks": "storage_tank", "mobilehomepark": "mobile_home_park", "baseballdiamond": "baseball_field",
    "denseresidential": "dense_residential", "sparseresidential": "sparse_residential",
}


@dataclass
class Datum:
    """dassl.data.datasets.Datum of the caption fork: impath, label, classname, caption."""
    impath: str
    label: int
    classname: str
    caption: Optional[str] = None


def listdir_nohidden(path: str, sort: bool = False) -> List[str]:
    """dassl.utils.listdir_nohidden."""
    items = [f for f in os.listdir(path) if not f.startswith(".")]
    if sort:
        items.sort()
    return items


def _read_caption(path: str) -> Optional[str]:
    if osp.exists(path):
        with open(path) as f:
            return f.read().strip()
    return None


def read_and_split_data(image_dir: str, caption_dir: str, p_trn: float = 0.5, p_val: float = 0.2,
                        ignored: Sequence[str] = ()) -> Tuple[List[Datum], List[Datum], List[Datum]]:
    """datasets/patternnet.py / ucmerced.py read_and_split_data: every image of the sorted categories in
    directory order, the caption from caption_dir/<category>/<file>.txt, then an unshuffled split."""
    categories = sorted(c for c in listdir_nohidden(image_dir) if c not in ignored)
    data = []
    for label, cat in enumerate(categories):
        for f in listdir_nohidden(osp.join(image_dir, cat)):
            cap = _read_caption(osp.join(caption_dir, cat, f.replace(".jpg", ".txt")))
            data.append(Datum(osp.join(image_dir, cat, f), label, cat, cap))
    n_trn, n_val = int(p_trn * len(data)), int(p_val * len(data))
    return data[:n_trn], data[n_trn:n_trn + n_val], data[n_trn + n_val:]


def dtd_read_and_split_data(image_dir: str, rng: random.Random, p_trn: float = 0.5, p_val: float = 0.2,
                            ignored: Sequence[str] = (), new_cnames: Optional[Dict[str, str]] = None):
    """datasets/dtd.py read_and_split_data (EuroSAT): per category the files shuffled, round(50 %) train,
    round(20 %) val, the rest test; classnames renamed by new_cnames."""
    categories = sorted(c for c in listdir_nohidden(image_dir) if c not in ignored)
    train, val, test = [], [], []
    for label, cat in enumerate(categories):
        ims = [osp.join(image_dir, cat, f) for f in listdir_nohidden(osp.join(image_dir, cat))]
        rng.shuffle(ims)
        n_trn, n_val = round(len(ims) * p_trn), round(len(ims) * p_val)
        if not (n_trn > 0 and n_val > 0 and len(ims) - n_trn - n_val > 0):
            raise ValueError(f"category {cat}: too few images to split ({len(ims)})")
        name = new_cnames.get(cat, cat) if new_cnames else cat
        train += [Datum(p, label, name) for p in ims[:n_trn]]
        val += [Datum(p, label, name) for p in ims[n_trn:n_trn + n_val]]
        test += [Datum(p, label, name) for p in ims[n_trn + n_val:]]
    return train, val, test


def save_split(train, val, test, filepath: str, path_prefix: str, with_caption: bool = True):
    def ext(items):
        out = []
        for it in items:
            p = it.impath.replace(path_prefix, "").lstrip("/")
            out.append((p, it.label, it.classname, it.caption) if with_caption else (p, it.label, it.classname))
        return out
    with open(filepath, "w") as f:
        json.dump({"train": ext(train), "val": ext(val), "test": ext(test)}, f, indent=4, separators=(",", ": "))


def read_split(filepath: str, path_prefix: str, caption_prefix: Optional[str] = None):
    """read_split of patternnet.py / ucmerced.py (captions from caption_prefix) and OxfordPets.read_split
    (EuroSAT: no caption_prefix); rows of 3 or 4 fields."""
    with open(filepath) as f:
        split = json.load(f)

    def conv(items):
        out = []
        for row in items:
            impath, label, classname = row[0], row[1], row[2]
            full = osp.join(path_prefix, impath)
            cap = None
            if caption_prefix is not None:
                cap = _read_caption(full.replace(path_prefix, caption_prefix).replace(".jpg", ".txt"))
            out.append(Datum(full, int(label), classname, cap))
        return out
    return conv(split["train"]), conv(split["val"]), conv(split["test"])


def generate_fewshot_dataset(data: List[Datum], num_shots: int, rng: random.Random) -> List[Datum]:
    """Dassl DatasetBase.generate_fewshot_dataset (repeat=False)."""
    if num_shots < 1:
        return data
    by_label: Dict[int, List[Datum]] = {}
    for it in data:
        by_label.setdefault(it.label, []).append(it)
    out = []
    for _, items in by_label.items():
        out += rng.sample(items, num_shots) if len(items) >= num_shots else items
    return out


@dataclass
class DatasetSplits:
    train_x: List[Datum]
    val: List[Datum]
    test: List[Datum]

    @property
    def lab2cname(self) -> Dict[int, str]:
        """Dassl DataManager.lab2cname: label -> classname over train_x."""
        out = {}
        for it in self.train_x + self.val + self.test:
            out.setdefault(it.label, it.classname)
        return dict(sorted(out.items()))


def load_dataset(name: str, root: str, num_shots: int = -1, seed: int = 1) -> DatasetSplits:
    """PatternNet / Ucmerced / EuroSAT as the reference's DATASET_REGISTRY builds them (few-shot on train
    and val, min(shots, 4) for val)."""
    rng = random.Random(seed)
    root = osp.abspath(osp.expanduser(root))
    if name == "PatternNet" or name == "Ucmerced":
        ddir = osp.join(root, name)
        image_dir = osp.join(ddir, "images" if name == "PatternNet" else "Images")
        caption_dir = osp.join(ddir, "Captions")
        split_path = osp.join(ddir, "patternnet.json" if name == "PatternNet" else "Ucmerced.json")
        if osp.exists(split_path):
            tr, va, te = read_split(split_path, image_dir, caption_dir)
        else:
            tr, va, te = read_and_split_data(image_dir, caption_dir)
            save_split(tr, va, te, split_path, image_dir)
    elif name == "EuroSAT":
        ddir = osp.join(root, "eurosat")
        image_dir, caption_dir = osp.join(ddir, "2750"), osp.join(ddir, "captions")
        split_path = osp.join(ddir, "split_zhou_EuroSAT.json")
        if osp.exists(split_path):
            tr, va, te = read_split(split_path, image_dir)
        else:
            tr, va, te = dtd_read_and_split_data(image_dir, rng, new_cnames=EUROSAT_NEW_CNAMES)
            save_split(tr, va, te, split_path, image_dir, with_caption=False)

        def add_captions(items):  # datasets/eurosat.py:84-104 (a missing caption file is an error there)
            out = []
            for it in items:
                rel = osp.relpath(it.impath, image_dir)
                cp = osp.splitext(osp.join(caption_dir, rel))[0] + ".txt"
                if not osp.exists(cp):
                    raise FileNotFoundError(f"Caption file missing: {cp}")
                out.append(Datum(it.impath, it.label, it.classname, _read_caption(cp)))
            return out
        tr, va, te = add_captions(tr), add_captions(va), add_captions(te)
    else:
        raise KeyError(f"dataset {name}: the federated clients read PatternNet, Ucmerced and EuroSAT")
    if num_shots >= 1:
        tr = generate_fewshot_dataset(tr, num_shots, rng)
        va = generate_fewshot_dataset(va, min(num_shots, 4), rng)
    return DatasetSplits(tr, va, te)


def union_and_remap(datasets: Dict[str, DatasetSplits]) -> Tuple[List[str], Dict[str, DatasetSplits]]:
    """trainers/maple_fed.py:80-131: UcMerced classnames renamed, the sorted union of every dataset's
    classnames, and the PatternNet / Ucmerced items relabelled to their union index (EuroSAT's are not,
    as in the reference)."""
    l2c = {k: dict(v.lab2cname) for k, v in datasets.items()}
    if "Ucmerced" in l2c:
        l2c["Ucmerced"] = {k: UCMERCED_RENAME.get(c, c) for k, c in l2c["Ucmerced"].items()}
    global_list = sorted(set().union(*[set(m.values()) for m in l2c.values()]))
    name2gid = {c: i for i, c in enumerate(global_list)}
    out = {}
    for name, ds in datasets.items():
        if name not in ("PatternNet", "Ucmerced"):
            out[name] = ds
            continue
        m = l2c[name]

        def remap(items):
            return [Datum(it.impath, name2gid[m[it.label]], m[it.label], it.caption) for it in items]
        out[name] = DatasetSplits(remap(ds.train_x), remap(ds.val), remap(ds.test))
    return global_list, out


def decode_rgb(paths: Sequence[str]) -> List[np.ndarray]:
    """PIL.Image.open(p).convert("RGB") as HxWx3 uint8 (Dassl's read_image); decoding stays on the host."""
    from PIL import Image
    out = []
    for p in paths:
        with Image.open(p) as im:
            out.append(np.asarray(im.convert("RGB"), dtype=np.uint8).copy())
    return out


def client_data_manager(client_id: int, classnames: List[str], ds: DatasetSplits, cfg, device, seed: int = 0):
    """ClientDataManager (trainers/client_datamanager.py:21-103) over a dataset's train_x / test: images
    decoded on the host, transformed on the device (DecodedClientDataManager), captions carried."""
    from .data import DecodedClientDataManager
    tr_imgs, te_imgs = decode_rgb([d.impath for d in ds.train_x]), decode_rgb([d.impath for d in ds.test])
    caps = lambda items: [d.caption if d.caption is not None else "" for d in items]
    return DecodedClientDataManager(client_id, classnames, tr_imgs, [d.label for d in ds.train_x], te_imgs,
                                    [d.label for d in ds.test], cfg.DATALOADER.TRAIN_X.BATCH_SIZE,
                                    cfg.DATALOADER.TEST.BATCH_SIZE, device, cfg=cfg, seed=seed,
                                    train_captions=caps(ds.train_x), test_captions=caps(ds.test))
