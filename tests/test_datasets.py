"""CPU tier: the clients' disk datasets and the class-union remap (federated_multi_modal_amd/datasets.py) on
small image trees written here, against the reference's rules (datasets/patternnet.py, ucmerced.py,
eurosat.py + dtd.py / oxford_pets.py split helpers, Dassl generate_fewshot_dataset,
trainers/maple_fed.py:48-159).  The reference's own datasets hold no image files (parity unpinned against
real data; the rules are restated)."""
import json
import os
import os.path as osp
import random

import numpy as np
import pytest

from federated_multi_modal_amd import datasets as D


def _write_tree(root, rel, classes, n, caption_dir=None, size=(20, 24)):
    from PIL import Image
    for ci, c in enumerate(classes):
        os.makedirs(osp.join(root, rel, c), exist_ok=True)
        if caption_dir:
            os.makedirs(osp.join(root, caption_dir, c), exist_ok=True)
        for k in range(n):
            arr = np.full((size[0], size[1], 3), (ci * 40 + k) % 256, dtype=np.uint8)
            Image.fromarray(arr).save(osp.join(root, rel, c, f"img_{k:03d}.jpg"), quality=95)
            if caption_dir and k % 3 != 2:  # some images without a caption file
                with open(osp.join(root, caption_dir, c, f"img_{k:03d}.txt"), "w") as f:
                    f.write(f"  a picture of {c} number {k}\n")


@pytest.fixture(scope="module")
def root(tmp_path_factory):
    r = str(tmp_path_factory.mktemp("data"))
    _write_tree(r, "PatternNet/images", ["forest", "parking_lot", "tennis_court"], 10, "PatternNet/Captions")
    _write_tree(r, "Ucmerced/Images", ["forest", "parkinglot", "tenniscourt", "beach"], 10, "Ucmerced/Captions")
    _write_tree(r, "eurosat/2750", ["AnnualCrop", "Forest"], 10, "eurosat/captions")
    # EuroSAT's captions are required for every image (datasets/eurosat.py:98-104)
    for c in ["AnnualCrop", "Forest"]:
        for k in range(10):
            with open(osp.join(r, "eurosat/captions", c, f"img_{k:03d}.txt"), "w") as f:
                f.write(f"eurosat {c} {k}")
    return r


def test_unshuffled_split_with_captions(root):
    ds = D.load_dataset("PatternNet", root)
    allitems = ds.train_x + ds.val + ds.test
    assert (len(ds.train_x), len(ds.val), len(ds.test)) == (15, 6, 9)  # int(0.5*30), int(0.2*30), rest
    # categories sorted, files in directory order, no shuffle: train holds the first classes only
    assert [d.classname for d in ds.train_x][:10] == ["forest"] * 10 and ds.test[-1].classname == "tennis_court"
    caps = {osp.basename(d.impath): d.caption for d in allitems if d.classname == "forest"}
    assert caps["img_000.jpg"] == "a picture of forest number 0" and caps["img_002.jpg"] is None
    # the split file round-trips (4-field rows, read back as the reference's read_split would want them)
    split = json.load(open(osp.join(root, "PatternNet", "patternnet.json")))
    assert len(split["train"][0]) == 4
    again = D.load_dataset("PatternNet", root)
    assert [(d.impath, d.label, d.classname, d.caption) for d in again.train_x] == \
           [(d.impath, d.label, d.classname, d.caption) for d in ds.train_x]


def test_eurosat_dtd_split_renames_and_captions(root):
    ds = D.load_dataset("EuroSAT", root, seed=3)
    assert sorted(set(d.classname for d in ds.train_x)) == ["Annual Crop Land", "Forest"]
    assert (len(ds.train_x), len(ds.val), len(ds.test)) == (10, 4, 6)  # per class round(5), round(2), rest
    assert all(d.caption.startswith("eurosat ") for d in ds.train_x + ds.val + ds.test)
    # the per-class shuffle is random.shuffle over the directory order
    rng = random.Random(3)
    ims = [osp.join(root, "eurosat/2750/AnnualCrop", f) for f in D.listdir_nohidden(osp.join(root, "eurosat/2750/AnnualCrop"))]
    rng.shuffle(ims)
    assert [d.impath for d in ds.train_x if d.label == 0] == ims[:5]


def test_fewshot_and_union_remap(root):
    ds = {n: D.load_dataset(n, root, num_shots=2, seed=1) for n in ("PatternNet", "Ucmerced", "EuroSAT")}
    assert all(sum(1 for d in ds["PatternNet"].train_x if d.label == y) == 2 for y in set(d.label for d in ds["PatternNet"].train_x))
    names, rm = D.union_and_remap(ds)
    assert names == sorted({"forest", "parking_lot", "tennis_court", "beach", "Annual Crop Land", "Forest"})
    g = {c: i for i, c in enumerate(names)}
    for d in rm["Ucmerced"].train_x + rm["Ucmerced"].test:
        assert names[d.label] == d.classname and d.classname in ("forest", "parking_lot", "tennis_court", "beach")
    assert {d.classname for d in rm["Ucmerced"].test} >= {"tennis_court"}
    assert all(d.label == g[d.classname] for d in rm["PatternNet"].train_x)
    assert rm["EuroSAT"] is ds["EuroSAT"]  # EuroSAT only contributes class names (trainers/maple_fed.py:119-125)
    imgs = D.decode_rgb([rm["PatternNet"].train_x[0].impath])
    assert imgs[0].shape == (20, 24, 3) and imgs[0].dtype == np.uint8
