"""Image transforms: the device `mf_augment` path against the oracle's
restatement of Pillow's resampling + torchvision's transforms, and the oracle against Pillow itself.

Bar: bit-exact (uint8 resampling is integer arithmetic; ToTensor/Normalize are correctly rounded
fp32 ops; the fp16 output is the RNE cast of the fp32 value).  Pillow is importable here and on the
GPU box (third-party, 12.2); torchvision is not, so its crop sampler is pinned only against the
oracle's restatement ("parity unpinned" against torchvision itself).
"""
import ctypes

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import transforms_oracle as T

MEAN = (0.48145466, 0.4578275, 0.40821073)
STD = (0.26862954, 0.26130258, 0.27577711)
PIL_INTERP = {"bicubic": Image.BICUBIC, "bilinear": Image.BILINEAR}


def _images(seed, shapes):
    rng = np.random.default_rng(seed)
    out = []
    for H, W in shapes:
        # smooth gradients + noise: exercises both the clipping and the interior of the taps
        yy, xx = np.mgrid[0:H, 0:W]
        base = (np.stack([xx * 255.0 / max(W - 1, 1), yy * 255.0 / max(H - 1, 1), (xx + yy) % 256], -1))
        noise = rng.integers(-60, 61, (H, W, 3))
        out.append(np.clip(base + noise, 0, 255).astype(np.uint8))
    return out


SHAPES = [(256, 256), (64, 64), (375, 500), (500, 333), (224, 224), (37, 51), (900, 1200), (1, 224)]


# ---- oracle pinned against Pillow -------------------------------------------------------------------

@pytest.mark.parametrize("interp", ["bicubic", "bilinear"])
def test_oracle_resize_matches_pillow(interp):
    rng = np.random.default_rng(1)
    cases = [(256, 256, 224, 224), (64, 64, 224, 224), (375, 500, 224, 298), (900, 1200, 224, 224),
             (10, 7, 3, 19), (224, 224, 224, 224), (1, 5, 4, 4), (300, 40, 224, 29)]
    cases += [tuple(int(v) for v in rng.integers(1, 320, 4)) for _ in range(12)]
    for H, W, oh, ow in cases:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        ref = np.asarray(Image.fromarray(img).resize((ow, oh), PIL_INTERP[interp]))
        np.testing.assert_array_equal(T.resize(img, oh, ow, interp), ref, err_msg=f"{(H, W, oh, ow)}")


def test_oracle_train_and_test_transform_match_pillow_pipeline():
    gen = torch.Generator().manual_seed(3)
    for img in _images(2, SHAPES[:6]):
        H, W, _ = img.shape
        i, j, h, w = T.rrc_get_params(H, W, gen)
        for flip in (False, True):
            p = Image.fromarray(img).crop((j, i, j + w, i + h)).resize((224, 224), Image.BICUBIC)
            if flip:
                p = p.transpose(Image.FLIP_LEFT_RIGHT)
            ref = T.to_tensor_normalize(np.asarray(p), MEAN, STD)
            np.testing.assert_array_equal(T.train_transform(img, i, j, h, w, flip, MEAN, STD), ref)
        rh, rw = T.resize_short_side(H, W, 224)
        p = Image.fromarray(img).resize((rw, rh), Image.BICUBIC)
        oy, ox = T.center_crop_offsets(rh, rw, 224, 224)
        ref = T.to_tensor_normalize(np.asarray(p)[oy:oy + 224, ox:ox + 224], MEAN, STD)
        np.testing.assert_array_equal(T.test_transform(img, MEAN, STD), ref)


# ---- host logic (no GPU) --------------------------------------------------------------------------------

def test_host_crop_sampler_and_sizes_follow_torchvision_restatement():
    from federated_multi_modal_amd import transforms as D
    for seed in range(5):
        g1, g2 = torch.Generator().manual_seed(seed), torch.Generator().manual_seed(seed)
        for H, W in SHAPES:
            assert D.rrc_get_params(H, W, g1) == T.rrc_get_params(H, W, g2)
            assert D.resize_short_side(H, W, 224) == T.resize_short_side(H, W, 224)
    # the ten-attempt fallback: a 1x224 strip can never hold a 3/4..4/3 crop of >= 8 % of its area
    i, j, h, w = D.rrc_get_params(1, 224, torch.Generator().manual_seed(0))
    assert (h, w) == (1, 1) and i == 0 and j == 111


def test_geometry_rows_and_config_surface():
    from types import SimpleNamespace
    from federated_multi_modal_amd import transforms as D
    cfg = SimpleNamespace(INPUT=SimpleNamespace(SIZE=(224, 224), INTERPOLATION="bicubic", PIXEL_MEAN=list(MEAN),
                                                PIXEL_STD=list(STD),
                                                TRANSFORMS=["random_resized_crop", "random_flip", "normalize"]))
    tr = D.build_transform(cfg, True, torch.Generator().manual_seed(0))
    te = D.build_transform(cfg, False)
    g = tr.geometry(SHAPES)
    assert g.shape == (len(SHAPES), 11) and set(g[:, 10]) <= {0, 1}
    assert np.all(g[:, 2] + g[:, 4] <= g[:, 0]) and np.all(g[:, 3] + g[:, 5] <= g[:, 1])
    gt = te.geometry([(375, 500)])
    assert gt.tolist() == [[375, 500, 0, 0, 375, 500, 224, 298, 0, 37, 0]]
    with pytest.raises(NotImplementedError):
        D.build_transform(SimpleNamespace(INPUT=SimpleNamespace(TRANSFORMS=["colorjitter"])), True)


def test_abi_validates_geometry_before_any_launch():
    from federated_multi_modal_amd import _lib
    h = _lib.lib()
    geom = np.array([[64, 64, 10, 0, 60, 64, 224, 224, 0, 0, 0]], np.int32)  # crop rows 10..70 > 64
    off = np.zeros(1, np.int64)
    fake = ctypes.c_void_p(16)
    rc = h.mf_augment(fake, 64 * 64 * 3, off.ctypes.data_as(ctypes.c_void_p), fake,
                      geom.ctypes.data_as(ctypes.c_void_p), 1, 224, 224, 0, 0, 0, 0, 1, 1, 1, fake, 1, fake,
                      1 << 30, None)
    assert rc != 0 and b"crop box" in h.mf_last_error()
    geom = np.array([[4000, 4000, 0, 0, 4000, 4000, 224, 224, 0, 0, 0]], np.int32)  # 17.9x downscale
    rc = h.mf_augment(fake, 4000 * 4000 * 3, off.ctypes.data_as(ctypes.c_void_p), fake,
                      geom.ctypes.data_as(ctypes.c_void_p), 1, 224, 224, 0, 0, 0, 0, 1, 1, 1, fake, 1, fake,
                      1 << 30, None)
    assert rc != 0 and b"downscale" in h.mf_last_error()
    assert h.mf_augment_ws_bytes(0, 224, 224, 1) < 0


# ---- device path against the oracle (bit-exact) ------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("path", ["fused", "3pass"])
@pytest.mark.parametrize("interp", ["bicubic", "bilinear"])
def test_device_train_transform_bit_exact(dev, interp, path):
    """Both device paths: the fused one-launch kernel, and the three-launch path mf_augment takes when a batch's
    taps + band rows exceed the fused kernel's 64 KB of LDS (whole-image crops downscaled 12x bicubic / 20x
    bilinear: 49 / 41 taps per output index, augment.hip)."""
    from federated_multi_modal_amd import transforms as D
    if path == "3pass":
        side = 2688 if interp == "bicubic" else 4480
        imgs = _images(5, [(side, side - 64), (side - 32, side)])
    else:
        imgs = _images(5, SHAPES)
    packed = D.pack_images(imgs, dev)
    tr = D.DeviceTransform(True, 224, interp, MEAN, STD, out_dtype=torch.float32,
                           generator=torch.Generator().manual_seed(7))
    geom = tr.geometry(packed.shapes)
    if path == "3pass":  # whole-image crops resized straight to 224 x 224
        for b, img in enumerate(imgs):
            H, W = img.shape[:2]
            geom[b] = np.array([H, W, 0, 0, H, W, 224, 224, 0, 0, b % 2], np.int32)
    geom[1, 10] = 1  # make sure both flip states are covered
    geom[0 if path == "3pass" else 2, 10] = 0
    out32 = tr(packed, geom).cpu().numpy()
    tr16 = D.DeviceTransform(True, 224, interp, MEAN, STD, out_dtype=torch.float16)
    out16 = tr16(packed, geom).cpu()
    for b, img in enumerate(imgs):
        H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip = geom[b].tolist()
        crop = img[y0:y0 + ch, x0:x0 + cw]
        r = T.resize(crop, 224, 224, interp)
        if flip:
            r = r[:, ::-1]
        ref = T.to_tensor_normalize(r, MEAN, STD)
        np.testing.assert_array_equal(out32[b], ref, err_msg=f"image {b} {geom[b].tolist()}")
        assert torch.equal(out16[b], torch.from_numpy(ref).half()), b


@pytest.mark.gpu
def test_device_test_transform_bit_exact_against_pillow(dev):
    from federated_multi_modal_amd import transforms as D
    imgs = _images(6, SHAPES)
    packed = D.pack_images(imgs, dev)
    te = D.DeviceTransform(False, 224, "bicubic", MEAN, STD, out_dtype=torch.float32)
    out = te(packed).cpu().numpy()
    for b, img in enumerate(imgs):
        H, W, _ = img.shape
        rh, rw = T.resize_short_side(H, W, 224)
        p = np.asarray(Image.fromarray(img).resize((rw, rh), Image.BICUBIC))
        oy, ox = T.center_crop_offsets(rh, rw, 224, 224)
        ref = T.to_tensor_normalize(p[oy:oy + 224, ox:ox + 224], MEAN, STD)
        np.testing.assert_array_equal(out[b], ref, err_msg=f"image {b} {img.shape}")


@pytest.mark.gpu
def test_device_transform_feeds_the_engine_batch(dev):
    """The fp16 transform output is the engine's image buffer layout ([B,3,224,224] fp16, contiguous)."""
    from federated_multi_modal_amd import transforms as D
    imgs = _images(8, [(256, 256)] * 4)
    packed = D.pack_images(imgs, dev)
    out = torch.empty(4, 3, 224, 224, device=dev, dtype=torch.float16)
    r = D.DeviceTransform(True, generator=torch.Generator().manual_seed(1))(packed, out=out)
    torch.cuda.synchronize()
    assert r.data_ptr() == out.data_ptr() and torch.isfinite(out.float()).all()
    assert D.DeviceTransform(True)(D.pack_images([], dev)).shape == (0, 3, 224, 224)


@pytest.mark.gpu
def test_decoded_client_data_manager_batches_match_oracle(dev):
    """The loader over decoded images: train batches equal the oracle's transform at the geometry the
    loader drew; test batches equal Resize + CenterCrop + Normalize; labels follow the sampled indices."""
    from federated_multi_modal_amd.data import DecodedClientDataManager
    shapes = [(256, 256), (300, 200), (64, 64), (480, 640), (224, 224), (250, 260)]
    imgs = _images(9, shapes)
    labels = [0, 1, 2, 0, 1, 2]
    dm = DecodedClientDataManager(0, ["a", "b", "c"], imgs, labels, imgs[:3], labels[:3], train_batch=4,
                                  test_batch=2, device=dev)
    assert len(dm.train_loader) == 1 and len(dm.test_loader) == 2
    for batch in dm.train_loader:
        img = batch["img"].cpu().numpy()
        assert img.dtype == np.float32 and img.shape == (4, 3, 224, 224)
        for r, k in enumerate(batch["index"].tolist()):
            H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip = batch["geom"][r].tolist()
            ref = T.train_transform(imgs[k], y0, x0, ch, cw, bool(flip), MEAN, STD)
            np.testing.assert_array_equal(img[r], ref)
            assert int(batch["label"][r]) == labels[k]
    seen = 0
    for batch in dm.test_loader:
        img = batch["img"].cpu().numpy()
        for r, k in enumerate(batch["index"].tolist()):
            np.testing.assert_array_equal(img[r], T.test_transform(imgs[k], MEAN, STD))
            seen += 1
    assert seen == 3


@pytest.mark.gpu
def test_device_transform_extreme_downscale_falls_back_bit_exact(dev):
    """A 3400x3400 image resized whole to 224 (63 taps per output index): too many taps for the fused
    kernel's LDS, so the three-launch path runs; mixed in one batch with an ordinary image."""
    from federated_multi_modal_amd import transforms as D
    imgs = _images(11, [(3400, 3400), (256, 256)])
    packed = D.pack_images(imgs, dev)
    geom = np.array([[3400, 3400, 0, 0, 3400, 3400, 224, 224, 0, 0, 1],
                     [256, 256, 16, 8, 200, 240, 224, 224, 0, 0, 0]], np.int32)
    out = D.DeviceTransform(True, out_dtype=torch.float32)(packed, geom).cpu().numpy()
    for b, img in enumerate(imgs):
        H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip = geom[b].tolist()
        ref = T.train_transform(img, y0, x0, ch, cw, bool(flip), MEAN, STD)
        np.testing.assert_array_equal(out[b], ref, err_msg=f"image {b}")


@pytest.mark.gpu
def test_device_train_transform_small_images_bit_exact(dev):
    """PatternNet / EuroSAT-size images (and ragged small ones) through the fused kernel: bit-exact."""
    from federated_multi_modal_amd import transforms as D
    shapes = [(256, 256), (64, 64), (224, 224), (37, 51), (250, 200), (256, 256)]
    imgs = _images(12, shapes)
    packed = D.pack_images(imgs, dev)
    tr = D.DeviceTransform(True, out_dtype=torch.float32, generator=torch.Generator().manual_seed(4))
    geom = tr.geometry(packed.shapes)
    geom[0, 10], geom[1, 10] = 1, 0
    out = tr(packed, geom).cpu().numpy()
    for b, img in enumerate(imgs):
        H, W, y0, x0, ch, cw, RH, RW, oy, ox, flip = geom[b].tolist()
        ref = T.train_transform(img, y0, x0, ch, cw, bool(flip), MEAN, STD)
        np.testing.assert_array_equal(out[b], ref, err_msg=f"image {b} {geom[b].tolist()}")
