"""Diagnostic (GPU box): the device train transform (mf_augment) on B decoded 256x256 RGB images,
fused one-launch path, timed with HIP events on the
launching stream.  Run under `rocprofv3 --kernel-trace --stats` for the per-kernel durations.

    python augment_bench.py [B]
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import transforms as T  # noqa: E402


def run(B, label, reps=50):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    packed = T.pack_images([rng.integers(0, 256, (256, 256, 3), dtype=np.uint8) for _ in range(B)], dev)
    tfm = T.DeviceTransform(True, generator=torch.Generator().manual_seed(0))
    out = torch.empty(B, 3, 224, 224, device=dev, dtype=torch.float16)
    geoms = [tfm.geometry(packed.shapes) for _ in range(reps)]
    tfm(packed, geoms[0], out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for g in geoms:
        tfm(packed, g, out=out)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    nbytes = float(np.mean([(g[:, 4] * g[:, 5] * 3).sum() for g in geoms])) + B * 3 * 224 * 224 * 2
    print(f"{label:6s} B={B}: {us:7.1f} us/batch  {B / us * 1e6:10.0f} img/s  {nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    run(B, "fused")
    run(4 * B, "fused")
    # (the three-launch path runs only where the fused kernel's LDS is too small: downscale beyond ~6x)
