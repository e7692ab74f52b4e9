"""Diagnostic (GPU box): fp16(float(h) * 1.702f) on every finite fp16 h, as the compiler emits it (v_fma_mixlo_f16)
and forced through an fp32 product, against numpy's two roundings (fp32 product then fp16 = the reference's fp16
op) and one rounding (exact product to fp16).  Build: hipcc -O3 -shared -fPIC --offload-arch=gfx950 mix.hip -o libmix.so"""
import ctypes
from pathlib import Path

import numpy as np
import torch

lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libmix.so"))
lib.run_mix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int]
f = np.arange(65536, dtype=np.uint16).view(np.float16)
f = f[np.isfinite(f) & (np.abs(f.astype(np.float64)) < 30000)]
c = np.float32(1.702)
double = (f.astype(np.float32) * c).astype(np.float16)
single = (f.astype(np.float64) * np.float64(c)).astype(np.float16)
h = torch.from_numpy(f.copy()).cuda()
for which, name in ((0, "compiler (fma_mix)"), (1, "fp32 product forced")):
    o = torch.empty_like(h)
    assert lib.run_mix(h.data_ptr(), o.data_ptr(), h.numel(), 1.702, which) == 0
    g = o.cpu().numpy()
    print(f"{name:22s}: differs from two roundings on {int((g.view(np.uint16) != double.view(np.uint16)).sum())}, "
          f"from one rounding on {int((g.view(np.uint16) != single.view(np.uint16)).sum())} of {f.size} inputs")
