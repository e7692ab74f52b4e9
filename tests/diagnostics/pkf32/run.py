"""Diagnostic (GPU box): packed vs scalar fp32 multiply / add on gfx950 (tests/diagnostics/pkf32/pkf32.hip; build:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC pkf32.hip -o libpkf32.so).  Prints the input classes where the
packed result differs from the scalar one."""
import ctypes
from pathlib import Path

import numpy as np
import torch

lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libpkf32.so"))
rng = np.random.default_rng(0)
n = 1 << 20
e = rng.uniform(-140, 10, size=(2, n))          # exponents from deep denormal to normal
a = (rng.choice([-1, 1], n) * rng.uniform(1, 2, n) * np.exp2(e[0])).astype(np.float32)
b = (rng.choice([-1, 1], n) * rng.uniform(1, 2, n) * np.exp2(e[1])).astype(np.float32)
ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
out = torch.empty(6 * n, device="cuda")
assert lib.pkf32_run(ctypes.c_void_p(ta.data_ptr()), ctypes.c_void_p(tb.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                     n, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
o = out.view(n, 6).cpu().numpy()
c = (-a * np.float32(1.7)).astype(np.float32)
tiny = np.float32(np.finfo(np.float32).tiny)
for name, s, p, ref in (("mul", o[:, 0], o[:, 1], (a.astype(np.float64) * b).astype(np.float32)),
                        ("add", o[:, 2], o[:, 3], (a.astype(np.float64) + b).astype(np.float32)),
                        ("fma", o[:, 4], o[:, 5], (a.astype(np.float64) * b + c).astype(np.float32))):
    d = s.view(np.uint32) != p.view(np.uint32)
    dref_s = s.view(np.uint32) != ref.view(np.uint32)
    dref_p = p.view(np.uint32) != ref.view(np.uint32)
    den_in = (np.abs(a) < tiny) | (np.abs(b) < tiny)
    den_out = np.abs(ref) < tiny
    print(f"{name}: packed != scalar at {int(d.sum())} of {n}; scalar != numpy {int(dref_s.sum())}, packed != numpy "
          f"{int(dref_p.sum())}; of the packed/scalar differences: denormal input {int((d & den_in).sum())}, "
          f"denormal result {int((d & den_out).sum())}, neither {int((d & ~den_in & ~den_out).sum())}", flush=True)
    idx = np.nonzero(d)[0][:4]
    for i in idx:
        print(f"   a={a[i]!r} b={b[i]!r} scalar={s[i]!r} packed={p[i]!r} numpy={ref[i]!r}")
