"""Diagnostic (GPU box): time lnbwd.hip's ln_bwd2 copy with parts switched off (MODE bits, see the .hip) at the
c4 vision shape, next to a same-traffic addcmul.  Build first (CPU box):
    hipcc -O3 -shared -fPIC --offload-arch=gfx950 lnbwd.hip -o liblnb.so
"""
import ctypes
import sys
from pathlib import Path

import torch

here = Path(__file__).resolve().parent
lib = ctypes.CDLL(str(here / "liblnb.so"))
P = ctypes.c_void_p
lib.lnb_launch.argtypes = [ctypes.c_int, P, P, P, P, P, P, P, P, P, ctypes.c_int, P]
dev = torch.device("cuda:0")


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e3)
    return best


rows = int(sys.argv[1]) if len(sys.argv) > 1 else 6368
D = 768
torch.manual_seed(0)
x, dy, dres = (torch.randn(rows, D, device=dev).half() for _ in range(3))
gamma = 1 + 0.1 * torch.randn(D, device=dev)
mean = torch.randn(rows, device=dev) * 0.1
rstd = 1 + torch.rand(rows, device=dev)
dx = torch.empty_like(x)
nb = (rows + 15) // 16
dg = torch.empty(nb, D, device=dev)
db = torch.empty(nb, D, device=dev)


def run(mode):
    st = torch.cuda.current_stream().cuda_stream
    rc = lib.lnb_launch(mode, dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                        dres.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), rows, st)
    assert rc == 0, rc


names = {0: "full", 1: "no gamma", 2: "no LDS reduce", 4: "no dx store", 8: "no dres load", 6: "no reduce+store",
         15: "loads of x,dy only", 16: "nt dx stores", 64: "x+dy+dres same shape",
         128: "1 row / half-wave", 144: "1 row / half-wave, nt"}
print(f"rows={rows}: addcmul (3 reads + 1 write) {timeit(lambda: torch.addcmul(x, dy, dres, out=dx)):.2f} us", flush=True)
for m in (0, 64, 16, 128, 144, 0, 128):
    print(f"  mode {m:3d} {names[m]:22s} {timeit(lambda: run(m)):6.2f} us", flush=True)
# bit-identity of the candidates against mode 0 (dx and the dgamma / dbeta partials)
outs = {}
for m in (0, 16, 128, 144):
    dx.zero_(), dg.zero_(), db.zero_()
    run(m)
    torch.cuda.synchronize()
    outs[m] = (dx.clone(), dg.clone(), db.clone())
for m in (16, 128, 144):
    print(f"  mode {m:3d} bit-identical to mode 0: " + ", ".join(
        f"{n} {torch.equal(a.view(torch.int16) if a.dtype == torch.float16 else a.view(torch.int32), b.view(torch.int16) if b.dtype == torch.float16 else b.view(torch.int32))}"
        for n, a, b in zip(("dx", "dg", "db"), outs[m], outs[0])), flush=True)

# ---- LayerNorm forward candidates (lnfwd.hip -> liblnf.so)
fl = ctypes.CDLL(str(here / "liblnf.so"))
fl.lnf_launch.argtypes = [ctypes.c_int, P, P, P, P, P, P, ctypes.c_int, P]
beta = 0.1 * torch.randn(D, device=dev)
y = torch.empty_like(x)
mo, ro = torch.empty(rows, device=dev), torch.empty(rows, device=dev)


def runf(mode):
    rc = fl.lnf_launch(mode, x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), mo.data_ptr(),
                       ro.data_ptr(), rows, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


print(f"rows={rows}: copy (1 read + 1 write) {timeit(lambda: y.copy_(x)):.2f} us", flush=True)
for m in (0, 1, 2, 0, 1):
    print(f"  fwd mode {m} {('library', 'gamma/beta in LDS', 'no gamma/beta')[m]:18s} {timeit(lambda: runf(m)):6.2f} us",
          flush=True)
fo = {}
for m in (0, 1):
    y.zero_(), mo.zero_(), ro.zero_()
    runf(m)
    torch.cuda.synchronize()
    fo[m] = (y.view(torch.int16).clone(), mo.view(torch.int32).clone(), ro.view(torch.int32).clone())
print("  fwd mode 1 bit-identical to mode 0:", [torch.equal(a, b) for a, b in zip(fo[0], fo[1])], flush=True)
