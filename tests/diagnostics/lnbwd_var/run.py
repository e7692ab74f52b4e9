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
         15: "loads of x,dy only", 16: "nt dx stores", 64: "x+dy+dres same shape"}
print(f"rows={rows}: addcmul (3 reads + 1 write) {timeit(lambda: torch.addcmul(x, dy, dres, out=dx)):.2f} us", flush=True)
for m in (0, 64, 16, 2, 4, 8, 0):
    print(f"  mode {m:2d} {names[m]:20s} {timeit(lambda: run(m)):6.2f} us", flush=True)
