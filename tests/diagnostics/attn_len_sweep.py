"""Diagnostic (GPU box): attention fwd / bwd time against the sequence length at the c4 head count (N = 32, H = 12):
where the 32-row padding of the backward (L = 199 -> 224) costs."""
import sys, torch
sys.path.insert(0, ".")
from federated_multi_modal_amd import ops
dev = torch.device("cuda:0")
def timeit(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it): fn()
    g.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record(); g.replay(); e.record(); torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / it * 1e3)
    return best
N, H = 32, 12
for L in (176, 192, 193, 199, 208, 224):
    qkv = (torch.randn(N * L, 3 * H * 64, device=dev) * 0.5).half()
    o, lse = ops.attention_fwd(qkv, N, L, H, False)
    do = torch.randn(N * L, H * 64, device=dev).half()
    tf = timeit(lambda: ops.attention_fwd(qkv, N, L, H, False, out=o, lse=lse))
    tb = timeit(lambda: ops.attention_bwd(qkv, o, do, lse, N, L, H, False))
    print(f"L={L}: fwd {tf:6.2f} us  bwd {tb:6.2f} us  (bwd per row^2 {tb / L / L * 1e3:.3f} ns)", flush=True)
