"""Diagnostic: K-scaling of mf_gemm_nt (fixed cost vs main-loop cost) and torch.matmul (hipBLASLt)
on the same shapes, for reference only."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = torch.device("cuda:0")
tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 9]
for (M, N) in [(6368, 2304), (6368, 768), (6368, 3072)]:
    for K in [64, 256, 768, 3072]:
        A = torch.randn(M, K, device=dev).half()
        B = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        row = f"M={M} N={N} K={K:5d}: "
        for t in tiles:
            us = timeit(lambda: ops.gemm_nt(A, B, C=C, epilogue=ops.EPI_NONE, tile=t))
            row += f" t{t} {us:7.1f}us {2 * M * N * K / us / 1e6:6.0f}TF |"
        us = timeit(lambda: torch.matmul(A, B.t(), out=C))
        row += f" torch {us:7.1f}us {2 * M * N * K / us / 1e6:6.0f}TF"
        print(row, flush=True)
