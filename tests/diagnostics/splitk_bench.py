"""Diagnostic (GPU box): weight-gradient GEMM dW = dY^T X (both operands K-major, K = tokens) as one
K-major GEMM vs split-K (mf_gemm_splitk), on the MaPLe block-11 shapes."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


dev = torch.device("cuda:0")
for name, M, N, K in [("v.dW_fc", 3072, 768, 6368), ("v.dW_proj", 768, 3072, 6368), ("v.dW_qkv", 2304, 768, 6368),
                      ("v.dW_out", 768, 768, 6368), ("t.dW_fc", 2048, 512, 2926), ("t.dW_out", 512, 512, 2926)]:
    dY = torch.randn(K, M, device=dev).half()
    X = torch.randn(K, N, device=dev).half()
    C = torch.empty(M, N, device=dev, dtype=torch.float16)
    fl = 2.0 * M * N * K
    res = [f"kmajor {fl / timeit(lambda: ops.gemm(dY, X, C, a_kmajor=True, b_kmajor=True)) / 1e6:6.0f}"]
    for sp in (0, 1, 2, 3, 4, 6, 8):
        ws = torch.empty(ops.gemm_splitk_ws_floats(M, N, K, sp), device=dev)
        us = timeit(lambda: ops.gemm_splitk(dY, X, C, ws, splits=sp, a_kmajor=True, b_kmajor=True))
        res.append(f"s{sp} {fl / us / 1e6:6.0f} ({us:5.1f}us)")
    print(f"{name:10s} " + "  ".join(res), flush=True)
