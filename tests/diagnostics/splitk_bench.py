"""Diagnostic (GPU box): weight-gradient GEMM dW = dY^T X (both operands K-major, K = tokens) as one
K-major GEMM vs split-K (mf_gemm_splitk), on the MaPLe block-11 shapes; microseconds per call.
    python splitk_bench.py [comma list of split counts; 0 = splitk_auto]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    """per-call time of `reps` calls captured in one hipGraph (no host overhead), best of 3 replays"""
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


dev = torch.device("cuda:0")
for name, M, N, K in [("v.dW_fc", 3072, 768, 6368), ("v.dW_proj", 768, 3072, 6368), ("v.dW_qkv", 2304, 768, 6368),
                      ("v.dW_out", 768, 768, 6368), ("t.dW_fc", 2048, 512, 2926), ("t.dW_proj", 512, 2048, 2926),
                      ("t.dW_qkv", 1536, 512, 2926), ("t.dW_out", 512, 512, 2926)]:
    dY = torch.randn(K, M, device=dev).half()
    X = torch.randn(K, N, device=dev).half()
    C = torch.empty(M, N, device=dev, dtype=torch.float16)
    fl = 2.0 * M * N * K
    res = [f"kmajor {timeit(lambda: ops.gemm(dY, X, C, a_kmajor=True, b_kmajor=True)):5.1f}"]
    for sp in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,6,8").split(",")]:
        ws = torch.empty(ops.gemm_splitk_ws_floats(M, N, K, sp), device=dev)
        us = timeit(lambda: ops.gemm_splitk(dY, X, C, ws, splits=sp, a_kmajor=True, b_kmajor=True))
        res.append(f"s{sp} {us:5.1f}")
    print(f"{name:10s} " + "  ".join(res), flush=True)
