"""Diagnostic (GPU box): attention fwd/bwd kernel time, TFLOP/s, algorithmic GB/s and roofline
fraction on the MaPLe shapes (vision N=32 L=199 H=12; text K=38 L=77 H=8 causal; the caption path's
longer vision sequences, L=263 and 455; the C5 text tower, K=1000 L=77 H=8 causal; the eval engine's
100- and 400-image launches)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def timeit(fn, it=20):
    """Kernel time per call: `it` calls captured in one hipGraph and replayed (no host overhead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * it) * 1e3


dev = torch.device("cuda:0")
SHAPES = [(32, 199, 12, False), (38, 77, 8, True), (4, 199, 12, False), (10, 77, 8, True), (32, 263, 12, False),
          (32, 455, 12, False), (1000, 77, 8, True), (100, 199, 12, False), (400, 199, 12, False)]
if len(sys.argv) > 1:  # e.g. "0,7,8": a subset of SHAPES (the eval engine's 100 / 400-image launches are 7, 8)
    SHAPES = [SHAPES[int(i)] for i in sys.argv[1].split(",")]
for (N, L, H, causal) in SHAPES:
    D = H * 64
    torch.manual_seed(L + N)
    qkv = torch.randn(N * L, 3 * D, device=dev).half()
    out, lse = ops.attention_fwd(qkv, N, L, H, causal)
    dout = torch.randn(N * L, D, device=dev).half()
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(N * H * L, device=dev)
    q, k, v = qkv.view(N, L, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    mask = torch.full((L, L), float("-inf"), device=dev).triu(1) if causal else None
    ref = F.scaled_dot_product_attention(q.float(), k.float(), v.float(), attn_mask=mask)
    err = (out.float().view(N, L, H, 64).permute(0, 2, 1, 3) - ref).abs().max().item()
    # bit pattern checksums: variants (MAPFED_ATTN_FWD) that claim bit-identity must print the same
    ck = (out.view(torch.int16).long().sum().item(), lse.double().sum().item())
    tf = timeit(lambda: ops.attention_fwd(qkv, N, L, H, causal, out=out, lse=lse))
    tb = timeit(lambda: ops.attention_bwd(qkv, out, dout, lse, N, L, H, causal, dqkv=dqkv, ws=ws))
    ckb = dqkv.view(torch.int16).long().sum().item()  # backward variants claiming bit-identity print the same
    fl_f = 4.0 * N * H * L * L * 64 * (0.5 if causal else 1.0)
    fl_b = 2.5 * fl_f  # QK^T, dP = dO V^T, dV = P^T dO, dQ, dK (5 products vs 2)
    by_f = 2.0 * 4 * N * L * D
    by_b = 2.0 * (3 + 2 + 3) * N * L * D  # qkv, O, dO in; dqkv out
    roof_f = min(2.5e15, fl_f / by_f * 8e12)
    print(f"N={N} L={L} H={H} causal={causal}: fwd {tf:7.1f}us {fl_f / tf / 1e6:6.0f} TF "
          f"{by_f / tf / 1e3:6.0f} GB/s frac(roof {roof_f / 1e12:.0f} TF)={fl_f / tf / 1e6 / (roof_f / 1e12):.3f} "
          f"| bwd {tb:7.1f}us {fl_b / tb / 1e6:6.0f} TF {by_b / tb / 1e3:6.0f} GB/s | max err {err:.2e} ck {ck} ckb {ckb}", flush=True)
