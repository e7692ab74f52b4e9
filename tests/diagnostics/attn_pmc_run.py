"""Diagnostic (GPU box): eager attention launches on the c4 shapes for PMC passes
(scripts/attn_pmc.sh -> tests/diagnostics/attn_pmc_summary.py).  Vision N=32 L=199 H=12 and text
K=38 L=77 H=8 causal, forward and backward, and the fused in-projection + attention forward
(qkv_attn_fwd_kernel), 5 launches each after one warm-up; no hipGraph, so every
dispatch is seen by the counter collection."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for (N, L, H, causal) in [(32, 199, 12, False), (38, 77, 8, True)]:
    D = H * 64
    torch.manual_seed(L + N)
    qkv = torch.randn(N * L, 3 * D, device=dev).half()
    out, lse = ops.attention_fwd(qkv, N, L, H, causal)
    dout = torch.randn(N * L, D, device=dev).half()
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(N * H * L, device=dev)
    x = torch.randn(N * L, D, device=dev).half()
    W = (torch.randn(3 * D, D, device=dev) * D ** -0.5).half()
    b = (torch.randn(3 * D, device=dev) * 0.02).half()
    for _ in range(6):
        ops.attention_fwd(qkv, N, L, H, causal, out=out, lse=lse)
        ops.attention_bwd(qkv, out, dout, lse, N, L, H, causal, dqkv=dqkv, ws=ws)
        ops.qkv_attention_fwd(x, W, b, qkv, out, lse, N, L, H, causal)  # the fused in-projection + attention
    torch.cuda.synchronize()
    print(f"N={N} L={L} H={H} causal={causal}: done", flush=True)
