"""Diagnostic (GPU box): the fused in-projection + attention forward (mf_qkv_attention_fwd) against the two
launches it replaces (mf_gemm_nt EPI_BIAS + mf_attention_fwd), on the c4 vision shape (N=32 L=199 H=12),
the c4 text shape (K=38 L=77 H=8 causal) and the C5 text shape (K=1000).  Times are per call from a
replayed hipGraph of 20 calls; every result is checked bit for bit against the unfused pair."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from attn_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
for (N, L, H, causal) in [(32, 199, 12, False), (38, 77, 8, True), (1000, 77, 8, True), (4, 199, 12, False)]:
    D = H * 64
    g = torch.Generator(device="cpu").manual_seed(N + L)
    x = torch.randn(N * L, D, generator=g).half().to(dev)
    W = (torch.randn(3 * D, D, generator=g) * D ** -0.5).half().to(dev)
    b = (torch.randn(3 * D, generator=g) * 0.02).half().to(dev)
    qkv_u = torch.empty(N * L, 3 * D, device=dev, dtype=torch.float16)
    o_u = torch.empty(N * L, D, device=dev, dtype=torch.float16)
    lse_u = torch.empty(N * H * L, device=dev)
    qkv_f, o_f, lse_f = torch.empty_like(qkv_u), torch.empty_like(o_u), torch.empty_like(lse_u)

    def unfused():
        ops.gemm_nt(x, W, qkv_u, bias=b, epilogue=ops.EPI_BIAS)
        ops.attention_fwd(qkv_u, N, L, H, causal, out=o_u, lse=lse_u)

    def fused():
        ops.qkv_attention_fwd(x, W, b, qkv_f, o_f, lse_f, N, L, H, causal)

    tg = timeit(lambda: ops.gemm_nt(x, W, qkv_u, bias=b, epilogue=ops.EPI_BIAS))
    tu = timeit(unfused)
    tf = timeit(fused)
    same = torch.equal(qkv_u, qkv_f) and torch.equal(o_u, o_f) and torch.equal(lse_u, lse_f)
    pairs = L * (L + 1) / 2 if causal else L * L
    flops = 2.0 * N * L * 3 * D * D + 4.0 * N * H * pairs * 64
    print(f"N={N} L={L} H={H} causal={causal}: in_proj {tg:6.1f}us  unfused {tu:6.1f}us ({flops / tu / 1e6:5.0f} TF)"
          f"  fused {tf:6.1f}us ({flops / tf / 1e6:5.0f} TF = {flops / tf / 1e6 / 2500:.3f} of the fp16 MFMA peak)"
          f"  bit-identical {same}", flush=True)
