"""Diagnostic (GPU box): LayerNorm fwd / bwd time and algorithmic GB/s on the MaPLe shapes
(vision 6368 x 768, text 2926 x 512).  MAPFED_LN=1 selects the wave-per-row kernels."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
for rows, D in [(6368, 768), (2926, 512)]:
    x = torch.randn(rows, D, device=dev).half()
    g = torch.rand(D, device=dev) + 0.5
    b = torch.randn(D, device=dev) * 0.1
    y, mean, rstd = ops.layernorm_fwd(x, g, b)
    dy = torch.randn(rows, D, device=dev).half()
    dres = torch.randn(rows, D, device=dev).half()
    dx = torch.empty_like(x)
    dg = torch.empty(D, device=dev)
    db = torch.empty(D, device=dev)
    ws = torch.empty(ops.layernorm_ws_floats(rows, D), device=dev)
    tf = timeit(lambda: ops.layernorm_fwd(x, g, b, y, mean, rstd))
    tb = timeit(lambda: ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dg, db, workspace=ws, dres=dres))
    print(f"rows={rows} D={D}: fwd {tf:6.2f} us {4 * rows * D / tf / 1e3:6.0f} GB/s | "
          f"bwd (+dres, dgamma/dbeta) {tb:6.2f} us {8 * rows * D / tb / 1e3:6.0f} GB/s", flush=True)
