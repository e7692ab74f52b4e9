"""Diagnostic (GPU box): LayerNorm forward / backward kernel time (hipGraph-timed) and algorithmic
GB/s on the c4 shapes (vision 6368 x 768, text 2926 x 512), with bit-pattern checksums so variants (two
builds of the library) that claim bit-identity can be compared across runs."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def timeit(fn, reps=20):
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
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * reps) * 1e3


dev = torch.device("cuda:0")
for rows, D in [(6368, 768), (2926, 512), (796, 768), (770, 512)]:
    torch.manual_seed(rows)
    x = torch.randn(rows, D, device=dev).half()
    dy = torch.randn(rows, D, device=dev).half()
    dres = torch.randn(rows, D, device=dev).half()
    gamma = 1 + 0.1 * torch.randn(D, device=dev)
    beta = 0.1 * torch.randn(D, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    dx = torch.empty_like(x)
    ws = torch.empty(ops.layernorm_ws_floats(rows, D), device=dev)
    dg = torch.empty(D, device=dev)
    db = torch.empty(D, device=dev)
    tf = timeit(lambda: ops.layernorm_fwd(x, gamma, beta, y, mean, rstd))
    tb = timeit(lambda: ops.layernorm_bwd(dy, x, gamma, mean, rstd, dx, dg, db, workspace=ws, dres=dres))
    ref = torch.nn.functional.layer_norm(x.float(), (D,), gamma, beta, 1e-5)
    err = (y.float() - ref).abs().max().item()
    ck = (y.view(torch.int16).long().sum().item(), dx.view(torch.int16).long().sum().item(), dg.double().sum().item())
    bf, bb = 4.0 * rows * D, 8.0 * rows * D
    # same-traffic streaming yardsticks: a copy (fwd's read + write) and addcmul (bwd's three reads + write)
    tc = timeit(lambda: y.copy_(x))
    ta = timeit(lambda: torch.addcmul(x, dy, dres, out=dx))
    print(f"rows={rows} D={D}: fwd {tf:6.2f} us {bf / tf / 1e3:6.0f} GB/s (copy {tc:6.2f} us) | bwd {tb:6.2f} us "
          f"{bb / tb / 1e3:6.0f} GB/s (addcmul {ta:6.2f} us) | max err {err:.2e} ck {ck}", flush=True)
