"""CPU tier: the fp16 reproducibility floor of the reference's logits (why the GPU parity gate on the
max logit error is 4e-3 and the 1e-3 gate is applied to the mean).

The reference runs every GEMM in fp16 with the CPU library's own fp32 summation order.  Re-running
the oracle (bit-identical to the reference, tests/test_oracle_golden.py) with ONLY the projection
GEMMs changed to the correctly rounded result — a strictly more accurate GEMM, no other change —
moves the C1 logits by several fp16 ulps.  Any implementation whose GEMMs sum in a different
order (every GPU kernel) inherits this floor."""
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

from federated_multi_modal_amd import synthetic as syn
from oracle import maple_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"


def _block_exact_gemm(x, P, pre, n_head, mask, f32):
    """oracle._block with every nn.Linear correctly rounded (float64 accumulate, one fp16 rounding)."""
    lin = lambda t, w, b: (t.double() @ w.double().t() + b.double()).to(t.dtype)
    Lq, N, D = x.shape
    h1 = O._ln(x, P[pre + "ln_1.weight"], P[pre + "ln_1.bias"], f32)
    qkv = lin(h1, P[pre + "attn.in_proj_weight"], P[pre + "attn.in_proj_bias"])
    q, k, v = qkv.unflatten(-1, (3, D)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
    hd = D // n_head
    f = lambda t: t.view(Lq, N * n_head, hd).transpose(0, 1).view(N, n_head, Lq, hd)
    m = None if mask is None else mask.to(x.dtype).view(1, 1, Lq, Lq)
    a = F.scaled_dot_product_attention(f(q), f(k), f(v), attn_mask=m)
    a = a.permute(2, 0, 1, 3).contiguous().view(Lq * N, D)
    x = x + lin(a, P[pre + "attn.out_proj.weight"], P[pre + "attn.out_proj.bias"]).view(Lq, N, D)
    h = O._ln(x, P[pre + "ln_2.weight"], P[pre + "ln_2.bias"], f32)
    h = O._quick_gelu(lin(h, P[pre + "mlp.c_fc.weight"], P[pre + "mlp.c_fc.bias"]))
    return x + lin(h, P[pre + "mlp.c_proj.weight"], P[pre + "mlp.c_proj.bias"])


def test_reference_logits_floor_under_exact_gemms(monkeypatch):
    g = np.load(GOLD / "c1_maple.npz")
    J, K, B, seed = int(g["J"]), int(g["K"]), int(g["B"]), int(g["seed"])
    M = O.build_model(seed, J, syn.synthetic_classnames(K, seed))
    img = torch.from_numpy(syn.client_batch(seed, 0, 0, B, K).images)
    monkeypatch.setattr(O, "_block", _block_exact_gemm)
    with torch.no_grad():
        lg = O.forward(M, img, train=False).float().numpy()
    d = np.abs(lg - g["logits"])
    print(f"exact-GEMM reference vs reference: max {d.max():.2e} mean {d.mean():.2e}")
    assert d.max() > 1e-3          # the 1e-3 max gate is below the floor ...
    assert d.max() <= 4e-3         # ... and the 4e-3 gate sits just above it
    assert d.mean() <= 1e-3
    assert np.array_equal(lg.argmax(1), g["logits"].argmax(1))
