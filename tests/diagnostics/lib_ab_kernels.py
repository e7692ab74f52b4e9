"""Diagnostic (GPU box): the same op on the same inputs through two builds of libmapfed.so in one process, outputs
compared bit for bit -- which kernels does a build change compute differently? (r06: the library with and without
packed fp32 VALU ops gave different step digests although v_pk_mul_f32 / v_pk_add_f32 match the scalar ops on
every input class in isolation, tests/diagnostics/pkf32/run.py.)

    python tests/diagnostics/lib_ab_kernels.py <libA.so> <libB.so>
"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import _lib, ops  # noqa: E402

libs = []
for p in sys.argv[1:3]:
    _lib._LIB = None
    os.environ["MAPFED_LIB"] = p
    libs.append(_lib.lib())
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(11)


def rnd(*s, scale=1.0, dt=torch.float16):
    return (torch.randn(*s, generator=g) * scale).to(dt).to(dev)


def both(fn):
    """fn() -> tensor or tuple of tensors, run once per library (outputs cloned)"""
    outs = []
    for h in libs:
        _lib._LIB = h
        o = fn()
        torch.cuda.synchronize()
        o = o if isinstance(o, (tuple, list)) else (o,)
        outs.append([t.clone() for t in o])
    return outs


def report(name, outs):
    a, b = outs
    diffs = []
    for i, (x, y) in enumerate(zip(a, b)):
        d = x.view(-1) != y.view(-1)
        if d.any():
            idx = int(d.nonzero()[0])
            diffs.append(f"out{i}: {int(d.sum())}/{d.numel()} differ, e.g. [{idx}] {x.view(-1)[idx].item()!r} vs "
                         f"{y.view(-1)[idx].item()!r}")
    print(f"{name:34s} {'IDENTICAL' if not diffs else 'DIFFER: ' + '; '.join(diffs)}", flush=True)


# GEMMs: every epilogue on the tiles the engine picks (c4 vision / text, C5 text, eval)
for (M, N, K) in [(6368, 2304, 768), (6368, 3072, 768), (6368, 768, 3072), (2926, 2048, 512), (77000, 2048, 512),
                  (77000, 512, 2048), (79600, 3072, 768)]:
    A, B = rnd(M, K), rnd(N, K, scale=K ** -0.5)
    bias, aux = rnd(N, scale=0.1), rnd(M, N)
    for epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU, ops.EPI_DGELU, ops.EPI_NONE):
        kw = {}
        if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU):
            kw["bias"] = bias
        if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU):
            kw["aux_in"] = aux
        for tile in (0, -1):
            def f():
                ao = torch.empty(M, N, device=dev, dtype=torch.float16) if epi == ops.EPI_BIAS_GELU else None
                c = ops.gemm_nt(A, B, epilogue=epi, tile=tile, aux_out=ao, **kw)
                return (c, ao) if ao is not None else c
            report(f"gemm {M}x{N}x{K} epi{epi} tile{tile}", both(f))
    del A, B, aux

# LayerNorm forward / backward (vision, text)
for rows, D in [(6368, 768), (2926, 512), (77000, 512)]:
    x, dy, dres = rnd(rows, D, scale=0.5), rnd(rows, D, scale=1e-3), rnd(rows, D, scale=1e-3)
    gm, bt = rnd(D, dt=torch.float32) * 0.1 + 1, rnd(D, dt=torch.float32) * 0.1

    def lf():
        y, m, r = torch.empty_like(x), torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        ops.layernorm_fwd(x, gm, bt, y, m, r)
        return y, m, r
    report(f"ln_fwd {rows}x{D}", both(lf))
    _lib._LIB = libs[0]
    _, mean, rstd = lf()

    def lb():
        dx, dgm, dbt = torch.empty_like(x), torch.empty(D, device=dev), torch.empty(D, device=dev)
        ops.layernorm_bwd(dy, x, gm, mean, rstd, dx, dgm, dbt, dres=dres)
        return dx, dgm, dbt
    report(f"ln_bwd {rows}x{D}", both(lb))

# attention forward / backward: vision (199 rows, 384 heads), text causal (77 rows, 304 and 8 000 heads), eval
for N, L, H, causal in [(32, 199, 12, False), (38, 77, 8, True), (1000, 77, 8, True), (400, 199, 12, False)]:
    D = H * 64
    qkv = rnd(N * L, 3 * D, scale=0.5)
    dout = rnd(N * L, D, scale=1e-2)

    def af():
        o, lse = torch.empty(N * L, D, device=dev, dtype=torch.float16), torch.empty(N * H * L, device=dev)
        ops.attention_fwd(qkv, N, L, H, causal, out=o, lse=lse)
        return o, lse
    report(f"attn_fwd N{N} L{L} causal{int(causal)}", both(af))
    _lib._LIB = libs[0]
    o, lse = af()

    def ab():
        return ops.attention_bwd(qkv, o, dout, lse, N, L, H, causal)
    if N * L <= 100000:
        report(f"attn_bwd N{N} L{L} causal{int(causal)}", both(ab))

# the fused in-projection + attention forward (the side tower's launches)
for N, L, H, causal in [(38, 77, 8, True), (32, 199, 12, False)]:
    D = H * 64
    if not ops.qkv_attention_supported(N, L, H, causal):
        continue
    x, w, bq = rnd(N * L, D, scale=0.5), rnd(3 * D, D, scale=D ** -0.5), rnd(3 * D, scale=0.1)

    def qf():
        qkv = torch.empty(N * L, 3 * D, device=dev, dtype=torch.float16)
        o, lse = torch.empty(N * L, D, device=dev, dtype=torch.float16), torch.empty(N * H * L, device=dev)
        ops.qkv_attention_fwd(x, w, bq, qkv, o, lse, N, L, H, causal)
        return qkv, o, lse
    report(f"qkv_attn_fwd N{N} L{L}", both(qf))
