"""Per-kernel numerics of libmapfed.so on the MI355X, each against a plain PyTorch fp32 (or fp64)
reference of the same op.  Tolerances are written per test; fp16 outputs are compared in units of
the fp16 ulp of the reference value."""
import math
import os
from pathlib import Path

import pytest
import torch
import torch.nn.functional as F

from federated_multi_modal_amd import ops

pytestmark = pytest.mark.gpu


def ulp16(x: torch.Tensor) -> torch.Tensor:
    a = x.abs().float().clamp_min(2.0 ** -14)
    return torch.exp2(torch.floor(torch.log2(a)) - 10)


def assert_ulps(out, ref, max_ulp=1.0, frac=1e-2, what="", floor=2e-5):
    """|out - ref| <= max_ulp fp16 ulps of the reference value, with an absolute floor of
    floor*max|ref| for values near zero (where fp32 accumulation order, not the fp16 rounding,
    sets the error); at most `frac` of elements off by more than half an ulp."""
    unit = torch.maximum(ulp16(ref), torch.tensor(floor * ref.abs().max().item(), device=ref.device))
    d = (out.float() - ref.float()).abs() / unit
    worst = d.max().item()
    bad = (d > 0.51).float().mean().item()
    assert worst <= max_ulp + 1e-6, f"{what}: worst {worst:.2f} ulp"
    assert bad <= frac, f"{what}: {bad:.4f} of elements beyond half an ulp"


@pytest.mark.parametrize("M,N,K", [(6368, 2304, 768), (513, 700, 256), (300, 516, 128)])
def test_gemm8_staggered_matches_unstaggered(dev, M, N, K):
    """The ping-pong 256x256 kernel (tile 20) issues every accumulator's MFMAs in the same k order as
    the unstaggered one (tile 22): outputs bit-identical."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + K)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    C20 = ops.gemm_nt(A, B, bias=b, epilogue=ops.EPI_BIAS, tile=20)
    C22 = ops.gemm_nt(A, B, bias=b, epilogue=ops.EPI_BIAS, tile=22)
    assert torch.equal(C20, C22)


@pytest.mark.parametrize("M,N,K", [(33000, 1024, 192), (77000, 2048, 512), (20001, 512, 128), (30000, 760, 128),
                                   (20001, 2304, 768), (1000, 256, 192), (6368, 2304, 768)])
def test_gemm8_fullline_matches_staggered(dev, M, N, K):
    """The full-line 256x256 kernel gemm8f (tile 40: [128 rows][64 k] half-tiles) against gemm8s (tile 20: [256
    rows][32 k]) -- bit-identical for every fp16 epilogue, ragged M / N included, and the pre-activation store
    skipped (aux_out null, the forward-only engine) without changing C."""
    g = torch.Generator(device="cpu").manual_seed(M + K)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    R = torch.randn(M, N, generator=g).half().to(dev)
    for epi in (ops.EPI_NONE, ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU, ops.EPI_DGELU, ops.EPI_RESID):
        kw = {"bias": b} if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU) else {}
        outs = []
        for tile in (20, 40):
            aux_out = torch.empty(M, N, device=dev, dtype=torch.float16) if epi == ops.EPI_BIAS_GELU else None
            aux_in = R if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU, ops.EPI_RESID) else None
            C = ops.gemm_nt(A, B, aux_in=aux_in, aux_out=aux_out, epilogue=epi, tile=tile, **kw)
            outs.append((C, aux_out))
        if epi == ops.EPI_BIAS_GELU:  # the forward-only engine's form: no pre-activation store
            for tile in (20, 40):
                outs.append((ops.gemm_nt(A, B, epilogue=epi, tile=tile, **kw), None))
        torch.cuda.synchronize()
        for k, (C, aux_out) in enumerate(outs[1:], 1):
            assert torch.equal(outs[0][0], C), f"epilogue {epi}, variant {k}"
            if aux_out is not None:
                assert torch.equal(outs[0][1], aux_out), f"epilogue {epi}, variant {k} (pre-activation)"


@pytest.mark.parametrize("M,N,K", [(79600, 2304, 768), (19900, 768, 3072), (3000, 512, 128), (77000, 512, 512)])
def test_gemm8p_persistent_matches_gemm8f(dev, M, N, K):
    """The persistent 256x256 kernel gemm8p (tile 41: one workgroup per CU walking its XCD's tiles, the next tile's
    prologue under this tile's register-direct epilogue) against gemm8f (tile 40) -- bit-identical for every fp16
    epilogue, ragged M included, with and without the pre-activation store."""
    g = torch.Generator(device="cpu").manual_seed(M + K + 1)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    R = torch.randn(M, N, generator=g).half().to(dev)
    for epi in (ops.EPI_NONE, ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU, ops.EPI_DGELU, ops.EPI_RESID):
        kw = {"bias": b} if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU) else {}
        aux_in = R if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU, ops.EPI_RESID) else None
        for with_aux_out in ((True, False) if epi == ops.EPI_BIAS_GELU else (False,)):
            outs = []
            for tile in (40, 41):
                aux_out = torch.full((M, N), 3.0, device=dev, dtype=torch.float16) if with_aux_out else None
                C = torch.full((M, N), 5.0, device=dev, dtype=torch.float16)
                ops.gemm_nt(A, B, C=C, aux_in=aux_in, aux_out=aux_out, epilogue=epi, tile=tile, **kw)
                outs.append((C, aux_out))
            torch.cuda.synchronize()
            assert torch.equal(outs[0][0], outs[1][0]), f"epilogue {epi}, aux_out {with_aux_out}"
            if with_aux_out:
                assert torch.equal(outs[0][1], outs[1][1]), f"epilogue {epi} (pre-activation)"


@pytest.mark.parametrize("M,N,K,epi", [(2926, 512, 2048, 2), (2926, 1536, 512, 1), (6368, 768, 3072, 0),
                                       (6368, 3072, 768, 3), (6368, 768, 768, 4), (770, 512, 512, 0)])
def test_gemm_side_tower_tile_hint_is_bit_identical(dev, M, N, K, epi):
    """tile -1 (the projections of the tower off the critical path: work-per-CU-second tiles, no hipBLASLt route)
    against the latency picks (tile 0): every tile accumulates each output in the same k order, so the outputs
    are bit-identical; below 2 048 rows the hint falls back to the latency picks."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    R = torch.randn(M, N, generator=g).half().to(dev)
    kw = {"bias": b} if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU) else {}
    if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU):
        kw["aux_in"] = R
    outs = []
    for tile in (0, -1):
        aux_out = torch.empty(M, N, device=dev, dtype=torch.float16) if epi == ops.EPI_BIAS_GELU else None
        outs.append((ops.gemm_nt(A, B, aux_out=aux_out, epilogue=epi, tile=tile, **kw), aux_out))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if epi == ops.EPI_BIAS_GELU:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("M,N,K,tile", [(796, 2304, 768, 0), (6368, 768, 3072, 0), (770, 512, 2048, 1),
                                        (130, 44, 64, 3), (257, 1536, 512, 2), (6368, 3072, 768, 0),
                                        # 8-wave phase-pipelined family (tiles 20 = staggered 256x256, 21,
                                        # 22 = unstaggered 256x256), ragged M / N, K down to two K-tiles
                                        (6368, 2304, 768, 20), (1000, 760, 192, 20), (6368, 3072, 768, 21),
                                        (300, 388, 64, 21), (777, 132, 128, 21), (129, 260, 320, 20),
                                        (300, 516, 128, 20), (6368, 2304, 768, 22), (129, 260, 320, 22),
                                        # 160x128 (tiles 10, 11)
                                        (6368, 768, 3072, 10), (333, 136, 128, 10), (6368, 768, 2304, 11),
                                        (170, 260, 192, 11),
                                        # 96x128, 160x64, 96x64 (tiles 15, 16, 26) as chosen by the heuristic
                                        (6368, 768, 3072, 0), (6368, 768, 768, 0), (2926, 1536, 512, 0),
                                        (97, 200, 64, 15), (161, 72, 128, 16), (100, 76, 192, 26),
                                        # the small clients' 4-stage rings (tiles 31, 33)
                                        (796, 768, 3072, 31), (770, 512, 2048, 33), (100, 72, 320, 31),
                                        (33, 136, 192, 33),
                                        # the full-line 8-wave 256x256 tile (gemm8f, 40)
                                        (6368, 2304, 768, 40), (1000, 760, 192, 40), (129, 260, 128, 40),
                                        (20001, 2304, 768, 40), (300, 516, 192, 40)])
def test_gemm_bias(dev, M, N, K, tile):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    b = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    C = ops.gemm_nt(A, B, bias=b, epilogue=ops.EPI_BIAS, tile=tile)
    ref = (A.double() @ B.double().t() + b.double())
    assert_ulps(C, ref, 1.0, 2e-2, "gemm+bias")
    # no-bias and fp32 epilogues
    C0 = ops.gemm_nt(A, B, epilogue=ops.EPI_NONE, tile=tile)
    assert_ulps(C0, A.double() @ B.double().t(), 1.0, 2e-2, "gemm")
    C32 = ops.gemm_nt(A, B, epilogue=ops.EPI_F32, tile=tile)
    torch.testing.assert_close(C32.double(), A.double() @ B.double().t(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,N,K,ak,bk,tile", [
    # weight gradients dW[out,in] = dY^T X: both operands K-major, K = rows (ragged: no padding)
    (3072, 768, 6368, True, True, 0), (768, 3072, 6368, True, True, 0), (2304, 768, 6368, True, True, 0),
    (512, 2048, 2926, True, True, 0), (64, 72, 100, True, True, 3), (136, 200, 1, True, True, 2),
    # dX = dY . W with W [out][in] read K-major
    (6368, 768, 3072, False, True, 0), (2926, 2048, 512, False, True, 1), (100, 64, 192, False, True, 3),
    (300, 200, 128, False, True, 2),
    # A K-major, B row-major
    (256, 128, 128, True, False, 1), (72, 64, 64, True, False, 3),
])
def test_gemm_kmajor(dev, M, N, K, ak, bk, tile):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    A = torch.randn(K, M, generator=g).half().to(dev) if ak else torch.randn(M, K, generator=g).half().to(dev)
    B = ((torch.randn(K, N, generator=g) if bk else torch.randn(N, K, generator=g)) * K ** -0.5).half().to(dev)
    Ad = A.double().t() if ak else A.double()
    Bd = B.double() if bk else B.double().t()
    ref = Ad @ Bd
    C = ops.gemm(A, B, epilogue=ops.EPI_NONE, tile=tile, a_kmajor=ak, b_kmajor=bk)
    assert_ulps(C, ref, 1.0, 2e-2, f"gemm kmajor {ak}{bk}")
    C32 = ops.gemm(A, B, epilogue=ops.EPI_F32, tile=tile, a_kmajor=ak, b_kmajor=bk)
    torch.testing.assert_close(C32.double(), ref, rtol=1e-5, atol=1e-4)
    # the NT form of the same product (explicit transposes) gives the identical fp32 accumulation order
    if K % 64 == 0:
        At = A.t().contiguous() if ak else A
        Bt = B.t().contiguous() if bk else B
        C0 = ops.gemm_nt(At, Bt, epilogue=ops.EPI_F32, tile=tile if tile in (1, 2, 3) else 1)
        assert torch.equal(C0, C32)



@pytest.mark.parametrize("M,N,K,ak,bk,splits", [(3072, 768, 6368, True, True, 0), (768, 768, 6368, True, True, 0),
                                                (2048, 512, 2926, True, True, 0), (256, 384, 1000, True, True, 3),
                                                (512, 256, 4096, False, False, 0), (384, 512, 2048, True, False, 5)])
def test_gemm_splitk(dev, M, N, K, ak, bk, splits):
    """Split-K weight-gradient GEMM: fp32 partial planes summed in a fixed order -- against fp64, and
    bit-reproducible run to run; one split equals the single-pass fp32 GEMM exactly."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(K, M, generator=g).half().to(dev) if ak else torch.randn(M, K, generator=g).half().to(dev)
    B = ((torch.randn(K, N, generator=g) if bk else torch.randn(N, K, generator=g)) * K ** -0.5).half().to(dev)
    ref = (A.double().t() if ak else A.double()) @ (B.double() if bk else B.double().t())
    ws = torch.empty(ops.gemm_splitk_ws_floats(M, N, K, splits), device=dev)
    C = torch.empty(M, N, device=dev, dtype=torch.float16)
    ops.gemm_splitk(A, B, C, ws, splits=splits, a_kmajor=ak, b_kmajor=bk)
    assert_ulps(C, ref, 1.0, 2e-2, "gemm splitk")
    C32 = torch.empty(M, N, device=dev)
    ops.gemm_splitk(A, B, C32, ws, splits=splits, a_kmajor=ak, b_kmajor=bk)
    torch.testing.assert_close(C32.double(), ref, rtol=1e-5, atol=1e-4)
    C32b = torch.empty_like(C32)
    ops.gemm_splitk(A, B, C32b, ws, splits=splits, a_kmajor=ak, b_kmajor=bk)
    assert torch.equal(C32, C32b)
    one = torch.empty_like(C32)
    ws1 = torch.empty(ops.gemm_splitk_ws_floats(M, N, K, 1), device=dev)
    ops.gemm_splitk(A, B, one, ws1, splits=1, a_kmajor=ak, b_kmajor=bk)
    assert torch.equal(one, ops.gemm(A, B, epilogue=ops.EPI_F32, tile=1, a_kmajor=ak, b_kmajor=bk))

def test_gemm_kmajor_dgelu(dev):
    torch.manual_seed(5)
    M, N, K = 600, 1024, 256
    dY = torch.randn(M, K).half().to(dev)
    W = (torch.randn(K, N) * K ** -0.5).half().to(dev)   # nn.Linear weight [out=K][in=N]
    F = torch.randn(M, N).half().to(dev)
    a = ops.gemm(dY, W, aux_in=F, epilogue=ops.EPI_DGELU, b_kmajor=True)
    b = ops.gemm_nt(dY, W.t().contiguous(), aux_in=F, epilogue=ops.EPI_DGELU, tile=1)
    assert torch.equal(a, b)


def _gelu16(f):
    t1 = (f.float() * 1.702).half()
    t2 = torch.sigmoid(t1.float()).half()
    return (f.float() * t2.float()).half()


@pytest.mark.parametrize("tile", [0, 10, 15, 20, 21])
def test_gemm_epilogues(dev, tile):
    torch.manual_seed(0)
    M, N, K = 600, 1024, 256
    A = torch.randn(M, K).half().to(dev)
    B = (torch.randn(N, K) * K ** -0.5).half().to(dev)
    b = (torch.randn(N) * 0.1).half().to(dev)
    R = torch.randn(M, N).half().to(dev)
    acc = A.double() @ B.double().t()
    y16 = (acc + b.double()).half()
    # residual
    C = ops.gemm_nt(A, B, bias=b, aux_in=R, epilogue=ops.EPI_BIAS_RESID, tile=tile)
    ref = (R.float() + y16.float()).half()
    assert (C.float() - ref.float()).abs().max().item() <= 2 * ulp16(ref).max().item()
    assert (C != ref).float().mean().item() < 2e-2
    # residual in place (C aliases R)
    R2 = R.clone()
    ops.gemm_nt(A, B, C=R2, bias=b, aux_in=R2, epilogue=ops.EPI_BIAS_RESID, tile=tile)
    assert torch.equal(R2, C)
    # gelu: stores pre-activation and QuickGELU with the reference's roundings
    Fpre = torch.empty(M, N, dtype=torch.float16, device=dev)
    G = ops.gemm_nt(A, B, bias=b, aux_out=Fpre, epilogue=ops.EPI_BIAS_GELU, tile=tile)
    assert (Fpre != y16).float().mean().item() < 2e-2
    assert (G != _gelu16(Fpre)).float().mean().item() < 1e-3
    # dgelu: the reference's autograd of QuickGELU on CPU torch (sigmoid_backward for Half runs in
    # fp16 op by op there), restated with explicit ops on the kernel's own fp16 GEMM output
    dG = ops.gemm_nt(A, B, aux_in=Fpre, epilogue=ops.EPI_DGELU, tile=tile)
    dg = ops.gemm_nt(A, B, epilogue=ops.EPI_NONE, tile=tile).float()
    h = lambda t: t.half().float()
    ff = Fpre.float()
    t2 = h(torch.sigmoid(h(ff * 1.702)))
    dt1 = h(h(h(dg * ff) * h(1 - t2)) * t2)
    man = (h(dg * t2) + h(dt1 * 1.702)).half()
    assert (dG != man).float().mean().item() < 1e-3
    # and within 2 ulp of GPU torch's own fp16 autograd (which computes sigmoid_backward in fp32)
    f = Fpre.clone().requires_grad_(True)
    (f * torch.sigmoid(1.702 * f)).backward(dg.half())
    assert_ulps(dG, f.grad.double(), 2.0, 0.5, "dgelu vs torch-gpu autograd", floor=1e-3)


# 6368 x 768 runs the two-rows-per-half-wave backward (398 row blocks); 2926 x 512, 796 x 768 and 770 x 512 the
# one-row form (< 256 blocks, layernorm.hip ln_bwd_wide)
@pytest.mark.parametrize("D,rows", [(768, 6368), (512, 2926), (768, 796), (512, 770), (768, 5)])
def test_layernorm(dev, D, rows):
    torch.manual_seed(D + rows)
    x = (torch.randn(rows, D) * 2 + 0.5).half().to(dev)
    g = (1 + 0.1 * torch.randn(D)).to(dev)
    b = (0.1 * torch.randn(D)).to(dev)
    y, mean, rstd = ops.layernorm_fwd(x, g, b)
    ref = F.layer_norm(x.double(), (D,), g.double(), b.double(), 1e-5)
    assert_ulps(y, ref, 1.0, 1e-2, "ln fwd")
    # backward vs autograd fp64, with residual accumulation
    dy = torch.randn(rows, D).half().to(dev)
    dres = torch.randn(rows, D).half().to(dev)
    xx = x.double().requires_grad_(True)
    gg = g.double().requires_grad_(True)
    bb = b.double().requires_grad_(True)
    F.layer_norm(xx, (D,), gg, bb, 1e-5).backward(dy.double())
    dx = torch.empty_like(x)
    dg = torch.empty(D, device=dev)
    db = torch.empty(D, device=dev)
    ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dg, db, dres=dres)
    refdx = (dres.double() + xx.grad.half().double())
    assert (dx.float() - refdx.float()).abs().max().item() <= 2 * ulp16(refdx).max().item()
    torch.testing.assert_close(dg.double(), gg.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db.double(), bb.grad, rtol=1e-4, atol=1e-3)


def test_layernorm_row_index(dev):
    torch.manual_seed(1)
    D, R = 768, 4 * 199
    x = torch.randn(R, D).half().to(dev)
    idx = torch.arange(0, R, 199, dtype=torch.int32, device=dev)
    g = torch.ones(D, device=dev)
    b = torch.zeros(D, device=dev)
    y, mean, rstd = ops.layernorm_fwd(x, g, b, row_index=idx)
    ref = F.layer_norm(x[idx.long()].double(), (D,), g.double(), b.double(), 1e-5)
    assert_ulps(y, ref, 1.0, 1e-2, "ln gather")
    dy = torch.randn(4, D).half().to(dev)
    dx = torch.zeros_like(x)
    dg = torch.empty(D, device=dev)
    db = torch.empty(D, device=dev)
    ops.layernorm_bwd(dy, x, g, mean, rstd, dx, dg, db, row_index=idx)
    mask = torch.ones(R, dtype=torch.bool, device=dev)
    mask[idx.long()] = False
    assert dx[mask].abs().max().item() == 0


@pytest.mark.parametrize("D,seqs,L_live,L_full,inject", [(512, 38, 10, 77, False), (512, 38, 10, 77, True),
                                                         (512, 1000, 13, 77, False), (768, 5, 40, 77, True)])
def test_layernorm_bwd_live_matches_full_layout(dev, D, seqs, L_live, L_full, inject):
    """mf_layernorm_bwd_live on the compact first-L_live rows of each sequence == mf_layernorm_bwd(_inject) on
    the full L_full-row layout whose other rows carry zero dy / dres: same dx rows, bit-identical dgamma / dbeta
    (and prompt gradient), both below and above the 256-block wide-kernel threshold."""
    torch.manual_seed(D + seqs)
    Rf, Rc = seqs * L_full, seqs * L_live
    live = (torch.arange(Rf, device=dev) % L_full) < L_live
    xf = (torch.randn(Rf, D, device=dev) * 2 + 0.5).half()
    g = (1 + 0.1 * torch.randn(D, device=dev))
    b = 0.1 * torch.randn(D, device=dev)
    _, mean_f, rstd_f = ops.layernorm_fwd(xf, g, b)
    dyf = torch.randn(Rf, D, device=dev).half() * live[:, None]
    dresf = torch.randn(Rf, D, device=dev).half() * live[:, None]
    xc, dyc, dresc = xf[live].contiguous(), dyf[live].contiguous(), dresf[live].contiguous()
    mean_c, rstd_c = mean_f[live].contiguous(), rstd_f[live].contiguous()
    outs = []
    for full in (True, False):
        lnb = ops.LNGradBatch(dev)
        dg = torch.empty(D, device=dev)
        db = torch.empty(D, device=dev)
        pg = torch.empty(2, D, device=dev) if inject else None
        if full:
            dx = dresf.clone()
            if inject:
                lnb.bwd_inject(dyf, xf, g, mean_f, rstd_f, dx, dg, db, dx, pg, L_full, 1, 2)
            else:
                lnb.bwd(dyf, xf, g, mean_f, rstd_f, dx, dg, db, dres=dx)
            dx = dx[live]
        else:
            dx = dresc.clone()
            if inject:
                lnb.bwd_inject(dyc, xc, g, mean_c, rstd_c, dx, dg, db, dx, pg, L_live, 1, 2, live=(L_live, L_full))
            else:
                lnb.bwd(dyc, xc, g, mean_c, rstd_c, dx, dg, db, dres=dx, live=(L_live, L_full))
        lnb.finish()
        torch.cuda.synchronize()
        outs.append((dx, dg, db, pg))
    (dx0, dg0, db0, pg0), (dx1, dg1, db1, pg1) = outs
    assert torch.equal(dx0, dx1)
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
    if inject:
        assert torch.equal(pg0, pg1)


def test_seq_scatter(dev):
    src = torch.randn(6 * 5, 24, device=dev).half()
    dst = torch.zeros(6 * 9, 32, device=dev).half()
    ops.seq_scatter(src, dst[:, :24], 6, 5, 9)
    ref = torch.zeros(6, 9, 32, device=dev).half()
    ref[:, :5, :24] = src.view(6, 5, 24)
    assert torch.equal(dst, ref.view(6 * 9, 32))


def _attn_ref(q, k, v, causal):
    """fp64 restatement of the kernel's numerics: P = exp(s - max) rounded to fp16, sum unrounded."""
    s = (q.double() @ k.double().transpose(-1, -2)) * 0.125
    if causal:
        L = s.shape[-1]
        s = s + torch.full((L, L), float("-inf"), device=s.device, dtype=s.dtype).triu(1)
    m = s.max(-1, keepdim=True).values
    e = torch.exp(s - m)
    return (e.half().double() @ v.double()) / e.sum(-1, keepdim=True)


@pytest.mark.parametrize("N,L,H,causal", [(4, 199, 12, False), (10, 77, 8, True), (3, 50, 2, False),
                                          (2, 256, 4, True), (2, 16, 3, True), (3, 40, 2, False),
                                          (1, 230, 2, True), (3, 455, 4, False), (2, 300, 3, False)])
def test_attention_fwd_bwd(dev, N, L, H, causal):
    torch.manual_seed(L)
    D = H * 64
    qkv = torch.randn(N * L, 3 * D).half().to(dev)
    out, lse = ops.attention_fwd(qkv, N, L, H, causal)
    q, k, v = qkv.view(N, L, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)  # [N,H,L,64]
    ref = _attn_ref(q, k, v, causal).permute(0, 2, 1, 3).reshape(N * L, D)
    assert_ulps(out, ref, 4.0, 2e-2, "attn fwd")
    # torch SDPA (the reference's op) within 1e-3 absolute
    mask = None
    if causal:
        mask = torch.full((L, L), float("-inf"), device=dev).triu(1).half()
    sd = F.scaled_dot_product_attention(q, k, v, attn_mask=mask).permute(0, 2, 1, 3).reshape(N * L, D)
    assert (out.float() - sd.float()).abs().max().item() < 2e-3
    # backward vs autograd fp32
    dout = torch.randn(N * L, D).half().to(dev)
    dqkv = ops.attention_bwd(qkv, out, dout, lse, N, L, H, causal)
    qq, kk, vv = [t.float().detach().requires_grad_(True) for t in (q, k, v)]
    m32 = mask.float() if mask is not None else None
    o32 = F.scaled_dot_product_attention(qq, kk, vv, attn_mask=m32)
    o32.backward(dout.float().view(N, L, H, 64).permute(0, 2, 1, 3))
    gref = torch.stack([qq.grad, kk.grad, vv.grad], 0).permute(1, 3, 0, 2, 4).reshape(N * L, 3 * D)
    err = (dqkv.float() - gref).abs()
    scale = gref.abs().max().item()
    assert err.max().item() < 1e-2 * scale + 2e-3, (err.max().item(), scale)
    rel = err.norm().item() / gref.norm().item()
    assert rel < 5e-3, rel


@pytest.mark.parametrize("L", [199, 150])
def test_attention_fwd_many_heads_bit_identical(dev, L):
    """>= 2 048 heads of > 128 rows run the persistent double-buffered forward (attn_fwdp_kernel): out and lse
    bit-identical to the per-head kernel run on slices of the batch (batch-invariant rows), and close to fp64."""
    N, H = 200, 12
    torch.manual_seed(L)
    D = H * 64
    qkv = torch.randn(N * L, 3 * D).half().to(dev)
    out, lse = ops.attention_fwd(qkv, N, L, H, False)
    n = 50  # 600 heads per slice: attn_fwd4_kernel
    for s in range(0, N, n):
        o_s, l_s = ops.attention_fwd(qkv[s * L:(s + n) * L], n, L, H, False)
        assert torch.equal(out[s * L:(s + n) * L], o_s)
        assert torch.equal(lse.view(N * H, -1)[s * H:(s + n) * H, :L], l_s.view(n * H, -1)[:, :L])
    q, k, v = qkv[:4 * L].view(4, L, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    ref = _attn_ref(q, k, v, False).permute(0, 2, 1, 3).reshape(4 * L, D)
    assert_ulps(out[:4 * L], ref, 4.0, 2e-2, "attn fwd persistent")


@pytest.mark.parametrize("N,L,H,causal,q_rows", [(400, 199, 12, False, 1), (32, 199, 12, False, 1),
                                                 (3, 199, 12, False, 40), (38, 77, 8, True, 1), (5, 80, 8, True, 17)])
def test_attention_fwd_rows_bit_identical(dev, N, L, H, causal, q_rows):
    """mf_attention_fwd_rows (query rows 0 .. q_rows-1 of every head: the forward-only engine's last vision block)
    against the full forward (attn_fwd4 or, at >= 2 048 heads, the persistent attn_fwdp): every computed query
    tile's out and lse rows bit-identical, the other rows untouched."""
    D = H * 64
    torch.manual_seed(q_rows + L)
    qkv = torch.randn(N * L, 3 * D).half().to(dev)
    out, lse = ops.attention_fwd(qkv, N, L, H, causal)
    o2 = torch.full_like(out, 7.0)
    l2 = torch.full_like(lse, 7.0)
    ops.attention_fwd_rows(qkv, N, L, H, causal, q_rows, o2, l2)
    rows = min(L, (q_rows + 15) // 16 * 16)
    o_v, o2_v = out.view(N, L, D), o2.view(N, L, D)
    assert torch.equal(o_v[:, :rows], o2_v[:, :rows])
    assert (o2_v[:, rows:] == 7.0).all()
    assert torch.equal(lse.view(N * H, L)[:, :rows], l2.view(N * H, L)[:, :rows])


@pytest.mark.parametrize("N,L,H,causal", [(4, 199, 12, False), (32, 199, 12, False), (3, 193, 12, False),
                                          (38, 77, 8, True), (5, 80, 8, True)])
def test_qkv_attention_fused_matches_unfused(dev, N, L, H, causal):
    """mf_qkv_attention_fwd (in-projection + attention in one launch) against the two launches it replaces
    (mf_gemm_nt with the bias epilogue, then mf_attention_fwd): qkv, out and lse bit-identical (same MFMA,
    same k order, same fp16 rounding points), incl. the last sequence of the buffer (rows past it read as 0)."""
    D = H * 64
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + L)
    x = torch.randn(N * L, D, generator=g).half().to(dev)
    W = (torch.randn(3 * D, D, generator=g) * D ** -0.5).half().to(dev)
    b = (torch.randn(3 * D, generator=g) * 0.02).half().to(dev)
    qkv_ref = ops.gemm_nt(x, W, bias=b, epilogue=ops.EPI_BIAS)
    o_ref, lse_ref = ops.attention_fwd(qkv_ref, N, L, H, causal)
    assert ops.qkv_attention_supported(N, L, H, causal)
    qkv = torch.full_like(qkv_ref, float("nan"))
    o = torch.full((N * L, D), float("nan"), device=dev, dtype=torch.float16)
    lse = torch.full((N * H * L,), float("nan"), device=dev, dtype=torch.float32)
    ops.qkv_attention_fwd(x, W, b, qkv, o, lse, N, L, H, causal)
    torch.cuda.synchronize()
    assert torch.equal(qkv, qkv_ref)
    assert torch.equal(o, o_ref)
    assert torch.equal(lse, lse_ref)
    assert not ops.qkv_attention_supported(N, 10, H, causal)  # the EOT-truncated text tower stays unfused


def test_assemble_inject_transpose_colsum(dev):
    torch.manual_seed(3)
    B, G2, D, n_ctx = 3, 196, 768, 2
    patch = torch.randn(B * G2, D).half().to(dev)
    cls = torch.randn(D).to(dev)
    pos = torch.randn(G2 + 1, D).to(dev)
    sc = torch.randn(n_ctx, D).half().to(dev)
    L = G2 + 1 + n_ctx
    x = torch.empty(B * L, D, dtype=torch.float16, device=dev)
    ops.vision_assemble(patch, cls, pos, sc, x, B, G2, n_ctx, D)
    ref = torch.cat([cls.half().expand(B, 1, D) + torch.zeros(B, 1, D, dtype=torch.float16, device=dev),
                     patch.view(B, G2, D)], 1) + pos.half()
    ref = torch.cat([ref, sc.expand(B, -1, -1)], 1).reshape(B * L, D)
    assert torch.equal(x, ref)
    # inject + its backward
    pr = torch.randn(n_ctx, D).to(dev)
    ops.prompt_inject_fwd(x, pr, B, L, L - n_ctx, n_ctx, D)
    assert torch.equal(x.view(B, L, D)[:, L - n_ctx:], pr.half().expand(B, -1, -1))
    dx = torch.randn(B * L, D).half().to(dev)
    d0 = dx.view(B, L, D)[:, L - n_ctx:].float().sum(0)
    out = torch.empty(n_ctx, D, device=dev)
    ops.prompt_inject_bwd(dx, B, L, L - n_ctx, n_ctx, D, out)
    torch.testing.assert_close(out, d0, rtol=1e-6, atol=1e-6)
    assert dx.view(B, L, D)[:, L - n_ctx:].abs().max().item() == 0
    # text assemble
    K, Lt, Dt = 5, 77, 512
    prefix = torch.randn(K, 1, Dt).half().to(dev)
    ctx = torch.randn(n_ctx, Dt).half().to(dev)
    suffix = torch.randn(K, Lt - 1 - n_ctx, Dt).half().to(dev)
    post = torch.randn(Lt, Dt).to(dev)
    xt = torch.empty(K * Lt, Dt, dtype=torch.float16, device=dev)
    ops.text_assemble(prefix, ctx, suffix, post, xt, K, Lt, n_ctx, Dt)
    reft = (torch.cat([prefix, ctx.expand(K, -1, -1), suffix], 1) + post.half()).reshape(K * Lt, Dt)
    assert torch.equal(xt, reft)
    # transpose / colsum
    a = torch.randn(300, 200).half().to(dev)
    t = torch.zeros(200, 320, dtype=torch.float16, device=dev)
    ops.transpose(a, t[:, :300])
    assert torch.equal(t[:, :300], a.t()) and t[:, 300:].abs().max().item() == 0
    for shape in ((3072, 768), (768, 2304), (130, 64)):  # 16-byte tile path + ragged fallback tiles
        w = torch.randn(*shape).half().to(dev)
        assert torch.equal(ops.transpose(w, torch.empty(shape[1], shape[0], dtype=torch.float16, device=dev)), w.t())
    cs = torch.empty(200, dtype=torch.float16, device=dev)
    ops.colsum(a, cs)
    assert (cs.float() - a.float().sum(0).half().float()).abs().max().item() <= ulp16(cs).max().item()


def test_small_linear(dev):
    torch.manual_seed(4)
    for dt in (torch.float32, torch.float16):
        X = torch.randn(2, 512, dtype=dt, device=dev)
        W = (torch.randn(768, 512) * 0.05).to(dt).to(dev)
        b = torch.randn(768, dtype=dt, device=dev)
        Y = torch.empty(2, 768, dtype=dt, device=dev)
        ops.small_linear_fwd(X, W, b, Y)
        ref = F.linear(X.double(), W.double(), b.double())
        tol = 1e-5 if dt == torch.float32 else 2e-3
        torch.testing.assert_close(Y.double(), ref, rtol=tol, atol=tol)
        dY = torch.randn(2, 768, dtype=dt, device=dev)
        dX = torch.empty_like(X)
        dW = torch.empty_like(W)
        db = torch.empty_like(b)
        ops.small_linear_bwd(dY, X, W, dX, dW, db)
        torch.testing.assert_close(dX.double(), dY.double() @ W.double(), rtol=tol * 5, atol=tol * 5)
        torch.testing.assert_close(dW.double(), dY.double().t() @ X.double(), rtol=tol * 5, atol=tol * 5)
        torch.testing.assert_close(db.double(), dY.double().sum(0), rtol=tol * 5, atol=tol * 5)


def test_small_linear_batch(dev):
    """The batched prompt-learner Linears equal the one-at-a-time kernels bit for bit (same per-output
    summation order), including the accumulate-into-dX form and mixed fp16 / fp32 entries."""
    torch.manual_seed(6)
    ents, singles = [], []
    for k, (dt, I, O) in enumerate([(torch.float16, 512, 768), (torch.float32, 512, 768), (torch.float32, 768, 512),
                                    (torch.float32, 512, 768)]):
        X = torch.randn(2, I, dtype=dt, device=dev)
        W = (torch.randn(O, I) * 0.05).to(dt).to(dev)
        b = torch.randn(O, dtype=dt, device=dev)
        dY = torch.randn(2, O, dtype=dt, device=dev)
        dX0 = torch.randn(2, I, dtype=dt, device=dev)
        e = dict(X=X, W=W, b=b, Y=torch.empty(2, O, dtype=dt, device=dev), dY=dY, dX=dX0.clone(), acc_dx=True,
                 dW=torch.empty_like(W), db=torch.empty_like(b))
        ents.append(e)
        s = dict(Y=torch.empty(2, O, dtype=dt, device=dev), dX=dX0.clone(), dW=torch.empty_like(W), db=torch.empty_like(b))
        ops.small_linear_fwd(X, W, b, s["Y"])
        ops.small_linear_bwd(dY, X, W, s["dX"], s["dW"], s["db"], accumulate_dx=True)
        singles.append(s)
    batch = ops.SmallLinearBatch(dev, ents)
    batch.fwd()
    batch.bwd()
    for e, s in zip(ents, singles):
        for key in ("Y", "dX", "dW", "db"):
            assert torch.equal(e[key], s[key]), key


def test_clip_head_loss(dev):
    torch.manual_seed(5)
    B, K, D = 8, 38, 512
    img = torch.randn(B, D).half().to(dev)
    txt = torch.randn(K, D).half().to(dev)
    label = torch.randint(0, K, (B,)).to(dev)
    ls = torch.tensor([math.log(1 / 0.07)], device=dev)
    img_n = torch.empty_like(img)
    txt_n = torch.empty_like(txt)
    norms = torch.empty(B + K, device=dev)
    mm = torch.empty(B, K, dtype=torch.float16, device=dev)
    logits = torch.empty_like(mm)
    ops.clip_head_fwd(img, txt, ls, img_n, txt_n, norms, mm, logits)
    # reference ops on the GPU in fp16 (trainers/maple.py:325,340-346)
    i_ = img.clone().requires_grad_(True)
    t_ = txt.clone().requires_grad_(True)
    inr = F.normalize(i_, dim=-1, eps=1e-8)
    tnr = F.normalize(t_, dim=-1, eps=1e-8)
    ref_logits = ls.exp().clamp(max=100) * (inr @ tnr.t())
    assert (logits.float() - ref_logits.float()).abs().max().item() <= 2e-2 * 1.0 + 1e-3
    dmm = torch.empty_like(mm)
    cos_ws = torch.empty(2 * B, device=dev)
    loss = torch.empty(4, device=dev)
    dimg_n, dtxt_n = torch.empty_like(img), torch.empty_like(txt)
    dimg, dtxt = torch.empty_like(img), torch.empty_like(txt)
    ops.clip_loss_fwd_bwd(img, txt, img_n, txt_n, norms, logits, label, ls, dmm, cos_ws, loss, dimg_n, dtxt_n,
                          dimg, dtxt)
    # fp32 reference of the loss and its gradient
    i32 = img.float().requires_grad_(True)
    t32 = txt.float().requires_grad_(True)
    a = F.normalize(i32, dim=-1, eps=1e-8)
    t = F.normalize(t32, dim=-1, eps=1e-8)
    lg = ls.exp().clamp(max=100) * (a @ t.t())
    tot = F.cross_entropy(lg, label) + 0.5 * (1 - F.cosine_similarity(a, t[label]).mean())
    tot.backward()
    assert abs(loss[0].item() - tot.item()) < 5e-3
    torch.testing.assert_close(dimg.float(), i32.grad, rtol=2e-2, atol=2e-4)
    torch.testing.assert_close(dtxt.float(), t32.grad, rtol=2e-2, atol=2e-4)



def _head_setup(dev, B, K, D, seed):
    torch.manual_seed(seed)
    img = torch.randn(B, D).half().to(dev)
    txt = torch.randn(K, D).half().to(dev)
    ls = torch.tensor([math.log(1 / 0.07)], device=dev)
    img_n, txt_n = torch.empty_like(img), torch.empty_like(txt)
    norms = torch.empty(B + K, device=dev)
    mm = torch.empty(B, K, dtype=torch.float16, device=dev)
    logits = torch.empty_like(mm)
    ops.clip_head_fwd(img, txt, ls, img_n, txt_n, norms, mm, logits)
    out = dict(img=img, txt=txt, ls=ls, img_n=img_n, txt_n=txt_n, norms=norms, logits=logits,
               dmm=torch.empty_like(mm), cos_ws=torch.empty(2 * B, device=dev), loss=torch.empty(4, device=dev),
               dimg_n=torch.empty_like(img), dtxt_n=torch.empty_like(txt), dimg=torch.empty_like(img),
               dtxt=torch.empty_like(txt), soft_ws=torch.empty(2 * B * D, dtype=torch.float16, device=dev))
    return out


def _soft(h, q):
    ops.clip_loss_soft_fwd_bwd(h["img"], h["txt"], h["img_n"], h["txt_n"], h["norms"], h["logits"], q, h["ls"],
                               h["dmm"], h["cos_ws"], h["soft_ws"], h["loss"], h["dimg_n"], h["dtxt_n"], h["dimg"],
                               h["dtxt"])


@pytest.mark.parametrize("B,K", [(8, 38), (32, 10), (3, 100)])
def test_clip_head_loss_soft(dev, B, K):
    """Soft-label branch (trainers/maple.py:356-360) against an fp32 torch restatement:
    KL(q.clamp(1e-8) || softmax(logits)) batchmean + 0.5 (1 - mean cos(img_n, q @ txt_n))."""
    D = 512
    h = _head_setup(dev, B, K, D, 7)
    q = torch.rand(B, K, device=dev) ** 4
    q[0, :] = 0.0
    q[0, K // 2] = 1.0                      # a one-hot row (zeros clamp to 1e-8 inside the KL)
    q = (q / q.sum(1, keepdim=True)).contiguous()
    _soft(h, q)
    i32 = h["img"].float().requires_grad_(True)
    t32 = h["txt"].float().requires_grad_(True)
    a = F.normalize(i32, dim=-1, eps=1e-8)
    t = F.normalize(t32, dim=-1, eps=1e-8)
    lg = h["ls"].exp().clamp(max=100) * (a @ t.t())
    kl = F.kl_div(F.log_softmax(lg, dim=1), q.clamp(min=1e-8), reduction="batchmean")
    tot = kl + 0.5 * (1 - F.cosine_similarity(a, q @ t).mean())
    tot.backward()
    loss = h["loss"].cpu()
    assert loss[3].item() == 0.0
    assert abs(loss[0].item() - tot.item()) < 5e-3, (loss[0].item(), tot.item())
    assert abs(loss[1].item() - kl.item()) < 5e-3
    torch.testing.assert_close(h["dimg"].float(), i32.grad, rtol=2e-2, atol=2e-4)
    torch.testing.assert_close(h["dtxt"].float(), t32.grad, rtol=2e-2, atol=2e-4)


def test_clip_head_loss_soft_onehot_matches_hard(dev):
    """One-hot soft labels reproduce the cross-entropy branch: the KL of a one-hot target is the CE
    (the 1e-8 clamps add < 1e-6), q @ txt_n selects txt_n[y] exactly, so the logit gradient and d img are
    bit-identical; d txt differs only in where the per-row cosine gradients are rounded."""
    B, K, D = 16, 38, 512
    h = _head_setup(dev, B, K, D, 8)
    y = torch.randint(0, K, (B,), device=dev)
    y[0] = y[1]                              # two rows on one class
    ops.clip_loss_fwd_bwd(h["img"], h["txt"], h["img_n"], h["txt_n"], h["norms"], h["logits"], y, h["ls"],
                          h["dmm"], h["cos_ws"], h["loss"], h["dimg_n"], h["dtxt_n"], h["dimg"], h["dtxt"])
    hard = {k: h[k].clone() for k in ("loss", "dmm", "dimg", "dtxt")}
    _soft(h, F.one_hot(y, K).float().contiguous())
    assert torch.equal(h["dmm"], hard["dmm"])
    assert torch.equal(h["dimg"], hard["dimg"])
    torch.testing.assert_close(h["dtxt"].float(), hard["dtxt"].float(), rtol=2e-3, atol=1e-6)
    assert abs(h["loss"][1].item() - hard["loss"][1].item()) <= 2e-3      # CE is rounded to fp16
    assert h["loss"][2].item() == hard["loss"][2].item()

def test_sgd_and_clip(dev):
    torch.manual_seed(6)
    n16, n32 = 10000, 5000
    p16 = torch.randn(n16).half().to(dev)
    p32 = torch.randn(n32).to(dev)
    g16 = (torch.randn(n16) * 0.05).half().to(dev)
    g32 = (torch.randn(n32) * 0.05).to(dev)
    # reference: torch clip_grad_norm_ + SGD on copies
    rp16 = p16.clone().requires_grad_(True)
    rp32 = p32.clone().requires_grad_(True)
    rp16.grad = g16.clone()
    rp32.grad = g32.clone()
    torch.nn.utils.clip_grad_norm_([rp16, rp32], 1.0)
    opt = torch.optim.SGD([rp16, rp32], lr=0.01, momentum=0.9, weight_decay=5e-4, foreach=False)
    opt.step()
    # ours: segments = two tensors of each flat buffer
    import ctypes
    import numpy as np
    ce = ops.optim_chunk_elems()
    chunks = []
    segs = [(0, 1, 0, n16), (1, 0, 0, n32)]
    for sid, is16, a0, a1 in segs:
        for s in range(a0, a1, ce):
            chunks.append((sid, is16, s, min(a1, s + ce)))
    arr = np.zeros(len(chunks), dtype=np.dtype([("seg", np.int32), ("is16", np.int32), ("s", np.int64),
                                                ("e", np.int64)]))
    for i, c in enumerate(chunks):
        arr[i] = c
    dchunks = torch.from_numpy(arr.view(np.uint8)).to(dev)
    part = torch.empty(len(chunks), device=dev)
    out = torch.empty(3, device=dev)
    ops.clip_grad_norm(g16, g32, dchunks, len(chunks), 1.0, part, out)
    tot_ref = math.sqrt(sum(float(t.float().norm()) ** 2 for t in (g16, g32)))
    assert abs(out[0].item() - tot_ref) < 1e-3 * tot_ref
    b16 = torch.empty_like(p16)
    b32 = torch.empty_like(p32)
    # halt set (a non-finite loss earlier in the epoch): nothing changes
    snap = [t.clone() for t in (p16, g16, p32, g32)]
    halted = torch.tensor([0.01, 0.9, 5e-4, 1.0, 1.0], device=dev)
    ops.sgd_step(p16, g16, b16, out, halted)
    ops.sgd_step(p32, g32, b32, out, halted)
    assert all(torch.equal(a, b) for a, b in zip(snap, (p16, g16, p32, g32)))
    hyper = torch.tensor([0.01, 0.9, 5e-4, 1.0, 0.0], device=dev)
    ops.sgd_step(p16, g16, b16, out, hyper)
    ops.sgd_step(p32, g32, b32, out, hyper)
    assert (p16 != rp16.detach()).float().mean().item() < 1e-3
    torch.testing.assert_close(p32, rp32.detach(), rtol=1e-6, atol=1e-7)


def test_fedavg_reduce_ordered_kernel(dev):
    """mf_fedavg_reduce_ordered == the client-order fp32 sum of torch.stack(...) (trainers/maple_fed.py:311-314),
    bit for bit, for 1..8 clients, ragged lengths and a row stride larger than the length."""
    g = torch.Generator(device="cpu").manual_seed(3)
    for nclients in (1, 2, 3, 8):
        for n in (1, 7, 4096 + 3):
            stride = n + 5
            host = torch.randn(nclients, stride, generator=g) * torch.exp2(torch.randint(-8, 8, (nclients, stride),
                                                                                          generator=g).float())
            out = torch.empty(n, device=dev)
            ops.fedavg_reduce_ordered(host.to(dev).reshape(-1), nclients, out)
            ref = host[0, :n].clone()
            for c in range(1, nclients):
                ref += host[c, :n]
            assert torch.equal(out.cpu(), ref), (nclients, n)


def test_fedavg_kernels_single_client(dev):
    """World size 1 through the HIP kernels: the mean of one client is its own weights rounded to
    fp16 (the `.half()` of trainers/maple_fed.py:314 on fp32 keys); a NaN client restores the
    previous global weights (round skipped)."""
    from federated_multi_modal_amd.federated import FedAvgBucket

    class Eng:
        device = dev
        n16, n32 = 1000, 777
        reloaded = 0

        def after_weights_loaded(self):
            self.reloaded += 1

    e = Eng()
    e.flat16 = torch.randn(e.n16, device=dev).half()
    e.flat32 = torch.randn(e.n32, device=dev) * 3
    fed = FedAvgBucket(e)
    g16, g32 = e.flat16.clone(), e.flat32.clone()
    e.flat32.add_(1e-3)  # local training moved the weights
    local32 = e.flat32.clone()
    assert fed.run() == 1
    assert torch.equal(e.flat16, g16)
    assert torch.equal(e.flat32, local32.half().float())
    new32 = e.flat32.clone()
    e.flat32[5] = float("nan")
    assert fed.run() == 0
    assert torch.equal(e.flat32, new32) and torch.equal(e.flat16, g16)


def test_argmax_correct(dev):
    torch.manual_seed(9)
    B, K = 100, 38
    logits = torch.randn(B, K, device=dev).half()
    logits[3, 5] = logits[3, 7] = 50.0          # tie: first index wins
    logits[4, 9] = float("nan")                 # NaN is the maximum (torch.argmax)
    label = torch.randint(0, K, (B,), device=dev)
    label[:10] = logits[:10].float().argmax(1)
    pred = torch.empty(B, dtype=torch.int64, device=dev)
    acc = torch.zeros(2, device=dev)
    ops.argmax_correct(logits, label, pred, acc)
    ref = logits.float().cpu().argmax(1)
    assert torch.equal(pred.cpu(), ref)
    assert acc[0].item() == (ref == label.cpu()).sum().item() and acc[1].item() == B


@pytest.mark.parametrize("N,L,D,row0", [(5, 199, 768, 197), (7, 77, 512, 1)])
def test_layernorm_fwd_inject_equals_inject_then_ln(dev, N, L, D, row0):
    """The fused deep-prompt injection + ln_1 is bit-identical to the two separate kernels."""
    torch.manual_seed(L)
    x = torch.randn(N * L, D).half().to(dev)
    prompt = torch.randn(2, D).to(dev)
    g, b = torch.randn(D).to(dev), torch.randn(D).to(dev)
    x1 = x.clone()
    ops.prompt_inject_fwd(x1, prompt, N, L, row0, 2, D)
    y1, m1, r1 = ops.layernorm_fwd(x1, g, b)
    x2 = x.clone()
    y2 = torch.empty_like(y1)
    m2, r2 = torch.empty_like(m1), torch.empty_like(r1)
    ops.layernorm_fwd_inject(x2, g, b, y2, m2, r2, prompt, L, row0, 2)
    assert torch.equal(x1, x2) and torch.equal(y1, y2) and torch.equal(m1, m2) and torch.equal(r1, r2)


@pytest.mark.parametrize("N,L,D,row0", [(5, 199, 768, 197), (7, 77, 512, 1)])
def test_layernorm_bwd_inject_equals_bwd_then_inject_bwd(dev, N, L, D, row0):
    """ln_1 backward with the deep prompt's gradient fused in: dx and dgamma/dbeta bit-identical to the
    separate kernels; the prompt gradient equal up to fp32 summation order."""
    torch.manual_seed(L + 1)
    rows = N * L
    x = torch.randn(rows, D).half().to(dev)
    g, b = torch.rand(D).to(dev) + 0.5, torch.randn(D).to(dev)
    _, mean, rstd = ops.layernorm_fwd(x, g, b)
    dy = torch.randn(rows, D).half().to(dev)
    dres = torch.randn(rows, D).half().to(dev)
    # reference: partial-mode LN backward + batched reduce, then inject_bwd
    ref = ops.LNGradBatch(dev)
    dx1 = dres.clone()
    dg1, db1 = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    ref.bwd(dy, x, g, mean, rstd, dx1, dg1, db1, dres=dx1)
    ref.finish()
    pg1 = torch.empty(2, D, device=dev)
    ops.prompt_inject_bwd(dx1, N, L, row0, 2, D, pg1, accumulate=False, zero_rows=True)
    fused = ops.LNGradBatch(dev)
    dx2 = dres.clone()
    dg2, db2 = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    pg2 = torch.empty(2, D, device=dev)
    fused.bwd_inject(dy, x, g, mean, rstd, dx2, dg2, db2, dx2, pg2, L, row0, 2)
    fused.finish()
    assert torch.equal(dx1, dx2) and torch.equal(dg1, dg2) and torch.equal(db1, db2)
    torch.testing.assert_close(pg2, pg1, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,N,K,epi", [(796, 768, 3072, 2), (796, 768, 2304, 0), (770, 512, 2048, 2),
                                       (770, 512, 1536, 0), (796, 3072, 768, 3), (770, 1536, 512, 1)])
def test_small_client_tiles_bit_identical(dev, M, N, K, epi):
    """The small clients' tile picks (4-stage 64x64 / 32x64 rings, 96x64; csrc/gemm.hip) keep the K order of the
    64x64 two-stage tile they replaced: outputs (and the pre-activation of the QuickGELU epilogue) bit-identical."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).half().to(dev)
    B = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(dev)
    kw = {}
    if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU):
        kw["bias"] = (torch.randn(N, generator=g) * 0.1).half().to(dev)
    if epi == ops.EPI_BIAS_RESID:
        kw["aux_in"] = torch.randn(M, N, generator=g).half().to(dev)
    outs = []
    for tile in (0, 3):
        aux_out = torch.empty(M, N, device=dev, dtype=torch.float16) if epi == ops.EPI_BIAS_GELU else None
        outs.append((ops.gemm_nt(A, B, aux_out=aux_out, epilogue=epi, tile=tile, **kw), aux_out))
    assert torch.equal(outs[0][0], outs[1][0])
    if epi == ops.EPI_BIAS_GELU:
        assert torch.equal(outs[0][1], outs[1][1])
