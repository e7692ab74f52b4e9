"""Diagnostic (GPU box): is the LayerNorm backward's result a function of its inputs alone?

Fixed inputs at the c4 vision shape (6 368 x 768, the deep-prompt injection of rows 1..2 of every 199-row sequence,
a residual gradient), the dgamma / dbeta block partials of one quiet launch as the reference, then `reps` launches
each racing a co-runner on a second stream (a long GEMM, or the text tower's D = 512 LayerNorm backward) and `reps`
launches alone.  Every launch's partials and dx are compared bit for bit with the reference; a mismatch is printed
with its columns mod 8 and half-wave lanes (r05's symptom: dgamma only, one even element slot, lanes 16..31 of a
half-wave).  Run it against two builds (MAPFED_LIB=...) to tell a kernel-internal hazard (mismatches with constant
inputs) from a buffer race in the engine (none here).

    python tests/diagnostics/ln_bwd_race_probe.py [reps] [inject|plain] [gemm|ln512|poison|none]

poison: before every launch, tests/diagnostics/poison/libpoison.so fills every VGPR / AGPR and 64 KB of LDS of every
wave slot with junk (a different seed per launch) on the same stream: a kernel that reads a register it never wrote
then gives results that change from launch to launch.
"""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from federated_multi_modal_amd._lib import call  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
mode = sys.argv[2] if len(sys.argv) > 2 else "inject"
co = sys.argv[3] if len(sys.argv) > 3 else "gemm"
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(7)
N, L, D = 32, 199, 768
rows = N * L
x = (torch.randn(rows, D, generator=g) * 0.5).half().to(dev)
dy = (torch.randn(rows, D, generator=g) * 1e-3).half().to(dev)
dres = (torch.randn(rows, D, generator=g) * 1e-3).half().to(dev)
gamma = (1.0 + 0.1 * torch.randn(D, generator=g)).float().to(dev)
beta = (0.1 * torch.randn(D, generator=g)).float().to(dev)
mean = torch.empty(rows, device=dev)
rstd = torch.empty(rows, device=dev)
y = torch.empty_like(x)
ops.layernorm_fwd(x, gamma, beta, y, mean, rstd)
nblk = call("mf_layernorm_bwd_blocks", rows)
P = ops._p


def launch(ws, dx, inj):
    if mode == "inject":
        call("mf_layernorm_bwd_inject", P(dy), D, P(x), D, P(gamma), P(mean), P(rstd), P(dres), D, P(dx), D, P(ws),
             rows, D, P(inj), L, 1, 2, ops._s())
    else:
        call("mf_layernorm_bwd", P(dy), D, P(x), D, None, P(gamma), P(mean), P(rstd), P(dres), D, P(dx), D, None,
             None, P(ws), rows, D, 0, ops._s())


def bufs():
    return (torch.full((2 * nblk * D,), float("nan"), device=dev), torch.empty_like(x),
            torch.full((N * 2 * D,), float("nan"), device=dev))


ref = bufs()
launch(*ref)
torch.cuda.synchronize()

# co-runners on a second stream
side = torch.cuda.Stream()
A = torch.randn(8192, 768, device=dev).half()
Bw = torch.randn(3072, 768, device=dev).half()
C = torch.empty(8192, 3072, device=dev).half()
xt = (torch.randn(2926, 512, device=dev) * 0.5).half()
dyt = (torch.randn(2926, 512, device=dev) * 1e-3).half()
gt = torch.ones(512, device=dev)
mt, rt = torch.empty(2926, device=dev), torch.empty(2926, device=dev)
ops.layernorm_fwd(xt, gt, torch.zeros(512, device=dev), torch.empty_like(xt), mt, rt)
wst = torch.empty(2 * call("mf_layernorm_bwd_blocks", 2926) * 512, device=dev)
dxt = torch.empty_like(xt)


poison = None
if co == "poison":
    poison = ctypes.CDLL(str(Path(__file__).resolve().parent / "poison" / "libpoison.so"))
    poison.mf_diag_poison.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
nseed = [0]


def corun():
    if poison is not None:
        nseed[0] += 1
        assert poison.mf_diag_poison(nseed[0], 2048, ops._s()) == 0
        return
    with torch.cuda.stream(side):
        for _ in range(4):
            if co == "gemm":
                ops.gemm_nt(A, Bw, C=C)
            elif co == "ln512":
                call("mf_layernorm_bwd", P(dyt), 512, P(xt), 512, None, P(gt), P(mt), P(rt), None, 0, P(dxt), 512,
                     None, None, P(wst), 2926, 512, 0, ops._s())


def compare(tag, i, out):
    ws, dx, inj = out
    bad = []
    dg = (ws[: nblk * D] != ref[0][: nblk * D]).nonzero().view(-1)
    db = (ws[nblk * D:] != ref[0][nblk * D:]).nonzero().view(-1)
    ddx = (dx.view(-1) != ref[1].view(-1)).nonzero().view(-1)
    dinj = (inj != ref[2]).nonzero().view(-1) if mode == "inject" else dg[:0]
    if len(dg) or len(db) or len(ddx) or len(dinj):
        cols = (dg % D).tolist()[:12]
        print(f"{tag} rep {i}: dgamma {len(dg)} db {len(db)} dx {len(ddx)} inj {len(dinj)}; dgamma blocks "
              f"{sorted(set((dg // D).tolist()))[:6]} cols {cols} col%8 {sorted(set(c % 8 for c in cols))} "
              f"half-wave lane {sorted(set((c // 8) % 32 for c in cols))}", flush=True)
        bad.append(i)
    return bad


outs = [bufs() for _ in range(8)]
nbad = {"corun": 0, "alone": 0}
for tag in ("corun", "alone"):
    for i in range(reps):
        o = outs[i % 8]
        o[0].fill_(float("nan"))
        torch.cuda.synchronize()
        if tag == "corun":
            corun()
        launch(*o)
        torch.cuda.synchronize()
        nbad[tag] += len(compare(tag, i, o))
    print(f"{tag}: {nbad[tag]} of {reps} launches differ from the reference", flush=True)
print("RESULT", mode, co, nbad, flush=True)
