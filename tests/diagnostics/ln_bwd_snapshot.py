"""Diagnostic (GPU box): where do the timing-dependent vision LayerNorm dgamma partials of r05 come from?

Two identical engines (EOT-truncated text towers, the r05 reproducer `eot_exact_steps.py ... tt`) step in lockstep.
Every vision LayerNorm backward launch is followed, on its own stream, by copies of what its dgamma / dbeta partials
depend on (dy, x, mean, rstd) and of the partials it wrote.  After each step the copies of the two engines are
compared launch by launch, and every launch whose partials differ is recomputed on a quiet GPU from the copied
inputs (mf_layernorm_bwd, partials only): if the inputs are equal and the quiet recompute equals one engine's
partials, the other engine's launch computed something its inputs do not determine -- a read of a value that was
different while the kernel ran (a cross-stream write, or a producer not yet finished), not an arithmetic defect.

    python tests/diagnostics/ln_bwd_snapshot.py [steps] [J,K,B] [plain|copyx|twice]

copyx: every vision LayerNorm backward reads private copies of x / mean / rstd made just before it on its stream
(nothing else can write them while it runs); twice: each launch is followed by a second launch on the same inputs
into a scratch workspace, and the two launches' partials are compared.
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd._lib import call  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
J, K, B = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "9,38,32").split(","))
variant = sys.argv[3] if len(sys.argv) > 3 else "plain"
dev = torch.device("cuda:0")
names = syn.synthetic_classnames(K, 0)
cb = [syn.client_batch(0, 1, s, B, K) for s in range(2)]
es = [MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=0, eot_truncate=True), device=dev)
      for _ in range(2)]
for e in es:
    e.set_lr(0.0026)

snaps = {0: [], 1: []}
cur = [0]
orig_bwd, orig_inj = ops.LNGradBatch.bwd, ops.LNGradBatch.bwd_inject


def _snap(self, dy, x, mean, rstd, dgamma):
    if self is not es[cur[0]].vis.lnb:
        return
    ws = self.ws[dgamma.data_ptr()]
    snaps[cur[0]].append({"dy": dy.clone(), "x": x.clone(), "mean": mean.clone(), "rstd": rstd.clone(),
                          "ws": ws.clone(), "name": es[cur[0]].G_name.get(dgamma.data_ptr(), hex(dgamma.data_ptr())),
                          "stream": torch.cuda.current_stream().cuda_stream})


twice_bad = []


def _mine(self):
    return self is es[cur[0]].vis.lnb


def _second(self, dy, x, mean, rstd, dgamma):
    if variant != "twice" or not _mine(self):
        return
    ws = self.ws[dgamma.data_ptr()]
    w2 = torch.full_like(ws, float("nan"))
    rows, D = dy.shape
    P = ops._p
    call("mf_layernorm_bwd", P(dy), D, P(x), D, None, P(torch.ones(D, device=dev)), P(mean), P(rstd), None, 0,
         P(torch.empty_like(dy)), D, None, None, P(w2), rows, D, 0, ops._s())
    twice_bad.append((cur[0], es[cur[0]].G_name.get(dgamma.data_ptr()), ws.clone(), w2))


def _private(self, x, mean, rstd):
    if variant == "copyx" and _mine(self):
        return x.clone(), mean.clone(), rstd.clone()
    return x, mean, rstd


def bwd(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres=None, row_index=None, live=None):
    x, mean, rstd = _private(self, x, mean, rstd)
    r = orig_bwd(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres=dres, row_index=row_index, live=live)
    _second(self, dy, x, mean, rstd, dgamma)
    _snap(self, dy, x, mean, rstd, dgamma)
    return r


def bwd_inject(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, prompt_grad, L, row0, nrows, live=None):
    x, mean, rstd = _private(self, x, mean, rstd)
    r = orig_inj(self, dy, x, gamma, mean, rstd, dx, dgamma, dbeta, dres, prompt_grad, L, row0, nrows, live=live)
    _second(self, dy, x, mean, rstd, dgamma)
    _snap(self, dy, x, mean, rstd, dgamma)
    return r


ops.LNGradBatch.bwd, ops.LNGradBatch.bwd_inject = bwd, bwd_inject
for e in es:
    e.G_name = {v.data_ptr(): k for k, v in e.G.items()}


def quiet_partials(s):
    rows, D = s["dy"].shape
    ws = torch.full_like(s["ws"], float("nan"))
    dx = torch.empty_like(s["dy"])
    P = ops._p
    call("mf_layernorm_bwd", P(s["dy"]), D, P(s["x"]), D, None, P(torch.ones(D, device=dev)), P(s["mean"]),
         P(s["rstd"]), None, 0, P(dx), D, None, None, P(ws), rows, D, 0, ops._s())
    torch.cuda.synchronize()
    return ws


for step in range(steps):
    for i, e in enumerate(es):
        snaps[i] = []
        cur[0] = i
        e.img_in.copy_(torch.from_numpy(cb[step % 2].images).to(dev))
        e.label_in.copy_(torch.from_numpy(cb[step % 2].labels).to(dev))
        e.train_step()
    torch.cuda.synchronize()
    for eng, name, w1, w2 in twice_bad:
        d = (w1 != w2).nonzero().view(-1)
        if len(d):
            print(f"step {step} engine {eng} {name}: first and second launch differ at {len(d)} "
                  f"(cols {(d % 768).tolist()[:6]})", flush=True)
    twice_bad.clear()
    n_diff = 0
    for k, (a, b) in enumerate(zip(snaps[0], snaps[1])):
        eq = {f: bool(torch.equal(a[f], b[f])) for f in ("dy", "x", "mean", "rstd", "ws")}
        if all(eq.values()):
            continue
        n_diff += 1
        D = a["dy"].shape[1]
        nb = a["ws"].numel() // 2
        d = (a["ws"] != b["ws"]).nonzero().view(-1)
        q = quiet_partials(a)
        qa, qb = bool(torch.equal(q, a["ws"])), bool(torch.equal(q, b["ws"]))
        cols = (d % D).tolist()[:8]
        print(f"step {step} launch {k} {a['name']}: equal {eq}; partials differ at {len(d)} "
              f"(dgamma {int((d < nb).sum())}, dbeta {int((d >= nb).sum())}); blocks {sorted(set((d // D).tolist()))[:4]} "
              f"cols {cols}; quiet recompute == engine0 {qa}, == engine1 {qb}", flush=True)
        if not (qa and qb):
            for tag, w in (("engine0", a["ws"]), ("engine1", b["ws"])):
                dq = (w != q).nonzero().view(-1)
                if len(dq):
                    i0 = int(dq[0])
                    print(f"    {tag} vs quiet: {len(dq)} differ, first idx {i0} (block {i0 // D}, col {i0 % D}): "
                          f"{w[i0].item()!r} vs {q[i0].item()!r}", flush=True)
    print(f"step {step}: loss {es[0].loss()} / {es[1].loss()}; {len(snaps[0])} vision LN launches, "
          f"{n_diff} with a difference", flush=True)
    if n_diff:
        break
