"""Diagnostic (GPU box): the 77-token and the EOT-truncated text tower stepped in lockstep (eager train steps,
alternating two batches of one client); after every step, every gradient and the weights are compared bit for bit and
the first differing elements are printed.

    python tests/diagnostics/eot_exact_steps.py [client] [steps] [J,K,B] [pair]
pair: "ft" (default: 77-token vs truncated), "ff" or "tt" (two identical engines: the run's own reproducibility),
"u" = truncated without the full-layout row reductions.
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

client = int(sys.argv[1]) if len(sys.argv) > 1 else 1
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
J, K, B = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "9,38,32").split(","))
seed = 0
dev = torch.device("cuda:0")
names = syn.synthetic_classnames(K, seed)
cb = [syn.client_batch(seed, client, s, B, K) for s in range(2)]
pair = sys.argv[4] if len(sys.argv) > 4 else "ft"
es = [MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=c in "tu"), device=dev)
      for c in pair]
for c, e in zip(pair, es):
    if c == "u":  # truncated without the full-layout reductions (the pre-r05 inexact mode)
        e.txt.live = None
    if "serial" in sys.argv[5:]:  # both towers on one stream (no concurrency between them)
        e.overlap_towers = False
print("text_len", [e.text_len for e in es], flush=True)
for e in es:
    e.set_lr(0.0026)
for s in range(steps):
    for e in es:
        e.img_in.copy_(torch.from_numpy(cb[s % 2].images).to(dev))
        e.label_in.copy_(torch.from_numpy(cb[s % 2].labels).to(dev))
        e.train_step()
    torch.cuda.synchronize()
    g0, g1 = es[0].grads(), es[1].grads()
    bad = []
    for n in g0:
        a, b = g0[n].float(), g1[n].float()
        d = (a != b)
        if d.any():
            idx = d.nonzero()[:3].tolist()
            bad.append((n, int(d.sum().item()), [(i, a[tuple(i)].item(), b[tuple(i)].item()) for i in idx]))
    w = int((es[0].flat16 != es[1].flat16).sum().item() + (es[0].flat32 != es[1].flat32).sum().item())
    # the LayerNorm dgamma / dbeta block partials of the vision tower (equal partials with unequal results: the
    # column reduction or a later write; unequal partials: the backward kernel's inputs)
    l0, l1 = es[0].vis.lnb, es[1].vis.lnb
    G0 = {v.data_ptr(): k for k, v in es[0].G.items()}
    for (k0, w0), (k1, w1) in zip(l0.ws.items(), l1.ws.items()):
        d = w0 != w1
        if d.any():
            half = w0.numel() // 2
            idx = d.nonzero().view(-1)
            print(f"   vision LN partials of {G0.get(k0, k0)} differ: {int(d[:half].sum())} in dgamma, "
                  f"{int(d[half:].sum())} in dbeta; element idx {idx[:6].tolist()} (block {int(idx[0]) // 768}, "
                  f"col {int(idx[0]) % 768}); ws ptr {w0.data_ptr():#x} / {w1.data_ptr():#x}", flush=True)
    # the saved forward activations of both towers after the backward (a write into them shows up here)
    for tname in ("vis", "txt"):
        t0, t1 = getattr(es[0], tname), getattr(es[1], tname)
        for attr in ("X", "X1", "QKV", "O", "Fp", "mean1", "rstd1", "mean2", "rstd2"):
            for i, (a, b) in enumerate(zip(getattr(t0, attr), getattr(t1, attr))):
                if a.shape == b.shape:
                    d = a.view(-1) != b.view(-1)
                    if d.any():
                        pos = d.nonzero()[:4].view(-1).tolist()
                        print(f"   {tname}.{attr}[{i}] differs in {int(d.sum())} elements, first flat idx {pos} "
                              f"(row {pos[0] // a.shape[-1] if a.dim() > 1 else pos[0]})", flush=True)
    print(f"step {s}: loss {es[0].loss()} / {es[1].loss()}, {len(bad)} gradients differ, {w} weights differ", flush=True)
    for n, c, ex in bad[:8]:
        print(f"   {n}: {c} elements, e.g. {ex}", flush=True)
    if bad or w:
        break
