"""Diagnostic (GPU box): an upper bound on what removing LayerNorm round trips could buy the c4 step.

Captures the c4 train step as a hipGraph four ways in one process, interleaved over 5 rounds of 20 replays:
  full     -- the product step;
  -fwd     -- every LayerNorm FORWARD launch (mf_layernorm_fwd / _inject) left out of the graph;
  -bwd     -- every LayerNorm BACKWARD launch left out;
  -fwdbwd  -- both;
  -fwd+scan -- every LayerNorm forward replaced by a read-only pass over its input (the nonfinite scan
              kernel): what a stats-only launch would cost if the normalisation moved into the consumer
              GEMM's operand load at no cost there.
The variants compute wrong numbers (the consumers read stale buffers); they only time what the step would
be if those launches cost nothing.  A normalise-on-load fusion (LN applied in the consumer GEMM's operand
load, row statistics from a stats-only pass) removes at most the forward's y write + re-read, and keeps a
launch per LayerNorm, so its gain is bounded well below the `-fwd` delta."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

J, K, B, seed = 9, 38, 32, 0
dev = torch.device("cuda:0")
e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, seed), prompt_depth=J, seed=seed),
                device=dev)
e.set_lr(0.0026)
b = syn.client_batch(seed, 0, 0, B, K)
e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
e.train_step()

# the forward launches are module functions of ops; the backward ones are LNGradBatch methods
real = {("ops", n): getattr(ops, n) for n in ("layernorm_fwd", "layernorm_fwd_inject")}
real.update({("lnb", n): getattr(ops.LNGradBatch, n) for n in ("bwd", "bwd_inject")})


def noop(*a, **k):
    return None


flag = torch.zeros(1, dtype=torch.int32, device=dev)


def scan(x, *a, **k):  # a read-only pass over the LayerNorm input: stands in for a stats-only launch
    ops.nonfinite_flag(x, flag)


def patch(skip, repl=noop):
    for (where, n), f in real.items():
        setattr(ops if where == "ops" else ops.LNGradBatch, n, repl if where in skip else f)


graphs = {}
for name, skip, repl in (("full", (), noop), ("-fwd", ("ops",), noop), ("-fwd+scan", ("ops",), scan),
                         ("-bwd", ("lnb",), noop), ("-fwdbwd", ("ops", "lnb"), noop)):
    patch(skip, repl)
    graphs[name] = e.capture_train_step()
patch(())
for g in graphs.values():
    g.replay()
torch.cuda.synchronize()
res = {k: [] for k in graphs}
for rnd in range(5):
    for k, g in graphs.items():
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        res[k].append(1e3 * (time.perf_counter() - a) / 20)
base = sorted(res["full"])[2]
for k in graphs:
    v = sorted(res[k])
    print(f"{k:8s}: median {v[2]:.3f} ms/step ({100 * (base - v[2]) / base:+.1f} % of the full step), "
          f"rounds {', '.join(f'{x:.3f}' for x in res[k])}", flush=True)
