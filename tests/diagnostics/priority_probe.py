"""Diagnostic (GPU box): does a stream priority survive hipGraph capture and shorten the c4 step?  The vision
tower (the step's critical path) is captured on a high-priority stream, the text tower on the engine's normal-
priority side stream; the two captures are timed alternately (graph replays, ms per step), and the weights after
the same number of replays are compared (priorities change scheduling only).

    python tests/diagnostics/priority_probe.py [rounds] [steps]
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
print("stream priority range (low, high):", torch.cuda.Stream.priority_range(), flush=True)
J, K, B, seed = 9, 38, 32, 0
names = syn.synthetic_classnames(K, seed)
cb = syn.client_batch(seed, 0, 0, B, K)


def build(prio):
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    e.set_lr(0.0026)
    e.img_in.copy_(torch.from_numpy(cb.images).to(dev))
    e.label_in.copy_(torch.from_numpy(cb.labels).to(dev))
    e.train_step()
    first = e.hyper[3].item()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev, priority=prio) if prio is not None else None
    with torch.cuda.graph(g, stream=cap):
        e.forward_backward()
        e.optimizer_step()
    e.hyper[3] = first
    return e, g


variants = {"default": build(None), "vision_high": build(-1)}
res = {k: [] for k in variants}
for r in range(rounds):
    for name, (e, g) in variants.items():
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        res[name].append(1e3 * (time.perf_counter() - t) / steps)
    print(f"round {r}: " + ", ".join(f"{k} {v[-1]:.3f} ms" for k, v in res.items()), flush=True)
(e0, _), (e1, _) = variants["default"], variants["vision_high"]
same = torch.equal(e0.flat16, e1.flat16) and torch.equal(e0.flat32, e1.flat32)
print({k: round(min(v), 3) for k, v in res.items()}, "weights equal:", same)
