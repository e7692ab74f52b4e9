"""Diagnostic (GPU box): can a client's test() pass share the GPU with its next local epoch?  Times, on one box,
an epoch's worth of c4 training steps (graph replays, main stream), a PatternNet test pass on the forward-only
eval engine (400-image launches, its own weights, a second stream), and both enqueued together.  Timing only:
the two engines hold separate weights, so nothing here says anything about results.
    python tests/diagnostics/overlap_train_eval.py [steps=19] [launches=23] [reps=3]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 19
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 23
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
names = syn.synthetic_classnames(38, 0)
eng = MapleEngine(EngineConfig(batch=32, classnames=names, prompt_depth=9, seed=0), device=dev)
eng.set_lr(0.0026)
cb = syn.client_batch(0, 0, 0, 32, 38)
eng.img_in.copy_(torch.from_numpy(cb.images).to(dev))
eng.label_in.copy_(torch.from_numpy(cb.labels).to(dev))
eng.train_step()
graph = eng.capture_train_step()
ev = MapleEngine(EngineConfig(batch=400, classnames=names, prompt_depth=9, seed=1, inference=True), device=dev)
imgs = torch.cat([torch.from_numpy(cb.images).to(dev)] * 13)[:400].contiguous()
labs = torch.cat([torch.from_numpy(cb.labels).to(dev)] * 13)[:400].contiguous()
acc = torch.zeros(2, device=dev)
side = torch.cuda.Stream(dev)
ev.img_in.copy_(imgs)
ev.eval_batch(labs, acc)
torch.cuda.synchronize()


def train():
    for _ in range(steps):
        graph.replay()


def test():
    with torch.cuda.stream(side):
        for _ in range(launches):
            ev.img_in.copy_(imgs)
            ev.eval_batch(labs, acc, reuse_text=True)


def timed(fn):
    torch.cuda.synchronize()
    a = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - a)


def both():
    test()
    train()


for r in range(reps):
    t_tr, t_te, t_both = timed(train), timed(test), timed(both)
    print(f"train {steps} steps {t_tr:7.1f} ms | test {launches} x 400 images {t_te:7.1f} ms | sum {t_tr + t_te:7.1f} "
          f"| overlapped {t_both:7.1f} ms ({100 * (1 - t_both / (t_tr + t_te)):.1f} % saved)", flush=True)
