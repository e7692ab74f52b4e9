"""Diagnostic (GPU box): would splitting the vision tower's batch into two halves on two streams fill
the step's vision-only phases?  Times the vision tower's forward + backward (hipGraph replays) as
  (a) one B = 32 tower on one stream, (b) two B = 16 towers on two streams, (c) the two halves in
  sequence on one stream.
Gradients are not combined (timing only)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import N_CTX, EngineConfig, MapleEngine, _Tower  # noqa: E402

J, K, B, seed = 9, 38, 32, 0
dev = torch.device("cuda:0")
e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, seed), prompt_depth=J, seed=seed),
                device=dev)
e.set_lr(0.0026)
b = syn.client_batch(seed, 0, 0, B, K)
e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
e.train_step()
torch.cuda.synchronize()
d = e.cfg.dims
halves = [_Tower(e, "image_encoder", B // 2, e.Lv, d.vision_width, d.vision_heads, d.vision_layers, False,
                 e.G2 + 1) for _ in range(2)]
g = torch.Generator(device="cpu").manual_seed(1)
pg = [[torch.zeros(N_CTX, d.vision_width, device=dev) for _ in range(J - 1)] for _ in range(3)]
for t in [e.vis] + halves:
    t.X[0].copy_(torch.randn(t.X[0].shape, generator=g).half() * 0.5)


def run(t, k):
    t.forward(e.vis_deep)
    t.dX[:t.Rs[-1]].copy_(t.X[-1])  # a stand-in d(loss)/d(output) of the right shape
    t.backward(J - 1, pg[k])
    t.lnb.finish()


def cap(fn):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    gr.replay()
    torch.cuda.synchronize()
    return gr


s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)


def two_streams():
    main = torch.cuda.current_stream(dev)
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        run(halves[0], 1)
    with torch.cuda.stream(s2):
        run(halves[1], 2)
    main.wait_stream(s1)
    main.wait_stream(s2)


graphs = {"a: B=32, one stream": cap(lambda: run(e.vis, 0)),
          "b: 2 x B=16, two streams": cap(two_streams),
          "c: 2 x B=16, one stream": cap(lambda: (run(halves[0], 1), run(halves[1], 2)))}
res = {k: [] for k in graphs}
for rnd in range(5):
    for k, gr in graphs.items():
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(10):
            gr.replay()
        torch.cuda.synchronize()
        res[k].append(1e3 * (time.perf_counter() - a) / 10)
for k, v in res.items():
    v = sorted(v)
    print(f"{k}: median {v[len(v) // 2]:.3f} ms, min {v[0]:.3f}")
