"""Diagnostic (GPU box): the c4 step's hipGraph replay time with the text tower on its side stream
(overlap_towers=True, the default) and with both towers on one stream, interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
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
graphs = {}
for ov in (True, False):
    e.overlap_towers = ov
    graphs[ov] = e.capture_train_step()
    graphs[ov].replay()
torch.cuda.synchronize()
res = {True: [], False: []}
for rnd in range(5):
    for ov in (True, False):
        g = graphs[ov]
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        res[ov].append(1e3 * (time.perf_counter() - a) / 20)
for ov in (True, False):
    v = sorted(res[ov])
    print(f"overlap_towers={ov}: median {v[len(v) // 2]:.3f} ms/step, min {v[0]:.3f} ({', '.join(f'{x:.3f}' for x in res[ov])})")
