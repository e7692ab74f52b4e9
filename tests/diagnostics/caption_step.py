"""Diagnostic (GPU box): the c4 client step on caption-carrying batches (K19: the vision sequence grows
199 -> 455 rows), hipGraph-replayed, for rocprofv3 kernel traces:
    rocprofv3 --kernel-trace --stats -d gpurun_out/cap -o run -- python3 tests/diagnostics/caption_step.py"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.captions import caption_tokens, draw_caption_weights  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

J, K, B, seed, steps = 9, 38, 32, 0, int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, seed), prompt_depth=J, seed=seed,
                             captions=True), device=dev)
e.set_lr(0.0026)
e.set_captions(caption_tokens(syn.synthetic_captions(seed, 0, 0, B)), draw_caption_weights(torch.Generator().manual_seed(1)))
b = syn.client_batch(seed, 0, 0, B, K)
e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
e.train_step()
g = e.capture_train_step()
g.replay()
torch.cuda.synchronize()
a = time.perf_counter()
for _ in range(steps):
    g.replay()
torch.cuda.synchronize()
print(f"caption step: {1e3 * (time.perf_counter() - a) / steps:.2f} ms, vision rows {e.vis.Ls}, loss {e.loss():.4f}")
