"""Diagnostic (GPU box): eager train step, hipGraph capture and one replay of a small engine, each
step printed -- isolates capture-time failures (e.g. a stream forked inside a captured side stream).
    python tests/diagnostics/capture_probe.py"""
import sys, torch
sys.path.insert(0, ".")
from federated_multi_modal_amd import synthetic as syn
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine
names = syn.synthetic_classnames(10, 0)
e = MapleEngine(EngineConfig(batch=4, classnames=names, prompt_depth=3, seed=0), device="cuda:0")
b = syn.client_batch(0, 0, 0, 4, 10)
e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
e.set_lr(0.001)
e.train_step()
torch.cuda.synchronize()
print("eager ok", e.loss(), flush=True)
g = e.capture_train_step()
print("captured", flush=True)
g.replay(); torch.cuda.synchronize()
print("replay ok", e.loss(), flush=True)
