"""Diagnostic: where the oracle's CPU training step spends its time on this host."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from oracle import maple_oracle as O  # noqa: E402

J, K, B = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (3, 10, 4)
t = time.perf_counter()
M = O.build_model(0, J, syn.synthetic_classnames(K, 0))
print(f"build {time.perf_counter() - t:.1f}s threads {torch.get_num_threads()}", flush=True)
b = syn.client_batch(0, 0, 0, B, K)
img, lab = torch.from_numpy(b.images), torch.from_numpy(b.labels)
t = time.perf_counter()
with torch.no_grad():
    O.forward(M, img, train=False)
print(f"eval fwd {time.perf_counter() - t:.1f}s", flush=True)
t = time.perf_counter()
loss = O.forward(M, img, lab, train=True)
print(f"train fwd {time.perf_counter() - t:.1f}s", flush=True)
from torch.profiler import profile
with profile() as p:
    t = time.perf_counter()
    loss.backward()
    print(f"bwd {time.perf_counter() - t:.1f}s", flush=True)
print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=12), flush=True)
