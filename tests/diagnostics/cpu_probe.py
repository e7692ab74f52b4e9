"""Diagnostic: host-CPU speed of the reference's fp16 ops on this machine (GPU box host)."""
import os
import time

import torch
import torch.nn.functional as F

print("threads", torch.get_num_threads(), "cpu_count", os.cpu_count(), "OMP", os.environ.get("OMP_NUM_THREADS"),
      "capability", torch.backends.cpu.get_cpu_capability(), flush=True)
try:
    print(open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0], flush=True)
except Exception:
    pass
for dt in (torch.float32, torch.float16, torch.bfloat16):
    a = torch.randn(796, 768).to(dt)
    w = torch.randn(2304, 768).to(dt)
    F.linear(a, w)
    t = time.perf_counter()
    for _ in range(3):
        F.linear(a, w)
    dtm = (time.perf_counter() - t) / 3
    print(f"linear 796x768x2304 {dt}: {dtm * 1e3:.1f} ms  ({2 * 796 * 768 * 2304 / dtm / 1e9:.1f} GFLOP/s)", flush=True)
q = torch.randn(4, 12, 199, 64).half()
t = time.perf_counter()
F.scaled_dot_product_attention(q, q, q)
print(f"sdpa fp16 4x12x199: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
