"""Diagnostic (GPU box, `torch.distributed.run --nproc-per-node 2`, MAPFED_DIST_BACKEND=gloo or nccl): two engines
per rank (the 77-token text tower and the EOT-truncated one) take the same steps from the same seed and batches, then
one FedAvg each (args: c4 = the bench's client shape, graph = replayed steps); prints, per rank, whether the weights agree before and after the exchange."""
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402
from federated_multi_modal_amd.federated import FedAvgBucket  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group(os.environ.get("MAPFED_DIST_BACKEND", "gloo"))
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
torch.cuda.set_device(dev)
J, K, B, seed = (9, 38, 32, 0) if "c4" in sys.argv[1:] else (3, 10, 4, 0)
graph = "graph" in sys.argv[1:]
names = syn.synthetic_classnames(K, seed)
cb = [syn.client_batch(seed, rank, s, B, K) for s in range(2)]
out = []
for trunc in (False, True):
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=trunc), device=dev)
    e.set_lr(0.0026)
    imgs = [(torch.from_numpy(c.images).to(dev), torch.from_numpy(c.labels).to(dev)) for c in cb]
    f = FedAvgBucket(e)
    e.img_in.copy_(imgs[0][0])
    e.label_in.copy_(imgs[0][1])
    e.train_step()
    g = e.capture_train_step() if graph else None
    for i in range(7):
        e.img_in.copy_(imgs[i % 2][0])
        e.label_in.copy_(imgs[i % 2][1])
        g.replay() if graph else e.train_step()
    pre = (e.flat16.clone(), e.flat32.clone())
    f.start()
    f.finish()
    torch.cuda.synchronize()
    out.append((pre, (e.flat16.clone(), e.flat32.clone())))
(p0, a0), (p1, a1) = out
eq = lambda x, y: bool(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]))
nd = lambda x, y: int((x[0] != y[0]).sum().item() + (x[1] != y[1]).sum().item())
print(f"rank {rank}: pre-FedAvg equal {eq(p0, p1)} ({nd(p0, p1)} differ), post-FedAvg equal {eq(a0, a1)} "
      f"({nd(a0, a1)} differ)", flush=True)
dist.barrier()
dist.destroy_process_group()
