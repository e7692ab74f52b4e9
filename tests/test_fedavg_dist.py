"""CPU tier: the FedAvg collective protocol (federated_multi_modal_amd/federated.py) across
world_size 2 and 3 gloo ranks, one client per rank, checked against the reference's
safe_average_weights / check_weights_valid semantics (trainers/maple_fed.py:271-325, restated in
oracle/maple_oracle.py and pinned to the reference by tests/golden/fedavg.npz).

The device kernels are replaced by host restatements here (no GPU in this tier); the GPU tier
(tests/test_kernels_gpu.py) checks the kernels themselves."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import maple_oracle as O


class HostKernels:
    @staticmethod
    def nonfinite_flag(x, flag):
        if not torch.isfinite(x.float()).all():
            flag.fill_(1)

    @staticmethod
    def fedavg_pack(p16, p32, invalid, bucket):
        n16, n32 = p16.numel(), p32.numel()
        bad = bool(invalid.item())
        bucket[:n16] = 0.0 if bad else p16.float()
        bucket[n16:n16 + n32] = 0.0 if bad else p32
        bucket[n16 + n32] = 0.0 if bad else 1.0

    @staticmethod
    def fedavg_unpack(bucket, p16, p32, g16, g32):
        n16, n32 = p16.numel(), p32.numel()
        n_valid = float(bucket[n16 + n32])
        if n_valid == 0:
            p16.copy_(g16)
            p32.copy_(g32)
            return
        v = (bucket[: n16 + n32] / n_valid).half()
        p16.copy_(v[:n16])
        p32.copy_(v[n16:].float())
        g16.copy_(p16)
        g32.copy_(p32)


class FakeEngine:
    def __init__(self, rank, n16=37, n32=29, bad=False):
        g = torch.Generator().manual_seed(100 + rank)
        self.device = torch.device("cpu")
        self.n16, self.n32 = n16, n32
        self.flat16 = torch.randn(n16, generator=g).half()
        self.flat32 = torch.randn(n32, generator=g)
        if bad:
            self.flat32[3] = float("nan")
        self.reloaded = 0

    def after_weights_loaded(self):
        self.reloaded += 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bad_ranks, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from federated_multi_modal_amd.federated import FedAvgBucket
    e = FakeEngine(rank, bad=rank in bad_ranks)
    g16, g32 = e.flat16.clone(), e.flat32.clone()
    e.flat16.copy_(FakeEngine(0).flat16)  # the previous global weights (identical on every rank)
    e.flat32.copy_(FakeEngine(0).flat32)
    fed = FedAvgBucket(e, kernels=HostKernels)
    e.flat16.copy_(g16)  # ... then this client's local training result
    e.flat32.copy_(g32)
    n_valid = fed.run()
    out[rank] = (n_valid, e.flat16.clone(), e.flat32.clone(), e.reloaded)
    dist.destroy_process_group()


def _run(world, bad_ranks=()):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, tuple(bad_ranks), out), nprocs=world, join=True)
    return dict(out)


@pytest.mark.parametrize("world,bad", [(2, ()), (3, (1,)), (2, (0, 1))])
def test_fedavg_allreduce_matches_reference(world, bad):
    res = _run(world, bad)
    clients = [FakeEngine(r, bad=r in bad) for r in range(world)]
    valid = [c for c in clients if O.check_weights_valid({"a": c.flat16, "b": c.flat32})]
    for r in range(world):
        n_valid, p16, p32, reloaded = res[r]
        assert n_valid == len(valid)
        if not valid:  # all clients failed: round skipped, every client back to the previous global
            assert torch.equal(p16, FakeEngine(0).flat16) and torch.equal(p32, FakeEngine(0).flat32)
            continue
        ref = O.safe_average_weights([{"a": c.flat16, "b": c.flat32} for c in valid])
        assert torch.equal(p16, ref["a"])                      # fp16 keys: bit-exact
        assert torch.equal(p32, ref["b"].float())              # fp32 keys take the .half() rounding
        assert reloaded == 1
    # every rank holds the same global weights (broadcast-free all-reduce)
    assert all(torch.equal(res[0][1], res[r][1]) for r in range(world))
