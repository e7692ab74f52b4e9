"""GPU tier: the sharded client-ordered FedAvg exchange (federated.FedAvgBucket, mode "ordered") over
RCCL, in a one-rank group on the box's GPU: all_to_all -> mf_fedavg_reduce_ordered -> all_gather on the
side stream, with the caller's stream waiting only in finish().  With one client the round result is
that client's weights rounded to fp16 (the reference's safe_average_weights of one state dict), and an
invalid client restores the previous global copy.  The multi-rank protocol itself is covered on CPU ranks
(tests/test_fedavg_dist.py, gloo world 2 / 3)."""
import os

import pytest
import torch
import torch.distributed as dist

from federated_multi_modal_amd.federated import FedAvgBucket

pytestmark = pytest.mark.gpu


class _Eng:
    def __init__(self, dev, n16, n32, seed):
        g = torch.Generator().manual_seed(seed)
        self.device = dev
        self.n16, self.n32 = n16, n32
        self.flat16 = (torch.randn(n16, generator=g) * 3).half().to(dev)
        self.flat32 = (torch.randn(n32, generator=g) * 1e-3).to(dev)
        self.loaded = 0

    def after_weights_loaded(self):
        self.loaded += 1


@pytest.fixture
def rccl_group(dev):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield
    dist.destroy_process_group()


def test_sharded_ordered_exchange_over_rccl(dev, rccl_group):
    e = _Eng(dev, 1_000_003, 77_777, 1)
    ref16 = e.flat16.clone()
    ref32 = e.flat32.half().float()
    fed = FedAvgBucket(e, mode="ordered", shard_single=True)
    assert fed.sharded and fed.side is not None
    fed.start()
    x = torch.randn(2048, 2048, device=dev)  # caller work queued under the exchange
    y = x @ x
    fed.finish()
    torch.cuda.synchronize()
    assert fed.n_valid() == 1 and torch.isfinite(y).all()
    assert torch.equal(e.flat16, ref16) and torch.equal(e.flat32, ref32)
    # an invalid client: no valid vote -> the previous global weights come back
    e.flat32[5] = float("nan")
    fed.start()
    fed.finish()
    torch.cuda.synchronize()
    assert fed.n_valid() == 0
    assert torch.equal(e.flat16, ref16) and torch.equal(e.flat32, ref32)
