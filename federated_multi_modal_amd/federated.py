"""Federated averaging of the MaPLe trainables across clients, one client per GPU.

Reference (trainers/maple_fed.py):
  * check_weights_valid (:317-325)  per-key isnan/isinf scan of a client's state dict, host sync per key;
  * safe_average_weights (:309-315) per key: stack(float) -> nan_to_num -> mean(0) -> .half(), over the
    clients whose weights were valid (:271-277); all invalid -> round skipped (:288-290);
  * broadcast_weights (:327-339)    load_state_dict + drop SGD momentum + rebuild the LR schedule.

MI355X form: client i runs on rank i.  Every rank
  1. scans its flat trainable buffers with one kernel (mf_nonfinite_flag) -> device int flag;
  2. packs them into one fp32 bucket [fp16 trainables | fp32 trainables | vote] with its validity vote
     (an invalid client packs zeros and vote 0; mf_fedavg_pack);
  3. exchanges the buckets over RCCL (xGMI), asynchronously, so the caller overlaps the collective with
     the client's last local test() (trainers/maple.py:646);
  4. unpacks mean = sum / n_valid rounded to fp16 into every trainable (mf_fedavg_unpack): the
     reference's `.half()` of every key, incl. fp32 LN params, deep prompts and logit_scale.

Two exchange modes (FED.AGGREGATION in the trainer config):
  * "ordered" (default): all_gather of the buckets (57 MB per client at J=9), then every rank sums them
    in client order on the device (mf_fedavg_reduce_ordered).  The fp32 summation order is the
    reference's torch.stack(...) order, so the fp16 result is bit-identical to safe_average_weights at any
    world size (CPU-torch mean semantics: sum then divide, which tests/golden/fedavg.npz pins).
  * "allreduce": one RCCL all_reduce(SUM) of the bucket.  Less traffic (a ring moves 2(N-1)/N of the
    bucket per link instead of (N-1) buckets), but RCCL's ring order changes the fp32 summation order
    per chunk; with three or more clients the fp16-rounded result can differ from the reference's in
    the last fp16 bit of rare elements.
Frozen tensors are bit-identical across clients, so leaving them out of the bucket is result-preserving
(an fp32 mean of identical fp16 values is exact).  With world_size 1 (or no process
group) the same kernels run with no collective.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import ops

MODES = ("ordered", "allreduce")


class _HipKernels:
    """The device kernels FedAvgBucket drives (libmapfed.so)."""
    nonfinite_flag = staticmethod(ops.nonfinite_flag)
    fedavg_pack = staticmethod(ops.fedavg_pack)
    fedavg_unpack = staticmethod(ops.fedavg_unpack)
    fedavg_reduce_ordered = staticmethod(ops.fedavg_reduce_ordered)


class FedAvgBucket:
    """`engine` needs: device, n16, n32, flat16 (fp16 trainables), flat32 (fp32 trainables) and
    after_weights_loaded().  `kernels` defaults to the HIP kernels; tests substitute host
    restatements to exercise the collective protocol on CPU ranks (gloo)."""

    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None, kernels=_HipKernels,
                 mode: str = "ordered"):
        if mode not in MODES:
            raise ValueError(f"FedAvg mode {mode!r}: one of {MODES}")
        self.e = engine
        self.group = group
        self.k = kernels
        self.mode = mode
        dev = engine.device
        n = engine.n16 + engine.n32
        # [bucket | count]: one contiguous buffer so the mean and the valid-client count travel in ONE
        # collective
        self.buf = torch.empty(n + 1, device=dev, dtype=torch.float32)
        self.bucket = self.buf[:n]
        self.count = self.buf[n:]
        self.flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.gathered = None
        self.world = dist.get_world_size(group) if self._distributed() else 1
        if mode == "ordered" and self.world > 1:
            self.gathered = torch.empty(self.world * (n + 1), device=dev, dtype=torch.float32)
        # the last global weights (what broadcast_weights would load): restored when a round fails
        self.global16 = engine.flat16.detach().clone()
        self.global32 = engine.flat32.detach().clone()
        self.work = None

    def _distributed(self) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def snapshot(self):
        """Take the engine's current weights as the global copy (after a checkpoint load or an explicit
        broadcast_weights: what an all-failed round reverts to)."""
        self.global16.copy_(self.e.flat16)
        self.global32.copy_(self.e.flat32)

    def start(self, collective: bool = True, failed: bool = False):
        """Validity scan + pack + (async) exchange; returns immediately (the caller overlaps the
        collective with test()).  failed=True: the client's local training raised (its weights are
        excluded, trainers/maple_fed.py:262-265).  collective=False packs only (several clients in one
        process reduce their buckets with reduce_local)."""
        e = self.e
        if failed:
            self.flag.fill_(1)
        else:
            self.flag.zero_()
            self.k.nonfinite_flag(e.flat16, self.flag)
            self.k.nonfinite_flag(e.flat32, self.flag)
        # an invalid client contributes zeros and no vote (trainers/maple_fed.py:272-277)
        self.k.fedavg_pack(e.flat16, e.flat32, self.flag, self.buf)
        self.work = None
        if collective and self._distributed():
            if self.gathered is not None:
                self.work = dist.all_gather_into_tensor(self.gathered, self.buf, group=self.group, async_op=True)
            else:
                self.work = dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        """Wait for the collective, then write the fp16-rounded mean into every trainable (device-side
        n_valid; n_valid == 0 leaves the weights at the previous global copy).  No host synchronisation."""
        gathered = False
        if self.work is not None:
            self.work.wait()
            self.work = None
            gathered = self.gathered is not None
        if gathered:
            self.k.fedavg_reduce_ordered(self.gathered, self.world, self.buf)
        e = self.e
        self.k.fedavg_unpack(self.buf, e.flat16, e.flat32, self.global16, self.global32)
        e.after_weights_loaded()

    def n_valid(self) -> int:
        """Valid clients of the last round (host sync)."""
        return int(round(float(self.count.item())))

    def run(self) -> int:
        self.start()
        self.finish()
        return self.n_valid()


def reduce_local(buckets) -> None:
    """In-process stand-in for the exchange when several clients share one process/GPU (the
    reference's sequential clients, trainers/maple_fed.py:247): SUM of every packed bucket in client
    order (== torch.stack(...) order), written back into each of them."""
    if len(buckets) < 2:
        return
    total = buckets[0].buf.clone()
    for b in buckets[1:]:
        total.add_(b.buf)
    for b in buckets:
        b.buf.copy_(total)
