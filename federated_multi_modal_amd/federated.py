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
  * "ordered" (default): a sharded client-ordered sum.  The bucket (57 MB per client at J=9, padded to
    a multiple of N) is cut into N shards; one all_to_all hands rank r shard r of every client, rank r
    sums its shard over the clients in client order on the device (mf_fedavg_reduce_ordered), and one
    all_gather returns every summed shard to every rank.  Each rank moves 2(N-1)/N of a bucket, the
    traffic of a ring all-reduce, but the fp32 summation order is the reference's torch.stack(...)
    order, so the fp16 result is bit-identical to safe_average_weights at any world size (CPU-torch
    mean semantics: sum then divide, which tests/golden/fedavg.npz pins).  On a GPU the chain runs on a
    side stream (all_to_all -> reduce -> all_gather), so start() returns at once and the caller's next
    kernels (the last local test()) run under it.
  * "allreduce": one RCCL all_reduce(SUM) of the bucket.  The same traffic, but RCCL's ring order
    changes the fp32 summation order per chunk; with three or more clients the fp16-rounded result can
    differ from the reference's in the last fp16 bit of rare elements.
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
                 mode: str = "ordered", shard_single: bool = False):
        if mode not in MODES:
            raise ValueError(f"FedAvg mode {mode!r}: one of {MODES}")
        self.e = engine
        self.group = group
        self.k = kernels
        self.mode = mode
        dev = engine.device
        n = engine.n16 + engine.n32
        self.world = dist.get_world_size(group) if self._distributed() else 1
        # shard_single: run the sharded ordered exchange even in a one-rank group (tests drive the RCCL
        # all_to_all -> reduce -> all_gather chain on a one-GPU box this way)
        self.shard_single = shard_single and dist.is_available() and dist.is_initialized()
        # [bucket | count | zero padding to a multiple of the world size]: one contiguous buffer so the
        # mean and the valid-client count travel in the same collectives
        padded = -(-(n + 1) // self.world) * self.world
        self.pbuf = torch.zeros(padded, device=dev, dtype=torch.float32)
        self.buf = self.pbuf[:n + 1]
        self.bucket = self.buf[:n]
        self.count = self.buf[n:]
        self.flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.sharded = mode == "ordered" and (self.world > 1 or self.shard_single)
        self.recv = self.shard = self.side = None
        self.host_stage = False
        if self.sharded:
            self.recv = torch.empty(padded, device=dev, dtype=torch.float32)  # [client][shard of this rank]
            self.shard = torch.empty(padded // self.world, device=dev, dtype=torch.float32)
            # RCCL on GPUs: the chain on a side stream.  Other backends (gloo: the CPU tests, and the
            # several-ranks-on-one-GPU rehearsal of bench.py) exchange host copies in finish().
            self.host_stage = dev.type == "cuda" and dist.get_backend(group) != "nccl"
            if dev.type == "cuda" and not self.host_stage:
                self.side = torch.cuda.Stream(device=dev)
        # the last global weights (what broadcast_weights would load): restored when a round fails
        self.global16 = engine.flat16.detach().clone()
        self.global32 = engine.flat32.detach().clone()
        self.work = None
        self.pending_a2a = None

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
        self.pending_a2a = None
        if collective and (self._distributed() or self.shard_single):
            if not self.sharded:
                self.work = dist.all_reduce(self.pbuf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            elif self.side is not None:
                # the whole chain on the side stream: the current stream only waits for it in finish()
                self.side.wait_stream(torch.cuda.current_stream(self.pbuf.device))
                with torch.cuda.stream(self.side):
                    a2a = dist.all_to_all_single(self.recv, self.pbuf, group=self.group, async_op=True)
                    a2a.wait()  # a stream dependency, not a host wait
                    self.k.fedavg_reduce_ordered(self.recv, self.world, self.shard)
                    self.work = dist.all_gather_into_tensor(self.pbuf, self.shard, group=self.group, async_op=True)
            else:  # gloo: reduce and gather in finish()
                src = self.pbuf.cpu() if self.host_stage else self.pbuf
                self.recv_x = torch.empty_like(src)
                self.pending_a2a = dist.all_to_all_single(self.recv_x, src, group=self.group, async_op=True)

    def finish(self):
        """Wait for the collective, then write the fp16-rounded mean into every trainable (device-side
        n_valid; n_valid == 0 leaves the weights at the previous global copy).  No host synchronisation."""
        if self.pending_a2a is not None:
            self.pending_a2a.wait()
            self.pending_a2a = None
            self.recv.copy_(self.recv_x)
            self.k.fedavg_reduce_ordered(self.recv, self.world, self.shard)
            if self.host_stage:
                out = torch.empty(self.pbuf.numel(), dtype=torch.float32)
                dist.all_gather_into_tensor(out, self.shard.cpu(), group=self.group)
                self.pbuf.copy_(out)
            else:
                dist.all_gather_into_tensor(self.pbuf, self.shard, group=self.group)
        if self.work is not None:
            self.work.wait()
            self.work = None
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
