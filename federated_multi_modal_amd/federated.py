"""Federated averaging of the MaPLe trainables across clients, one or more clients per GPU.

Reference (trainers/maple_fed.py):
  * check_weights_valid (:317-325)  per-key isnan/isinf scan of a client's state dict, host sync per key;
  * safe_average_weights (:309-315) per key: stack(float) -> nan_to_num -> mean(0) -> .half(), over the
    clients whose weights were valid (:271-277); all invalid -> round skipped (:288-290);
  * broadcast_weights (:327-339)    load_state_dict + drop SGD momentum + rebuild the LR schedule.

MI355X form: the N clients are spread over the ranks in contiguous blocks (rank r trains clients
r*C .. r*C + C - 1 one after another, C = N / world; C = 1 is one client per GPU).  For every client
  1. one kernel scans its flat trainable buffers (mf_nonfinite_flag) -> device int flag;
  2. its buffers are packed into one fp32 bucket [fp16 trainables | fp32 trainables | vote] with its
     validity vote (an invalid client packs zeros and vote 0; mf_fedavg_pack);
then FedAvgExchange moves every rank's buckets over RCCL (xGMI), asynchronously, so the caller overlaps
the collective with the last client's last local test() (trainers/maple.py:646), and finally
  3. every bucket unpacks mean = sum / n_valid rounded to fp16 into its client's trainables
     (mf_fedavg_unpack): the reference's `.half()` of every key, incl. fp32 LN params, deep prompts and
     logit_scale.

Two exchange modes (FED.AGGREGATION in the trainer config):
  * "ordered" (default): a sharded client-ordered sum.  Every bucket (57 MB per client at J=9, padded to
    a multiple of the world size W) is cut into W shards; one all_to_all hands rank r shard r of every
    client ([source rank][local client] = global client order), rank r sums its shard over the N clients
    in client order on the device (mf_fedavg_reduce_ordered), and one all_gather returns every summed
    shard to every rank.  Each rank moves 2(W-1)/W of C buckets, the traffic of a ring all-reduce, but
    the fp32 summation order is the reference's torch.stack(...) order, so the fp16 result is
    bit-identical to safe_average_weights at any world size (CPU-torch mean semantics: sum then divide,
    which tests/golden/fedavg.npz pins).  On a GPU the chain runs on a side stream (all_to_all -> reduce
    -> all_gather), so start() returns at once and the caller's next kernels run under it; under gloo (the
    world-size 2 / 3 / 8 CPU tests) the same _ordered_chain runs with host waits, so those tests cover its
    collective order and arithmetic -- not the RCCL stream dependencies, nor the start() / finish() overlap
    with caller kernels, which only an RCCL run with more than one GPU exercises (the driver's 8-GPU bench).
  * "allreduce": the rank's buckets summed in client order, then one RCCL all_reduce(SUM).  The same
    traffic, but RCCL's ring order changes the fp32 summation order per chunk; with three or more ranks the
    fp16-rounded result can differ from the reference's in the last fp16 bit of rare elements.
A client that fails after its bucket was packed (its last test() raising, after the exchange started) is
still excluded, as the reference's `continue` excludes it (trainers/maple_fed.py:262-265): finish() agrees
on such late failures with one 4-byte all_reduce and, when there is one, re-packs every local bucket
(failed ones with vote 0; the weights are untouched until unpack) and exchanges again.
Frozen tensors are bit-identical across clients, so leaving them out of the bucket is result-preserving
(an fp32 mean of identical fp16 values is exact).  With world_size 1 (or no process
group) the same kernels run with no collective.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist

from . import ops

MODES = ("ordered", "allreduce")


class FederatedAbort(RuntimeError):
    """Raised on every rank when one rank stops the run (FedAvgExchange.finish(abort=True))."""


class _HipKernels:
    """The device kernels FedAvgBucket drives (libmapfed.so)."""
    nonfinite_flag = staticmethod(ops.nonfinite_flag)
    fedavg_pack = staticmethod(ops.fedavg_pack)
    fedavg_unpack = staticmethod(ops.fedavg_unpack)
    fedavg_reduce_ordered = staticmethod(ops.fedavg_reduce_ordered)


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


class FedAvgBucket:
    """One client's bucket.  `engine` needs: device, n16, n32, flat16 (fp16 trainables), flat32 (fp32
    trainables) and after_weights_loaded().  `kernels` defaults to the HIP kernels; tests substitute host
    restatements to exercise the collective protocol on CPU ranks (gloo).

    pack() / unpack() are the per-client halves; start() / finish() / run() exchange this one bucket
    alone (one client per rank: the bench and the single-client tests).  Several clients per rank
    exchange through one FedAvgExchange over all their buckets."""

    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None, kernels=_HipKernels,
                 mode: str = "ordered", shard_single: bool = False):
        if mode not in MODES:
            raise ValueError(f"FedAvg mode {mode!r}: one of {MODES}")
        self.e = engine
        self.group = group
        self.k = kernels
        self.mode = mode
        self.shard_single = shard_single
        dev = engine.device
        n = engine.n16 + engine.n32
        self.world = _world(group)
        # [bucket | count | zero padding to a multiple of the world size]: one contiguous buffer so the
        # mean and the valid-client count travel in the same collectives
        padded = -(-(n + 1) // self.world) * self.world
        self.pbuf = torch.zeros(padded, device=dev, dtype=torch.float32)
        self.buf = self.pbuf[:n + 1]
        self.bucket = self.buf[:n]
        self.count = self.buf[n:]
        self.flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.failed = False
        # the last global weights (what broadcast_weights would load): restored when a round fails
        self.global16 = engine.flat16.detach().clone()
        self.global32 = engine.flat32.detach().clone()
        self._x: Optional[FedAvgExchange] = None

    # -- per client
    def pack(self, failed: bool = False):
        """Validity scan + pack.  failed=True: the client's local training raised (its weights are
        excluded, trainers/maple_fed.py:262-265); an invalid client contributes zeros and no vote
        (:272-277)."""
        e = self.e
        self.failed = failed
        if failed:
            self.flag.fill_(1)
        else:
            self.flag.zero_()
            self.k.nonfinite_flag(e.flat16, self.flag)
            self.k.nonfinite_flag(e.flat32, self.flag)
        self.k.fedavg_pack(e.flat16, e.flat32, self.flag, self.buf)

    def unpack(self):
        """The fp16-rounded mean into every trainable (device-side n_valid; n_valid == 0 leaves the weights
        at the previous global copy).  No host synchronisation."""
        e = self.e
        self.k.fedavg_unpack(self.buf, e.flat16, e.flat32, self.global16, self.global32)
        e.after_weights_loaded()

    def snapshot(self):
        """Take the engine's current weights as the global copy (after a checkpoint load or an explicit
        broadcast_weights: what an all-failed round reverts to)."""
        self.global16.copy_(self.e.flat16)
        self.global32.copy_(self.e.flat32)

    def n_valid(self) -> int:
        """Valid clients of the last round (host sync)."""
        return int(round(float(self.count.item())))

    # -- this bucket alone
    @property
    def exchange(self) -> "FedAvgExchange":
        if self._x is None:
            self._x = FedAvgExchange([self], group=self.group, mode=self.mode, shard_single=self.shard_single)
        return self._x

    @property
    def sharded(self) -> bool:
        return self.exchange.sharded

    @property
    def side(self):
        return self.exchange.side

    def start(self, collective: bool = True, failed: bool = False):
        """pack + (async) exchange; returns immediately (the caller overlaps the collective with test()).
        collective=False packs only."""
        self.pack(failed)
        if collective:
            self.exchange.start()

    def finish(self, late_failed: Optional[bool] = None):
        """Wait for the exchange, then unpack.  late_failed: whether the client failed after start()
        (None: the caller ran nothing that can fail in between -- no agreement collective)."""
        if self._x is not None and self._x.started:
            self._x.finish(None if late_failed is None else ([0] if late_failed else []))
        self.unpack()

    def run(self) -> int:
        self.start()
        self.finish()
        return self.n_valid()


class FedAvgExchange:
    """The exchange of one rank's buckets (its C clients, in client order) with every other rank's."""

    def __init__(self, buckets: Sequence[FedAvgBucket], group: Optional[dist.ProcessGroup] = None,
                 mode: str = "ordered", shard_single: bool = False):
        if mode not in MODES:
            raise ValueError(f"FedAvg mode {mode!r}: one of {MODES}")
        self.b = list(buckets)
        assert self.b and len({x.pbuf.numel() for x in self.b}) == 1
        b0 = self.b[0]
        self.group, self.mode, self.k = group, mode, b0.k
        self.C = len(self.b)
        self.world = _world(group)
        self.distributed = dist.is_available() and dist.is_initialized() and (self.world > 1 or shard_single)
        dev = b0.pbuf.device
        padded = b0.pbuf.numel()
        self.S = padded // self.world
        # shard_single: run the sharded ordered exchange even in a one-rank group (tests drive the RCCL
        # all_to_all -> reduce -> all_gather chain on a one-GPU box this way)
        self.sharded = self.distributed and mode == "ordered"
        self.side = None
        self.host_stage = False
        # the exchange's send image: C == 1 sends the bucket itself; C > 1 stages [dest rank][client][shard]
        self.stage = None if self.C == 1 else torch.empty(self.world, self.C, self.S, device=dev, dtype=torch.float32)
        # where the exchanged sum lands (C == 1: back into the bucket; C > 1: a total copied into every bucket)
        self.total = b0.pbuf if self.C == 1 else torch.empty(padded, device=dev, dtype=torch.float32)
        self.recv = self.shard = None
        if self.sharded:
            self.recv = torch.empty(self.world * self.C * self.S, device=dev, dtype=torch.float32)
            self.shard = torch.empty(self.S, device=dev, dtype=torch.float32)
        if self.distributed:
            # RCCL on GPUs: the chain on a side stream.  Other backends (gloo: the CPU tests, and the
            # several-ranks-on-one-GPU rehearsal of bench.py) exchange host copies in finish().
            self.host_stage = dev.type == "cuda" and dist.get_backend(group) != "nccl"
            if dev.type == "cuda" and not self.host_stage:
                self.side = torch.cuda.Stream(device=dev)
        self.started = False
        self.work = None

    def _send_image(self) -> torch.Tensor:
        if self.C == 1:
            return self.b[0].pbuf
        for j, x in enumerate(self.b):
            self.stage[:, j, :].copy_(x.pbuf.view(self.world, self.S))
        return self.stage.view(-1)

    def _local_sum(self) -> torch.Tensor:
        """The rank's buckets summed in client order (== torch.stack(...) order over these clients)."""
        if self.C == 1:
            return self.b[0].pbuf
        self.total.copy_(self.b[0].pbuf)
        for x in self.b[1:]:
            self.total.add_(x.pbuf)
        return self.total

    def start(self):
        """Launch the exchange of the packed buckets (asynchronously where the backend allows)."""
        self.started = True
        self.work = None
        if not self.distributed:
            return  # one process: the sum is formed in finish()
        if not self.sharded:
            src = self._local_sum()
            if src is not self.total:
                self.total.copy_(src)
            self.work = dist.all_reduce(self.total, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return
        send = self._send_image()
        if self.side is not None:
            # the whole chain on the side stream: the current stream only waits for it in finish()
            self.side.wait_stream(torch.cuda.current_stream(send.device))
            with torch.cuda.stream(self.side):
                self.work = self._ordered_chain(send)
        else:  # gloo: the same chain, its waits host waits
            self.work = self._ordered_chain(send)

    def _ordered_chain(self, send: torch.Tensor):
        """all_to_all of the shards -> client-ordered sum of this rank's shard -> all_gather of the sums.
        One code path for every backend: under RCCL (on the side stream) a2a.wait() is a stream dependency;
        under gloo it is a host wait, and with device buckets (host_stage) the collectives move host copies.
        Returns the all_gather's work handle (None when it completed here)."""
        hs = self.host_stage
        recv = torch.empty(self.recv.numel(), dtype=torch.float32) if hs else self.recv
        a2a = dist.all_to_all_single(recv, send.cpu() if hs else send, group=self.group, async_op=True)
        a2a.wait()
        if hs:
            self.recv.copy_(recv)
        self.k.fedavg_reduce_ordered(self.recv, self.world * self.C, self.shard)
        if hs:
            out = torch.empty(self.total.numel(), dtype=torch.float32)
            dist.all_gather_into_tensor(out, self.shard.cpu(), group=self.group)
            self.total.copy_(out)
            return None
        return dist.all_gather_into_tensor(self.total, self.shard, group=self.group, async_op=True)

    def _complete(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        if not self.distributed:
            self._local_sum()
        if self.total is not self.b[0].pbuf:
            for x in self.b:
                x.pbuf.copy_(self.total)

    def _agree(self, code: int) -> int:
        """Max over the ranks of a small status code (0 ok, 1 a late client failure, 2 a rank aborts)."""
        if not self.distributed:
            return code
        dev = self.b[0].pbuf.device
        on_dev = dev.type == "cuda" and not self.host_stage
        t = torch.tensor([code], dtype=torch.int32, device=dev if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def finish(self, late_failed: Optional[Iterable[int]] = (), abort: bool = False):
        """Wait for the exchange; afterwards every local bucket holds the sum over all clients (unpack
        follows).  late_failed: local client indices that failed after they were packed (None: nothing ran
        between start and finish that can fail, so the ranks skip agreeing on it).  abort: this rank hit an
        error the reference does not catch (e.g. the ValueError of a non-finite input, trainers/maple.py:
        526-535); every rank then raises FederatedAbort instead of waiting in the next round's collectives."""
        late = sorted(set(late_failed)) if late_failed is not None else None
        code = self._agree(2 if abort else int(bool(late))) if late is not None else 0
        if code == 2:
            self._complete()
            self.started = False
            raise FederatedAbort("a rank stopped the federated run (an error the round loop does not catch)")
        if code == 1:
            self._complete()  # drain the exchange in flight (every rank does, in the same order)
            for j, x in enumerate(self.b):
                x.pack(failed=x.failed or j in late)
            self.start()
        self._complete()
        self.started = False

    def n_valid(self) -> int:
        return self.b[0].n_valid()
