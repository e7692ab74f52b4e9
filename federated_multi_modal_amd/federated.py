"""Federated averaging of the MaPLe trainables across clients, one client per GPU.

Reference (trainers/maple_fed.py):
  * check_weights_valid (:317-325)  per-key isnan/isinf scan of a client's state dict, host sync per key;
  * safe_average_weights (:309-315) per key: stack(float) -> nan_to_num -> mean(0) -> .half(), over the
    clients whose weights were valid (:271-277); all invalid -> round skipped (:288-290);
  * broadcast_weights (:327-339)    load_state_dict + drop SGD momentum + rebuild the LR schedule.

MI355X form: client i runs on rank i.  Every rank
  1. scans its flat trainable buffers with one kernel (mf_nonfinite_flag) -> device int flag;
  2. packs them into one fp32 bucket scaled by its validity (0/1) (mf_fedavg_pack + a scale);
  3. all-reduces (SUM) the bucket and the validity count over RCCL (xGMI) -- one collective of
     n16+n32 floats (57 MB at J=9) plus 4 bytes;
  4. unpacks mean = sum / n_valid rounded to fp16 into every trainable (mf_fedavg_unpack): the
     reference's `.half()` of every key, incl. fp32 LN params, deep prompts and logit_scale.
Frozen tensors are bit-identical across clients, so leaving them out of the bucket is
result-preserving (an fp32 mean of identical fp16 values is exact).
With world_size 1 (or no process group) the same kernels run with no collective.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import ops


class FedAvgBucket:
    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None):
        self.e = engine
        self.group = group
        dev = engine.device
        n = engine.n16 + engine.n32
        # [bucket | count]: one contiguous buffer so the mean and the valid-client count travel in ONE
        # all-reduce
        self.buf = torch.empty(n + 1, device=dev, dtype=torch.float32)
        self.bucket = self.buf[:n]
        self.count = self.buf[n:]
        self.flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.work = None

    def _distributed(self) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def start(self):
        """Validity scan + pack + (async) all-reduce; returns immediately (overlap with test())."""
        e = self.e
        self.flag.zero_()
        ops.nonfinite_flag(e.flat16, self.flag)
        ops.nonfinite_flag(e.flat32, self.flag)
        ops.fedavg_pack(e.flat16, e.flat32, self.bucket)
        valid = (self.flag == 0).to(torch.float32)
        self.bucket.mul_(valid)  # an invalid client contributes nothing (trainers/maple_fed.py:272-277)
        self.count.copy_(valid)
        self.work = None
        if self._distributed():
            self.work = dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self) -> int:
        """Wait, then write the fp16-rounded mean into every trainable; returns n_valid (0 -> skipped)."""
        if self.work is not None:
            self.work.wait()
            self.work = None
        n_valid = int(round(float(self.count.item())))
        if n_valid == 0:
            return 0  # every client failed: keep the global weights (trainers/maple_fed.py:288-290)
        e = self.e
        ops.fedavg_unpack(self.bucket, float(n_valid), e.flat16, e.flat32)
        e.after_weights_loaded()
        return n_valid

    def run(self) -> int:
        self.start()
        return self.finish()
