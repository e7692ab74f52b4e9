"""Learning-rate schedule of the reference's client trainers.

trainers/maple.py:498-499 builds the optimizer and scheduler with Dassl's build_optimizer /
build_lr_scheduler (Dassl is un-vendored and unpinned; restated here from its published source):
SGD(lr, momentum, weight_decay, dampening, nesterov) and, for LR_SCHEDULER="cosine",
torch.optim.lr_scheduler.CosineAnnealingLR(T_max=MAX_EPOCH) wrapped in a ConstantWarmupScheduler
(WARMUP_EPOCH epochs at WARMUP_CONS_LR) when WARMUP_EPOCH > 0.  The scheduler is stepped once per
local epoch (trainers/maple.py:645,655-658) and REBUILT at every broadcast with
last_epoch = epoch - 1 (trainers/maple_fed.py:336-339), which is what makes the per-epoch LR of
later rounds differ from a single cosine cycle (SURVEY.md §7 "LR / optimizer semantics").

The schedule is evaluated on the host with torch's own CosineAnnealingLR over a one-element dummy
parameter group (so its recursive update is reproduced exactly); the value is handed to the device
SGD kernel through the engine's hyper-parameter buffer.
"""
from __future__ import annotations

import warnings

import torch
from torch.optim.lr_scheduler import CosineAnnealingLR, _LRScheduler


class _BaseWarmupScheduler(_LRScheduler):
    def __init__(self, optimizer, successor, warmup_epoch, last_epoch=-1):
        self.successor = successor
        self.warmup_epoch = warmup_epoch
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        raise NotImplementedError

    def step(self, epoch=None):
        if self.last_epoch >= self.warmup_epoch:
            self.successor.step(epoch)
            self._last_lr = self.successor.get_last_lr()
        else:
            super().step(epoch)


class ConstantWarmupScheduler(_BaseWarmupScheduler):
    def __init__(self, optimizer, successor, warmup_epoch, cons_lr, last_epoch=-1):
        self.cons_lr = cons_lr
        super().__init__(optimizer, successor, warmup_epoch, last_epoch)

    def get_lr(self):
        if self.last_epoch >= self.warmup_epoch:
            return self.successor.get_last_lr()
        return [self.cons_lr for _ in self.base_lrs]


class LinearWarmupScheduler(_BaseWarmupScheduler):
    def __init__(self, optimizer, successor, warmup_epoch, min_lr, last_epoch=-1):
        self.min_lr = min_lr
        super().__init__(optimizer, successor, warmup_epoch, last_epoch)

    def get_lr(self):
        if self.last_epoch >= self.warmup_epoch:
            return self.successor.get_last_lr()
        if self.last_epoch == 0:
            return [self.min_lr for _ in self.base_lrs]
        return [lr * self.last_epoch / self.warmup_epoch for lr in self.base_lrs]


def build_lr_scheduler(optimizer, optim_cfg):
    """Dassl build_lr_scheduler for the schedulers the MaPLe configs use."""
    name = optim_cfg.LR_SCHEDULER
    max_epoch = optim_cfg.MAX_EPOCH
    if name == "cosine":
        sched = CosineAnnealingLR(optimizer, float(max_epoch))
    elif name == "single_step":
        step = optim_cfg.STEPSIZE
        step = step[-1] if isinstance(step, (list, tuple)) else step
        if step <= 0:
            step = max_epoch
        sched = torch.optim.lr_scheduler.StepLR(optimizer, step_size=step, gamma=optim_cfg.GAMMA)
    elif name == "multi_step":
        sched = torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=list(optim_cfg.STEPSIZE),
                                                     gamma=optim_cfg.GAMMA)
    else:
        raise ValueError(f"Unsupported scheduler: {name}")
    if optim_cfg.WARMUP_EPOCH > 0:
        if not optim_cfg.WARMUP_RECOUNT:
            sched.last_epoch = optim_cfg.WARMUP_EPOCH
        if optim_cfg.WARMUP_TYPE == "constant":
            sched = ConstantWarmupScheduler(optimizer, sched, optim_cfg.WARMUP_EPOCH, optim_cfg.WARMUP_CONS_LR)
        elif optim_cfg.WARMUP_TYPE == "linear":
            sched = LinearWarmupScheduler(optimizer, sched, optim_cfg.WARMUP_EPOCH, optim_cfg.WARMUP_MIN_LR)
        else:
            raise ValueError(f"Unknown warmup type: {optim_cfg.WARMUP_TYPE}")
    return sched


# the dummy optimizer never steps (the SGD runs on the device), which torch would warn about
warnings.filterwarnings("ignore", message="Detected call of `lr_scheduler.step\\(\\)` before")


class HostLR:
    """The scheduler state of one client: a one-element torch SGD whose param group carries the LR
    (the reference's optimizer.param_groups[0]['lr'])."""

    def __init__(self, optim_cfg):
        self.cfg = optim_cfg
        self._p = torch.zeros(1, requires_grad=True)
        self.optim = torch.optim.SGD([self._p], lr=optim_cfg.LR, momentum=optim_cfg.MOMENTUM,
                                     weight_decay=optim_cfg.WEIGHT_DECAY)
        self.sched = build_lr_scheduler(self.optim, optim_cfg)

    @property
    def lr(self) -> float:
        return float(self.optim.param_groups[0]["lr"])

    def step(self):
        """update_lr (trainers/maple.py:655-658)."""
        self.sched.step()

    def rebuild(self, epoch: int | None):
        """broadcast_weights: rebuild the scheduler, last_epoch = epoch - 1 (trainers/maple_fed.py:336-339)."""
        self.sched = build_lr_scheduler(self.optim, self.cfg)
        if epoch is not None:
            self.sched.last_epoch = epoch - 1
