"""LR schedules: gradual warm-up then multi-step decay (``distar/ctools/torch_utils/lr_scheduler_util.py``
GradualWarmupScheduler + MultiStepLR, wired by ``base_learner.py:157-181``)."""
from __future__ import annotations

import torch


class GradualWarmup(torch.optim.lr_scheduler.LRScheduler):
    """Linear warm-up from ``lr/multiplier``-ish start to ``lr * multiplier`` over ``total_epoch`` steps,
    then hand over to ``after_scheduler`` (if any)."""

    def __init__(self, optimizer, multiplier: float = 1.0, total_epoch: int = 1000, after_scheduler=None):
        self.multiplier = multiplier
        self.total_epoch = max(int(total_epoch), 1)
        self.after_scheduler = after_scheduler
        self.finished = False
        super().__init__(optimizer)

    def get_lr(self):
        e = self.last_epoch
        if e > self.total_epoch:
            if self.after_scheduler is not None:
                if not self.finished:
                    self.after_scheduler.base_lrs = [b * self.multiplier for b in self.base_lrs]
                    self.finished = True
                return self.after_scheduler.get_last_lr()
            return [b * self.multiplier for b in self.base_lrs]
        if self.multiplier == 1.0:
            return [b * float(e) / self.total_epoch for b in self.base_lrs]
        return [b * ((self.multiplier - 1.0) * e / self.total_epoch + 1.0) for b in self.base_lrs]

    def step(self, epoch=None):
        if self.finished and self.after_scheduler is not None:
            self.after_scheduler.step()
            self._last_lr = self.after_scheduler.get_last_lr()
            self.last_epoch += 1
        else:
            super().step()


class _Const(torch.optim.lr_scheduler.LRScheduler):
    def get_lr(self):
        return list(self.base_lrs)


def build_lr_scheduler(optimizer, cfg=None):
    cfg = cfg or {}
    t = cfg.get('type', 'none')
    multi = torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=list(cfg.get('milestones', [])),
                                                 gamma=cfg.get('decay_rate', 1.0)) if t in ('multistep', 'warmup') else None
    if t == 'warmup':
        return GradualWarmup(optimizer, cfg.get('multiplier', 1.0), cfg.get('warm_up_steps', 1000), multi)
    if t == 'multistep':
        return multi
    return _Const(optimizer)
