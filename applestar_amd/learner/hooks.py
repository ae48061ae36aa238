"""Learner hooks (``distar/ctools/worker/learner/learner_hook.py``): priority-sorted callables run at
``before_run`` / ``before_iter`` / ``after_iter`` / ``after_run``.

Built-ins: ``lr_scheduler``, ``load_ckpt``, ``save_ckpt`` (``freq``), ``log_show`` (``freq``),
``log_reduce``.  Config keys and defaults follow ``base_learner_default_config.yaml:19-55``.
``log_reduce`` packs every numeric log value into ONE tensor and does ONE all-reduce (the reference
issues ~43 one-element all-reduces with a host sync each).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List

import torch

from ..parallel import dist as pdist

POSITIONS = ('before_run', 'before_iter', 'after_iter', 'after_run')


class LearnerHook:
    def __init__(self, name: str = '', priority: int = 0, position: str = 'after_iter', ext_args=None):
        assert position in POSITIONS, position
        self.name = name or type(self).__name__
        self.priority = priority
        self.position = position
        self.ext_args = dict(ext_args or {})
        self.freq = int(self.ext_args.get('freq', 1))

    def __call__(self, engine) -> None:
        raise NotImplementedError


class LrSchedulerHook(LearnerHook):
    def __call__(self, engine):
        if engine.lr_scheduler is not None:
            engine.lr_scheduler.step()
            engine.log_buffer['cur_lr'] = engine.optimizer.param_groups[0]['lr']


class LoadCkptHook(LearnerHook):
    def __call__(self, engine):
        path = engine.load_path
        if not path or path in ('none', 'default') or not os.path.exists(path):
            return
        obj = engine.checkpoint_helper.load(path, engine.model, engine.optimizer,
                                            load_optimizer=engine.cfg.learner.get('load_optimizer', True),
                                            logger=engine.logger, loader=engine.model_loader())
        engine.last_iter.update(int(obj.get('last_iter', 0)))
        if engine.lr_scheduler is not None:
            engine.lr_scheduler.last_epoch = engine.last_iter.val
        engine.info(f'{engine.name} loaded checkpoint {path} (iter {engine.last_iter.val})')


class SaveCkptHook(LearnerHook):
    def __call__(self, engine):
        if engine.rank != 0 or engine.last_iter.val % self.freq != 0:
            return
        path = engine.checkpoint_path(engine.last_iter.val)
        engine.checkpoint_helper.save(path, engine.model, engine.optimizer, last_iter=engine.last_iter.val,
                                      state_dict=engine.model_state_dict())
        engine.last_checkpoint_path = path
        engine.info(f'{engine.name} saved checkpoint {path}')


class LogShowHook(LearnerHook):
    def __call__(self, engine):
        if engine.rank != 0:
            engine.log_buffer.clear()
            return
        engine.record.update_var(engine.log_buffer)
        if engine.scalar_logger is not None:
            frames = engine.last_iter.val * engine.world_size * engine.samples_per_iter
            for k, v in engine.log_buffer.items():
                engine.scalar_logger.add_scalar(k, v, frames)
        engine.log_buffer.clear()
        if engine.last_iter.val % self.freq == 0:
            engine.info(f'=== Training Iteration {engine.last_iter.val} Result ===\n{engine.record.get_vars_text()}')


class LogReduceHook(LearnerHook):
    def __call__(self, engine):
        if engine.world_size <= 1 or not engine.log_buffer:
            return
        keys = [k for k, v in engine.log_buffer.items() if isinstance(v, (int, float)) or
                (torch.is_tensor(v) and v.numel() == 1)]
        vals = pdist.allreduce_scalars({k: engine.log_buffer[k] for k in keys}, average=True)
        engine.log_buffer.update(vals)


HOOK_TYPES: Dict[str, Callable] = {
    'lr_scheduler': LrSchedulerHook,
    'load_ckpt': LoadCkptHook,
    'save_ckpt': SaveCkptHook,
    'log_show': LogShowHook,
    'log_reduce': LogReduceHook,
}

DEFAULT_HOOK_CONFIG = {
    'lr_scheduler': {'name': 'lr_scheduler', 'type': 'lr_scheduler', 'priority': 20, 'position': 'after_iter'},
    'log_reduce': {'name': 'log_reduce', 'type': 'log_reduce', 'priority': 1, 'position': 'after_iter',
                   'ext_args': {'freq': 1}},
    'load_ckpt': {'name': 'load_ckpt', 'type': 'load_ckpt', 'priority': 20, 'position': 'before_run'},
    'save_ckpt_after_iter': {'name': 'save_ckpt_after_iter', 'type': 'save_ckpt', 'priority': 40,
                             'position': 'after_iter', 'ext_args': {'freq': 200}},
    'save_ckpt_after_run': {'name': 'save_ckpt_after_run', 'type': 'save_ckpt', 'priority': 20,
                            'position': 'after_run'},
    'log_show': {'name': 'log_show', 'type': 'log_show', 'priority': 20, 'position': 'after_iter',
                 'ext_args': {'freq': 10}},
}


def register_hook_type(name: str, cls) -> None:
    HOOK_TYPES[name] = cls


def build_learner_hooks(hook_cfg: Dict) -> Dict[str, List[LearnerHook]]:
    hooks: Dict[str, List[LearnerHook]] = {p: [] for p in POSITIONS}
    for _, c in (hook_cfg or {}).items():
        h = HOOK_TYPES[c['type']](name=c.get('name', ''), priority=c.get('priority', 0),
                                  position=c.get('position', 'after_iter'), ext_args=c.get('ext_args'))
        add_learner_hook(hooks, h)
    return hooks


def add_learner_hook(hooks: Dict[str, List[LearnerHook]], hook: LearnerHook) -> None:
    hooks[hook.position].append(hook)
    hooks[hook.position].sort(key=lambda h: h.priority)
