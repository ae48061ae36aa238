"""Checkpoint save/load with the reference artefact format, and crash-safe auto-checkpointing.

* ``rl_model.pth`` / ``sl_model.pth`` / learner checkpoints are ``torch.save`` dicts with a
  ``'model'`` state_dict (+ ``'optimizer'``, ``'last_iter'``, optional ``map_name``,
  ``fake_reward_prob``, ``z_path``, ``z_idx``) — ``checkpoint_helper.py:34-278``, ``actor.py:65-73``.
* Loading is shape-matched and non-strict with a report of missing / unexpected / mismatched keys;
  ``drop`` filters key substrings (actors drop ``value_networks``).
* Reference checkpoints are loaded with ``weights_only=True`` (no unpickling of code).
* ``auto_checkpoint`` saves on exceptions and on SIGINT/SIGTERM/SIGUSR1 (``checkpoint_helper.py:325-369``).
"""
from __future__ import annotations

import functools
import os
import signal
import tempfile
from typing import Callable, Dict, Iterable, Optional

import torch


def load_file(path: str, map_location='cpu') -> Dict:
    return torch.load(path, map_location=map_location, weights_only=True)


def save_file(obj: Dict, path: str) -> None:
    """Atomic save (write to a temp file in the same directory, then rename)."""
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, suffix='.tmp')
    os.close(fd)
    try:
        torch.save(obj, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def load_state_dict_matched(module: torch.nn.Module, state: Dict[str, torch.Tensor],
                            drop: Iterable[str] = (), prefix_strip: str = 'module.', loader=None) -> Dict[str, list]:
    """Copy every key whose name and shape match; report the rest."""
    own = module.state_dict()
    matched, mismatched, unexpected = {}, [], []
    for k, v in state.items():
        kk = k[len(prefix_strip):] if prefix_strip and k.startswith(prefix_strip) else k
        if any(d in kk for d in drop):
            continue
        if kk not in own:
            unexpected.append(kk)
        elif own[kk].shape != v.shape:
            mismatched.append(kk)
        else:
            matched[kk] = v
    missing = [k for k in own if k not in matched and not any(d in k for d in drop)]
    (loader or (lambda sd: module.load_state_dict(sd, strict=False)))(matched)
    return {'missing': missing, 'unexpected': unexpected, 'mismatched': mismatched, 'loaded': list(matched)}


class CheckpointHelper:
    def save(self, path: str, model: torch.nn.Module, optimizer=None, last_iter: Optional[int] = None,
             extra: Optional[Dict] = None, policy_only: bool = False, state_dict: Optional[Dict] = None) -> None:
        sd = model.state_dict() if state_dict is None else state_dict
        if policy_only:
            sd = {k: v for k, v in sd.items() if 'value_networks' not in k and 'value_encoder' not in k}
        obj = {'model': {k: v.detach().cpu() for k, v in sd.items()}}
        if optimizer is not None:
            obj['optimizer'] = optimizer.state_dict()
        if last_iter is not None:
            obj['last_iter'] = int(last_iter)
        if extra:
            obj.update(extra)
        save_file(obj, path)

    def load(self, path: str, model: torch.nn.Module, optimizer=None, load_optimizer: bool = True,
             drop: Iterable[str] = (), logger=None, loader=None) -> Dict:
        """``loader(matched_state_dict)`` replaces ``model.load_state_dict`` (master-weight trainers)."""
        obj = load_file(path)
        sd = obj['model'] if 'model' in obj else obj
        report = load_state_dict_matched(model, sd, drop=drop, loader=loader)
        if logger is not None:
            for k in ('missing', 'unexpected', 'mismatched'):
                if report[k]:
                    logger.info(f'checkpoint {os.path.basename(path)}: {k} keys ({len(report[k])}): {report[k][:8]}')
        if optimizer is not None and load_optimizer and 'optimizer' in obj:
            try:
                optimizer.load_state_dict(obj['optimizer'])
            except Exception as e:  # param groups changed
                if logger is not None:
                    logger.warning(f'optimizer state not loaded: {e}')
        obj['report'] = report
        return obj


class CountVar:
    def __init__(self, init_val: int = 0):
        self.val = init_val

    def add(self, n: int = 1):
        self.val += n

    def update(self, v: int):
        self.val = v


def auto_checkpoint(save_fn_name: str = 'save_checkpoint') -> Callable:
    """Decorate a ``run`` method: on exception or SIGINT/SIGTERM/SIGUSR1 call ``self.<save_fn_name>()``."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(self, *a, **kw):
            def handler(signum, frame):
                getattr(self, save_fn_name)()
                raise SystemExit(128 + signum)
            old = {}
            for sig in (signal.SIGINT, signal.SIGTERM, signal.SIGUSR1):
                try:
                    old[sig] = signal.signal(sig, handler)
                except ValueError:  # not main thread
                    pass
            try:
                return fn(self, *a, **kw)
            except Exception:
                getattr(self, save_fn_name)()
                raise
            finally:
                for sig, h in old.items():
                    signal.signal(sig, h)
        return wrapper
    return deco
