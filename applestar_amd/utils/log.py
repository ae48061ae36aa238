"""Logging: per-role text logs, scalar summaries and running meters.

Covers ``distar/ctools/utils/log_helper.py`` (TextLogger, TensorBoardLogger, VariableRecord,
AverageMeter / EmaMeter / MoveAverageMeter, LogDict).  TensorBoard is optional: when
``torch.utils.tensorboard`` is unavailable (as on these images) scalars go to a JSON-lines file
(``<path>/scalars.jsonl``) that tools can plot; the API is the same.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from collections import defaultdict, deque
from typing import Dict, Iterable, Optional

__all__ = ['build_logger', 'TextLogger', 'ScalarLogger', 'AverageMeter', 'EmaMeter', 'MoveAverageMeter',
           'VariableRecord', 'LogDict', 'pretty_table', 'AlphaStarVarRecord']


class TextLogger:
    def __init__(self, path: str, name: str = 'log', to_stdout: bool = True, level=logging.INFO):
        os.makedirs(path, exist_ok=True)
        self.logger = logging.getLogger(f'applestar.{name}.{id(self)}')
        self.logger.setLevel(level)
        self.logger.propagate = False
        fmt = logging.Formatter('[%(asctime)s][%(name)s] %(message)s', '%Y-%m-%d %H:%M:%S')
        fh = logging.FileHandler(os.path.join(path, f'{name}.txt'))
        fh.setFormatter(fmt)
        self.logger.addHandler(fh)
        if to_stdout:
            sh = logging.StreamHandler(sys.stdout)
            sh.setFormatter(fmt)
            self.logger.addHandler(sh)

    def info(self, msg, *a):
        self.logger.info(msg, *a)

    def warning(self, msg, *a):
        self.logger.warning(msg, *a)

    def error(self, msg, *a):
        self.logger.error(msg, *a)


class ScalarLogger:
    """TensorBoard-compatible ``add_scalar`` sink; registered-variable gate like the reference."""

    def __init__(self, path: str, name: str = 'scalars'):
        os.makedirs(path, exist_ok=True)
        self._writer = None
        try:  # pragma: no cover - depends on image
            from torch.utils.tensorboard import SummaryWriter
            self._writer = SummaryWriter(path)
        except Exception:
            self._fh = open(os.path.join(path, f'{name}.jsonl'), 'a')
        self._vars = set()

    def register_var(self, name: str):
        self._vars.add(name)

    def add_scalar(self, tag: str, value: float, step: int):
        if self._writer is not None:
            self._writer.add_scalar(tag, value, step)
        else:
            self._fh.write(json.dumps({'tag': tag, 'value': float(value), 'step': int(step), 't': time.time()}) + '\n')

    def add_scalars(self, values: Dict[str, float], step: int, only_registered: bool = False):
        for k, v in values.items():
            if only_registered and k not in self._vars:
                continue
            self.add_scalar(k, v, step)

    def flush(self):
        if self._writer is not None:
            self._writer.flush()
        else:
            self._fh.flush()

    def close(self):
        if self._writer is not None:
            self._writer.close()
        else:
            self._fh.close()


class AverageMeter:
    def __init__(self, length: int = 0):
        self.length = length
        self.reset()

    def reset(self):
        self.history = deque(maxlen=self.length or None)
        self.val = 0.0
        self.sum = 0.0
        self.count = 0

    def update(self, val: float, n: int = 1):
        self.val = float(val)
        if self.length:
            self.history.append(self.val)
        self.sum += self.val * n
        self.count += n

    @property
    def avg(self) -> float:
        if self.length:
            return sum(self.history) / max(len(self.history), 1)
        return self.sum / max(self.count, 1)


class EmaMeter:
    def __init__(self, decay: float = 0.99):
        self.decay = decay
        self.val = None

    def update(self, v: float):
        self.val = float(v) if self.val is None else self.decay * self.val + (1 - self.decay) * float(v)


class MoveAverageMeter(AverageMeter):
    def __init__(self, length: int = 100):
        super().__init__(length)


class VariableRecord:
    """Named running averages printed as a table every ``print_freq`` updates (actor / learner)."""

    def __init__(self, length: int = 10):
        self.length = length
        self.vars: Dict[str, AverageMeter] = {}

    def register_var(self, name: str, length: Optional[int] = None):
        self.vars[name] = AverageMeter(length or self.length)

    def update_var(self, values: Dict[str, float]):
        for k, v in values.items():
            if k not in self.vars:
                self.register_var(k)
            self.vars[k].update(v)

    def get_vars_text(self) -> str:
        return pretty_table({k: m.avg for k, m in self.vars.items()})

    def get_vars_dict(self) -> Dict[str, float]:
        return {k: m.avg for k, m in self.vars.items()}


class LogDict(dict):
    """Buffer of per-iteration log values; tensors are converted lazily in one batch."""

    def update_tensors(self, d: Dict):
        for k, v in d.items():
            self[k] = v

    def to_floats(self) -> Dict[str, float]:
        import torch
        tensors = {k: v for k, v in self.items() if torch.is_tensor(v)}
        out = {k: float(v) for k, v in self.items() if not torch.is_tensor(v) and isinstance(v, (int, float))}
        if tensors:
            keys = sorted(tensors)
            vec = torch.stack([tensors[k].detach().float().reshape(()) for k in keys]).cpu().tolist()
            out.update(dict(zip(keys, vec)))
        return out


def pretty_table(values: Dict[str, float], cols: int = 4) -> str:
    items = [(k, f'{v:.4g}' if isinstance(v, float) else str(v)) for k, v in values.items()]
    w = max((len(k) + len(v) + 3 for k, v in items), default=10)
    lines, row = [], []
    for k, v in items:
        row.append(f'{k}: {v}'.ljust(w))
        if len(row) == cols:
            lines.append(' | '.join(row))
            row = []
    if row:
        lines.append(' | '.join(row))
    return '\n'.join(lines)


def build_logger(path: str, name: str = 'learner', need_scalar: bool = True, to_stdout: bool = True):
    text = TextLogger(path, name, to_stdout=to_stdout)
    scalar = ScalarLogger(os.path.join(path, 'scalars'), name) if need_scalar else None
    return text, scalar


class AlphaStarVarRecord(VariableRecord):
    """RL learner table layout (``log_helper.py:689-749``): rows = loss families (winloss, bo, bu,
    effect, upgrade, battle, upgo, kl, ent), columns = per-head / value / reward terms."""
    ROWS = ['winloss', 'build_order', 'built_unit', 'effect', 'upgrade', 'battle', 'upgo', 'kl', 'entropy']
    COLS = ['reward', 'value', 'td', 'action_type', 'delay', 'queued', 'selected_units', 'target_unit',
            'target_location', 'total']
    GENERAL = ['cur_lr', 'data_time', 'train_time', 'total_loss', 'gradient', 'kl/extra_at',
               'staleness/mean', 'staleness/max']

    def get_vars_text(self) -> str:
        vals = self.get_vars_dict()
        head = ['name', 'val', 'loss'] + [c[:8] for c in self.COLS]
        rows = [head]
        for i in range(max(len(self.ROWS), len(self.GENERAL))):
            g = self.GENERAL[i] if i < len(self.GENERAL) else ''
            row = [g, f'{vals[g]:.5g}' if g in vals else '']
            if i < len(self.ROWS):
                r = self.ROWS[i]
                row += [r] + [f'{vals[f"{r}/{c}"]:.4g}' if f'{r}/{c}' in vals else '' for c in self.COLS]
            rows.append(row)
        w = [max(len(r[j]) if j < len(r) else 0 for r in rows) for j in range(len(head))]
        return '\n'.join(' | '.join((r[j] if j < len(r) else '').ljust(w[j]) for j in range(len(head))) for r in rows)
