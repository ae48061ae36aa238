"""Hierarchical wall-clock stopwatch (the role of ``pysc2/lib/stopwatch.py``): named, nestable
sections with sum / avg / dev / min / max / count, usable as a decorator or context manager.  Used
on the actor's host path (featurization, action translation, replay decoding).  Disabled (no-op)
unless ``enable()`` is called or ``APPLESTAR_STOPWATCH=1``."""
from __future__ import annotations

import functools
import math
import os
import threading
import time
from collections import defaultdict


class Stat:
    __slots__ = ('num', 'sum', 'sum_sq', 'min', 'max')

    def __init__(self):
        self.num, self.sum, self.sum_sq, self.min, self.max = 0, 0.0, 0.0, math.inf, 0.0

    def add(self, v: float):
        self.num += 1
        self.sum += v
        self.sum_sq += v * v
        self.min = min(self.min, v)
        self.max = max(self.max, v)

    @property
    def avg(self):
        return self.sum / self.num if self.num else 0.0

    @property
    def dev(self):
        if self.num < 2:
            return 0.0
        return math.sqrt(max(self.sum_sq / self.num - self.avg ** 2, 0.0))

    def merge(self, o: 'Stat'):
        self.num += o.num
        self.sum += o.sum
        self.sum_sq += o.sum_sq
        self.min = min(self.min, o.min)
        self.max = max(self.max, o.max)


class StopWatch:
    def __init__(self, enabled: bool = None):
        self.enabled = bool(int(os.environ.get('APPLESTAR_STOPWATCH', '0'))) if enabled is None else enabled
        self.times = defaultdict(Stat)
        self._local = threading.local()

    def enable(self):
        self.enabled = True

    def disable(self):
        self.enabled = False

    def _stack(self):
        if not hasattr(self._local, 'stack'):
            self._local.stack = []
        return self._local.stack

    def __call__(self, name: str):
        return _Section(self, name)

    def decorate(self, name_or_fn):
        def deco(fn, name):
            @functools.wraps(fn)
            def wrapper(*a, **kw):
                if not self.enabled:
                    return fn(*a, **kw)
                with self(name):
                    return fn(*a, **kw)
            return wrapper
        if callable(name_or_fn):
            return deco(name_or_fn, name_or_fn.__name__)
        return lambda fn: deco(fn, name_or_fn)

    def clear(self):
        self.times.clear()

    def str(self, threshold: float = 0.0) -> str:
        rows = [('name', 'num', 'sum(ms)', 'avg(ms)', 'dev', 'min', 'max')]
        total = sum(s.sum for k, s in self.times.items() if '.' not in k) or 1.0
        for k in sorted(self.times):
            s = self.times[k]
            if s.sum / total < threshold:
                continue
            rows.append((k, str(s.num), f'{s.sum * 1e3:.2f}', f'{s.avg * 1e3:.3f}', f'{s.dev * 1e3:.3f}',
                         f'{s.min * 1e3:.3f}', f'{s.max * 1e3:.3f}'))
        w = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
        return '\n'.join('  '.join(c.ljust(w[i]) for i, c in enumerate(r)) for r in rows)


class _Section:
    __slots__ = ('sw', 'name', 't0')

    def __init__(self, sw: StopWatch, name: str):
        self.sw, self.name = sw, name

    def __enter__(self):
        if self.sw.enabled:
            st = self.sw._stack()
            st.append(self.name)
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sw.enabled:
            dt = time.perf_counter() - self.t0
            st = self.sw._stack()
            self.sw.times['.'.join(st)].add(dt)
            st.pop()
        return False


sw = StopWatch()
