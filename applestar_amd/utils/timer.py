"""Timers: device-event timing for GPU phases and wall-clock timing elsewhere
(``distar/ctools/utils/time_helper.py`` EasyTimer, with HIP events instead of CUDA events), plus
optional roctx ranges so rocprofv3 ``--marker-trace`` can attribute kernels to phases."""
from __future__ import annotations

import contextlib
import time
from typing import Optional

import torch


class EasyTimer:
    """``with timer: ...`` then ``timer.value`` (seconds).  On GPU uses events (no per-phase sync
    until ``value`` is read)."""

    def __init__(self, cuda: Optional[bool] = None):
        self.cuda = torch.cuda.is_available() if cuda is None else cuda
        self._value = 0.0
        self._start = self._end = None

    def __enter__(self):
        if self.cuda:
            self._start = torch.cuda.Event(enable_timing=True)
            self._end = torch.cuda.Event(enable_timing=True)
            self._start.record()
        else:
            self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self._end.record()
        else:
            self._value = time.perf_counter() - self._t0

    @property
    def value(self) -> float:
        if self.cuda and self._end is not None:
            self._end.synchronize()
            self._value = self._start.elapsed_time(self._end) / 1000.0
            self._end = None
        return self._value


class WallTimer:
    def __init__(self):
        self.t = time.perf_counter()

    def lap(self) -> float:
        now = time.perf_counter()
        d, self.t = now - self.t, now
        return d


@contextlib.contextmanager
def range_marker(name: str):
    """roctx range (visible to ``rocprofv3 --marker-trace``); no-op on CPU."""
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)  # routed to roctx on ROCm builds
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield
