"""HIP-graph capture of static-shape model sections (forward AND backward).

An RL learner step launches ~3000 kernels; at ~10-15 us of host time each the step is host-bound in
places (bench: host time per step ~= wall time).  Sections whose tensor shapes depend only on the
learner config (batch, unroll) - the value baselines, the core LSTM, the location head - are captured
once per input signature with ``torch.cuda.make_graphed_callables`` and then replayed: one graph launch
for the whole forward and one for the whole backward instead of ~100-300 individual launches.

The wrapped module keeps its parameters (the bf16 compute weights are updated in place by the
optimizer, so replays see new values); each captured graph owns a private memory pool whose static
outputs are overwritten by the next replay, which is fine for a learner that consumes a step's outputs
before starting the next.  Graphs are used only when: CUDA, grad mode on, module in training mode and enabled (constructor
argument, else ``APPLESTAR_GRAPHS=1``); anything else calls the module directly.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.nn as nn

__all__ = ['GraphedSection', 'graphs_enabled']


def graphs_enabled() -> bool:
    """Off by default for the learner: its step is GPU-bound (tools/ab_bench.py: graphing the value
    baselines measured +0.4 ms, i.e. no host time to win back); ``APPLESTAR_GRAPHS=1`` turns it on."""
    return os.environ.get('APPLESTAR_GRAPHS', '0') == '1'


class _Holder(nn.Module):
    """make_graphed_callables rewrites the forward of the Module it is given; wrap so the user's module
    object itself is never modified (eval / no-grad / CPU calls keep the eager path)."""

    def __init__(self, m: nn.Module):
        super().__init__()
        self.m = m

    def forward(self, *args):
        return self.m(*args)


class GraphedSection:
    """Callable wrapper: ``GraphedSection(module)(*tensors)``."""

    def __init__(self, module: nn.Module, warmup: int = 3, max_signatures: int = 4, enabled=None):
        self.module = module
        self.enabled = enabled
        self.warmup = warmup
        self.max_signatures = max_signatures
        self._graphs: Dict[Tuple, nn.Module] = {}
        self.replays = 0

    def _signature(self, args) -> Tuple:
        return tuple((tuple(a.shape), a.dtype, a.requires_grad, a.device.index) for a in args) + (
            torch.is_autocast_enabled(), torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled() else None)

    def __call__(self, *args):
        on = graphs_enabled() if self.enabled is None else self.enabled
        use = (on and self.module.training and torch.is_grad_enabled() and
               all(torch.is_tensor(a) and a.is_cuda for a in args))
        if not use:
            return self.module(*args)
        sig = self._signature(args)
        g = self._graphs.get(sig)
        if g is None:
            if len(self._graphs) >= self.max_signatures:   # shapes keep changing: not a static section
                return self.module(*args)
            sample = tuple(a.detach().clone().requires_grad_(a.requires_grad) for a in args)
            with torch.autocast('cuda', dtype=sig[-1], enabled=sig[-2], cache_enabled=False):
                g = torch.cuda.make_graphed_callables(_Holder(self.module), sample, num_warmup_iters=self.warmup,
                                                      allow_unused_input=True)
            self._graphs[sig] = g
        self.replays += 1
        return g(*args)
