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

import contextlib
import gc
import os
from typing import Dict, Tuple

import torch
import torch.nn as nn

# inference graphs: capture the scalar encoder on a side stream (APPLESTAR_GRAPH_SIDE_STREAMS=0: one stream)
GRAPH_SIDE_STREAMS = os.environ.get('APPLESTAR_GRAPH_SIDE_STREAMS', '0') == '1'

__all__ = ['GraphedSection', 'graphs_enabled']


@contextlib.contextmanager
def gc_paused():
    """Python's cyclic garbage collector paused while a HIP graph is captured (collected once before).  A collection
    inside the capture runs the destructors of unrelated garbage from earlier eager steps against the capturing
    process - one aborted the whole-step capture of test_graphed_train_step_matches_eager mid-forward
    ("Garbage-collecting" frame on the aborting thread)."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


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
            with torch.autocast('cuda', dtype=sig[-1], enabled=sig[-2], cache_enabled=False), gc_paused():
                g = torch.cuda.make_graphed_callables(_Holder(self.module), sample, num_warmup_iters=self.warmup,
                                                      allow_unused_input=True)
            self._graphs[sig] = g
        self.replays += 1
        return g(*args)


# ---------------------------------------------------------------------------------------------------
def _tree_clone(x):
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, dict):
        return {k: _tree_clone(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_tree_clone(v) for v in x)
    return x


def _tree_pairs(dst, src, out):
    if torch.is_tensor(dst):
        if dst.shape != src.shape:
            raise ValueError(f'graphed input shape {tuple(src.shape)} != captured {tuple(dst.shape)}')
        out.append((dst, src))
    elif isinstance(dst, dict):
        for k in dst:
            _tree_pairs(dst[k], src[k], out)
    elif isinstance(dst, (list, tuple)):
        for a, b in zip(dst, src):
            _tree_pairs(a, b, out)
    return out


def _tree_copy_(dst, src):
    """Refresh the captured inputs.  A policy request has ~70 tensor leaves: one blit per leaf was ~70 copy launches
    in front of every replay (profiles/r6j_timeline_b1_policy_graph.txt); same-device leaves of one dtype class go
    through the native multi-tensor copy (raw bytes, 64 leaves per launch)."""
    dev, rest = [], []
    for d, s in _tree_pairs(dst, src, []):
        ok = d.is_cuda and s.is_cuda and d.device == s.device and d.dtype == s.dtype and d.is_contiguous() and \
            s.is_contiguous()
        (dev if ok else rest).append((d, s))
    if len(dev) > 1:
        from ..ops import native
        native.ensure_loaded().multi_copy([d for d, _ in dev], [s for _, s in dev])
    else:
        rest += dev
    for d, s in rest:
        d.copy_(s, non_blocking=True)


def _signature(x):
    if torch.is_tensor(x):
        return (tuple(x.shape), x.dtype)
    if isinstance(x, dict):
        return tuple((k, _signature(v)) for k, v in sorted(x.items()))
    if isinstance(x, (list, tuple)):
        return tuple(_signature(v) for v in x)
    return x


class GraphedPolicy:
    """Actor inference (``compute_logp_action`` / ``compute_teacher_logit``) replayed from HIP graphs,
    one graph per input signature (batch size x padded entity count): the B = 1 agent step is ~500
    small kernels whose launch chain, not the GPU, sets the latency.

    Inputs must keep a fixed padded shape per signature (the inference server pads entities to
    ``MAX_ENTITY_NUM``); the entity encoder switches to its shape-static dense path while capturing.
    Outputs are the graph's static tensors: consume (or clone) them before the next call."""

    def __init__(self, model: nn.Module, method: str = 'compute_logp_action', max_graphs: int = 8):
        self.model = model
        self.method = method
        self.max_graphs = max_graphs
        self._graphs: Dict[Tuple, tuple] = {}
        self.captures = 0

    def _run(self, kwargs):
        fn = getattr(self.model, self.method)
        with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            return fn(**kwargs)

    def __call__(self, **kwargs):
        from ..models import encoders, model as model_mod
        sig = _signature(kwargs)
        entry = self._graphs.get(sig)
        if entry is None:
            if len(self._graphs) >= self.max_graphs:
                self._graphs.pop(next(iter(self._graphs)))
            static_in = _tree_clone(kwargs)
            flags = (encoders.STATIC_SHAPES, encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED)
            # GRAPH_SIDE_STREAMS: the scalar encoder (build-order transformer included) is captured on its own side
            # stream, forked from and joined into the capture stream, so its kernels overlap the entity / spatial path
            encoders.STATIC_SHAPES, encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED = \
                True, GRAPH_SIDE_STREAMS, GRAPH_SIDE_STREAMS
            try:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(2):                      # warm-up (allocator, lazy tables) off-capture
                        self._run(static_in)
                torch.cuda.current_stream().wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with gc_paused(), torch.cuda.graph(g):
                    static_out = self._run(static_in)
            finally:
                encoders.STATIC_SHAPES, encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED = flags
            entry = self._graphs[sig] = (g, static_in, static_out)
            self.captures += 1
        g, static_in, static_out = entry
        _tree_copy_(static_in, kwargs)
        g.replay()
        return static_out
