"""Whole learner step as HIP graphs: forward + loss + backward in one graph, clip + Adam + weight
publish in a second; the data-parallel gradient all-reduce (RCCL) runs eagerly between the two.

An RL learner step is ~1,250 kernel launches (bf16); eagerly each costs ~16 us of host time (PyTorch
dispatch + autograd).  Measured on MI355X / ROCm 7 (profiles/r3l_graph_sync_probe.txt): a replay issues in
~1.5 ms of host time and the step is then GPU-bound at 29.8 ms, vs 27.3 ms for the eager step (the captured
step keeps torch's capturable Adam and per-call weight forms instead of the fused clip+Adam and the cached
derived weights), so RLTrainer keeps this opt-in (``learner.graph_step``): it pays where the host is the
bottleneck (many ranks per node contending for CPU), not on an idle host.  The machinery (static shapes, eager
warm-up, shared pool, the DP all-reduce between the two graphs) is tested for equivalence.

Host waits: round 2 needed a host synchronize after each replay (without it, eager work behind a replay read
an inf gradient norm).  The probe (tools/diag/graph_sync_diag.py) snapshots the graph's outputs from the
stream right behind the replay and compares them with the settled values: with the current code every
snapshot matches and nothing is non-finite over 12 replays - alone, interleaved with an eager trainer, with
private pools, and even with the round-2 split-LSTM poll budget rebuilt in (the 'shortpoll' variant), which
rules the LSTM exchange out.  The change on this path since round 2 is the removal of the per-parameter
gradient hooks (parallel/dp.py, round 3), whose AccumulateGrad work was bound to the stream of an earlier
step - the likely cause, not reproduced in isolation.  The waits are gone (APPLESTAR_GRAPH_HOST_SYNC=1 puts
them back when debugging).

Shapes must be static per graph.  The one data-dependent shape of the learner step, the packed entity
count, is fixed by packing to ``encoders.entity_pad_for(total, N)`` rows (``EntityEncoder._forward_padded``:
padding rows ride along as extra attention segments and get zero gradient).  Everything else is keyed:
one graph pair per input signature (tensor shapes/dtypes, python scalars, value-pretrain flag), LRU-bounded,
all sharing one memory pool (graphs replay strictly one after another).

Protocol per signature: the first occurrence runs eagerly (a real training step that also warms up
lazily-created state: optimizer moments, library workspaces, cached weight folds); the second
occurrence captures and then replays.  Outputs are the graph's static tensors, packed and copied once
so callers may keep them across steps.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Callable, Dict, Optional, Tuple

import torch

from .graphs import gc_paused

__all__ = ['GraphedTrainStep', 'batch_signature']


def _tree_clone(x):
    if torch.is_tensor(x):
        return x.clone()
    if isinstance(x, dict):
        return {k: _tree_clone(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_tree_clone(v) for v in x)
    return x


def _tree_pairs(dst, src, out, path='batch'):
    if torch.is_tensor(dst):
        if dst.shape != src.shape or dst.dtype != src.dtype:
            raise ValueError(f'{path}: {tuple(src.shape)}/{src.dtype} != captured {tuple(dst.shape)}/{dst.dtype}')
        out.append((dst, src))
    elif isinstance(dst, dict):
        for k in dst:
            _tree_pairs(dst[k], src[k], out, f'{path}.{k}')
    elif isinstance(dst, (list, tuple)):
        for i, (a, b) in enumerate(zip(dst, src)):
            _tree_pairs(a, b, out, f'{path}[{i}]')
    return out


def _tree_copy_(dst, src):
    """Refresh the captured input tensors from a new batch.  A learner batch has ~130 leaves: copied one by
    one that is ~130 blit launches per replay (rocprof r4n: 1.1 ms of copyBuffer per bf16 step), so device
    leaves go through the native multi-tensor copy (raw bytes, 64 leaves per launch)."""
    dev, rest = [], []
    for d, s in _tree_pairs(dst, src, []):
        (dev if d.is_cuda and s.is_cuda and d.device == s.device else rest).append((d, s))
    if dev:
        from ..ops import native
        native.ensure_loaded().multi_copy([d for d, _ in dev], [s for _, s in dev])
    for d, s in rest:
        d.copy_(s, non_blocking=True)


def batch_signature(x):
    """Hashable description of everything a captured step depends on: tensor shapes/dtypes/devices and
    plain python values (batch_size, unroll_len, entity_pad...)."""
    if torch.is_tensor(x):
        return ('T', tuple(x.shape), str(x.dtype), x.device.type)
    if isinstance(x, dict):
        return tuple((k, batch_signature(v)) for k, v in sorted(x.items()))
    if isinstance(x, (list, tuple)):
        return tuple(batch_signature(v) for v in x)
    return x


class _Entry:
    __slots__ = ('fb', 'upd', 'static_in', 'keys', 'packed', 'grad_norm')   # upd None: update inside fb


class GraphedTrainStep:
    """``GraphedTrainStep(fwd_bwd, reduce, update)(batch, extra_key)``.

    * ``fwd_bwd(batch) -> Dict[str, 0-d tensor]``: forward, loss and backward into the gradient buffers;
    * ``reduce()``: the cross-rank gradient reduction (eager, between the graphs; no-op on one rank);
    * ``update() -> 0-d tensor``: clip + optimizer + weight publish, returns the pre-clip gradient norm;
    * ``pre_replay()`` (attribute, optional): the update's host work, run before every replay.
    """

    def __init__(self, fwd_bwd: Callable[[Dict], Dict[str, torch.Tensor]], reduce: Callable[[], None],
                 update: Callable[[], torch.Tensor], max_graphs: int = 6, device=None):
        self.fwd_bwd, self.reduce, self.update = fwd_bwd, reduce, update
        self.max_graphs = max_graphs
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self._graphs: 'OrderedDict[Tuple, _Entry]' = OrderedDict()
        self._seen = set()
        self._pool = None
        self.captures = 0
        self.replays = 0
        self.eager_steps = 0
        self.host_time: Dict[str, float] = {}     # summed host seconds per replay phase
        self.check_fn: Optional[Callable[[], None]] = None
        # one graph for the whole step when there is no cross-rank reduction between backward and update
        import torch.distributed as dist
        self.single_graph = not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)
        # forked side streams (value / scalar encoders) inside the capture; off: captured on one stream
        self.side_streams = os.environ.get('APPLESTAR_GRAPH_SIDE_STREAMS', '0') == '1'
        # host waits after the replays (module docstring: no longer needed on one rank); APPLESTAR_GRAPH_HOST_SYNC=1
        # for debugging.  Multi-rank keeps the wait between the two graphs (before the RCCL reduce) unless the
        # variable is set to 0: the probe that retired it ran single-process only
        env = os.environ.get('APPLESTAR_GRAPH_HOST_SYNC')
        self.host_sync = env == '1'
        self.host_sync_between = self.host_sync or (env is None and not self.single_graph)
        # one private memory pool per graph instead of one shared pool (diagnostics)
        self.private_pools = os.environ.get('APPLESTAR_GRAPH_PRIVATE_POOLS', '0') == '1'
        self.after_replay: Optional[Callable[[_Entry], None]] = None    # diagnostics hook, before any host wait
        # host work of the update that cannot live in a graph (optimizer step count, bias corrections uploaded
        # to the device buffer the captured update reads): run before every replay
        self.pre_replay: Optional[Callable[[], None]] = None

    def _eager(self, batch):
        info = self.fwd_bwd(batch)
        self.reduce()
        info['gradient'] = self.update()
        self.eager_steps += 1
        return info

    def _capture(self, key, batch) -> _Entry:
        if len(self._graphs) >= self.max_graphs:
            self._graphs.popitem(last=False)
        if self._pool is None or self.private_pools:
            self._pool = torch.cuda.graph_pool_handle()
        e = _Entry()
        e.static_in = _tree_clone(batch)
        torch.cuda.synchronize(self.device)
        e.fb = torch.cuda.CUDAGraph()
        from ..models import encoders, model as model_mod
        flags = (encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED)
        if not self.side_streams:
            encoders.SCALAR_SIDE_STREAM = model_mod.SIDE_STREAMS_ENABLED = False
        try:
            with gc_paused(), torch.cuda.graph(e.fb, pool=self._pool):
                info = self.fwd_bwd(e.static_in)
                e.keys = sorted(k for k, v in info.items() if torch.is_tensor(v) and v.numel() == 1)
                e.packed = torch.stack([info[k].detach().float().reshape(()) for k in e.keys]) if e.keys else None
                if self.single_graph:
                    self.reduce()          # one rank: no collective, only the step's health gate
                    e.grad_norm = self.update().detach().float().reshape(())
        finally:
            encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED = flags
        e.upd = None
        if not self.single_graph:
            e.upd = torch.cuda.CUDAGraph()
            with gc_paused(), torch.cuda.graph(e.upd, pool=self._pool):
                e.grad_norm = self.update().detach().float().reshape(())
        self.captures += 1
        self._graphs[key] = e
        return e

    def __call__(self, batch: Dict, extra_key=()) -> Dict[str, torch.Tensor]:
        key = (batch_signature(batch), extra_key)
        e = self._graphs.get(key)
        if e is None:
            if key not in self._seen:
                self._seen.add(key)
                return self._eager(batch)
            e = self._capture(key, batch)
        else:
            self._graphs.move_to_end(key)
        t = self.host_time
        t0 = time.perf_counter()
        if self.pre_replay is not None:
            self.pre_replay()
        _tree_copy_(e.static_in, batch)
        t1 = time.perf_counter()
        e.fb.replay()
        if self.after_replay is not None:
            self.after_replay(e)
        if self.check_fn is not None:      # debugging hook between the two graphs
            self.check_fn()
        t2 = time.perf_counter()
        if e.upd is not None:
            if self.host_sync_between:
                torch.cuda.current_stream(self.device).synchronize()
            self.reduce()
        t3 = time.perf_counter()
        if e.upd is not None:
            e.upd.replay()
        if self.host_sync:
            torch.cuda.current_stream(self.device).synchronize()
        t4 = time.perf_counter()
        for k, dt in (('copy_in', t1 - t0), ('replay_fwd_bwd', t2 - t1), ('reduce', t3 - t2), ('replay_update', t4 - t3)):
            t[k] = t.get(k, 0.0) + dt
        self.replays += 1
        out: Dict[str, torch.Tensor] = {}
        if e.packed is not None:
            vals = torch.cat([e.packed, e.grad_norm.reshape(1)]).clone()
            out = {k: vals[i] for i, k in enumerate(e.keys)}
            out['gradient'] = vals[-1]
        else:
            out['gradient'] = e.grad_norm.clone()
        return out

    def replay_fwd_bwd_only(self):
        """Debugging aid: replay the forward/backward graph of the most recently used signature again
        (gradients left in the buffers, no optimizer update)."""
        if self._graphs:
            next(reversed(self._graphs.values())).fb.replay()

    def reset(self):
        """Drop every captured graph (e.g. after the optimizer or the parameter set was replaced)."""
        self._graphs.clear()
        self._seen.clear()
