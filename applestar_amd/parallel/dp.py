"""Bucketed, backward-overlapped gradient all-reduce for the data-parallel learner.

The reference (``dist_helper.py:421-431``) all-reduces each of 394-474 parameter tensors one by one
after backward.  Here every parameter's ``.grad`` is a *view* into a small number of flat buckets;
a post-accumulate-grad hook counts arrivals and, as soon as a bucket is complete, launches one async
RCCL all-reduce for it while backward continues into earlier layers.  ``synchronize()`` (called
before clip/optimizer) only waits for the tail bucket.

Bucket size is chosen for xGMI rings (7 point-to-point links at ~153 GB/s per MI355X): a ring
all-reduce moves 2(n-1)/n of the bucket over each link, so fewer, larger buckets (default 32 MB)
amortise RCCL launch latency while still leaving several buckets to overlap with backward on a
~33 M-parameter model (132 MB of fp32 gradients -> ~5 buckets).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

from . import dist as pdist


def _cur_stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device) if t.is_cuda else None


def join_hook_stream(main, t: Optional[torch.Tensor] = None):
    """Called from a gradient hook.  The autograd engine runs a parameter's hooks on the stream its
    gradient was produced on: the stream its forward ran on (the scalar encoder runs on a side stream,
    models/model.py ``_side_stream_call``).  Bucket copies and collectives are always issued on ``main``
    (the stream backward was started from), so ``main`` must first wait for that producer stream, and a
    hook-captured gradient ``t`` read later on ``main`` must not be recycled by the allocator early.
    Without this, a bucket completed from a side-stream hook was copied / reduced while main-stream
    gradients of the same bucket were still being computed (non-finite gradients with world > 1)."""
    if main is None:
        return
    cur = torch.cuda.current_stream(main.device)
    if cur != main:
        main.wait_stream(cur)
        if t is not None:
            t.record_stream(main)


class _on_stream:
    """``with torch.cuda.stream(main)`` that is a no-op for CPU (``main`` None)."""

    def __init__(self, main):
        self.ctx = torch.cuda.stream(main) if main is not None else None

    def __enter__(self):
        if self.ctx is not None:
            self.ctx.__enter__()

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)


class _Bucket:
    __slots__ = ('params', 'flat', 'ready', 'handle', 'comm')

    def __init__(self, params: List[torch.nn.Parameter], dtype, device):
        self.params = params
        n = sum(p.numel() for p in params)
        self.flat = torch.zeros(n, dtype=dtype, device=device)
        self.ready = 0
        self.handle = None
        self.comm = None


class GradientReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 32.0,
                 comm_dtype: Optional[torch.dtype] = None, group=None, overlap: bool = True):
        self.group = group
        self.world = pdist.get_world_size()
        self.overlap = overlap
        self.comm_dtype = comm_dtype
        self.keep_comm = False  # master-weight mode reads the fp32 reduction directly (reduced())
        params = [p for p in params if p.requires_grad]
        self.params = params
        self.buckets: List[_Bucket] = []
        self._owner = {}
        # backward visits layers roughly in reverse registration order; parameters of different dtypes
        # (bf16 GEMM weights + fp32 norm affines under master weights) go to separate bucket chains so
        # the interleaving does not fragment the buckets
        limit = int(bucket_mb * 1024 * 1024)
        keys = []
        for p in reversed(params):
            if (p.dtype, p.device) not in keys:
                keys.append((p.dtype, p.device))
        for key in keys:
            cur, cur_bytes = [], 0
            for p in reversed(params):
                if (p.dtype, p.device) != key:
                    continue
                if cur and cur_bytes + p.numel() * p.element_size() > limit:
                    self._add_bucket(cur)
                    cur, cur_bytes = [], 0
                cur.append(p)
                cur_bytes += p.numel() * p.element_size()
            if cur:
                self._add_bucket(cur)
        self._hooks = []
        if self.world > 1 and overlap:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self.use_avg = self.world > 1 and dist.get_backend(group) == 'nccl'
        self._main = None        # stream backward was started from (bucket collectives are issued there)

    def _add_bucket(self, params):
        b = _Bucket(params, params[0].dtype, params[0].device)
        off = 0
        for p in params:
            n = p.numel()
            # same strides as the parameter (channels_last conv weights) so fused optimizers that walk
            # param and grad storage in lockstep see matching elements
            p.grad = b.flat[off:off + n].as_strided(p.shape, p.stride())
            self._owner[p] = b
            off += n
        self.buckets.append(b)

    @property
    def num_buckets(self) -> int:
        return len(self.buckets)

    def _launch(self, b: _Bucket):
        if b.handle is not None or self.world == 1:
            return
        buf = b.flat
        comm_dtype = self.comm_dtype
        if comm_dtype is None and buf.dtype == torch.bfloat16 and self.keep_comm:
            comm_dtype = torch.float32  # bf16 gradients are summed across ranks in fp32
        if comm_dtype is not None and comm_dtype != buf.dtype:
            b.comm = buf.to(comm_dtype)
            buf = b.comm
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        b.handle = dist.all_reduce(buf, op=op, group=self.group, async_op=True)

    def _on_grad(self, p):
        join_hook_stream(self._main)
        b = self._owner[p]
        b.ready += 1
        if b.ready == len(b.params):
            with _on_stream(self._main):
                self._launch(b)

    def backward(self, loss: torch.Tensor):
        """``loss.backward()`` into the bucket views.

        Multi-rank: plain backward, so the post-accumulate hooks launch each bucket's all-reduce as soon
        as its last gradient lands (overlap with the rest of backward).  Single rank: there is nothing to
        overlap, so the gradients are taken with ``autograd.grad`` (no per-parameter AccumulateGrad
        ``add_`` into the zeroed buckets - ~240 launches per RL step) and written with one multi-tensor
        copy."""
        if self.world > 1:
            self._main = _cur_stream(loss)
            loss.backward()
            return
        grads = torch.autograd.grad(loss, self.params, allow_unused=True)
        dst, src = [], []
        for p, g in zip(self.params, grads):
            if g is not None:
                dst.append(p.grad)
                src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)

    def zero_grad(self):
        for b in self.buckets:
            b.flat.zero_()
            b.ready = 0
            b.handle = None
            b.comm = None
        for p in self.params:  # re-attach in case someone set grads to None
            if p.grad is None or p.grad.data_ptr() == 0:
                raise RuntimeError('gradient view detached from its bucket; use GradientReducer.zero_grad()')

    def synchronize(self):
        if self.world == 1:
            return
        for b in self.buckets:
            self._launch(b)  # buckets with unused params (or overlap disabled) go now
        for b in self.buckets:
            b.handle.wait()
            if b.comm is not None:
                if not self.use_avg:
                    b.comm.div_(self.world)
                if not self.keep_comm:
                    b.flat.copy_(b.comm)
            elif not self.use_avg:
                b.flat.div_(self.world)
            b.handle = None

    def reduced(self, b: _Bucket) -> torch.Tensor:
        """The bucket's averaged gradient (the fp32 communication copy when one was used)."""
        return b.comm if b.comm is not None else b.flat

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
