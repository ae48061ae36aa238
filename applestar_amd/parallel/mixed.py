"""bf16 compute weights backed by fp32 master weights in the optimizer.

Under plain autocast every GEMM/conv weight is cast fp32->bf16 on every forward (~450 cast kernels per
learner iteration) and its bf16 gradient is cast back to fp32 (~450 more).  Here the GEMM/conv/LSTM
weights *are* bf16 (identical forward numerics: autocast rounded them to bf16 anyway); their fp32
master copy lives in ONE flat buffer laid out exactly like the gradient buckets, so an iteration's
optimizer work is: cast the reduced bf16 (or fp32-reduced) gradient buckets into one flat fp32
gradient (one kernel per bucket), one fused Adam over [flat master + fp32 norm params], one cast of
the master back into the flat bf16 weight storage.  Norm affines and other small parameters stay
fp32 end to end.  ``state_dict`` exports the fp32 master values (reference checkpoint format).
"""
from __future__ import annotations

import os
from typing import Dict, List

import torch
import torch.nn as nn

from .dp import GradientReducer, join_hook_stream, _on_stream

LOWP_MODULES = (nn.Linear, nn.Conv2d, nn.ConvTranspose2d)


def lowp_parameter_names(model: nn.Module) -> List[str]:
    """Names of the parameters autocast would cast to bf16: GEMM / conv weights and biases, LSTM gate
    matrices.  LayerNorm affines, embeddings and loose parameters stay fp32."""
    names = []
    for mname, m in model.named_modules():
        if isinstance(m, LOWP_MODULES):
            names += [f'{mname}.{n}' if mname else n for n, _ in m.named_parameters(recurse=False)]
        elif type(m).__name__ == 'LNLSTMCell':
            names += [f'{mname}.weight_ih', f'{mname}.weight_hh']
    return names


class MasterWeights:
    def __init__(self, model: nn.Module, bucket_mb: float = 32.0, comm_dtype=None):
        self.model = model
        params = dict(model.named_parameters())
        lowp = set(lowp_parameter_names(model))
        self.names = {p: n for n, p in params.items()}
        for n in lowp:
            p = params[n]
            p.data = p.data.to(torch.bfloat16)  # keeps strides (channels_last conv weights)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.reducer = GradientReducer(self.params, bucket_mb=bucket_mb, comm_dtype=comm_dtype)
        self.reducer.keep_comm = True
        # fp32 master in bucket order: master slice i <-> bf16 bucket i (same per-parameter offsets)
        self.lowp_buckets = [b for b in self.reducer.buckets if b.flat.dtype == torch.bfloat16]
        n = sum(b.flat.numel() for b in self.lowp_buckets)
        dev = self.params[0].device
        self.master = nn.Parameter(torch.empty(n, dtype=torch.float32, device=dev))
        self.master.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.weight_flat = torch.empty(n, dtype=torch.bfloat16, device=dev)
        self._slices = []
        off = 0
        for b in self.lowp_buckets:
            k = b.flat.numel()
            self._slices.append((b, off, k))
            o2 = off
            for p in b.params:
                m = p.numel()
                self.master.data[o2:o2 + m].as_strided(p.shape, p.stride()).copy_(p.data.float())
                view = self.weight_flat[o2:o2 + m].as_strided(p.shape, p.stride())
                view.copy_(p.data)
                p.data = view  # the module computes with a view of the flat bf16 storage
                o2 += m
            off += k
        self.fp32_params = [p for b in self.reducer.buckets if b.flat.dtype != torch.bfloat16 for p in b.params]
        self.opt_params = [self.master] + self.fp32_params
        # fp32 biases / transposed GEMM weights / flipped conv weights the kernels read: rebuilt in one launch
        # per step by after_step instead of one cast or transpose per layer (ops/native.py DerivedWeights)
        self.derived = None
        if dev.type == 'cuda' and os.environ.get('APPLESTAR_DERIVED_WEIGHTS', '1') != '0':   # A/B switch
            from ..ops.native import DerivedWeights
            self.derived = DerivedWeights()
            for p in self.params:
                p._derived_forms = self.derived
        # multi-rank: False = per-bucket all-reduce overlapped with backward (eager step); True = backward
        # writes the local gradient and synchronize() reduces the flat buffers (graph-captured step)
        self.defer_allreduce = False

    # ---------------------------------------------------------------- per iteration
    def zero_grad(self):
        self.reducer.zero_grad()

    def backward(self, loss: torch.Tensor):
        """Backward straight into the fp32 master gradient (``autograd.grad``: no per-parameter
        AccumulateGrad ``add_`` into zeroed buckets, ~240 launches per RL step).

        Single rank: ONE native multi-tensor copy writes every bf16 gradient, converted, into its fp32
        master-grad slot (and the fp32 ones into their buckets).  Multi-rank: a tensor hook per
        parameter collects the gradients of each bucket as backward produces them; when a bucket is
        complete, one multi-tensor copy writes them (converted) into the bucket's slice of the fp32 master
        gradient and ONE async RCCL all-reduce of that slice starts, overlapping the rest of backward
        (:meth:`synchronize` waits for the tail).  The reduction is fp32 and lands in place: no bf16
        bucket, no gather into the master afterwards."""
        self._direct = False
        self._overlapped = False
        world = self.reducer.world
        if world > 1 and not self.defer_allreduce:
            self._backward_overlapped(loss)
            return
        if not loss.is_cuda and world == 1:
            self.reducer.backward(loss)
            return
        grads = torch.autograd.grad(loss, self.reducer.params, allow_unused=True)
        mg = self._master_grad_views()
        dst, src = [], []
        for p, g in zip(self.reducer.params, grads):
            if g is not None:
                dst.append(mg.get(p, p.grad))
                src.append(g)
        if len(dst) < len(self.reducer.params):   # unused parameters (e.g. value pre-training) get zeros
            self.master.grad.zero_()
            for b in self.reducer.buckets:
                if b.flat.dtype != torch.bfloat16:
                    b.flat.zero_()
        if loss.is_cuda:
            from ..ops import native
            native.ensure_loaded().multi_copy(dst, src)
        else:
            torch._foreach_copy_(dst, src)
        self._direct = True

    def reduce_flat(self):
        """All-reduce (average) the whole fp32 master gradient and the fp32 buckets: two RCCL calls,
        used when backward ran without per-bucket overlap (``defer_allreduce``, e.g. between the two
        halves of a graph-captured step)."""
        import torch.distributed as dist
        if self.reducer.world == 1:
            return
        bufs = [self.master.grad] + [b.flat for b in self.reducer.buckets if b.flat.dtype != torch.bfloat16]
        avg = self.reducer.use_avg
        for buf in bufs:
            dist.all_reduce(buf, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=self.reducer.group)
            if not avg:
                buf.div_(self.reducer.world)

    # ---------------------------------------------------------------- multi-rank, overlapped
    def _comm_buffers(self):
        """Per bucket: the fp32 buffer that is all-reduced (a master-grad slice for bf16 buckets, the
        bucket itself for fp32 ones) and, per parameter, its destination view in that buffer."""
        plan = getattr(self, '_plan', None)
        if plan is None:
            mg = self._master_grad_views()
            slot = {id(b): (off, k) for b, off, k in self._slices}
            plan = {}
            for b in self.reducer.buckets:
                if id(b) in slot:
                    off, k = slot[id(b)]
                    buf = self.master.grad[off:off + k]
                else:
                    buf = b.flat
                plan[id(b)] = (buf, {p: mg.get(p, p.grad) for p in b.params})
            self._plan = plan
            self._bucket_of = {p: b for b in self.reducer.buckets for p in b.params}
            self._hook_handles = [p.register_hook(self._make_hook(p)) for p in self.reducer.params]
        return plan

    def _make_hook(self, p):
        def hook(g):
            if getattr(self, '_overlapped', False):
                join_hook_stream(self._main, g)
                b = self._bucket_of[p]
                st = self._pending[id(b)]
                st.append((p, g))
                if len(st) == len(b.params):
                    with _on_stream(self._main):
                        self._flush(b)
            return None
        return hook

    def _flush(self, b):
        """Copy the collected gradients of bucket ``b`` into its fp32 buffer and start its all-reduce."""
        import torch.distributed as dist
        if id(b) in self._handles:
            return
        buf, dst_of = self._plan[id(b)]
        got = self._pending[id(b)]
        if len(got) < len(b.params):           # unused parameters contribute zeros
            buf.zero_()
        dst = [dst_of[p] for p, _ in got]
        src = [g for _, g in got]
        if dst:
            if buf.is_cuda:
                from ..ops import native
                native.ensure_loaded().multi_copy(dst, src)
            else:
                torch._foreach_copy_(dst, src)
        op = dist.ReduceOp.AVG if self.reducer.use_avg else dist.ReduceOp.SUM
        self._handles[id(b)] = dist.all_reduce(buf, op=op, group=self.reducer.group, async_op=True)

    def _backward_overlapped(self, loss: torch.Tensor):
        self._comm_buffers()
        self._pending = {id(b): [] for b in self.reducer.buckets}
        self._handles = {}
        self._main = torch.cuda.current_stream(loss.device) if loss.is_cuda else None
        self._overlapped = True
        try:
            torch.autograd.grad(loss, self.reducer.params, allow_unused=True)
        finally:
            self._overlapped = False
        self._overlap_done = True

    def _master_grad_views(self):
        views = getattr(self, '_mg_views', None)
        if views is None:
            views = {}
            g = self.master.grad
            for b, off, _ in self._slices:
                o2 = off
                for p in b.params:
                    m = p.numel()
                    views[p] = g[o2:o2 + m].as_strided(p.shape, p.stride(), g.storage_offset() + o2)
                    o2 += m
            self._mg_views = views
        return views

    def synchronize(self):
        """All-reduce (if distributed) and gather the bf16 gradients into the flat fp32 master grad."""
        if getattr(self, '_direct', False):
            self.reduce_flat()
            return
        if getattr(self, '_overlap_done', False):
            self._overlap_done = False
            for b in self.reducer.buckets:         # buckets whose parameters all went unused
                self._flush(b)
            world = self.reducer.world
            for b in self.reducer.buckets:
                self._handles[id(b)].wait()
                if not self.reducer.use_avg:
                    self._plan[id(b)][0].div_(world)
            self._handles = {}
            return
        self.reducer.synchronize()
        g = self.master.grad
        for b, off, k in self._slices:
            g[off:off + k].copy_(self.reducer.reduced(b))

    def after_step(self):
        """Publish the updated master weights to the bf16 compute weights."""
        with torch.no_grad():
            self.weight_flat.copy_(self.master.detach())
            if self.derived is not None:
                self.derived.refresh()

    # ---------------------------------------------------------------- state
    def _master_views(self) -> Dict[str, torch.Tensor]:
        out = {}
        for b, off, _ in self._slices:
            o2 = off
            for p in b.params:
                m = p.numel()
                out[self.names[p]] = self.master.data[o2:o2 + m].as_strided(p.shape, p.stride())
                o2 += m
        return out

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Model state dict with fp32 master values for the bf16 parameters."""
        sd = self.model.state_dict()
        for n, v in self._master_views().items():
            if n in sd:
                sd[n] = v.detach().clone()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = False):
        """Load fp32 values into the masters (no bf16 round trip), everything else into the model."""
        views = self._master_views()
        rest = {}
        with torch.no_grad():
            for k, v in sd.items():
                kk = k[7:] if k.startswith('module.') else k
                if kk in views and views[kk].shape == v.shape:
                    views[kk].copy_(v)
                else:
                    rest[kk] = v
            res = self.model.load_state_dict(rest, strict=False)
            self.after_step()
        return res

    def sync_from_model(self):
        """Re-derive the masters from the current (bf16) compute weights, e.g. after an in-place reset."""
        if self.derived is not None:
            self.derived.invalidate()
        with torch.no_grad():
            for n, v in self._master_views().items():
                v.copy_(dict(self.model.named_parameters())[n].data.float())
