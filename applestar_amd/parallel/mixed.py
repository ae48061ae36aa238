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

from .dp import GradientReducer, copy_into

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
        # kept for the graph-captured step (runtime/step_graph.py), which runs the reduction between its two
        # graphs: backward never launches a collective, so this only documents that contract
        self.defer_allreduce = False

    # ---------------------------------------------------------------- per iteration
    def zero_grad(self):
        self.reducer.zero_grad()

    def backward(self, loss: torch.Tensor):
        """Backward straight into the fp32 master gradient, with the same launches at every world size:
        ``autograd.grad`` (no per-parameter ``AccumulateGrad`` add into zeroed buckets) and ONE native
        multi-tensor copy that writes every bf16 gradient, converted, into its fp32 master-grad slot (and the
        fp32 ones into their buckets).  Multi-rank, :meth:`synchronize` then all-reduces the flat fp32
        buffers (fp32 reduction of the bf16 gradients; parallel/dp.py explains why the collective is not
        overlapped with backward through per-parameter hooks)."""
        self._direct = False
        if not loss.is_cuda:
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
        copy_into(dst, src)
        self._direct = True

    def reduce_flat(self):
        """All-reduce (average) the whole fp32 master gradient and the fp32 buckets: one RCCL call each,
        issued back to back (async) and then waited for."""
        import torch.distributed as dist
        if self.reducer.world == 1:
            return
        bufs = [self.master.grad] + [b.flat for b in self.reducer.buckets if b.flat.dtype != torch.bfloat16]
        avg = self.reducer.use_avg
        op = dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM
        handles = [dist.all_reduce(buf, op=op, group=self.reducer.group, async_op=True) for buf in bufs]
        for h, buf in zip(handles, bufs):
            h.wait()
            if not avg:
                buf.div_(self.reducer.world)

    def segments(self):
        """(offset, numel) of every bf16 parameter inside the flat master, in master order (per-layer pieces
        for per-tensor gradient clips such as momentum_norm)."""
        out = []
        for b, off, _ in self._slices:
            o2 = off
            for p in b.params:
                out.append((o2, p.numel()))
                o2 += p.numel()
        return out

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
        """Average the gradients across ranks (no-op on one rank)."""
        if getattr(self, '_direct', False):
            self.reduce_flat()
            return
        self.reducer.synchronize()        # CPU path: the plain bucket reducer, then bucket -> master
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
