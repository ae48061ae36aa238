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
    def __init__(self, model: nn.Module, bucket_mb: float = 32.0, comm_dtype=None, phase_of=None):
        self.model = model
        params = dict(model.named_parameters())
        lowp = set(lowp_parameter_names(model))
        self.names = {p: n for n, p in params.items()}
        for n in lowp:
            p = params[n]
            p.data = p.data.to(torch.bfloat16)  # keeps strides (channels_last conv weights)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.reducer = GradientReducer(self.params, bucket_mb=bucket_mb, comm_dtype=comm_dtype, phase_of=phase_of)
        self.reducer.keep_comm = True
        # gradients on the wire: fp32 (default) or bf16 (half the bytes; averaged by RCCL, widened back to fp32)
        self.comm_dtype = comm_dtype if comm_dtype == torch.bfloat16 else None
        self._pending = []
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
        # the master range of the phase-0 parameters (parallel/dp.py backward_phased): buckets are built phase by
        # phase, so it is the prefix [0, n0)
        ph0 = set(id(b) for b in self.reducer.phase_buckets[0])
        self.master_n0 = sum(k for b, _, k in self._slices if id(b) in ph0)
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

    def backward(self, loss: torch.Tensor, boundary=None):
        """Backward straight into the fp32 master gradient, with the same launches at every world size:
        ``autograd.grad`` (no per-parameter ``AccumulateGrad`` add into zeroed buckets) and ONE native
        multi-tensor copy that writes every bf16 gradient, converted, into its fp32 master-grad slot (and the
        fp32 ones into their buckets).  Multi-rank, :meth:`synchronize` then all-reduces the flat fp32
        buffers (fp32 reduction of the bf16 gradients; parallel/dp.py explains why the collective is not
        overlapped with backward through per-parameter hooks)."""
        self._direct = False
        self._pending = []
        self._phase0_issued = False
        if not loss.is_cuda:
            self.reducer.backward(loss)
            return
        if boundary is None:
            grads = torch.autograd.grad(loss, self.reducer.params, allow_unused=True)
            self._store(self.reducer.params, grads, None)
            self._direct = True
            return
        # two phases (parallel/dp.py backward_phased): the phase-0 master range and fp32 buckets are final after
        # phase 1; their all-reduce is issued before the encoders' backward
        p0, p1 = self.reducer.phase_params
        outs, leaves = [o for o, _ in boundary], [lf for _, lf in boundary]
        g = torch.autograd.grad(loss, p0 + leaves, allow_unused=True)
        self._store(p0, g[:len(p0)], 0)
        self._direct = True
        self._issue(0)
        self._phase0_issued = True
        roots = [(t, gt) for t, gt in zip(outs, g[len(p0):]) if gt is not None]
        g2 = torch.autograd.grad([t for t, _ in roots], p1, grad_outputs=[gt for _, gt in roots],
                                 allow_unused=True) if roots and p1 else [None] * len(p1)
        self._store(p1, g2, 1)

    def _store(self, params, grads, phase):
        """Every gradient, converted, into its fp32 master-grad slot (fp32 ones into their buckets); ``phase``:
        which master range / fp32 buckets these parameters own (None: all)."""
        mg = self._master_grad_views()
        dst, src = [], []
        for p, g in zip(params, grads):
            if g is not None:
                dst.append(mg.get(p, p.grad))
                src.append(g)
        if len(dst) < len(params):   # unused parameters (e.g. value pre-training) get zeros
            lo, hi = self._range(phase)
            self.master.grad[lo:hi].zero_()
            for b in self._fp32_buckets(phase):
                b.flat.zero_()
        copy_into(dst, src)

    def _range(self, phase):
        n = self.master.grad.numel()
        return (0, n) if phase is None else ((0, self.master_n0) if phase == 0 else (self.master_n0, n))

    def _fp32_buckets(self, phase):
        bs = self.reducer.buckets if phase is None else self.reducer.phase_buckets[phase]
        return [b for b in bs if b.flat.dtype != torch.bfloat16]

    def _issue(self, phase):
        """Async all-reduce (AVG) of one phase's master range + fp32 buckets (None: everything)."""
        import torch.distributed as dist
        if self.reducer.world == 1:
            return
        lo, hi = self._range(phase)
        bufs = ([self.master.grad[lo:hi]] if hi > lo else []) + [b.flat for b in self._fp32_buckets(phase)]
        op = dist.ReduceOp.AVG if self.reducer.use_avg else dist.ReduceOp.SUM
        for buf in bufs:
            wire = buf.to(self.comm_dtype) if self.comm_dtype is not None and buf.dtype != self.comm_dtype else buf
            self._pending.append((dist.all_reduce(wire, op=op, group=self.reducer.group, async_op=True), buf, wire))

    def reduce_flat(self):
        """All-reduce (average) the fp32 master gradient and the fp32 buckets: one RCCL call each, issued back to
        back (async) and then waited for; after a two-phase backward only phase 1's ranges are still to issue."""
        if self.reducer.world == 1:
            return
        self._issue(1 if getattr(self, '_phase0_issued', False) else None)
        for h, buf, wire in self._pending:
            h.wait()
            if wire is not buf:
                buf.copy_(wire)
            if not self.reducer.use_avg:
                buf.div_(self.reducer.world)
        self._pending = []

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
