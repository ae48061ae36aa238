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

from typing import Dict, List

import torch
import torch.nn as nn

from .dp import GradientReducer

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

    # ---------------------------------------------------------------- per iteration
    def zero_grad(self):
        self.reducer.zero_grad()

    def backward(self, loss: torch.Tensor):
        """Backward into the master gradient.  Multi-rank: into the bf16 buckets (hooks overlap the
        all-reduces with backward; :meth:`synchronize` then gathers them into the fp32 master grad).
        Single rank: ``autograd.grad`` and ONE native multi-tensor copy that writes every bf16 gradient,
        converted, straight into its fp32 master-grad slot (and the fp32 ones into their buckets) - no
        per-parameter accumulate / copy launches, no bucket round trip."""
        self._direct = False
        if self.reducer.world > 1 or not loss.is_cuda:
            self.reducer.backward(loss)
            return
        from ..ops import native
        C = native.ensure_loaded()
        grads = torch.autograd.grad(loss, self.reducer.params, allow_unused=True)
        mg = self._master_grad_views()
        dst, src = [], []
        for p, g in zip(self.reducer.params, grads):
            if g is not None:
                dst.append(mg.get(p, p.grad))
                src.append(g)
        if len(dst) < len(self.reducer.params):   # unused parameters (e.g. value pre-training) get zeros
            self.master.grad.zero_()
        C.multi_copy(dst, src)
        self._direct = True

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
            return
        self.reducer.synchronize()
        g = self.master.grad
        for b, off, k in self._slices:
            g[off:off + k].copy_(self.reducer.reduced(b))

    def after_step(self):
        """Publish the updated master weights to the bf16 compute weights."""
        with torch.no_grad():
            self.weight_flat.copy_(self.master.detach())

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
        with torch.no_grad():
            for n, v in self._master_views().items():
                v.copy_(dict(self.model.named_parameters())[n].data.float())
