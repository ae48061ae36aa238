"""Autograd wrappers around the HIP kernels in ``applestar_amd/_C`` (gfx950).

Each wrapper is a ``torch.autograd.Function`` whose forward and backward both run native kernels.
Shapes/dtypes the kernels do not cover raise instead of silently using torch.
"""
from __future__ import annotations

import torch

from . import _ext

_ACT = {None: 0, 'relu': 1, 'sigmoid': 2, 'tanh': 3}
_C = None


def ensure_loaded():
    global _C
    if _C is None:
        _C = _ext.require()
    return _C


_IMPLEMENTED = {'layer_norm', 'gated_residual', 'reverse_scan'}


def has(name: str) -> bool:
    """True when this wrapper module implements ``name`` (the extension is loaded by ensure_loaded)."""
    return name in _IMPLEMENTED


def _dt_code(dtype) -> int:
    return 1 if dtype == torch.bfloat16 else 0


# ---------------------------------------------------------------------------- layer norm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, act, eps, out_dtype):
        x_c = x.contiguous()
        res_c = res.contiguous() if res is not None else None
        y, mean, rstd, xsum = _C.layer_norm_fwd(x_c, res_c, w, b, _dt_code(out_dtype), eps, _ACT[act], True)
        xin = xsum if res is not None else x_c
        ctx.save_for_backward(xin, y, w, mean, rstd)
        ctx.act = act
        ctx.has_res = res is not None
        ctx.x_dtype = x.dtype
        ctx.res_dtype = res.dtype if res is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        xin, y, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        dx, dw, db = _C.layer_norm_bwd(dy, xin, y, w, mean, rstd, _dt_code(ctx.x_dtype), _ACT[ctx.act])
        dres = None
        if ctx.has_res:
            dres = dx if ctx.res_dtype == ctx.x_dtype else dx.to(ctx.res_dtype)
        return dx, dres, dw, db, None, None, None


def layer_norm(x, w, b, residual=None, act=None, eps=1e-5, out_dtype=None):
    C = x.shape[-1]
    if C % 64 != 0 or C > 1536 or w.dtype != torch.float32:
        from . import reference
        return reference.layer_norm(x, w, b, residual, act, eps)
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    if residual is not None and residual.dtype not in (torch.float32, torch.bfloat16):
        residual = residual.float()
    out_dtype = out_dtype or torch.float32
    return _LayerNorm.apply(x, residual, w, b, act, float(eps), out_dtype)


# ---------------------------------------------------------------------------- gated residual
class _GatedResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, g, sp, x):
        out = _C.gated_residual_fwd(y, g, sp, x)
        ctx.save_for_backward(y, g, sp, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, g, sp, out = ctx.saved_tensors
        dy, dg, dx, dsp = _C.gated_residual_bwd(dout.contiguous().to(y.dtype), y, g, sp, out)
        return dy, dg, dsp, dx


def gated_residual(y, g, sp, x):
    dt = torch.promote_types(torch.promote_types(y.dtype, g.dtype), x.dtype)
    y, g, x = (t.to(dt).contiguous() for t in (y, g, x))
    return _GatedResidual.apply(y, g, sp.float(), x)


# ---------------------------------------------------------------------------- reverse scan (no grad)
def reverse_scan(a, b, init):
    a = a.float().contiguous()
    b = b.float().contiguous()
    init = init.float().contiguous().expand(b.shape[:-2] + b.shape[-1:]).contiguous()
    return _C.reverse_scan(a, b, init)
