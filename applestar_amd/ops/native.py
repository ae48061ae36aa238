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


_IMPLEMENTED = {'layer_norm', 'gated_residual', 'reverse_scan', 'lnlstm_layer'}


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


# ---------------------------------------------------------------------------- LN-LSTM layer
class _LNLSTMRecurrence(torch.autograd.Function):
    """Recurrent part of an LN-LSTM layer: xp [T,B,4H] (already LN_i(x W_ih^T)) -> h [T,B,H]."""

    @staticmethod
    def forward(ctx, xp, h0, c0, w_hh, lnh_w, lnh_b, lnc_w, lnc_b, w_dtype):
        wq = w_hh.detach().to(w_dtype)
        wT = wq.t().contiguous()
        out, hT, cT, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c = _C.lnlstm_fwd(
            xp.contiguous(), h0.contiguous(), c0.contiguous(), wT, lnh_w.detach(), lnh_b.detach(),
            lnc_w.detach(), lnc_b.detach(), 1e-5)
        ctx.save_for_backward(h0, out, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, wq.contiguous(), lnh_w, lnc_w)
        return out, hT, cT

    @staticmethod
    def backward(ctx, dout, dhT, dcT):
        h0, out, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, wq, lnh_w, lnc_w = ctx.saved_tensors
        T, B, H = out.shape
        z = lambda t: torch.zeros(B, H, device=out.device) if t is None else t.float().contiguous()
        dout = torch.zeros_like(out) if dout is None else dout.float().contiguous()
        dgates, dhg, dc_ln, dh0, dc0 = _C.lnlstm_bwd(dout, z(dhT), z(dcT), gates, c_all, xhat_c, rstd_c, xhat_h,
                                                     rstd_h, wq, lnh_w.detach(), lnc_w.detach())
        h_prev = torch.cat([h0.float().unsqueeze(0), out[:-1]], 0).view(T * B, H)
        dw = dhg.view(T * B, 4 * H).t() @ h_prev
        dlnh_w = (dgates * xhat_h).sum((0, 1))
        dlnh_b = dgates.sum((0, 1))
        dlnc_w = (dc_ln * xhat_c).sum((0, 1))
        dlnc_b = dc_ln.sum((0, 1))
        return dgates, dh0, dc0, dw, dlnh_w, dlnh_b, dlnc_w, dlnc_b, None


def lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b):
    """x [T,B,I] -> (out [T,B,H], h_T, c_T).  Input GEMM (+ LN_i) for all T at once; recurrence native."""
    T, B, _ = x.shape
    H = w_hh.shape[1]
    if H not in (384, 32):
        from . import reference
        return reference.lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b)
    xg = torch.nn.functional.linear(x.reshape(T * B, -1), w_ih)
    xp = layer_norm(xg, lni_w, lni_b, out_dtype=torch.float32).view(T, B, 4 * H)
    w_dtype = torch.bfloat16 if torch.is_autocast_enabled() else torch.float32
    out, hT, cT = _LNLSTMRecurrence.apply(xp, h0.float(), c0.float(), w_hh, lnh_w, lnh_b, lnc_w, lnc_b, w_dtype)
    return out, hT, cT
