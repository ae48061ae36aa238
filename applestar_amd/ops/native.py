"""Autograd wrappers around the HIP kernels in ``applestar_amd/_C`` (gfx950).

Each wrapper is a ``torch.autograd.Function`` whose forward and backward both run native kernels.
Shapes/dtypes the kernels do not cover raise instead of silently using torch.
"""
from __future__ import annotations

import collections
import os
import weakref

import torch

from . import _ext

_ACT = {None: 0, 'relu': 1, 'sigmoid': 2, 'tanh': 3}
_C = None


def ensure_loaded():
    global _C
    if _C is None:
        _C = _ext.require()
    return _C


_IMPLEMENTED = {'entity_mean_pool', 'layer_norm', 'gated_residual', 'reverse_scan', 'lnlstm_layer', 'entity_embed', 'upsample2x',
                'spatial_embed', 'varlen_attention', 'su_sample', 'upsample_conv_out', 'maxpool2x2', 'segment_sum',
                'gather_rows', 'conv2d', 'linear', 'resblock', 'gated_resblock', 'head_stats', 'bo_encoder', 'resmlp',
                'location_input', 'value_spatial_proj', 'spatial_embed_pool', 'value_spatial_proj_pool',
                'rl_loss', 'embed_relu', 'col_assemble', 'entity_pack', 'action_logp'}


def has(name: str) -> bool:
    """True when this wrapper module implements ``name`` (the extension is loaded by ensure_loaded)."""
    return name in _IMPLEMENTED


def nhwc(t):
    """[B,C,H,W] (any layout) -> contiguous [B,H,W,C]; free for channels_last tensors."""
    return t.permute(0, 2, 3, 1).contiguous()


def from_nhwc(t):
    """contiguous [B,H,W,C] -> [B,C,H,W] view with channels_last strides."""
    return t.permute(0, 3, 1, 2)


def _lowp(x) -> bool:
    """True when ``x`` is computed at bf16 precision: a bf16 tensor, or any tensor under bf16 autocast."""
    return x.dtype == torch.bfloat16 or torch.is_autocast_enabled()


def _dt_code(dtype) -> int:
    return 1 if dtype == torch.bfloat16 else 0


# ---------------------------------------------------------------------------- layer norm
RESID_LINK = os.environ.get('APPLESTAR_RESID_LINK', '1') == '1'   # A/B switch
_DEBUG_GRADLINK = os.environ.get('APPLESTAR_DEBUG_GRADLINK', '0') == '1'


class GradLink:
    """Hands the residual gradient of ``LN(f(x) + x)`` from the LayerNorm backward to the backward of the
    branch's first linear (``f = ... o linear(x)``), which adds it in the dX GEMM epilogue
    (``addmm(g, dY, W)``): x then receives one gradient instead of two that the autograd engine sums with a
    separate [T, C] add (two per entity-transformer layer).  Autograd runs the LayerNorm backward before the
    linear's (the linear feeds the LayerNorm), so the hand-off is ordered.  The LayerNorm only hands off
    when the linear armed the link in forward on the native path with the residual itself as its input
    (``armed`` is that tensor), so an unarmed link leaves the plain two-gradient path in place.

    Aliasing invariant: when the residual has the LayerNorm input's dtype, ``g`` IS the LayerNorm's input
    gradient, which autograd also passes on as the gradient of the branch output (the attention projection /
    MLP output).  The linear adds into it in place, so every reader of that gradient must run before the
    branch's first linear's backward - true for the plain autograd order on one stream (the branch's later
    layers consume it first).  A ``retain_grad`` / stored tensor hook on the branch output, or a consumer on
    another stream, would see the sum: do not add either to a GradLink block.  ``APPLESTAR_DEBUG_GRADLINK=1``
    checks at the hand-over that nothing wrote to ``g`` in between (tensor version counter)."""
    __slots__ = ('armed', 'g', 'version')

    def __init__(self):
        self.armed = None
        self.g = None
        self.version = None


LN_RELU_MASK = os.environ.get('APPLESTAR_LN_RELU_MASK', '1') == '1'   # A/B switch


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, act, eps, out_dtype, link=None):
        x_c = x.contiguous()
        res_c = res.contiguous() if res is not None else None
        y, mean, rstd, xsum = _C.layer_norm_fwd(x_c, res_c, w, b, _dt_code(out_dtype), eps, _ACT[act], True)
        xin = xsum if res is not None else x_c
        # residual LN over an fp32 ReLU output (the transformer FFN's last layer): the backward writes x's gradient
        # masked as a second output beside the residual's unmasked one, so the ReLU's producer skips its threshold
        ctx.mask_x = LN_RELU_MASK and res is not None and x_c.dtype == torch.float32 and _relu_src(x_c)
        ctx.save_for_backward(xin, y, w, mean, rstd, x_c if ctx.mask_x else None)
        ctx.act = act
        ctx.has_res = res is not None
        ctx.x_dtype = x.dtype
        ctx.res_dtype = res.dtype if res is not None else None
        ctx.link = link if (link is not None and res is not None and link.armed is res) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        xin, y, w, mean, rstd, xm = ctx.saved_tensors
        dy = dy.contiguous()
        dxm = None
        if xm is not None and ctx.needs_input_grad[0]:
            dx, dw, db, dxm = _C.layer_norm_bwd(dy, xin, y, w, mean, rstd, _dt_code(ctx.x_dtype), _ACT[ctx.act], xm)
            _MASKED_DX[xm.data_ptr()] = (dxm, dxm._version)
        else:
            dx, dw, db = _C.layer_norm_bwd(dy, xin, y, w, mean, rstd, _dt_code(ctx.x_dtype), _ACT[ctx.act])
        dres = None
        if ctx.has_res:
            dres = dx if ctx.res_dtype == ctx.x_dtype else dx.to(ctx.res_dtype)
            if ctx.link is not None and ctx.needs_input_grad[1]:
                ctx.link.g, dres = dres, None      # added by the branch linear's dX GEMM (GradLink)
                ctx.link.version = ctx.link.g._version if _DEBUG_GRADLINK else None
        return dx if dxm is None else dxm, dres, dw, db, None, None, None, None


def layer_norm(x, w, b, residual=None, act=None, eps=1e-5, out_dtype=None, grad_link=None):
    C = x.shape[-1]
    if C % 64 != 0 or C > 1536 or w.dtype != torch.float32:
        from . import reference
        return reference.layer_norm(x, w, b, residual, act, eps)
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    if residual is not None and residual.dtype not in (torch.float32, torch.bfloat16):
        residual = residual.float()
    out_dtype = out_dtype or torch.float32
    return _LayerNorm.apply(x, residual, w, b, act, float(eps), out_dtype, grad_link if RESID_LINK else None)


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
    if x.dim() == 4:  # NCHW logical, run on the NHWC storage (channels_last end to end)
        y, g, x = (nhwc(t.to(dt)) for t in (y, g, x))
        return from_nhwc(_GatedResidual.apply(y, g, sp.float(), x))
    y, g, x = (t.to(dt).contiguous() for t in (y, g, x))
    return _GatedResidual.apply(y, g, sp.float(), x)


# ---------------------------------------------------------------------------- reverse scan (no grad)
def reverse_scan(a, b, init):
    a = a.float().contiguous()
    b = b.float().contiguous()
    init = init.float().contiguous().expand(b.shape[:-2] + b.shape[-1:]).contiguous()
    return _C.reverse_scan(a, b, init)


# ---------------------------------------------------------------------------- LN-LSTM layer
def lstm_exchange_ok(device):
    """Device scalar 1.0 while the split LSTM recurrence's cross-workgroup exchange has never timed out on
    ``device``, else 0.0 (lstm.hip kSplitPollLimit): the trainers multiply it into the optimizer update and log
    it, so a timed-out step never reaches the weights.  None off the GPU."""
    if device.type != 'cuda':
        return None
    return (ensure_loaded().lstm_split_flag(device.index or 0) == 0).float().reshape(())



LSTM_BF16_OUT = os.environ.get('APPLESTAR_LSTM_BF16_OUT', '1') == '1'     # A/B switch


class _LNLSTMRecurrence(torch.autograd.Function):
    """Recurrent part of an LN-LSTM layer: xp [T,B,4H] (already LN_i(x W_ih^T)) -> h [T,B,H]."""

    @staticmethod
    def forward(ctx, xp, h0, c0, w_hh, lnh_w, lnh_b, lnc_w, lnc_b, w_dtype, need_bwd=True):
        # W_hh in the recurrence's dtype, for the backward only (inference skips the cast)
        wq = w_hh.detach().to(w_dtype) if need_bwd else w_hh.detach()
        wT = _wT(w_hh, w_dtype)          # a derived form: transposed once per optimizer step, not per layer call
        # inference under autocast: the recurrence also writes h in bf16, registered as out's cast (_bf16_rows), so
        # the next layer's input projection and the heads read it without a cast launch per layer
        want_bf16 = LSTM_BF16_OUT and not need_bwd and CAST_CACHE and torch.is_autocast_enabled() and xp.is_cuda
        out, hT, cT, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, out_bf = _C.lnlstm_fwd(
            xp.contiguous(), h0.contiguous(), c0.contiguous(), wT, lnh_w.detach(), lnh_b.detach(),
            lnc_w.detach(), lnc_b.detach(), 1e-5, want_bf16)
        if out_bf is not None:
            _note_bf16_copy(out, out_bf)
        ctx.save_for_backward(h0, out, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, wq.contiguous(), lnh_w, lnc_w)
        ctx.set_materialize_grads(False)     # unused hT / cT: None (a cached zero) instead of two fills per layer
        return out, hT, cT

    @staticmethod
    def backward(ctx, dout, dhT, dcT):
        h0, out, c_all, xhat_h, rstd_h, gates, xhat_c, rstd_c, wq, lnh_w, lnc_w = ctx.saved_tensors
        T, B, H = out.shape
        z = lambda t: _zeros_const((B, H), out.device) if t is None else t.float().contiguous()
        dout = torch.zeros_like(out) if dout is None else dout.float().contiguous()
        dgates, dhg, dc_ln, dh0, dc0 = _C.lnlstm_bwd(dout, z(dhT), z(dcT), gates, c_all, xhat_c, rstd_c, xhat_h,
                                                     rstd_h, wq, lnh_w.detach(), lnc_w.detach())
        # the recurrence is launched (its 8-workgroup rows are dispatched first): the heads' queued weight
        # gradients now fill the CUs it leaves idle (_Deferred)
        defer_flush()
        h_prev = torch.cat([h0.float().unsqueeze(0), out[:-1]], 0).view(T * B, H)
        dw = _mm_tn(dhg.view(T * B, 4 * H), h_prev)
        # LN_h / LN_c affine gradients: one column-sum launch each (four products + reductions as torch ops
        # were ~17 launches at ~19 us per LSTM backward, r2dl)
        dlnh_w, dlnh_b = _C.ln_affine_grads(dgates.contiguous(), xhat_h.contiguous()).unbind(0)
        dlnc_w, dlnc_b = _C.ln_affine_grads(dc_ln.contiguous(), xhat_c.contiguous()).unbind(0)
        return dgates, dh0, dc0, dw, dlnh_w, dlnh_b, dlnc_w, dlnc_b, None, None


_ZEROS = {}


def _zeros_const(shape, device):
    """A cached all-zero fp32 tensor (read-only input of a kernel, e.g. the LSTM's absent final-state
    gradients): no fill launch per use.  Callers must never write into it."""
    key = (tuple(shape), str(device))
    t = _ZEROS.get(key)
    if t is None or t._version != 0:
        t = _ZEROS[key] = torch.zeros(shape, device=device)
    return t


def entity_mean_pool(x, valid, num):
    """Mean of x [B,N,C] over the valid rows (valid [B,N] bool), divided by max(num, 1), in x's dtype with fp32
    accumulation: one launch (inference only - no autograd node)."""
    if valid.dtype != torch.bool or num.dtype not in (torch.int64, torch.int32) or x.dtype not in (torch.float32,
                                                                                                  torch.bfloat16):
        return None
    return ensure_loaded().entity_mean_pool(x.contiguous(), valid.contiguous(), num.contiguous())


def lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b):
    """x [T,B,I] -> (out [T,B,H], h_T, c_T).  Input GEMM (+ LN_i) for all T at once; recurrence native."""
    T, B, _ = x.shape
    H = w_hh.shape[1]
    if H not in (384, 32):
        from . import reference
        return reference.lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b)
    x2 = x.reshape(T * B, -1)
    # bf16 input projection through linear(): its dW takes the split-R MFMA kernel, not a library GEMM that
    # tiles only the 4H x I output over T*B = 24576 rows (the selected-units head's LSTM)
    xg = linear(x2, w_ih) if x2.dtype in (torch.bfloat16, torch.float32) and \
        (x2.dtype == w_ih.dtype or torch.is_autocast_enabled()) else torch.nn.functional.linear(x2, w_ih)
    xp = layer_norm(xg, lni_w, lni_b, out_dtype=torch.float32).view(T, B, 4 * H)
    w_dtype = torch.bfloat16 if torch.is_autocast_enabled() else torch.float32
    need_bwd = torch.is_grad_enabled() and any(t.requires_grad for t in (xp, h0, c0, w_hh, lnh_w, lnh_b, lnc_w, lnc_b))
    out, hT, cT = _LNLSTMRecurrence.apply(xp, h0.float(), c0.float(), w_hh, lnh_w, lnh_b, lnc_w, lnc_b, w_dtype,
                                          need_bwd)
    return out, hT, cT


# ---------------------------------------------------------------------------- entity embedding
_KIND = {'one_hot': 0, 'binary': 1, 'scalar': 2}


def _entity_table(entity_info):
    from ..models.encoders import ENTITY_LAYOUT
    fields, kind, offset, width = [], [], [], []
    for name, enc, off, w in ENTITY_LAYOUT:
        fields.append(entity_info[name].contiguous())
        kind.append(_KIND[enc])
        offset.append(off)
        width.append(w)
    return fields, kind, offset, width


# bf16 dW of the entity embedding on MFMA with the sparse input scattered per 32-token step (entity.hip):
# A/B 35.65 -> 34.74 ms/step vs the materialised one-hot + library GEMM (APPLESTAR_ENTITY_SPARSE_WGRAD=0)
ENTITY_SPARSE_WGRAD = os.environ.get('APPLESTAR_ENTITY_SPARSE_WGRAD', '1') != '0'


class _EntityEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, b, index, out_dtype, *fields):
        from ..models.encoders import ENTITY_LAYOUT
        kind = [_KIND[e] for _, e, _, _ in ENTITY_LAYOUT]
        offset = [o for _, _, o, _ in ENTITY_LAYOUT]
        width = [x for _, _, _, x in ENTITY_LAYOUT]
        wq = _wT(w, out_dtype)                              # [997, 256]
        out = _C.entity_embed_fwd(list(fields), kind, offset, width, index, wq, b.detach().float(),
                                  _dt_code(out_dtype))
        ctx.save_for_backward(out, index, *fields)
        ctx.meta = (kind, offset, width, w.shape[1], out_dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        out, index, *fields = ctx.saved_tensors
        kind, offset, width, k_in, out_dtype = ctx.meta
        if ENTITY_SPARSE_WGRAD and out.dtype == torch.bfloat16:   # bf16 MFMA: the autocast path's precision
            dw, db = _C.entity_embed_wgrad(list(fields), kind, offset, width, index,
                                           dout.to(out.dtype).contiguous(), out, k_in)
            return (dw, db, None, None) + (None,) * len(fields)
        dpre = (dout * (out > 0)).to(out_dtype)
        if out_dtype == torch.float32 and dpre.shape[1] % 4 == 0:
            # fp32 step: the split-R f32 weight gradient over the one-hot input padded to a multiple of 4 columns
            kp = (k_in + 3) // 4 * 4
            X = _C.entity_onehot(list(fields), kind, offset, width, index, kp, _dt_code(out_dtype))
            dw, db = _C.wgrad_f32(dpre.contiguous(), X, 0, True)
            return (dw[:, :k_in], db, None, None) + (None,) * len(fields)
        X = _C.entity_onehot(list(fields), kind, offset, width, index, k_in, _dt_code(out_dtype))
        dw = (dpre.t() @ X).float()
        db = dpre.float().sum(0)
        return (dw, db, None, None) + (None,) * len(fields)


def entity_embed(entity_info, flat_index, w, b):
    """relu(one_hot_997(entity rows flat_index) @ w^T + b) without materialising the 997-wide input."""
    fields, _, _, _ = _entity_table(entity_info)
    flat = [f.reshape(-1) for f in fields]
    out_dtype = torch.bfloat16 if torch.is_autocast_enabled() else torch.float32
    return _EntityEmbed.apply(w, b, flat_index.contiguous(), out_dtype, *flat)


# ---------------------------------------------------------------------------- bilinear x2 (NHWC)
class _Upsample2x(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_nhwc):
        # an fp32 ReLU output as input: the backward applies its mask (the producer conv skips its threshold)
        relu_in = x_nhwc.dtype == torch.float32 and x_nhwc.is_contiguous() and _relu_src(x_nhwc)
        ctx.save_for_backward(x_nhwc if relu_in else None)
        return _C.upsample2x_fwd(x_nhwc)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        dx = _C.upsample2x_bwd(dy.contiguous(), x)
        if x is not None:
            _MASKED_DX[x.data_ptr()] = (dx, dx._version)
        return dx


def upsample2x(x):
    """F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=False) for [B,C,H,W] with C%4==0;
    computed in x's dtype (bf16 stays bf16) on the channels_last storage."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return from_nhwc(_Upsample2x.apply(nhwc(x)))


# ---------------------------------------------------------------------------- spatial input embedding
class _SpatialEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w_dense, bias, rows, ex, ey, entity_num, out_dtype, n_planes, *tensors):
        planes = list(tensors[:n_planes])
        effects = list(tensors[n_planes:])
        _, out = _C.spatial_embed_fwd(planes, effects, _w32(w_dense),
                                      _w32(bias), rows.contiguous(), ex, ey, entity_num,
                                      _dt_code(out_dtype))
        ctx.save_for_backward(out, ex, ey, entity_num, *tensors)
        ctx.n_planes = n_planes
        ctx.N = rows.shape[1]
        ctx.rows_dtype = rows.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        out, ex, ey, entity_num, *tensors = ctx.saved_tensors
        planes, effects = list(tensors[:ctx.n_planes]), list(tensors[ctx.n_planes:])
        if dout.dtype == out.dtype and dout.is_contiguous():
            # NHWC gradient of the same dtype: the ReLU mask is applied inside the two consumers (no
            # dpre round trip over the 9.5M-pixel map)
            drows = _C.spatial_gather_rows(dout, ex, ey, entity_num, ctx.N, out).to(ctx.rows_dtype)
            dw, db = _C.spatial_dense_wgrad(planes, effects, dout, out)
            return (dw, db, drows) + (None,) * (5 + len(tensors))
        if out.dtype == torch.bfloat16:   # one pass: ReLU mask + cast + NHWC
            dpre = _C.act_grad_nhwc(dout, out, True)
        else:
            dpre = (dout * (out > 0)).to(out.dtype).contiguous()                # [B,H,W,32]
        drows = _C.spatial_gather_rows(dpre, ex, ey, entity_num, ctx.N).to(ctx.rows_dtype)
        # dense-column weight gradient straight from dpre and the planes (no [npix, 24] input matrix)
        dw, db = _C.spatial_dense_wgrad(planes, effects, dpre.contiguous())
        return (dw, db, drows) + (None,) * (5 + len(tensors))


def spatial_embed(spatial_info, rows, entity_x, entity_y, entity_num, w_dense, bias):
    """relu(1x1conv(56 input planes)) where the 32 scatter channels arrive pre-multiplied per entity
    (``rows`` = scatter_project(entity) @ W[:, 24:56]^T).  Returns [B,32,H,W] channels_last."""
    from ..lib.features import SPATIAL_ONE_HOT, EFFECT_KEYS
    planes = [spatial_info['height_map']] + [spatial_info[k] for k, _ in SPATIAL_ONE_HOT]
    planes = [p.to(torch.uint8).contiguous() for p in planes]
    effects = [spatial_info[k].to(torch.int16).contiguous() for k in EFFECT_KEYS]
    out_dtype = torch.bfloat16 if torch.is_autocast_enabled() else torch.float32
    ex = entity_x.to(torch.uint8).contiguous()
    ey = entity_y.to(torch.uint8).contiguous()
    out = _SpatialEmbed.apply(w_dense, bias, rows, ex, ey, entity_num.long().contiguous(), out_dtype, len(planes),
                              *planes, *effects)
    return from_nhwc(out)


SPATIAL_POOL_FUSED = os.environ.get('APPLESTAR_SPATIAL_POOL_FUSED', '1') == '1'


class _SpatialEmbedPool(torch.autograd.Function):
    """relu(embed) -> max_pool2x2 of the spatial encoder's first stage in one kernel (spatial.hip
    spatial_embed_pool_kernel): the full-resolution map (607 MB at the learner batch) is neither written nor
    re-read by a separate pool.  Backward: one pass builds the full-resolution dpre from the pooled gradient,
    the argmax bytes and the pooled ReLU output (maxpool2_bwd_relu), then the unfused gather / dense-wgrad
    kernels run on it without a gate."""

    @staticmethod
    def forward(ctx, w_dense, bias, rows, ex, ey, entity_num, n_planes, *tensors):
        planes = list(tensors[:n_planes])
        effects = list(tensors[n_planes:])
        pooled, pos = _C.spatial_embed_pool_fwd(planes, effects, _w32(w_dense),
                                                _w32(bias), rows.contiguous(), ex, ey,
                                                entity_num)
        ctx.save_for_backward(pooled, pos, ex, ey, entity_num, *tensors)
        ctx.n_planes = n_planes
        ctx.N = rows.shape[1]
        ctx.rows_dtype = rows.dtype
        ctx.HW = (planes[0].shape[1], planes[0].shape[2])
        return pooled

    @staticmethod
    def backward(ctx, dpooled):
        pooled, pos, ex, ey, entity_num, *tensors = ctx.saved_tensors
        planes, effects = list(tensors[:ctx.n_planes]), list(tensors[ctx.n_planes:])
        H, W = ctx.HW
        if POOLED_BWD and pooled.dtype == torch.float32 and H % 2 == 0 and W % 2 == 0:
            # fp32: the row gather and the dense weight gradient compute dpre from the pooled gradient, the argmax bytes
            # and the pooled ReLU output on the fly - no 1.2 GB full-resolution dpre written and read back twice
            dy = dpooled.to(torch.float32).contiguous()
            drows = _C.spatial_gather_rows_pooled(dy, pooled.contiguous(), pos.contiguous(), ex, ey, entity_num, ctx.N,
                                                  H, W).to(ctx.rows_dtype)
            dw, db = _C.spatial_dense_wgrad_pooled(planes, effects, dy, pooled.contiguous(), pos.contiguous())
            return (dw, db, drows) + (None,) * (4 + len(tensors))
        dpre = _C.maxpool2_bwd_relu(dpooled.to(pooled.dtype).contiguous(), pos, pooled, H, W)
        drows = _C.spatial_gather_rows(dpre, ex, ey, entity_num, ctx.N).to(ctx.rows_dtype)
        dw, db = _C.spatial_dense_wgrad(planes, effects, dpre)
        return (dw, db, drows) + (None,) * (4 + len(tensors))


SPATIAL_POOL_FUSED_F32 = os.environ.get('APPLESTAR_SPATIAL_POOL_FUSED_F32', '1') == '1'
# the fp32 fused embed + pool backward without the full-resolution dpre (spatial.hip *_pooled; A/B switch)
POOLED_BWD = os.environ.get('APPLESTAR_POOLED_BWD', '1') == '1'


def spatial_embed_pool(spatial_info, rows, entity_x, entity_y, entity_num, w_dense, bias):
    """max_pool2x2(spatial_embed(...)) as [B,32,H/2,W/2] channels_last (bf16 under autocast / bf16 rows; fp32 in
    the fp32 step: the projection on three exact bf16 parts of W against the exact-in-bf16 planes), or None when
    the fused stage does not apply (odd or wide maps)."""
    from ..lib.features import SPATIAL_ONE_HOT, EFFECT_KEYS
    H, W = spatial_info['height_map'].shape[-2:]
    lowp = torch.is_autocast_enabled() or rows.dtype == torch.bfloat16
    f32 = not lowp and rows.dtype == torch.float32 and SPATIAL_POOL_FUSED_F32
    if not SPATIAL_POOL_FUSED or not (lowp or f32) or not _C.spatial_pool_supported(H, W):
        return None
    planes = [spatial_info['height_map']] + [spatial_info[k] for k, _ in SPATIAL_ONE_HOT]
    planes = [p.to(torch.uint8).contiguous() for p in planes]
    effects = [spatial_info[k].to(torch.int16).contiguous() for k in EFFECT_KEYS]
    ex = entity_x.to(torch.uint8).contiguous()
    ey = entity_y.to(torch.uint8).contiguous()
    with torch.autocast('cuda', enabled=False):
        out = _SpatialEmbedPool.apply(w_dense, bias, rows.contiguous() if f32 else rows.to(torch.bfloat16), ex, ey,
                                      entity_num.long().contiguous(), len(planes), *planes, *effects)
    return from_nhwc(out)


class _RLLossTail(torch.autograd.Function):
    """The RL loss after the per-head statistics (rl_loss.hip): one kernel computes the total, the info
    vector and the closed-form gradients w.r.t. the stacked log-probs / entropies / KLs / values; backward
    only scales them by the incoming gradient."""

    @staticmethod
    def forward(ctx, alp, ent, kl, v, blp, hm, r, wm, atflag, sc, upgo_f, only_value):
        c = lambda t: t.detach().float().contiguous()  # noqa: E731
        info, dalp, dent, dkl, dv = _C.rl_loss(c(alp), c(blp), c(hm), c(ent), c(kl), c(v), c(r), c(wm), c(atflag),
                                               sc, int(upgo_f), bool(only_value))
        ctx.save_for_backward(dalp, dent, dkl, dv)
        ctx.dtypes = (alp.dtype, ent.dtype, kl.dtype, v.dtype)
        ctx.mark_non_differentiable(info)
        return info[-1], info

    @staticmethod
    def backward(ctx, gtotal, ginfo):
        dalp, dent, dkl, dv = ctx.saved_tensors
        da, de, dk, dvv = (g * gtotal for g in (dalp, dent, dkl, dv))
        return (da.to(ctx.dtypes[0]), de.to(ctx.dtypes[1]), dk.to(ctx.dtypes[2]), dvv.to(ctx.dtypes[3])) + (None,) * 8


def rl_loss_tail(alp, ent, kl, v, blp, hm, r, wm, atflag, sc, upgo_f, only_value):
    """(total loss 0-d, info vector) of the fused RL loss tail; see rl/loss.py _compute_loss_fused."""
    return _RLLossTail.apply(alp, ent, kl, v, blp, hm, r, wm, atflag, sc, upgo_f, only_value)


# ---------------------------------------------------------------------------- varlen attention
class _VarlenAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cu, max_len, heads):
        out, lse = _C.varlen_attn_fwd(qkv, cu, max_len, heads)
        ctx.save_for_backward(qkv, out, lse, cu)
        ctx.max_len, ctx.heads = max_len, heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, cu = ctx.saved_tensors
        dqkv = _C.varlen_attn_bwd(qkv, out, dout.to(torch.bfloat16).contiguous(), lse, cu, ctx.max_len, ctx.heads)
        return dqkv, None, None, None


class _VarlenAttentionF32(torch.autograd.Function):
    """fp32 operands end to end (attention_f32.hip): the like-for-like path of the fp32 learner step."""

    @staticmethod
    def forward(ctx, qkv, cu, max_len, heads):
        out, lse = _C.varlen_attn_fwd_f32(qkv, cu, max_len, heads)
        ctx.save_for_backward(qkv, out, lse, cu)
        ctx.max_len, ctx.heads = max_len, heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, cu = ctx.saved_tensors
        dqkv = _C.varlen_attn_bwd_f32(qkv, out, dout.float().contiguous(), lse, cu, ctx.max_len, ctx.heads)
        return dqkv, None, None, None


def varlen_attention(qkv, cu_seqlens, max_len: int, num_heads: int, head_dim: int):
    """Packed self-attention over variable-length entity sets, head_dim 128: the bf16 flash kernel for bf16
    operands (the mixed-precision step), the fp32 flash kernel (f32-input MFMA) for fp32 operands - an fp32
    input is never rounded to bf16."""
    if head_dim != 128 or qkv.dtype not in (torch.float32, torch.bfloat16):
        from . import reference
        return reference.varlen_attention(qkv, cu_seqlens, max_len, num_heads, head_dim)
    cu = cu_seqlens.to(torch.int32).contiguous()
    if qkv.dtype == torch.float32:
        if not hasattr(ensure_loaded(), 'varlen_attn_fwd_f32'):
            from . import reference
            return reference.varlen_attention(qkv, cu_seqlens, max_len, num_heads, head_dim)
        return _VarlenAttentionF32.apply(qkv.contiguous(), cu, int(max_len), int(num_heads))
    return _VarlenAttention.apply(qkv.contiguous(), cu, int(max_len), int(num_heads))


def linear_f32_rows(x, w, b=None):
    """fp32 x W^T + b without autograd (inference): the native f32 GEMM when it takes the shape (few rows: one wave
    per 32 x 32 tile), else torch.addmm; the weight / bias read as fp32 derived forms."""
    C = ensure_loaded()
    R, K = x.shape
    if x.is_cuda and _gemm_f32_ok(R, w.shape[0], K):
        return C.gemm_f32(x.contiguous(), _w32(w), None if b is None else _w32(b), None, 0)
    return torch.addmm(b.float(), x, w.float().t()) if b is not None else x @ w.float().t()


def su_sample(key, c0, u, entity_num, su_mask, wf_bf16, bf, wq2, bq2, cell, we1, be1, temperature: float,
              max_steps: int, extra_units: bool):
    """Persistent selected-units sampler (inference only; see csrc/kernels/pointer.hip)."""
    C = ensure_loaded()
    f = lambda t: t.detach().float().contiguous()
    key = key.detach()
    if key.dtype not in (torch.float32, torch.bfloat16):
        key = key.float()
    return C.su_sample(key.contiguous(), f(c0), f(u), entity_num.long().contiguous(),
                       su_mask.to(torch.uint8).contiguous(), wf_bf16.contiguous(), f(bf), f(wq2), f(bq2),
                       f(cell.weight_ih), f(cell.weight_hh), f(cell.layernorm_i.weight), f(cell.layernorm_i.bias),
                       f(cell.layernorm_h.weight), f(cell.layernorm_h.bias), f(cell.layernorm_c.weight),
                       f(cell.layernorm_c.bias), f(we1), f(be1), float(temperature), 1e-5, int(max_steps),
                       bool(extra_units))


# ---------------------------------------------------------------------------- upsample x2 + conv -> 1 ch
UPCONV_RELU = os.environ.get('APPLESTAR_UPCONV_RELU', '1') == '1'   # A/B switch


class _UpsampleConvOut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_nhwc, w, b):
        w32 = w.detach().float().reshape(-1).contiguous()
        bias = b.detach().float().reshape(1).contiguous() if b is not None else w32.new_zeros(1)
        y = _C.upconv1_fwd(x_nhwc, w32, bias)
        ctx.save_for_backward(x_nhwc, w32)
        ctx.has_bias = b is not None
        ctx.w_shape, ctx.w_dtype = w.shape, w.dtype
        # an fp32 ReLU conv output as input: dX takes its mask in the kernel (the conv skips its threshold pass)
        relu_in = UPCONV_RELU and x_nhwc.dtype == torch.float32 and x_nhwc.is_contiguous() and _relu_src(x_nhwc)
        ctx.x_ptr = x_nhwc.data_ptr() if relu_in else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x_nhwc, w32 = ctx.saved_tensors
        dx, dwb = _C.upconv1_bwd(x_nhwc, w32, dy.float().contiguous(), ctx.x_ptr is not None)
        if ctx.x_ptr is not None:
            _MASKED_DX[ctx.x_ptr] = (dx, dx._version)
        dw = dwb[:-1].view(ctx.w_shape).to(ctx.w_dtype)
        db = dwb[-1:].to(ctx.w_dtype) if ctx.has_bias else None
        return dx, dw, db


def upsample_conv_out(x, weight, bias):
    """conv3x3(upsample_bilinear_x2(x), weight[1,32,3,3], padding 1) + bias for [B,32,H,W] -> [B,2H*2W]
    fp32 logits, fused (the 32-channel upsampled map never reaches HBM)."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return _UpsampleConvOut.apply(nhwc(x), weight, bias).reshape(x.shape[0], -1)


# ---------------------------------------------------------------------------- max-pool 2x2 (NHWC)
POOL_BWD_RELU = os.environ.get('APPLESTAR_POOL_BWD_RELU', '1') == '1'


class _MaxPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_nhwc):
        y, pos = _C.maxpool2_fwd(x_nhwc)
        # an fp32 ReLU output as input: the backward applies its mask (the producer conv skips its threshold).  The
        # mask at the argmax is (pooled value > 0) - the pooled value IS the input there - so the backward reads the
        # pooled output (maxpool2_bwd_relu: one thread per pooled pixel) instead of the full-resolution input
        relu_in = x_nhwc.dtype == torch.float32 and x_nhwc.is_contiguous() and _relu_src(x_nhwc)
        H, W = x_nhwc.shape[1], x_nhwc.shape[2]
        ctx.pooled_mask = relu_in and POOL_BWD_RELU and H % 2 == 0 and W % 2 == 0 and x_nhwc.shape[3] % 8 == 0
        ctx.save_for_backward(pos, y if ctx.pooled_mask else (x_nhwc if relu_in else None))
        ctx.x_ptr = x_nhwc.data_ptr() if relu_in else None
        ctx.hw = (H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        pos, m = ctx.saved_tensors
        if ctx.pooled_mask:
            dx = _C.maxpool2_bwd_relu(dy.to(m.dtype).contiguous(), pos, m, *ctx.hw)
        else:
            dx = _C.maxpool2_bwd(dy.contiguous(), pos, *ctx.hw, m)
        if ctx.x_ptr is not None:
            _MASKED_DX[ctx.x_ptr] = (dx, dx._version)
        return dx


def maxpool2x2(x):
    """F.max_pool2d(x, 2, 2) for [B,C,H,W] (C % 8 == 0) on the channels_last storage."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return from_nhwc(_MaxPool2.apply(nhwc(x)))


# ---------------------------------------------------------------------------- packed-segment sum
class _SegmentSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cu, seg):
        ctx.save_for_backward(seg)
        ctx.dtype = x.dtype
        return _C.segment_sum(x.contiguous(), cu)

    @staticmethod
    def backward(ctx, dout):
        seg, = ctx.saved_tensors
        return dout.index_select(0, seg).to(ctx.dtype), None, None


def segment_sum(x, cu, seg):
    """Row sums of packed x [T,C] per segment (cu int32 [S+1]; seg [T] = segment of each row) -> fp32 [S,C]."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return _SegmentSum.apply(x, cu.to(torch.int32).contiguous(), seg)


# ---------------------------------------------------------------------------- small-table row gather
class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, idx):
        ctx.save_for_backward(idx)
        ctx.V, ctx.dtype = table.shape[0], table.dtype
        return table.index_select(0, idx)

    @staticmethod
    def backward(ctx, dout):
        idx, = ctx.saved_tensors
        d = dout.reshape(idx.numel(), -1)
        if d.dtype not in (torch.float32, torch.bfloat16):
            d = d.float()
        return _C.table_grad(d.contiguous(), idx, ctx.V).to(ctx.dtype), None


def gather_rows(table, idx):
    """table[idx] whose backward accumulates in LDS per block (tiny tables hit by ~1e5 indices)."""
    if table.shape[0] * table.shape[1] > 16384:
        return table.index_select(0, idx)
    return _GatherRows.apply(table, idx.long().contiguous())


def entity_pack(entity_num, N: int, total: int):
    """(valid [B, N] bool, flat [total] int64, seg [total] int64, cu [B + 1] int32) of the packed entity rows in one
    launch (pool_reduce.hip entity_pack_kernel)."""
    num = entity_num.reshape(-1)
    if num.dtype not in (torch.int64, torch.int32):
        num = num.long()
    return tuple(_C.entity_pack(num.contiguous(), int(N), int(total)))


class _ColAssemble(torch.autograd.Function):
    """Concatenations of one set of [R, w_i] pieces along columns into several outputs (output j takes the pieces
    flagged in masks[j], in order) in ONE launch (multi_copy.hip col_sum); backward: each piece's gradient as the sum
    of its column blocks of the output gradients, one launch - instead of a cat per output and an autograd add per
    extra use of a piece (the scalar encoder: 3 cats + 12 adds)."""

    @staticmethod
    def forward(ctx, masks, *pieces):
        R = pieces[0].shape[0]
        widths = [p.shape[1] for p in pieces]
        outs, offs = [], []
        for m in masks:
            outs.append(pieces[0].new_empty(R, sum(w for w, f in zip(widths, m) if f)))
            o, acc = [], 0
            for w, f in zip(widths, m):
                o.append(acc if f else -1)
                acc += w if f else 0
            offs.append(o)
        dsts, dcols, ws, srcs, scols = [], [], [], [], []
        for j, o in enumerate(offs):
            for i, off in enumerate(o):
                if off >= 0:
                    dsts.append(outs[j]), dcols.append(off), ws.append(widths[i])
                    srcs.append([pieces[i]]), scols.append([0])
        for k in range(0, len(dsts), 32):
            _C.col_sum(dsts[k:k + 32], dcols[k:k + 32], ws[k:k + 32], srcs[k:k + 32], scols[k:k + 32])
        ctx.offs, ctx.widths = offs, widths
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        douts = [None if d is None else d.float().contiguous() for d in douts]
        R = next(d.shape[0] for d in douts if d is not None)
        grads, dsts, dcols, ws, srcs, scols = [], [], [], [], [], []
        for i, w in enumerate(ctx.widths):
            ss = [(douts[j], ctx.offs[j][i]) for j in range(len(douts)) if douts[j] is not None and ctx.offs[j][i] >= 0]
            if not ss:
                grads.append(None)
                continue
            g = douts[0].new_empty(R, w) if douts[0] is not None else ss[0][0].new_empty(R, w)
            grads.append(g)
            dsts.append(g), dcols.append(0), ws.append(w)
            srcs.append([t for t, _ in ss]), scols.append([c for _, c in ss])
        for k in range(0, len(dsts), 32):
            _C.col_sum(dsts[k:k + 32], dcols[k:k + 32], ws[k:k + 32], srcs[k:k + 32], scols[k:k + 32])
        return (None, *grads)


def col_assemble(pieces, masks):
    """tuple of outputs, output j = cat([p for p, f in zip(pieces, masks[j]) if f], 1); None when not covered."""
    if not COL_ASSEMBLE or not pieces or \
            any(p.dtype != torch.float32 or p.dim() != 2 or not p.is_cuda or p.stride(1) != 1 for p in pieces) or \
            len({p.shape[0] for p in pieces}) != 1:
        return None
    return _ColAssemble.apply(tuple(tuple(bool(f) for f in m) for m in masks), *pieces)


class _EmbedRelu(torch.autograd.Function):
    """relu(table[clamp(idx, 0, V - 1)]) in one launch; backward: the ReLU-masked rows summed per index in LDS
    (pool_reduce.hip embed_relu_*).  The scalar encoder's small embedding tables."""

    @staticmethod
    def forward(ctx, table, idx):
        out = _C.embed_relu_fwd(table.detach().contiguous(), idx)
        ctx.save_for_backward(idx, out)
        ctx.V, ctx.dtype = table.shape[0], table.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        idx, out = ctx.saved_tensors
        return _C.embed_relu_bwd(dout.to(out.dtype).contiguous(), out, idx, ctx.V).to(ctx.dtype), None


def embed_relu(table, idx):
    """relu(table[clamp(idx, max=V - 1)]) as [*idx.shape, D]; None when the table is too large for the LDS
    accumulation (caller falls back)."""
    V, D = table.shape
    if V * D > 16384 or table.dtype not in (torch.float32, torch.bfloat16) or \
            idx.dtype not in (torch.int64, torch.int32, torch.int16, torch.uint8, torch.int8):
        return None
    out = _EmbedRelu.apply(table, idx.contiguous().reshape(-1))
    return out.view(*idx.shape, D)


# ---------------------------------------------------------------------------- dtype-generic conv / GEMM pieces
# Every conv / linear autograd node below runs on bf16 operands (the mixed-precision step: bf16 MFMA kernels) or
# on fp32 operands (the fp32 step: f32-MFMA kernels conv3x3_f32.hip / wgrad_f32.hip); an fp32 operand is never
# rounded to bf16.
def _conv3(x, wk, bias, res, act_code, w=None, dx=False, res2=None, mask=None):
    """3x3 / pad 1 conv on NHWC x with a [Cout, 3, 3, Cin] weight wk, epilogue act code (_ACT / 4 = ReLU mask).
    ``w``: the conv parameter wk derives from (wk = _conv_w(w), or _conv_wt(w) for ``dx``): fp32 convs with 128-multiple
    outputs then run on its pre-split planes (gemm_f32_psb.hip conv3x3_f32_psb_kernel).  res2 / mask: the extended
    input-gradient epilogue (conv3x3_f32_epi2)."""
    if x.dtype == torch.float32:
        B, H, W, Cin = x.shape
        Cout = wk.shape[0]
        if w is not None and CONV_PSB and _C.conv3x3_f32_psb_supported(B * H * W, Cin, Cout):
            return _C.conv3x3_f32_psb(x, _psb_conv(w, dx), Cout, bias, res, res2, mask, act_code)
        if res2 is not None or mask is not None:
            return _C.conv3x3_f32_epi2(x, wk, res, res2, mask)
        return _C.conv3x3_f32(x, wk, bias, res, act_code)
    return _C.conv3x3_fwd(x, wk, bias, res, act_code)


def _act_grad(dout, out, relu):
    """dout * (out > 0) (relu) or dout, as a contiguous tensor of out's shape and dtype (one pass)."""
    if out.dtype == torch.bfloat16:
        return _C.act_grad_nhwc(dout, out, relu)
    dout = dout.to(out.dtype).contiguous()
    return torch.ops.aten.threshold_backward(dout, out, 0.0) if relu else dout


def _wgrad(dy2d, x, cin, has_b, bf16_out, param=None):
    """(dW, db) of a dense GEMM (cin == 0, x [R, K]) or a 3x3 conv (x NHWC image, Cin = cin) in dy's precision.
    ``param``: the weight, when the caller lets the product be deferred (_Deferred: single-use weights only)."""
    if _ABL_NO_WGRAD:
        return _abl_zero_wgrad(dy2d, x, cin, has_b, bf16_out)
    if dy2d.dtype == torch.float32:
        if _Deferred.on and dy2d.is_cuda and param is not None and _single_use(param):
            return _Deferred.add(dy2d, x, cin, has_b, param)
        return _C.wgrad_f32(dy2d, x, cin, has_b)
    return _C.wgrad(dy2d, x, cin, has_b, bf16_out)


# timing ablation only (tools/host_gpu_timeline.py): every weight gradient of the native kernels is a cached zero
# tensor, no launch - the step without its weight-gradient work, i.e. how much of it the side streams hide
_ABL_NO_WGRAD = os.environ.get('APPLESTAR_ABL_NO_WGRAD', '0') == '1'
_ABL_ZEROS = {}


def _abl_zero_wgrad(dy2d, x, cin, has_b, bf16_out):
    N, K = dy2d.shape[1], (9 * cin if cin else x.shape[-1])
    dt = dy2d.dtype if dy2d.dtype == torch.float32 or not bf16_out else torch.bfloat16
    key = (N, K, dt, dy2d.device)
    if key not in _ABL_ZEROS:
        _ABL_ZEROS[key] = (torch.zeros(N, K, dtype=dt, device=dy2d.device), torch.zeros(N, dtype=dt, device=dy2d.device))
    dw, db = _ABL_ZEROS[key]
    return dw, (db if has_b else None)


# ---------------------------------------------------------------------------- deferred weight gradients
DEFER_WGRAD = os.environ.get('APPLESTAR_DEFER_WGRAD', '1') == '1'     # A/B switch


_FWD_EPOCH = [0]


def _count_use(p) -> None:
    """Record one forward use of parameter ``p`` in the current step (``_FWD_EPOCH``)."""
    if isinstance(p, torch.nn.Parameter):
        u = getattr(p, '_as_uses', None)
        p._as_uses = (_FWD_EPOCH[0], u[1] + 1) if u is not None and u[0] == _FWD_EPOCH[0] else (_FWD_EPOCH[0], 1)


def _single_use(p) -> bool:
    """``p`` fed exactly one native node in this step's forward AND has exactly one consumer in this step's
    autograd graph (``single_consumer_params``, checked by :func:`defer_begin`): autograd returns that node's
    gradient as is.  A weight with a second consumer - another native node, or an uncounted path such as
    ``F.linear`` or a torch fallback - would have its gradients summed by autograd on the main stream into a
    buffer the side stream has not written yet."""
    u = getattr(p, '_as_uses', None)
    return u is not None and u == (_FWD_EPOCH[0], 1) and getattr(p, '_as_one_consumer', False)


def single_consumer_params(root) -> list:
    """The leaf tensors that exactly ONE edge of ``root``'s autograd graph reaches (their AccumulateGrad node has
    one producer of its gradient)."""
    return [t for t, c in _consumer_counts(root).values() if c == 1]


def _consumer_counts(root) -> dict:
    """{id(AccumulateGrad node): (leaf tensor, edges reaching it)} over ``root``'s autograd graph: one iterative
    walk.  Visited nodes are held in ``seen`` (node wrappers are created on access: an id is unique only while its
    object lives)."""
    counts, seen, stack = {}, {}, [root.grad_fn] if root.grad_fn is not None else []
    while stack:
        fn = stack.pop()
        for nxt, _ in fn.next_functions:
            if nxt is None:
                continue
            if type(nxt).__name__ == 'AccumulateGrad':
                k = id(nxt)
                c = counts.get(k)
                counts[k] = (nxt, 1) if c is None else (nxt, c[1] + 1)
            elif id(nxt) not in seen:
                seen[id(nxt)] = nxt
                stack.append(nxt)
    return {k: (node.variable, c) for k, (node, c) in counts.items()}


class _Deferred:
    """Weight gradients of the policy heads, run beside the core LSTM's backward (fp32 step).

    The LSTM backward is three latency-bound recurrences on 8 workgroups per batch row (~1 ms in which ~200
    of the 256 CUs idle); the heads' backward before it is a dX chain whose weight-gradient kernels (the
    location head's gated ResBlocks, gate GEMMs, up-convolutions, head MLPs: a few ms) lie off its critical
    path.  Between :func:`defer_begin` (the trainer, before autograd) and the first LSTM backward, every fp32
    ``_wgrad`` only allocates its result buffer and queues the product (with an event on the stream that
    produced its operands); the LSTM backward launches its recurrence and then :func:`defer_flush` issues the
    queue on a side stream, so the products fill the CUs the recurrence leaves idle.  :func:`defer_end` (the
    trainer, after autograd) makes the main stream wait for them before the gradients are read.  Operands
    and results are held by the queue and recorded on the side stream (the caching allocator never recycles
    them early); autograd cannot accumulate in place into a held tensor.  Not while a HIP graph is captured."""
    on = False
    q = []
    streams = {}
    flushed = None

    issued = []          # (param, dW view): checked against what autograd returns (defer_verify)
    walks = 0            # graph walks so far (single_consumer_params), one per REWALK deferral steps
    steps = 0

    @classmethod
    def add(cls, dy2d, x, cin, has_b, param=None):
        N = dy2d.shape[1]
        K = 9 * cin if cin > 0 else x.shape[1]
        out = torch.empty(N * K + (N if has_b else 0), dtype=torch.float32, device=dy2d.device)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dy2d.device))
        cls.q.append((ev, dy2d, x, cin, has_b, out))
        dw = out[:N * K].view(N, K)
        if param is not None:
            cls.issued.append((param, dw))
        return dw, (out[N * K:] if has_b else None)


# the single-consumer walk (defer_begin) runs on the first deferral step and then every DEFER_REWALK steps (a walk of
# the ~2,000-node graph is ~1-2 ms of host time the GPU would wait for between the loss and the backward); every step
# defer_verify checks what autograd actually returned, so a weight that gained a second consumer in between fails
# loudly instead of receiving a half-written gradient.  APPLESTAR_DEFER_CHECK=1: walk every step.
DEFER_REWALK = 1 if os.environ.get('APPLESTAR_DEFER_CHECK', '0') == '1' else 256


def defer_verify(params, grads) -> None:
    """Every deferred weight gradient must reach the buckets exactly as the native node returned it: autograd adds
    a second consumer's gradient by replacing it (another tensor) or in place (a version bump)."""
    issued, _Deferred.issued = _Deferred.issued, []
    if not issued:
        return
    got = {id(p): g for p, g in zip(params, grads)}
    for p, dw in issued:
        g = got.get(id(p))
        if g is None:
            continue
        if g.data_ptr() != dw.data_ptr() or g._version != dw._version:
            p._as_one_consumer = False
            raise RuntimeError('deferred fp32 weight gradient was accumulated by autograd (a second consumer of the '
                               f'weight {tuple(p.shape)}): run with APPLESTAR_DEFER_WGRAD=0 or APPLESTAR_DEFER_CHECK=1')


def defer_begin(device, loss=None, owner=None) -> None:
    """Start queueing fp32 weight gradients (see :class:`_Deferred`).  ``loss``: the root of the backward about to
    run; only parameters with one consumer in its graph may be deferred (without it nothing is).  ``owner``: the
    object whose steps these are (the trainer): the graph is walked on ITS first step and every DEFER_REWALK-th
    after, so a second trainer in the process (new parameters) is walked on its own first step."""
    if DEFER_WGRAD and torch.device(device).type == 'cuda' and not torch.cuda.is_current_stream_capturing():
        steps = getattr(owner, '_defer_steps', 0) if owner is not None else _Deferred.steps
        if loss is not None and steps % DEFER_REWALK == 0:
            for t, c in _consumer_counts(loss).values():
                t._as_one_consumer = c == 1
            _Deferred.walks += 1
        if owner is not None:
            owner._defer_steps = steps + 1
        _Deferred.steps += 1
        _Deferred.issued = []
        _Deferred.on = True
        _Deferred.q = []
        _Deferred.flushed = None


# side streams the deferred weight gradients are spread over (APPLESTAR_DEFER_STREAMS, default 1): each product goes
# to the stream with the least queued work (rows x N x K plus a per-launch constant).  Measured: 2 streams neutral
# (54.89 / 54.66 vs 54.66 / 54.68 ms), 3 slower (55.24 / 55.25; profiles/r10f_bench_defer_streams.txt) - the
# products already fill the CUs the recurrence leaves idle, and more queues than the box's 4 hardware queues share
DEFER_STREAMS = max(1, int(os.environ.get('APPLESTAR_DEFER_STREAMS', '1')))


def defer_flush() -> None:
    """Issue the queued weight gradients on the side stream(s) (ordered after each operand's producer) and stop
    queueing."""
    if not _Deferred.on:
        return
    _Deferred.on = False
    q, _Deferred.q = _Deferred.q, []
    if not q:
        return
    dev = q[0][1].device
    sides = _Deferred.streams.get(dev)
    if sides is None:
        sides = _Deferred.streams[dev] = [torch.cuda.Stream(device=dev) for _ in range(DEFER_STREAMS)]
    load = [0] * len(sides)
    for ev, dy2d, x, cin, has_b, out in q:
        i = min(range(len(sides)), key=load.__getitem__)
        load[i] += dy2d.shape[0] * out.numel() + (1 << 22)
        side = sides[i]
        with torch.cuda.stream(side):
            side.wait_event(ev)
            for t in (dy2d, x, out):
                t.record_stream(side)
            _C.wgrad_f32(dy2d, x, cin, has_b, out)
    _Deferred.flushed = [s for s, n in zip(sides, load) if n]


def defer_end(device) -> None:
    """Flush anything still queued (no LSTM in this backward) and join the side stream(s)."""
    if _Deferred.on:
        defer_flush()
    sides, _Deferred.flushed = _Deferred.flushed, None
    main = torch.cuda.current_stream(torch.device(device))
    for side in sides or ():
        main.wait_stream(side)
    _FWD_EPOCH[0] += 1          # the next forward counts weight uses afresh


# ---------------------------------------------------------------------------- weight gradients on a side stream
SIDE_WGRAD = os.environ.get('APPLESTAR_SIDE_WGRAD', '0') == '1'     # A/B switch (off: measured slower, r3j)
_SIDE_MIN_ROWS = 1 << 15
_SIDE_STREAMS = {}


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NULL_CTX = _NullCtx()


class _SideWork:
    """Runs a backward node's weight-gradient kernels on a second HIP stream, concurrently with the input-
    gradient kernels that stay on the main stream: the dW (split-R) and dX (implicit GEMM) kernels of a layer
    are independent, and either alone leaves the chip partly idle in its last round of workgroups (a 19x20
    ResBlock conv is 1158 tiles = 1.5 rounds of the ~768 resident workgroups).  ``fork()`` makes the side
    stream wait for the main stream's work so far (the side kernels read tensors the main stream produced);
    ``join(*outs)`` makes the main stream wait for the side kernels and marks their outputs (allocated from
    the side stream's pool) as used on the main stream.  The caller keeps the inputs referenced until the
    join, so the main stream cannot recycle them while the side stream reads.  Only for large products (the
    event hops cost more than the overlap buys on small ones).  Off by default (APPLESTAR_SIDE_WGRAD=1 turns
    it on): measured 87.5 -> 88.7 ms (fp32) and 27.3 -> 29.8 ms (bf16) per learner step on one MI355X
    (profiles/r3j_side_stream_ab.txt) - the two streams contend for the same CUs and the dX chain, which is
    the critical path, slows down more than the tails it fills."""
    __slots__ = ('on', 'main', 'side')

    def __init__(self, ref, rows):
        self.on = SIDE_WGRAD and ref.is_cuda and rows >= _SIDE_MIN_ROWS
        if self.on:
            self.main = torch.cuda.current_stream(ref.device)
            s = _SIDE_STREAMS.get(ref.device)
            if s is None:
                s = _SIDE_STREAMS[ref.device] = torch.cuda.Stream(device=ref.device)
            self.side = s

    def fork(self):
        """Context manager: the enclosed launches go to the side stream, ordered after the main stream's work."""
        if not self.on:
            return _NULL_CTX
        self.side.wait_stream(self.main)
        return torch.cuda.stream(self.side)

    def join(self, *outs):
        if self.on:
            self.main.wait_stream(self.side)
            for t in outs:
                if t is not None:
                    t.record_stream(self.main)
        return outs


# ---------------------------------------------------------------------------- conv3x3 implicit GEMM
class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_nhwc, w_lp, b, res_nhwc, act):
        _count_use(w_lp)
        wk = w_lp.detach().permute(0, 2, 3, 1)          # [Cout,3,3,Cin]: a view for channels_last weights
        if not wk.is_contiguous():
            wk = wk.contiguous()
        bias = _w32(b) if b is not None else None
        out = _conv3(x_nhwc, wk, bias, res_nhwc, _ACT[act], w_lp)
        if act == 'relu' and out.dtype == torch.float32:
            _note_relu_out(out)
        ctx.save_for_backward(x_nhwc, w_lp, out)
        ctx.act, ctx.has_res = act, res_nhwc is not None
        ctx.b_dtype = b.dtype if b is not None else None
        if _DEBUG_PREMASK:
            ctx.site = _fwd_site()
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, out = ctx.saved_tensors
        if ctx.act == 'relu' and _premasked(out, dout):
            dpre = dout.contiguous()                       # the consumer's backward applied the mask
        else:
            if ctx.act == 'relu':
                _premask_miss(ctx, 'conv3x3', out)
            dpre = _act_grad(dout, out, ctx.act == 'relu')    # one pass: mask + cast + NHWC
        has_b = ctx.b_dtype is not None
        cout, cin = w.shape[0], w.shape[1]
        bf = _bf16_grads(w.dtype, ctx.b_dtype)
        side = _SideWork(dpre, dpre.numel() // cout)
        with side.fork():
            dw, db = _wgrad(dpre.view(-1, cout), x, cin, has_b, bf, w)   # dW in [Cout,3,3,Cin] (channels_last) order
            dw = dw.view(cout, 3, 3, cin).permute(0, 3, 1, 2).to(w.dtype)
            db = db.to(ctx.b_dtype) if has_b else None
        dx = _conv3(dpre, _conv_wt(w), None, None, 0, w, True)
        side.join(dw, db)
        return (dx, dw, db, dpre if ctx.has_res else None, None)


def _conv_w(w):
    """[Cout,Cin,3,3] -> [Cout,3,3,Cin] (a view for channels_last weights)."""
    wk = w.detach().permute(0, 2, 3, 1)
    return wk if wk.is_contiguous() else wk.contiguous()


def _conv_wt(w):
    """flipped, transposed weight [Cin,3,3,Cout] for the input gradient (bf16: a derived form rebuilt once per
    optimizer step for parameters; fp32: built per call, a few hundred KB)."""
    if w.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f'native conv3x3 backward needs bf16 or fp32 weights, got {w.dtype}')

    def make():
        s0, s1, s2, s3 = w.stride()
        spec = [w.shape[1], 3, 3, w.shape[0], s1, -s2, -s3, s0, 2 * s2 + 2 * s3]
        if w.dtype == torch.float32:
            return w.detach().flip(2, 3).permute(1, 2, 3, 0).contiguous(), spec
        return _C.conv_wt(w.detach()), spec
    return _derived(w, 'convwt', make)


# ---------------------------------------------------------------------------- derived weight forms
class DerivedWeights:
    """Layout / dtype forms of the compute weights that the kernels consume - fp32 biases and small fp32
    weights, transposed GEMM weights for the dX products, flipped+transposed conv weights - built ONCE per
    optimizer step instead of once per layer per step (~110 cast / transpose launches per RL step).

    Owned by :class:`~applestar_amd.parallel.mixed.MasterWeights`, which tags its parameters with it
    (``p._derived_forms``) and calls :meth:`refresh` after publishing new bf16 weights: one
    ``multi_strided_copy`` launch per 24 forms rebuilds every form in place (the buffers keep their
    addresses).  A form is served only while it matches the owner's weight epoch and the parameter's version
    counter; any other write path (state-dict load, resync) calls :meth:`invalidate`, after which the next
    use rebuilds the form per call, as the uncached path does.  Untagged tensors (casts of fp32 weights,
    activations) are never cached."""

    def __init__(self):
        self.enabled = True
        self.epoch = 0
        self.forms = {}          # (id(param), key) -> [param, out, spec, epoch, version]

    def lookup(self, p, key, make):
        f = self.forms.get((id(p), key))
        if f is not None and f[3] == self.epoch and f[4] == p._version:
            return f[1]
        if f is not None and callable(f[2]):
            f[2](f[1])           # a custom form (e.g. pre-split planes): rebuilt in place by its own kernel
            f[3], f[4] = self.epoch, p._version
            return f[1]
        out, spec = make()
        if spec is None or out.data_ptr() == p.data_ptr():
            return out
        if f is not None and f[1].shape == out.shape and f[1].dtype == out.dtype:
            f[1].copy_(out)      # rebuilt in the form's own buffer: its address may be baked into a HIP graph
            out = f[1]
        self.forms[(id(p), key)] = [p, out, spec, self.epoch, p._version]
        return out

    def invalidate(self):
        self.epoch += 1

    def refresh(self):
        """New weights were published: rebuild every known form in place (same stream as the writer)."""
        self.epoch += 1
        if not (self.enabled and self.forms):
            return
        fs = [f for f in self.forms.values() if not callable(f[2])]
        spec = []
        for f in fs:
            spec += f[2]
        if fs:
            ensure_loaded().multi_strided_copy([f[1] for f in fs], [f[0].detach() for f in fs], spec)
        for f in fs:                # current before the pre-split rebuilds read them (a conv's transposed form)
            f[3], f[4] = self.epoch, f[0]._version
        # pre-split weight planes: every form in one batched launch (multi_presplit); other custom forms one by one
        ps = [f for f in self.forms.values() if callable(f[2]) and getattr(f[2], 'psb_src', None) is not None]
        if ps:
            ensure_loaded().multi_presplit([f[2].psb_src() for f in ps], [f[2].psb_trans for f in ps],
                                           [f[1] for f in ps])
        for f in self.forms.values():
            if callable(f[2]) and getattr(f[2], 'psb_src', None) is None:
                f[2](f[1])
        for f in self.forms.values():
            f[3], f[4] = self.epoch, f[0]._version


def _derived(p, key, make):
    reg = getattr(p, '_derived_forms', None) if isinstance(p, torch.nn.Parameter) else None
    if reg is None or not reg.enabled or not p.is_cuda:
        return make()[0]
    return reg.lookup(p, key, make)


def _view_spec(view, src):
    """multi_strided_copy spec of a strided view of ``src`` (<= 4 dims, element units)."""
    if view.dim() > 4:
        return None
    pad = 4 - view.dim()
    return [1] * pad + list(view.shape) + [0] * pad + list(view.stride()) + \
        [view.storage_offset() - src.storage_offset()]


# fp32 GEMMs on pre-split weight planes (gemm_f32_psb.hip: the weight split once per optimizer step into MFMA
# fragment-order bf16 planes instead of in every wave of every M-tile); APPLESTAR_GEMM_PSB=0: the split ring GEMM
GEMM_PSB = os.environ.get('APPLESTAR_GEMM_PSB', '1') == '1'
GEMM_PSB_VARIANT = int(os.environ.get('APPLESTAR_GEMM_PSB_VARIANT', '1'))


def _psb_ok(M, N, K):
    """The pre-split GEMM replaces the split ring kernel (tile-count rule of gemm_f32; few-row products keep the
    small-tile kernel): N % 128, K % 4."""
    return GEMM_PSB and (M + 127) // 128 * ((N + 63) // 64) >= 128 and _C.gemm_f32_psb_supported(M, N, K)


def _psb(w, transposed=False):
    """Pre-split planes of the GEMM B operand: w [N, K] itself, or (transposed) w^T [K_in, N_out] for the dX
    product; a derived form of a parameter (rebuilt in place by presplit_b after each optimizer step)."""
    def src():
        t = w.detach().reshape(w.shape[0], -1)
        return t if t.is_contiguous() else t.contiguous()

    def build(into=None):
        return _C.presplit_b(src(), transposed, into)
    build.psb_src, build.psb_trans = src, transposed        # DerivedWeights.refresh batches these rebuilds
    return _derived(w, 'psbT' if transposed else 'psb', lambda: (build(), build))


CONV_PSB = os.environ.get('APPLESTAR_CONV_PSB', '1') == '1'


def _psb_conv(w, dx=False):
    """Pre-split planes of a 3x3 conv's weight operand: [Cout, 3, 3, Cin] (forward) or the flipped transpose
    [Cin, 3, 3, Cout] (input gradient, built from the _conv_wt form); a derived form of the parameter."""
    def src():
        wk = _conv_wt(w) if dx else _conv_w(w)
        wk = wk.reshape(wk.shape[0], -1)
        return wk if wk.is_contiguous() else wk.contiguous()

    def build(into=None):
        return _C.presplit_b(src(), False, into)
    build.psb_src, build.psb_trans = src, False             # DerivedWeights.refresh batches these rebuilds
    return _derived(w, 'psbcT' if dx else 'psbc', lambda: (build(), build))


def _w32(t):
    """t as a contiguous fp32 tensor (a bias, a small weight); a derived form for parameters."""
    if t.dtype == torch.float32 and t.is_contiguous():
        return t.detach()
    return _derived(t, 'f32', lambda: (t.detach().float().contiguous(), _view_spec(t.detach(), t)))


def _wT(t, dtype=None):
    """t viewed as [shape0, -1], transposed, contiguous, in ``dtype`` (default t's); a derived form for
    parameters."""
    dtype = dtype or t.dtype

    def make():
        v = t.detach().reshape(t.shape[0], -1).t()
        out = v.to(dtype).contiguous() if dtype != t.dtype else v.contiguous()
        try:
            spec = _view_spec(t.detach().view(t.shape[0], -1).t(), t)
        except RuntimeError:          # not viewable as 2-D: keep the per-call copy
            spec = None
        return out, spec
    return _derived(t, ('T', dtype), make)


FUSED_DRELU = os.environ.get('APPLESTAR_CONV_DRELU', '1') != '0'   # A/B switch


def _conv_dx_drelu(dpre, w, y):
    """Input gradient of a 3x3 conv whose input y is a ReLU output, already gated by (y > 0): the gate
    is the dX conv's epilogue mode 4 (no separate read-modify-write pass over the activation)."""
    if FUSED_DRELU:
        return _conv3(dpre, _conv_wt(w), None, y, 4, w, True)
    return _act_grad(_conv3(dpre, _conv_wt(w), None, None, 0, w, True), y, True)


def _conv_dw(dpre, x, w, b_dtype):
    """dW (in w's dtype) and db of a 3x3 conv; callers cast db to b_dtype (a no-op when both are bf16:
    the cast is then fused into the split reduction)."""
    cout, cin = w.shape[0], w.shape[1]
    dw, db = _wgrad(dpre.view(-1, cout), x, cin, b_dtype is not None, _bf16_grads(w.dtype, b_dtype), w)
    return dw.view(cout, 3, 3, cin).permute(0, 3, 1, 2).to(w.dtype), db


class SkipLink:
    """Hands the location head's gradient of an encoder skip map (``model._TakeRows``: the first T*B rows of a
    ResBlock input) to the backward of the ResBlock that consumes the map, which adds it in its dX conv's
    epilogue (``conv3x3_f32_epi2``: + res2 on the first rows) - together with the ReLU mask of the map (the
    previous layer's ReLU): the map then receives ONE gradient, already masked, instead of a full-height
    copy + tail fill (_TakeRows), an autograd add of the two gradients and a threshold pass (~120 us per
    19x20x128 level, four levels per fp32 step).  The link rides on the map tensor object itself
    (``x._skip_link``, set when the ResBlock is called on it), so it can never be picked up by another tensor.
    Autograd runs the location head's backward (which consumes the heads' outputs) before any encoder
    ResBlock's (the encoder feeds the heads), so the hand-off is normally ordered.  The order is not relied on:
    the ResBlock's backward marks the link ``consumed``, and a ``_TakeRows`` backward that finds it consumed
    returns its full-height gradient through autograd instead (an ordinary add; the map's producer then sees an
    unmasked gradient and applies its own ReLU mask), so a late hand-over is never dropped."""
    __slots__ = ('g', 'consumed')

    def __init__(self):
        self.g = None
        self.consumed = False


SKIP_LINK = os.environ.get('APPLESTAR_SKIP_LINK', '1') == '1'    # A/B switch
# the location head's skip-map adds in the gated residual blocks' output pass (APPLESTAR_POST_ADD=0: separate adds)
POST_ADD = os.environ.get('APPLESTAR_POST_ADD', '1') == '1'
# the scalar encoder's three concatenations in one launch (APPLESTAR_COL_ASSEMBLE=0: torch.cat + autograd adds)
COL_ASSEMBLE = os.environ.get('APPLESTAR_COL_ASSEMBLE', '1') == '1'


class _ResBlock(torch.autograd.Function):
    """relu(conv2(relu(conv1(x))) + x) (res_block.py:50-65) as ONE autograd node: the input gradient of
    conv1 and the skip gradient are summed in the dX conv's epilogue (the residual input of the same MFMA
    kernel) instead of a separate autograd add over the whole activation.  fp32: the output is registered as
    a ReLU output (its consumer may apply the mask, _premasked), and the input gradient takes the location
    head's hand-over (SkipLink) and the input's own ReLU mask in the same epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, link=None):
        _count_use(w1)
        _count_use(w2)
        y1 = _conv3(x, _conv_w(w1), _w32(b1), None, 1, w1)
        out = _conv3(y1, _conv_w(w2), _w32(b2), x, 1, w2)
        ctx.save_for_backward(x, w1, w2, y1, out)
        ctx.b_dtypes = (b1.dtype, b2.dtype)
        ctx.link = link
        ctx.mask_in = False
        if out.dtype == torch.float32 and SKIP_LINK:
            _note_relu_out(out)
            ctx.mask_in = _relu_src(x)
        if _DEBUG_PREMASK:
            ctx.site = _fwd_site()
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w1, w2, y1, out = ctx.saved_tensors
        if out.dtype == torch.float32 and _premasked(out, dout):
            dpre2 = dout.contiguous()           # the consumer's dX epilogue already applied this block's ReLU
        else:
            _premask_miss(ctx, 'resblock', out)
            dpre2 = _act_grad(dout, out, True)
        side = _SideWork(dpre2, dpre2.numel() // dpre2.shape[-1])
        with side.fork():       # weight gradients concurrent with the dX convs
            dw2, db2 = _conv_dw(dpre2, y1, w2, ctx.b_dtypes[1])
            db2 = db2.to(ctx.b_dtypes[1])
        dpre1 = _conv_dx_drelu(dpre2, w2, y1)
        with side.fork():
            dw1, db1 = _conv_dw(dpre1, x, w1, ctx.b_dtypes[0])
            db1 = db1.to(ctx.b_dtypes[0])
        g = None
        if ctx.link is not None:
            g, ctx.link.g = ctx.link.g, None
            ctx.link.consumed = True          # a later _TakeRows backward takes the autograd path (SkipLink)
        C = x.shape[-1]
        if x.dtype == torch.float32 and (g is not None or ctx.mask_in) and _C.conv3x3_f32_epi2_supported(C, C):
            # + skip gradient + the location head's hand-over (first rows), masked by this input's own ReLU
            dx = _conv3(dpre1, _conv_wt(w1), None, dpre2, 0, w1, True, g, x if ctx.mask_in else None)
            if ctx.mask_in:
                _MASKED_DX[x.data_ptr()] = (dx, dx._version)
        else:
            dx = _conv3(dpre1, _conv_wt(w1), None, dpre2, 0, w1, True)       # + skip gradient, fused
            if g is not None:
                dx[:g.shape[0]] += g
        side.join(dw1, db1, dw2, db2)
        return dx, dw1, db1, dw2, db2, None


def _f32_conv_ok(x, w, cin, cout):
    """fp32 step (fp32 operands, no autocast) and a shape the f32-MFMA conv takes in both directions."""
    return x.dtype == torch.float32 and w.dtype == torch.float32 and not torch.is_autocast_enabled() and \
        _C.conv3x3_f32_supported(cin, cout) and _C.conv3x3_f32_supported(cout, cin)


def resblock(x, w1, b1, w2, b2):
    """Native fused ResBlock; None when the shapes / dtypes are not covered (caller falls back)."""
    C = x.shape[1]
    if x.dim() != 4 or b1 is None or b2 is None or tuple(w1.shape) != (C, C, 3, 3) or tuple(w2.shape) != (C, C, 3, 3):
        return None
    if _f32_conv_ok(x, w1, C, C):
        link = None
        if SKIP_LINK and x.is_cuda and _C.conv3x3_f32_epi2_supported(C, C):
            link = SkipLink()
            x._skip_link = link          # read by the location head's row view of this map (model._take_rows)
        return from_nhwc(_ResBlock.apply(nhwc(x), w1, b1, w2, b2, link))
    lowp = x.dtype == torch.bfloat16 or torch.is_autocast_enabled()
    if not lowp or not _C.conv3x3_supported(C, C):
        return None
    xl = nhwc(x.to(torch.bfloat16))
    w1l = w1 if w1.dtype == torch.bfloat16 else _bf16w(w1)
    w2l = w2 if w2.dtype == torch.bfloat16 else _bf16w(w2)
    with torch.autocast('cuda', enabled=False):
        return from_nhwc(_ResBlock.apply(xl, w1l, b1, w2l, b2))


GATE_CHAIN = os.environ.get('APPLESTAR_GATE_CHAIN', '1') == '1'
# the fp32 step's gate chain in one launch per direction (gate_chain.hip gate_chain_f32_kernel): measured equal to the
# four f32 GEMMs on the step (profiles/r4z_gate_chain_f32.txt), off by default
GATE_CHAIN_F32 = os.environ.get('APPLESTAR_GATE_CHAIN_F32', '0') == '1'
GATE_PSB = os.environ.get('APPLESTAR_GATE_PSB', '1') == '1'       # A/B: the fp32 gate GEMMs on pre-split planes
# the fp32 gate chain (four K = 128 GEMMs: pipeline-bound, ~70 us each) on its own stream beside the conv branch, forward
# and backward: neutral (51.18 / 51.23 / 51.12 vs 51.16 / 51.17 / 51.19 ms, profiles/r10x_bench_gate_side.txt - the convs
# already fill the chip); off, APPLESTAR_GATE_SIDE=1 turns it on
GATE_SIDE = os.environ.get('APPLESTAR_GATE_SIDE', '0') == '1'
_GATE_STREAMS = {}


class _GateSide:
    """Run a block of launches on the gated blocks' side stream (ordered after the main stream's work so far) and join:
    ``with g.run(): ...`` then ``g.join(*outs)`` makes the main stream wait and marks the outputs as used there."""

    def __init__(self, ref, on):
        self.on = on and ref.is_cuda and not torch.cuda.is_current_stream_capturing()
        if self.on:
            self.main = torch.cuda.current_stream(ref.device)
            key = ref.device.index
            if key not in _GATE_STREAMS:
                _GATE_STREAMS[key] = torch.cuda.Stream(ref.device)
            self.side = _GATE_STREAMS[key]

    def run(self, *inputs):
        if not self.on:
            return _NULL_CTX
        self.side.wait_stream(self.main)
        for t in inputs:
            if t is not None:
                t.record_stream(self.side)
        return torch.cuda.stream(self.side)

    def join(self, *outs):
        if self.on:
            self.main.wait_stream(self.side)
            for t in outs:
                if t is not None:
                    t.record_stream(self.main)


class _GatedResBlock(torch.autograd.Function):
    """Location-head GatedResBlock (module_utils.py:204-231) as one autograd node on NHWC bf16:

        y = conv2(relu(conv1(x)));  g = G4(relu(G3(relu(G2(relu(G1(x)))))))   (G* = 1x1 convs = GEMMs)
        out = relu(tanh(y * sigmoid(g)) * sp + x)

    x feeds three consumers (conv1, G1, the skip); their input gradients are accumulated inside
    kernels that run anyway: the G1 dX GEMM adds the skip gradient (addmm), and the conv1 dX kernel adds
    that sum in its epilogue - no separate whole-activation adds."""

    @staticmethod
    def forward(ctx, x, sp, post, w1, b1, w2, b2, *gate):
        for p in (w1, w2, *gate[0::2]):
            _count_use(p)
        B, H, W, C = x.shape
        h = x.view(-1, C)
        acts = [h]
        gate_join = None
        gate_first = GATE_SIDE and x.dtype == torch.float32 and x.is_cuda and not GATE_CHAIN_F32
        if not gate_first:
            y1 = _conv3(x, _conv_w(w1), _w32(b1), None, 1, w1)
            y = _conv3(y1, _conv_w(w2), _w32(b2), None, 0, w2)
        if GATE_CHAIN and C == 128 and x.dtype == torch.bfloat16:
            # the four gate layers in one launch, activation tile resident in LDS (gate_chain.hip)
            acts += _C.gate_chain(h, [gate[2 * i].detach().view(C, C) for i in range(4)],
                                  [_w32(gate[2 * i + 1]) for i in range(4)],
                                  [None] * 4, [None] * 4, 0b0111)
            h = acts[-1]
        elif GATE_CHAIN_F32 and C == 128 and x.dtype == torch.float32 and h.shape[0] * C < 2 ** 31:
            # fp32 step: the four gate layers in one launch, the split activation tile resident in LDS
            acts += _C.gate_chain_f32(h, [gate[2 * i].detach().view(C, C) for i in range(4)],
                                      [_w32(gate[2 * i + 1]) for i in range(4)], [None] * 4, [None] * 4, 0b0111)
            h = acts[-1]
        elif x.dtype == torch.float32 and _gemm_f32_ok(h.shape[0], C, C):
            # fp32 step: the four gate layers on the f32 GEMM with bias (+ ReLU) in the epilogue - on the gate stream,
            # beside the two 3x3 convs above (independent branches of the block)
            psb = GATE_PSB and _psb_ok(h.shape[0], C, C)     # the pre-split weight planes (gemm_f32_psb.hip)
            pw = [_psb(gate[2 * i]) if psb else gate[2 * i].detach().view(C, C) for i in range(4)]   # (main stream)
            pb = [_w32(gate[2 * i + 1]) for i in range(4)]
            gs = _GateSide(x, GATE_SIDE)
            with gs.run(x):
                for i in range(4):
                    act = 1 if i < 3 else 0
                    h = _C.gemm_f32_psb(h, pw[i], C, C, pb[i], None, act, GEMM_PSB_VARIANT) if psb \
                        else _C.gemm_f32(h, pw[i], pb[i], None, act)
                    acts.append(h)
            gate_join = gs      # joined after the convs are issued (a join here would order them behind the chain)
        else:
            for i in range(4):
                gw, gb = gate[2 * i].detach().view(C, C), gate[2 * i + 1].detach()
                R = h.shape[0]
                if _bf16_small_ok(h, R, C, C) or _bf16_pipe_ok(h, R, C, C):
                    # the per-op path's kernels (_Linear): fp32 bias in the epilogue, so both paths agree bit for bit
                    fn = _C.gemm_bf16_small if _bf16_small_ok(h, R, C, C) else _C.gemm_bf16
                    h = fn(h, gw.contiguous(), _w32(gb), None, 1 if i < 3 else 0)
                else:
                    gb = gb.to(h.dtype)
                    h = torch._addmm_activation(gb, h, gw.t(), use_gelu=False) if i < 3 else torch.addmm(gb, h, gw.t())
                acts.append(h)
        if gate_first:
            # the convs after the gate chain's issue: the gate stream waited only for x's producer, so its GEMMs run
            # beside these
            y1 = _conv3(x, _conv_w(w1), _w32(b1), None, 1, w1)
            y = _conv3(y1, _conv_w(w2), _w32(b2), None, 0, w2)
        if gate_join is not None:
            gate_join.join(*acts[1:])
        # post: the next encoder skip map, added to the block output in the same pass (LocationHead)
        out = _C.gated_residual_fwd(y, h.view(B, H, W, C), sp, x, post)
        ctx.save_for_backward(x, sp, w1, w2, y1, y, out if post is None else None, *acts[1:], *gate[0::2])
        ctx.dtypes = (b1.dtype, b2.dtype, gate[1].dtype)
        ctx.has_post = post is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, sp, w1, w2, y1, y, out, a1, a2, a3, g, gw1, gw2, gw3, gw4 = ctx.saved_tensors
        B, H, W, C = x.shape
        dout = dout.contiguous().to(y.dtype)
        # with a post-add the saved output is not the ReLU output: the mask is recomputed from the block input
        dy, dg, dx_res, dsp = _C.gated_residual_bwd(dout, y, g.view(B, H, W, C), sp, out,
                                                    x if ctx.has_post else None)
        # gate chain (1x1 convs as GEMMs over the pixels)
        grads_g = []
        gate_bwd = None
        d = dg.view(-1, C)
        acts_in = [x.view(-1, C), a1, a2, a3]
        gws = [gw1, gw2, gw3, gw4]
        if GATE_CHAIN and C == 128 and x.dtype == torch.bfloat16:
            # d3, d2, d1 and the gate-path input gradient (+ the skip gradient) in one launch; the weight
            # gradients from the saved layer inputs and these
            d3, d2, d1, dx_gate = _C.gate_chain(d, [_wT(gws[i]) for i in (3, 2, 1, 0)],
                                                [None] * 4, [a3, a2, a1, None], [None, None, None, dx_res.view(-1, C)],
                                                0)
            for i, di in ((3, d), (2, d3), (1, d2), (0, d1)):
                dw_i, db_i = _wgrad(di, acts_in[i], 0, True, _bf16_grads(gws[i].dtype, ctx.dtypes[2]))
                grads_g.append((i, dw_i.view_as(gws[i]).to(gws[i].dtype), db_i.to(ctx.dtypes[2])))
        elif GATE_CHAIN_F32 and C == 128 and x.dtype == torch.float32 and d.shape[0] * C < 2 ** 31:
            # fp32 step: d3, d2, d1 and the gate-path input gradient (+ the skip gradient) in one launch
            d3, d2, d1, dx_gate = _C.gate_chain_f32(d.contiguous(), [_wT(gws[i]) for i in (3, 2, 1, 0)], [None] * 4,
                                                    [a3, a2, a1, None],
                                                    [None, None, None, dx_res.view(-1, C).contiguous()], 0)
            for i, di in ((3, d), (2, d3), (1, d2), (0, d1)):
                dw_i, db_i = _wgrad(di, acts_in[i], 0, True, False)
                grads_g.append((i, dw_i.view_as(gws[i]).to(gws[i].dtype), db_i.to(ctx.dtypes[2])))
        elif x.dtype == torch.float32 and _gemm_f32_ok(d.shape[0], C, C):
            # fp32 step: each input gradient on the f32 GEMM with the previous layer's ReLU mask (ACT_DRELU on its
            # saved output) or the skip gradient in the epilogue - no threshold_backward / addmm passes
            psb = GATE_PSB and _psb_ok(d.shape[0], C, C)
            pwt = [_psb(gws[i], True) if psb else _wT(gws[i]) for i in range(4)]      # (main stream)

            def dgemm(d, i, r, mode):
                return _C.gemm_f32_psb(d, pwt[i], C, C, None, r, mode, GEMM_PSB_VARIANT) if psb \
                    else _C.gemm_f32(d, pwt[i], None, r, mode)
            # the gate chain's backward on the gate stream, beside the conv branch's dX below; joined before the
            # conv1 dX kernel that adds dx_gate in its epilogue
            gate_bwd = _GateSide(x, GATE_SIDE)
            dxr = dx_res.view(-1, C).contiguous()
            with gate_bwd.run(d, dxr, *acts_in):
                for i in (3, 2, 1, 0):
                    dw_i, db_i = _wgrad(d, acts_in[i], 0, True, False, gws[i])
                    grads_g.append((i, dw_i.view_as(gws[i]).to(gws[i].dtype), db_i.to(ctx.dtypes[2])))
                    if i > 0:
                        d = dgemm(d, i, acts_in[i], 4)
                dx_gate = dgemm(d, 0, dxr, 0)
        else:
            for i in (3, 2, 1, 0):
                dw_i, db_i = _wgrad(d, acts_in[i], 0, True, _bf16_grads(gws[i].dtype, ctx.dtypes[2]))
                grads_g.append((i, dw_i.view_as(gws[i]).to(gws[i].dtype), db_i.to(ctx.dtypes[2])))
                if i > 0:
                    dh = torch.mm(d, gws[i].view(C, C))
                    P = dh.shape[0]
                    d = _act_grad(dh.view(1, 1, P, C), acts_in[i].view(1, 1, P, C), True).view(P, C)
            dx_gate = torch.addmm(dx_res.view(-1, C), d, gw1.view(C, C))      # skip + G1 input gradients
        # conv path: its weight gradients on the side stream, concurrent with the dX convs
        side = _SideWork(dy, B * H * W)
        with side.fork():
            dw2, db2 = _conv_dw(dy, y1, w2, ctx.dtypes[1])
            db2 = db2.to(ctx.dtypes[1])
        dpre1 = _conv_dx_drelu(dy, w2, y1)
        with side.fork():
            dw1, db1 = _conv_dw(dpre1, x, w1, ctx.dtypes[0])
            db1 = db1.to(ctx.dtypes[0])
        if gate_bwd is not None:
            gate_bwd.join(dx_gate, *[t for _, dw_i, db_i in grads_g for t in (dw_i, db_i)])
        dx = _conv3(dpre1, _conv_wt(w1), None, dx_gate.view(B, H, W, C).contiguous(), 0, w1, True)
        side.join(dw1, db1, dw2, db2)
        gate_grads = [None] * 8
        for i, dw_i, db_i in grads_g:
            gate_grads[2 * i], gate_grads[2 * i + 1] = dw_i, db_i
        return (dx, dsp.to(sp.dtype), dout if ctx.has_post else None, dw1, db1, dw2, db2, *gate_grads)


def gated_resblock(x, conv1, conv2, gates, sp, post=None):
    """Fused GatedResBlock (see _GatedResBlock); None when not covered (caller falls back).  ``post``: a tensor of
    x's shape added to the block output in the same pass (None when it cannot be: the caller adds it)."""
    C = x.shape[1]
    ws = [conv1.weight, conv1.bias, conv2.weight, conv2.bias]
    for gc in gates:
        ws += [gc.weight, gc.bias]
    if x.dim() != 4 or any(t is None for t in ws) or C % 8:
        return None
    if post is not None and (post.shape != x.shape or not post.is_contiguous(memory_format=torch.channels_last)
                             or not POST_ADD):
        return None
    if _f32_conv_ok(x, conv1.weight, C, C) and all(t.dtype == torch.float32 for t in ws) and \
            (post is None or post.dtype == torch.float32):
        return from_nhwc(_GatedResBlock.apply(nhwc(x), sp.float(), None if post is None else nhwc(post), *ws))
    lowp = x.dtype == torch.bfloat16 or torch.is_autocast_enabled()
    if not lowp or not _C.conv3x3_supported(C, C):
        return None
    # conv / GEMM weights and the GEMM biases in bf16 (the per-op path's casts); the conv biases stay as
    # given: the conv epilogue adds them in fp32
    # (with the one-launch bf16 gate chain the gate biases stay fp32 too: it reads them as fp32)
    # (the four-GEMM gate path keeps them fp32 as well: its native GEMMs add an fp32 bias, as the per-op path's do)
    keep = {1, 3, 5, 7, 9, 11}
    ws = [t if (t.dtype == torch.bfloat16 or i in keep) else _bf16w(t) for i, t in enumerate(ws)]
    xl = nhwc(x.to(torch.bfloat16))
    pl = None if post is None else nhwc(post.to(torch.bfloat16))
    with torch.autocast('cuda', enabled=False):
        return from_nhwc(_GatedResBlock.apply(xl, sp.float(), pl, *ws))


def _bf16w(w):
    """bf16 compute form of an fp32 weight / bias (autocast semantics).  With autograd: a _CastWeight node (fp32
    gradient).  Without (actor inference, frozen teachers): a derived form of the parameter, cast once and
    reused until its weights change - the inference server tags its models' parameters
    (:func:`attach_inference_forms`) and refreshes the forms in place after every weight update, so the HIP graphs
    that captured a form's buffer read the new values; untagged tensors are cast per call."""
    if torch.is_grad_enabled() and w.requires_grad:
        return _CastWeight.apply(w)
    if w.dim() == 4 and not w.is_contiguous() and w.is_contiguous(memory_format=torch.channels_last):
        # a channels_last conv weight: the form keeps that layout ([Cout, kh, kw, Cin] storage, what the conv
        # kernels read through _conv_w without a copy); returned as the NCHW-logical view of it
        src = w.detach().permute(0, 2, 3, 1)
        f = _derived(w, 'bf16_cl', lambda: (src.to(torch.bfloat16).contiguous(), _view_spec(src, w)))
        return f.permute(0, 3, 1, 2)
    return _derived(w, 'bf16', lambda: (w.detach().to(torch.bfloat16).contiguous(), _view_spec(w.detach(), w)
                                        if w.is_contiguous() else None))


def attach_inference_forms(model):
    """Tag ``model``'s parameters with one DerivedWeights registry (bf16 / fp32 / transposed forms cached across
    inference calls); returns it - call ``.refresh()`` after loading new weights into the model."""
    reg = DerivedWeights()
    for p in model.parameters():
        p._derived_forms = reg
    return reg


class _CastWeight(torch.autograd.Function):
    """bf16 view of an fp32 weight for the native conv (autocast semantics) with an fp32 gradient."""

    @staticmethod
    def forward(ctx, w):
        return w.detach().to(torch.bfloat16)

    @staticmethod
    def backward(ctx, g):
        return g.float()


def conv2d(x, w, b, stride, padding, act, residual):
    """Native convolution paths; returns None when the call should go to MIOpen.

    * 3x3 / stride 1 / pad 1 with Cin, Cout multiples of 32: MFMA implicit GEMM (bf16, under autocast
      or with bf16 inputs) with bias / residual / ReLU fused;
    * 1x1 / stride 1 / pad 0: a GEMM over the NHWC pixels (hipBLASLt, bias fused) - no transposes."""
    if x.dim() != 4 or stride != 1:
        return None
    kh, kw = w.shape[2], w.shape[3]
    cout, cin = w.shape[0], w.shape[1]
    lowp = x.dtype == torch.bfloat16 or torch.is_autocast_enabled()
    if kh == 3 and kw == 3 and padding == 1 and _f32_conv_ok(x, w, cin, cout) and \
            (residual is None or residual.dtype == torch.float32):
        rl = nhwc(residual) if residual is not None else None
        return from_nhwc(_Conv3x3.apply(nhwc(x), w, b, rl, act))
    if kh == 3 and kw == 3 and padding == 1 and lowp and _C.conv3x3_supported(cin, cout) \
            and _C.conv3x3_supported(cout, cin):
        xl = nhwc(x.to(torch.bfloat16))
        wl = w if w.dtype == torch.bfloat16 else _bf16w(w)
        rl = nhwc(residual.to(torch.bfloat16)) if residual is not None else None
        with torch.autocast('cuda', enabled=False):
            return from_nhwc(_Conv3x3.apply(xl, wl, b, rl, act))
    if kh == 1 and kw == 1 and padding == 0:
        B, _, H, W = x.shape
        if residual is None and lowp and act in (None, 'relu') and _C.pointwise_supported(cin, cout):
            xl = nhwc(x.to(torch.bfloat16)).view(-1, cin)
            with torch.autocast('cuda', enabled=False):
                y = _Pointwise.apply(xl, w.view(cout, cin), b, act == 'relu')
            return from_nhwc(y.view(B, H, W, cout))
        if residual is None:
            y = linear(nhwc(x).view(-1, cin), w.view(cout, cin), b, act)
        else:
            y = linear(nhwc(x).view(-1, cin), w.view(cout, cin), b) + nhwc(residual).view(-1, cout)
            if act is not None:
                from . import reference
                y = reference.act_fn(y, act)
        return from_nhwc(y.view(B, H, W, cout))
    return None


# ---------------------------------------------------------------------------- value spatial input (value_spatial.hip)
VSP_FUSED = os.environ.get('APPLESTAR_VSP_FUSED', '1') == '1'
VSP_POOL_FUSED = os.environ.get('APPLESTAR_VSP_POOL_FUSED', '1') == '1'


class _ValueSpatialProj(torch.autograd.Function):
    """relu(conv1x1(cat([scatter map (8 ch), own, enemy]))) of the value encoder over the 9.5M-pixel map
    without building the 10-channel input (value_spatial.hip); backward is one pass for the ReLU mask, the
    scatter map's gradient and dW / db."""

    @staticmethod
    def forward(ctx, sc2d, own, enemy, w2, b):
        wf, bf = w2.detach().float().contiguous(), b.detach().float().contiguous()
        out = _C.vsp_fwd(sc2d, own, enemy, wf, bf)
        ctx.save_for_backward(sc2d, own, enemy, wf, out)
        ctx.dtypes = (w2.dtype, b.dtype)
        return out

    @staticmethod
    def backward(ctx, dout):
        sc2d, own, enemy, wf, out = ctx.saved_tensors
        dsc, dwb = _C.vsp_bwd(dout.to(sc2d.dtype).contiguous(), out, sc2d, own, enemy, wf)
        w_dtype, b_dtype = ctx.dtypes
        return dsc, None, None, dwb[:, :-1].to(w_dtype), dwb[:, -1].to(b_dtype)


class _ValueSpatialProjPool(torch.autograd.Function):
    """max_pool2x2(relu(conv1x1(cat([scatter map, own, enemy])))) in one pass per pooled pixel
    (value_spatial.hip vsp_pool_*): neither the 16-channel full-resolution map nor its pool gradient is built."""

    @staticmethod
    def forward(ctx, sc2d, own, enemy, w2, b, B, H, W):
        wf, bf = w2.detach().float().contiguous(), b.detach().float().contiguous()
        pooled, pos = _C.vsp_pool_fwd(sc2d, own, enemy, wf, bf, B, H, W)
        ctx.save_for_backward(sc2d, own, enemy, wf, pooled, pos)
        ctx.meta = (w2.dtype, b.dtype, B, H, W)
        return pooled

    @staticmethod
    def backward(ctx, dpooled):
        sc2d, own, enemy, wf, pooled, pos = ctx.saved_tensors
        w_dtype, b_dtype, B, H, W = ctx.meta
        dsc, dwb = _C.vsp_pool_bwd(dpooled.to(sc2d.dtype).contiguous(), pos, pooled, sc2d, own, enemy, wf, B, H, W)
        return dsc, None, None, dwb[:, :-1].to(w_dtype), dwb[:, -1].to(b_dtype), None, None, None


def value_spatial_proj_pool(sc, own, enemy, w, b):
    """max_pool2x2 of :func:`value_spatial_proj` as a channels_last [B, 16, H/2, W/2] view (even H, W);
    None when it does not apply."""
    if not (VSP_FUSED and VSP_POOL_FUSED):
        return None
    B, C, H, W = sc.shape
    cout, cin = w.shape[0], w.shape[1]
    if H % 2 or W % 2 or cout != _C.vsp_out_channels() or cin != _C.vsp_in_channels() or C != cin - 2 or b is None \
            or own.dtype != torch.bool or enemy.dtype != torch.bool or own.numel() != B * H * W \
            or enemy.numel() != B * H * W:
        return None
    # bf16 maps under autocast; the fp32 step keeps fp32 maps (the kernel's math is fp32 FMA either way)
    sc2d = nhwc(sc.to(torch.bfloat16) if _lowp(sc) else sc.float()).view(-1, C)
    with torch.autocast('cuda', enabled=False):
        y = _ValueSpatialProjPool.apply(sc2d, own.reshape(-1).view(torch.uint8), enemy.reshape(-1).view(torch.uint8),
                                        w.view(cout, cin), b, B, H, W)
    return from_nhwc(y.view(B, H // 2, W // 2, cout))


def value_spatial_proj(sc, own, enemy, w, b):
    """sc [B, 8, H, W] (NHWC-contiguous scatter map), own / enemy [B, 1, H, W] bool, 1x1 conv weight
    [16, 10, 1, 1] + bias -> relu(conv(cat([sc, own, enemy]))) as a channels_last [B, 16, H, W] view;
    None when the shapes are not the kernel's."""
    if not VSP_FUSED:
        return None
    B, C, H, W = sc.shape
    cout, cin = w.shape[0], w.shape[1]
    if cout != _C.vsp_out_channels() or cin != _C.vsp_in_channels() or C != cin - 2 or b is None \
            or own.dtype != torch.bool or enemy.dtype != torch.bool or own.numel() != B * H * W \
            or enemy.numel() != B * H * W:
        return None
    sc2d = nhwc(sc.to(torch.bfloat16) if _lowp(sc) else sc.float()).view(-1, C)
    with torch.autocast('cuda', enabled=False):
        y = _ValueSpatialProj.apply(sc2d, own.reshape(-1).view(torch.uint8), enemy.reshape(-1).view(torch.uint8),
                                    w.view(cout, cin), b)
    return from_nhwc(y.view(B, H, W, cout))


# ---------------------------------------------------------------------------- location-head input (locin.hip)
LOC_FUSED = os.environ.get('APPLESTAR_LOC_FUSED', '1') == '1'


class _LocationInput(torch.autograd.Function):
    """relu(conv1x1(relu(cat([p, skip], 1)))) of the location head without the concat: y0 = skip W_s^T + b
    as a K = 128 library GEMM, then the rank-4 term W_p relu(p) + ReLU per pixel in one pass (locin.hip),
    reading p in the fc output's [B, 4*HW] layout.  Backward: one pass for the ReLU mask, dP and the
    128 x 4 dW_p; dSkip on the library, dW_s / db on the split-R MFMA wgrad.  The cat-based path wrote the
    38 MB concat (0.25 ms on channels_last), ran the K = 132 GEMMs and a ReLU pass each way."""

    @staticmethod
    def forward(ctx, pf, skip2d, w2, b, HW):
        C, CP = w2.shape
        ws = w2[:, CP - C:].contiguous()
        wp = w2[:, :CP - C].float().contiguous()
        y0 = torch.addmm(b.to(skip2d.dtype), skip2d, ws.t())
        y = _C.loc_in_fwd(y0, pf, wp, HW)
        ctx.save_for_backward(pf, skip2d, ws, wp, y)
        ctx.meta = (HW, w2.dtype, b.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        pf, skip2d, ws, wp, y = ctx.saved_tensors
        HW, w_dtype, b_dtype = ctx.meta
        dym, dp, dwp = _C.loc_in_bwd(dy.to(torch.bfloat16).contiguous(), y, pf, wp, HW)
        dskip = torch.mm(dym, ws) if ctx.needs_input_grad[1] else None
        dws, db = _C.wgrad(dym, skip2d, 0, True, _bf16_grads(w_dtype, b_dtype))
        dw = torch.cat([dwp.to(dws.dtype), dws], 1).to(w_dtype)
        return dp, dskip, dw, db.to(b_dtype), None


def location_input(pf, skip, w, b):
    """pf [B, P*H*W] (ReLU'd fc output), skip [B, C, H, W] channels_last bf16 (a ReLU output), conv1x1
    weight [C, P + C, 1, 1] + bias -> relu(conv(relu(cat([pf.view(B, P, H, W), skip], 1)))) as a
    channels_last [B, C, H, W] view; None when the shapes are not the kernel's."""
    if not LOC_FUSED:
        return None
    B, C, H, W = skip.shape
    cout, cin = w.shape[0], w.shape[1]
    if skip.dtype != torch.bfloat16 or not skip.is_contiguous(memory_format=torch.channels_last) or b is None \
            or cout != C or not _C.loc_in_supported(C, cin - C) or pf.numel() != B * (cin - C) * H * W:
        return None
    w2 = w.view(cout, cin)
    w2 = w2 if w2.dtype == torch.bfloat16 else _bf16w(w2)
    bb = b if b.dtype == torch.bfloat16 else _bf16w(b)
    with torch.autocast('cuda', enabled=False):
        y = _LocationInput.apply(pf.to(torch.bfloat16).reshape(B, -1).contiguous(), nhwc(skip).view(-1, C), w2, bb,
                                 H * W)
    return from_nhwc(y.view(B, H, W, C))


# ---------------------------------------------------------------------------- narrow 1x1 conv (pointwise.hip)
class _Pointwise(torch.autograd.Function):
    """act(x W^T + b) per NHWC pixel for Cin, Cout <= 32: one thread per pixel (the library GEMM runs
    16x256 tiles at ~0.85 ms on the value encoder's 9.5M-pixel 16->16 projection); dX is the same kernel
    with W^T, dW / db the split-R MFMA kernel."""

    @staticmethod
    def forward(ctx, x2, w, b, relu):
        y = _C.pointwise_conv(x2, _w32(w), _w32(b) if b is not None else None, 1 if relu else 0)
        ctx.save_for_backward(x2, w, y)
        ctx.relu = relu
        ctx.b_dtype = b.dtype if b is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        P, cout = y.shape
        dpre = _C.act_grad_nhwc(dy.reshape(1, 1, P, cout), y.view(1, 1, P, cout), ctx.relu).view(P, cout)
        dx = _C.pointwise_conv(dpre, _wT(w, torch.float32), None, 0) if ctx.needs_input_grad[0] \
            else None
        has_b = ctx.b_dtype is not None
        dw, db = _C.wgrad(dpre, x2, 0, has_b, _bf16_grads(w.dtype, ctx.b_dtype))
        return dx, dw.to(w.dtype), (db.to(ctx.b_dtype) if has_b else None), None, None


WGRAD_BF16_OUT = True    # tools/ab_bench.py --variant wgrad_bf16


def _bf16_grads(w_dtype, b_dtype):
    """Have wgrad emit dW/db in bf16 (cast fused into its split reduction) when the parameters are the
    bf16 compute copies of master weights; fp32 parameters keep the fp32 reduction."""
    return WGRAD_BF16_OUT and w_dtype == torch.bfloat16 and b_dtype in (None, torch.bfloat16)


# ---------------------------------------------------------------------------- linear with MFMA split-R wgrad
class _Linear(torch.autograd.Function):
    """y = act(x W^T + b) on hipBLASLt (ReLU fused into the GEMM epilogue via ``_addmm_activation``; dX
    is a well-shaped library GEMM); dW and db come from the split-R MFMA kernel (``wgrad.hip``): the
    library tiles only the small N x K output of dW = dY^T X and runs a handful of workgroups for
    R ~ 10^5..10^7 rows.  The ReLU mask is applied to dY by the one-pass ``act_grad`` kernel."""

    @staticmethod
    def forward(ctx, x2, w, b, relu, link=None):
        _count_use(w)
        ctx.link = link
        R, K = x2.shape
        if SMALL_NATIVE and SPLITK_NATIVE and x2.is_cuda and R <= 2048 and K > F32_SMALL_K_MAX and \
                (R + 127) // 128 * ((w.shape[0] + 63) // 64) < 128 and R * K < (1 << 31) and w.shape[0] * K < (1 << 31):
            # few rows, long reduction (the spatial encoder's 48,640 -> 256 fc, the location head's 12,160 -> 128):
            # split-K over workgroup slices + one ordered sum with the bias / ReLU epilogue (gemm_small.hip),
            # in the operands' precision
            y = _C.small_gemm_splitk(x2, w.detach().contiguous(), _w32(b) if b is not None else None, 1 if relu else 0)
            if relu and y.dtype == torch.float32 and RELU_LINK:
                _note_relu_out(y)
        elif GEMM_REFORM and R <= 2048 and K >= 16384 and K % (32 * 8) == 0:
            # few rows, huge reduction (the spatial encoder's 48640 -> 256 fc): the library ran a 256x16 tile
            # over the whole K (0.14-0.30 ms); 32 K-chunks as one batched GEMM + an fp32 sum: 48 us
            S = 32
            kc = K // S
            p = torch.bmm(x2.view(R, S, kc).transpose(0, 1), w.view(w.shape[0], S, kc).permute(1, 2, 0))
            y = p.sum(0, dtype=torch.float32)
            if b is not None:
                y = y + b.float()
            y = (torch.relu(y) if relu else y).to(x2.dtype)
        elif x2.dtype == torch.float32 and _gemm_f32_ok(R, w.shape[0], K):
            # fp32 step: f32-MFMA GEMM with the bias and ReLU in its epilogue (gemm_f32.hip; on the pre-split weight
            # planes when the shape allows, gemm_f32_psb.hip)
            bias = _w32(b) if b is not None else None
            if w.dim() == 2 and _psb_ok(R, w.shape[0], K):
                y = _C.gemm_f32_psb(x2, _psb(w), w.shape[0], K, bias, None, 1 if relu else 0, GEMM_PSB_VARIANT)
            else:
                y = _C.gemm_f32(x2, w.detach().contiguous(), bias, None, 1 if relu else 0)
            if relu and RELU_LINK:
                _note_relu_out(y)
        elif _bf16_small_ok(x2, R, w.shape[0], K):
            # bf16 step, few rows: one workgroup per 32 x 32 tile (gemm_bf16_small_kernel), bias + ReLU fused
            y = _C.gemm_bf16_small(x2, w.detach().contiguous(), _w32(b) if b is not None else None, None,
                                   1 if relu else 0)
        elif _bf16_pipe_ok(x2, R, w.shape[0], K):
            # bf16 step, many rows (the entity transformer, the pointer heads' key MLPs): the LDS-DMA ring kernel
            # (gemm_bf16.hip), bias + ReLU in its epilogue
            y = _C.gemm_bf16(x2, w.detach().contiguous(), _w32(b) if b is not None else None, None, 1 if relu else 0)
        elif relu and b is not None:
            y = torch._addmm_activation(b.to(x2.dtype), x2, w.t(), use_gelu=False)
        else:
            y = torch.nn.functional.linear(x2, w, None if b is None else b.to(x2.dtype))
            if relu:
                y = torch.relu(y)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu = relu
        ctx.b_dtype = b.dtype if b is not None else None
        ctx.mask_in = x2.dtype == torch.float32 and link is None and _relu_src(x2)
        if _DEBUG_PREMASK:
            ctx.site = _fwd_site()
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        if ctx.relu and y.dtype == torch.float32 and _premasked(y, dy):
            dy = dy.contiguous().view(y.shape)      # the consumer's dX epilogue applied this ReLU's mask
        elif ctx.relu:
            R, N = y.shape
            _premask_miss(ctx, 'linear', y)
            dy = _act_grad(dy.view(1, 1, R, N) if dy.is_contiguous() else dy.contiguous().view(1, 1, R, N),
                           y.view(1, 1, R, N), True).view(R, N)
        else:
            dy = dy.to(x2.dtype).contiguous()
        has_b = ctx.b_dtype is not None
        side = _SideWork(dy, dy.shape[0])
        with side.fork():       # dW / db concurrent with the dX GEMM below
            dw, db = _wgrad(dy, x2, 0, has_b, _bf16_grads(w.dtype, ctx.b_dtype), w)
            dw = dw.to(w.dtype)
            db = db.to(ctx.b_dtype) if has_b else None
        dx = None
        g = None
        if ctx.link is not None:
            g, ctx.link.g = ctx.link.g, None
            if g is not None and (_Deferred.on or _Deferred.flushed is not None):
                # g is written in place below; queued / side-stream weight gradients may still read it
                defer_end(g.device)
            if _DEBUG_GRADLINK and g is not None and g._version != ctx.link.version:
                raise RuntimeError('GradLink: the handed-over residual gradient was modified before the dX GEMM')
        if dy.dtype == torch.float32 and _gemm_f32_ok(dy.shape[0], w.shape[1], dy.shape[1]) and \
                (g is not None or ctx.needs_input_grad[0]):
            # fp32: dX = dY W (+ the handed-over residual gradient) on the f32-MFMA GEMM, out of place; when x is
            # the ReLU output of another fp32 linear, that ReLU's mask is applied here (epilogue mode 4) and
            # the producer's backward skips its own threshold pass (_premasked)
            psb = w.dim() == 2 and _psb_ok(dy.shape[0], w.shape[1], dy.shape[1])
            if g is None and ctx.mask_in:
                dx = _C.gemm_f32_psb(dy, _psb(w, True), w.shape[1], w.shape[0], None, x2, 4, GEMM_PSB_VARIANT) if psb \
                    else _C.gemm_f32(dy, _wT(w), None, x2, 4)
                _MASKED_DX[x2.data_ptr()] = (dx, dx._version)
            else:
                r = None if g is None else g.view(dy.shape[0], w.shape[1])
                if psb and r is not None and not r.is_contiguous():
                    psb = False
                dx = _C.gemm_f32_psb(dy, _psb(w, True), w.shape[1], w.shape[0], None, r, 0, GEMM_PSB_VARIANT) if psb \
                    else _C.gemm_f32(dy, _wT(w), None, r, 0)
        elif (g is not None or ctx.needs_input_grad[0]) and _bf16_small_ok(dy, dy.shape[0], w.shape[1], dy.shape[1]) \
                and (g is None or g.dtype == torch.bfloat16):
            # bf16 step, few rows: dX = dY W (+ the handed-over residual gradient) on the small-tile kernel
            dx = _C.gemm_bf16_small(dy.contiguous(), _wT(w), None,
                                    None if g is None else g.view(dy.shape[0], w.shape[1]).contiguous(), 0)
        elif (g is not None or ctx.needs_input_grad[0]) and _bf16_pipe_ok(dy, dy.shape[0], w.shape[1], dy.shape[1]) \
                and (g is None or g.dtype == torch.bfloat16) and not (g is None and dy.shape[1] == 32):
            # bf16 step, many rows: dX = dY W (+ the handed-over residual gradient) on the LDS-DMA ring kernel
            dx = _C.gemm_bf16(dy.contiguous(), _wT(w), None,
                              None if g is None else g.view(dy.shape[0], w.shape[1]).contiguous(), 0)
        elif g is not None:
            # + the residual gradient the closing LayerNorm handed over (GradLink), in the GEMM epilogue
            # in place: g is the LayerNorm's input gradient, which the branch's later layers (backward
            # runs earlier, same stream) have already consumed; out-of-place addmm copied g first
            wt = _wT(w).t() if GEMM_REFORM and dy.shape[0] * w.shape[1] >= (1 << 22) else w
            dx = g.view(dy.shape[0], w.shape[1]).addmm_(dy, wt)
        elif ctx.needs_input_grad[0]:
            if dy.shape[1] == 32 and x2.shape[1] % 16 == 0 and dy.is_contiguous() and dy.dtype == torch.bfloat16:
                # thin-K product (the heads' 256 -> 32 key projections): one MFMA per output tile, a pure
                # store stream (gemm_k32.hip); the library took 0.19 ms per 196k-row call
                dx = _C.mm_k32(dy, _wT(w))
            elif GEMM_REFORM and dy.shape[0] * w.shape[1] >= (1 << 22):
                # dY W as an "NT" product against a transposed weight copy (the layout of the forward):
                # hipBLASLt's "NN" kernels ran the transformer FFN dX at 132 vs 106 us and the value fc's
                # 390 x 12160 dX at 32 vs 19 us (tools/bench_gemm_alts.py)
                dx = torch.nn.functional.linear(dy, _wT(w))
            else:
                dx = torch.mm(dy, w)
        side.join(dw, db)
        return dx, dw, db, None, None


# ---------------------------------------------------------------------------- ReLU-mask hand-off (fp32 linears)
RELU_LINK = os.environ.get('APPLESTAR_RELU_LINK', '1') == '1'   # A/B switch
_RELU_OUTS = {}      # data_ptr -> weakref of an fp32 _Linear ReLU output (recorded in forward)
_MASKED_DX = {}      # data_ptr of such an output -> (dX of its consumer, version): already ReLU-masked

# debug (APPLESTAR_DEBUG_PREMASK=1): ReLU backward passes that could not be folded into a consumer's epilogue,
# counted by (op, shape, forward call site) - tools/glue_sites.py prints them
_DEBUG_PREMASK = os.environ.get('APPLESTAR_DEBUG_PREMASK', '0') == '1'
PREMASK_MISSES = collections.Counter()


def _fwd_site():
    import traceback
    fr = [f for f in traceback.extract_stack() if 'applestar_amd' in f.filename and 'ops/native.py' not in f.filename]
    return ' < '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in fr[-2:][::-1])


def _premask_miss(ctx, kind, t):
    if _DEBUG_PREMASK:
        PREMASK_MISSES[(kind, tuple(t.shape), getattr(ctx, 'site', '?'))] += 1


def _relu_src(x2):
    """x2 is (the storage of, same size) the ReLU output of an fp32 ``_Linear``: its consumer's dX may apply
    that ReLU's mask in the GEMM epilogue (mask(x2 > 0) = relu'(pre) exactly, since x2 = relu(pre))."""
    if not RELU_LINK:
        return False
    r = _RELU_OUTS.get(x2.data_ptr())
    t = r() if r is not None else None
    return t is not None and t.data_ptr() == x2.data_ptr() and t.numel() == x2.numel() and t.dtype == x2.dtype


def _note_relu_out(y):
    if len(_RELU_OUTS) > 4096:
        for k in [k for k, r in _RELU_OUTS.items() if r() is None]:
            del _RELU_OUTS[k]
    _RELU_OUTS[y.data_ptr()] = weakref.ref(y)


def _premasked(y, dy):
    """The incoming gradient dy of ReLU output y is exactly the dX its sole consumer already masked by
    (y > 0) (same storage, unmodified): the separate threshold_backward pass is skipped.  Any other
    gradient (a sum over several consumers is a new tensor) takes the mask as usual; masking is idempotent,
    so a missed hand-off costs one pass, never correctness.  As with GradLink, a ``retain_grad`` / hook on
    such an intermediate ReLU output would observe the masked gradient."""
    if len(_MASKED_DX) > 256:
        _MASKED_DX.clear()
    rec = _MASKED_DX.pop(y.data_ptr(), None)
    return rec is not None and rec[0].data_ptr() == dy.data_ptr() and rec[0]._version == rec[1] and \
        rec[0].numel() == dy.numel()


_WGRAD_MIN_ROWS = 256     # tools/ab_bench.py --variant wgrad_small: -0.7 ms/step vs 4096


def _gemm_f32_ok(M, N, K):
    """The native f32 GEMM takes this [M, K] x [N, K]^T product: K % 4 and 32-bit buffer offsets.  Products with
    >= 128 of its 128 x 64 tiles run the LDS-DMA pipe kernel; fewer (the few-row linears: heads, scalar encoder,
    value projections) run one wave per 32 x 32 tile straight from L2 (``gemm_f32_small_kernel``), which replaced
    ~170 library calls per fp32 step (r4) - up to a reduction of ``F32_SMALL_K_MAX`` (the spatial encoder's
    48,640-wide fc keeps its batched split-K form)."""
    return K % 4 == 0 and M * K * 4 < 0x7ffffff0 and N * K * 4 < 0x7ffffff0 and \
        ((M + 127) // 128 * ((N + 63) // 64) >= 128 or (F32_SMALL and K <= F32_SMALL_K_MAX))


F32_SMALL = os.environ.get('APPLESTAR_F32_SMALL_GEMM', '1') == '1'     # A/B switch
BF16_SMALL = os.environ.get('APPLESTAR_BF16_SMALL_GEMM', '1') == '1'   # A/B switch


def _bf16_small_ok(a, M, N, K):
    """A bf16 [M, K] x [N, K]^T product for gemm_bf16_small_kernel: few tiles (as the fp32 small path), K % 8."""
    return BF16_SMALL and a.dtype == torch.bfloat16 and a.is_cuda and K % 8 == 0 and K <= F32_SMALL_K_MAX and \
        (M + 127) // 128 * ((N + 63) // 64) < 128 and M * K * 2 < 0x7ffffff0 and N * K * 2 < 0x7ffffff0
F32_SMALL_K_MAX = 4096
BF16_PIPE = os.environ.get('APPLESTAR_BF16_GEMM', '1') != '0'          # A/B switch ('all': every shape)
BF16_PIPE_ALL = os.environ.get('APPLESTAR_BF16_GEMM', '1') == 'all'


def _bf16_pipe_ok(a, M, N, K):
    """A bf16 [M, K] x [N, K]^T product of >= 128 tiles for gemm_bf16.hip: K % 8, 32-bit byte offsets.  Shapes with
    K >= 256 and N >= 256 over many rows (the entity transformer's projections / FFN, both directions) stay on
    hipBLASLt, which measured 1.0-1.5x faster there (profiles/r4o_gemm_bf16_vs_hipblaslt.jsonl); the native kernel
    wins the thin-output and few-row products (N or K <= 128: 0.5-0.93x the library's time)."""
    return BF16_PIPE and a.dtype == torch.bfloat16 and a.is_cuda and K % 8 == 0 and K < 16384 and \
        M * K * 2 < 0x7ffffff0 and N * K * 2 < 0x7ffffff0 and M * N < (1 << 31) and \
        (M + 127) // 128 * ((N + 63) // 64) >= 128 and (BF16_PIPE_ALL or not (K >= 256 and N >= 256 and M > 2048))
F32_KPAD = False         # tools/ab_bench.py --variant f32_kpad: neutral (64.06 vs 64.14 ms, r3z4), off
GEMM_REFORM = os.environ.get('APPLESTAR_GEMM_REFORM', '1') == '1'


def _mm_tn(a, b):
    """a^T b for a [R, M], b [R, N] with R >> M, N (recurrent weight gradients): 32 row chunks as one batched
    GEMM + a sum when R is large (the library tiled only the small M x N output: 45 vs 25 us at R = 24576)."""
    R = a.shape[0]
    if GEMM_REFORM and R >= 8192 and R % 32 == 0 and a.shape[1] * b.shape[1] <= (1 << 18):
        return torch.bmm(a.view(32, R // 32, -1).transpose(1, 2), b.view(32, R // 32, -1)).sum(0)
    return a.t() @ b


class _LinearSplitK(torch.autograd.Function):
    """act(x W^T + b) for a reduction dim the native kernels do not take (K % 8 != 0): library GEMMs
    for y and dX, dW / db reduced over 64 row chunks with one batched GEMM + a sum."""

    @staticmethod
    def forward(ctx, x2, w, b, relu):
        y = torch.nn.functional.linear(x2, w, b)
        if relu:
            y = torch.relu(y)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu, ctx.has_b = relu, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        if ctx.relu:
            dy = dy * (y > 0)
        dy = dy.to(x2.dtype).contiguous()
        R, N = dy.shape
        K = x2.shape[1]
        dx = dy @ w if ctx.needs_input_grad[0] else None
        c = 64
        Rc = R // c
        dw = torch.bmm(dy[:Rc * c].view(c, Rc, N).transpose(1, 2), x2[:Rc * c].view(c, Rc, K)).float().sum(0)
        if Rc * c < R:
            dw += dy[Rc * c:].t().float() @ x2[Rc * c:].float()
        db = dy.float().sum(0) if ctx.has_b else None
        return dx, dw.to(w.dtype), (db.to(w.dtype) if db is not None else None), None


_SMALL_LINEAR_ROWS = 4096
_ONES = {}


def _ones_row(R, dtype, device):
    """A cached [1, R] ones row (bias gradients as a GEMV)."""
    key = (R, dtype, device)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(1, R, dtype=dtype, device=device)
    return t


class _SmallLinear(torch.autograd.Function):
    """act(x W^T + b) over a few rows, or with K / N not a multiple of 8 (the scalar encoders' one-hot inputs,
    the 2- and 1-wide head / value outputs): library GEMMs both ways, the bias gradient as a ones-row GEMV
    (torch's column reduction over a few hundred rows took ~15 us per layer, r2dl) and the ReLU mask as one
    threshold_backward."""

    @staticmethod
    def forward(ctx, x2, w, b, relu):
        if relu and b is not None:
            y = torch._addmm_activation(b, x2, w.t(), use_gelu=False)
        else:
            y = torch.nn.functional.linear(x2, w, b)
            if relu:
                y = torch.relu(y)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu, ctx.has_b = relu, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy = dy.to(x2.dtype)
        if ctx.relu:
            dy = torch.ops.aten.threshold_backward(dy, y, 0.0)
        dx = dy @ w if ctx.needs_input_grad[0] else None
        dw = dy.t() @ x2
        db = (_ones_row(dy.shape[0], dy.dtype, dy.device) @ dy).view(-1) if ctx.has_b else None
        return dx, dw, db, None


SMALL_NATIVE = os.environ.get('APPLESTAR_SMALL_NATIVE', '1') == '1'     # A/B switch
_MASK = {None: 0, 'relu': 1, 'sigmoid': 2}


class _SmallLinearNative(torch.autograd.Function):
    """act(x W^T + b) over a few rows for ANY K / N (gemm_small.hip), fp32 or bf16: forward one launch with the
    bias and ReLU / sigmoid in the epilogue; backward two launches - dX = mask(dY) W against the transposed
    weight form, dW and db in one TN kernel - where mask(dY) = dY * act'(y) is applied as dY is loaded (no
    threshold pass, no ones-row GEMV).  Replaces the library path of the odd-width scalar-encoder / head /
    value layers and the GLU gates (three library GEMMs + one or two elementwise passes per layer)."""

    @staticmethod
    def forward(ctx, x2, w, b, act):
        if SPLITK_NATIVE and x2.shape[1] > F32_SMALL_K_MAX and _ACT[act] in (0, 1, 2):
            # long reduction (the actor's B = 1..16 spatial-encoder fc, 48,640 wide): split-K slices + an ordered
            # sum; one workgroup per output tile walked all of K (142 us at B = 1, profiles/r5v_timeline_*)
            y = _C.small_gemm_splitk(x2, w.detach().contiguous(), _w32(b) if b is not None else None, _ACT[act])
        else:
            y = _C.small_gemm(x2, w.detach().contiguous(), _w32(b) if b is not None else None, None, None, 0,
                              _ACT[act])
        ctx.save_for_backward(x2, w, y if act else None)
        ctx.act, ctx.has_b = act, b is not None
        ctx.b_dtype = b.dtype if b is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy = dy.to(x2.dtype).contiguous()
        mode = _MASK[ctx.act]
        dx = _C.small_gemm(dy, _wT(w), None, None, y, mode, 0) if ctx.needs_input_grad[0] else None
        bf = x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
        dw, db = _C.small_wgrad(dy, x2, y, mode, ctx.has_b, bf)
        return dx, dw.to(w.dtype), (db.to(ctx.b_dtype) if ctx.has_b else None), None


_SMALL_SIGMOID = os.environ.get('APPLESTAR_SMALL_SIGMOID', '1') == '1'    # bisection switches
_SMALL_ODD = os.environ.get('APPLESTAR_SMALL_ODD', '1') == '1'
SPLITK_NATIVE = os.environ.get('APPLESTAR_SPLITK_NATIVE', '1') == '1'


def _small_native_ok(x, R, N, K, act):
    if act == 'sigmoid' and not _SMALL_SIGMOID:
        return False
    if act != 'sigmoid' and not _SMALL_ODD:
        return False
    return SMALL_NATIVE and x.is_cuda and act in _MASK and 0 < R < _SMALL_LINEAR_ROWS and N > 0 and K > 0 and \
        R * K < (1 << 31) and R * N < (1 << 31)


_CAST_CACHE = {}      # (data_ptr, R, K) of an fp32 activation -> (weakref, version, bf16 copy)
CAST_CACHE = os.environ.get('APPLESTAR_CAST_CACHE', '1') == '1'


def _cast_key(x, R, K):
    return (x.data_ptr(), R, K) if x.is_contiguous() and x.numel() == R * K else None


def _cast_lookup(x, R, K):
    key = _cast_key(x, R, K)
    e = _CAST_CACHE.get(key) if key is not None else None
    if e is None:
        return None
    src = e[0]()
    # the source object alive at the same address and unmodified (views share its version counter)
    if src is None or src.data_ptr() != x.data_ptr() or src._version != e[1] or x._version != e[1]:
        return None
    return e[2]


def _cast_store(x, R, K, xb):
    import weakref
    key = _cast_key(x, R, K)
    if key is None:
        return
    if len(_CAST_CACHE) > 64:
        for k in [k for k, v in _CAST_CACHE.items() if v[0]() is None]:
            del _CAST_CACHE[k]
    try:
        _CAST_CACHE[key] = (weakref.ref(x), x._version, xb)
    except TypeError:
        pass


def _note_bf16_copy(x, xb):
    """Register xb (bf16, same shape) as the cast of the fp32 activation x (written by x's producer kernel)."""
    R = x.shape[0] * x.shape[1] if x.dim() == 3 else x.shape[0]
    K = x.numel() // R if R else 0
    _cast_store(x, R, K, xb.view(R, K))


def _bf16_rows(x, R, K):
    """x as a contiguous bf16 [R, K].  An fp32 activation feeding several linears (the core LSTM output, the scalar
    context: 3-4 heads each) is cast once: the copy is kept while the source tensor is alive and unmodified (same
    storage address, same version counter, so a reshaped view of it hits too) - one launch instead of one per
    consumer; the LSTM recurrence registers its own bf16 output here (no launch at all)."""
    if x.dtype == torch.bfloat16:
        return x.reshape(R, K).contiguous()
    if not (CAST_CACHE and x.is_cuda and x.dtype == torch.float32) or (torch.is_grad_enabled() and x.requires_grad):
        # (no caching under autograd: an entry would keep the step's graph alive)
        return x.reshape(R, K).to(torch.bfloat16).contiguous()
    xb = _cast_lookup(x, R, K)
    if xb is not None:
        return xb
    xb = x.reshape(R, K).to(torch.bfloat16).contiguous()
    _cast_store(x, R, K, xb)
    return xb


def linear(x, w, b=None, act=None, grad_link=None):
    """bf16 act(x W^T + b) over the last dim of x with the native weight gradient when the row count is
    large; other shapes take F.linear (+ the activation).  ``grad_link``: a :class:`GradLink` the residual
    LayerNorm downstream hands x's residual gradient over (armed only on the native path below)."""
    N, K = w.shape
    R = x.numel() // K if K else 0
    lowp = x.dtype == torch.bfloat16 or torch.is_autocast_enabled()
    if lowp and K % 8 and R >= 4 * _WGRAD_MIN_ROWS and act in (None, 'relu'):
        # K not a multiple of 8 (e.g. the location head's 4 + 128 = 132-channel 1x1 conv over 146k
        # pixels): library forward / dX, weight gradient as a split-K batched GEMM (the plain library
        # dW = dY^T X on [146k, 132] runs a couple of output tiles for 0.42 ms; zero-padding K to 136
        # instead made both the dX GEMM and the native dW pick slow tiles: +5 ms, r2ap)
        with torch.autocast('cuda', enabled=False):
            xb = x.reshape(R, K).to(torch.bfloat16)
            wb = w if w.dtype == torch.bfloat16 else _bf16w(w)
            bb = None if b is None else (b if b.dtype == torch.bfloat16 else _bf16w(b))
            y = _LinearSplitK.apply(xb, wb, bb, act == 'relu')
        return y.view(*x.shape[:-1], N)
    if lowp and _small_native_ok(x, R, N, K, act) and (R < _WGRAD_MIN_ROWS or N % 8 or K % 8 or act == 'sigmoid'):
        # few rows, odd widths or a sigmoid gate: the native any-shape kernels both ways (gemm_small.hip)
        ensure_loaded()
        with torch.autocast('cuda', enabled=False):
            xb = _bf16_rows(x, R, K)
            wb = w if w.dtype == torch.bfloat16 else _bf16w(w)
            y = _SmallLinearNative.apply(xb, wb, b, act)
        return y.view(*x.shape[:-1], N)
    if lowp and x.is_cuda and act in (None, 'relu') and R < _SMALL_LINEAR_ROWS and \
            (R < _WGRAD_MIN_ROWS or N % 8 or K % 8):
        with torch.autocast('cuda', enabled=False):
            xb = x.reshape(R, K).to(torch.bfloat16)
            wb = w if w.dtype == torch.bfloat16 else _bf16w(w)
            bb = None if b is None else (b if b.dtype == torch.bfloat16 else _bf16w(b))
            y = _SmallLinear.apply(xb, wb, bb, act == 'relu')
        return y.view(*x.shape[:-1], N)
    if not lowp and x.dtype == torch.float32 and w.dtype == torch.float32 and x.is_cuda and \
            R >= _WGRAD_MIN_ROWS and N % 4 == 0 and K % 4 == 0 and R * max(N, K) * 4 < 0x7ffffff0 and \
            act in (None, 'relu') and (b is None or b.dtype == torch.float32):
        # fp32 step: library fp32 GEMMs forward / dX (exact f32 on gfx950), dW / db on the f32-MFMA split-R kernel
        ensure_loaded()
        link = None
        if grad_link is not None and RESID_LINK and x.dim() == 2 and x.is_contiguous() and x.requires_grad:
            grad_link.armed, link, x2 = x, grad_link, x
        else:
            x2 = x.reshape(R, K).contiguous()
        y = _Linear.apply(x2, w, b, act == 'relu', link)
        return y.view(*x.shape[:-1], N)
    if not lowp and x.dtype == torch.float32 and w.dtype == torch.float32 and (b is None or b.dtype == torch.float32) \
            and _small_native_ok(x, R, N, K, act):
        # fp32, few rows with odd widths / under the split-R threshold, or a sigmoid gate (gemm_small.hip)
        ensure_loaded()
        y = _SmallLinearNative.apply(x.reshape(R, K).contiguous(), w, b, act)
        return y.view(*x.shape[:-1], N)
    if F32_KPAD and not lowp and x.is_cuda and K % 4 and R < _SMALL_LINEAR_ROWS and act in (None, 'relu') and \
            x.dtype == torch.float32 and w.dtype == torch.float32:
        # fp32, a few rows, K not a multiple of 4 (the scalar encoder's 167- / 269-wide inputs): the library's
        # weight-gradient GEMM on the odd K ran 0.33 ms for a 390 x 167 x 128 product; zero-padded to K % 4 == 0
        # (two copies of a few hundred KB) it takes the aligned kernels
        pad = 4 - K % 4
        y = torch.nn.functional.linear(torch.nn.functional.pad(x, (0, pad)), torch.nn.functional.pad(w, (0, pad)), b)
        return torch.relu(y) if act == 'relu' else y
    if not lowp or R < _WGRAD_MIN_ROWS or N % 8 or K % 8 or R * max(N, K) * 2 >= 0x7ffffff0 or \
            act not in (None, 'relu'):
        y = torch.nn.functional.linear(x, w, b)
        if act is None:
            return y
        from . import reference
        return reference.act_fn(y, act)
    ensure_loaded()
    link = None
    if grad_link is not None and RESID_LINK and x.dim() == 2 and x.dtype == torch.bfloat16 and \
            x.is_contiguous() and x.requires_grad:
        grad_link.armed, link, xb = x, grad_link, x
    else:
        xb = _bf16_rows(x, R, K)
    wb = w if w.dtype == torch.bfloat16 else _bf16w(w)
    # the bias as given: the native epilogues add it in fp32 (an fp32 parameter is used as is - no fp32 -> bf16
    # -> fp32 round trip of casts); _Linear's library fallbacks cast it to the operand dtype themselves
    with torch.autocast('cuda', enabled=False):
        y = _Linear.apply(xb, wb, b, act == 'relu', link)
    return y.view(*x.shape[:-1], N)


# ---------------------------------------------------------------------------- fused loss-head statistics
class _HeadStats(torch.autograd.Function):
    """(logp_a, entropy, KL) per row in one kernel; backward one pass over the row (loss.hip)."""

    @staticmethod
    def forward(ctx, logits, teacher, action):
        out, stats = _C.head_stats_fwd(logits, teacher, action)
        ctx.save_for_backward(logits, teacher, action, stats)
        ctx.set_materialize_grads(False)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, ga, gh, gk):
        logits, teacher, action, stats = ctx.saved_tensors
        R = logits.shape[0]
        z = logits.new_zeros(R, dtype=torch.float32)
        g = torch.stack([z if x is None else x.float() for x in (ga, gh, gk)]).contiguous()
        return _C.head_stats_bwd(logits, teacher, action, stats, g), None, None


def head_stats(logits, teacher, actions):
    """Fused ``reference.head_stats`` for fp32 / bf16 logits [..., C]."""
    C = logits.shape[-1]
    lead = logits.shape[:-1]
    l2 = logits if logits.dtype in (torch.float32, torch.bfloat16) else logits.float()
    l2 = l2.reshape(-1, C).contiguous()
    t2 = None
    if teacher is not None:
        t2 = teacher.detach()
        t2 = (t2 if t2.dtype in (torch.float32, torch.bfloat16) else t2.float()).reshape(-1, C).contiguous()
    a = actions.reshape(-1).long().contiguous()
    logp_a, ent, kl = _HeadStats.apply(l2, t2, a)
    return logp_a.view(lead), ent.view(lead), kl.view(lead)


# ---------------------------------------------------------------------------- fused build-order transformer
class _BOEncoder(torch.autograd.Function):
    """Embedding + 3 pre-LN layers + token mean of the beginning-build-order encoder in one kernel per
    direction (bo_encoder.hip); parameter gradients accumulated in one fp32 buffer, then cast into the
    parameters' dtypes with one multi-tensor copy."""

    @staticmethod
    def forward(ctx, bo, loc, *params):
        out, rec = _C.bo_encoder_fwd(bo, loc, list(params), True)
        ctx.save_for_backward(bo, loc, rec, *params)
        return out

    @staticmethod
    def backward(ctx, dmean):
        bo, loc, rec, *params = ctx.saved_tensors
        flat = _C.bo_encoder_bwd(bo, loc, list(params), rec, dmean.float().contiguous())
        grads, srcs, off = [], [], 0
        for p in params:
            n = p.numel()
            src = flat[off:off + n].view(p.shape)
            grads.append(src if p.dtype == torch.float32 else torch.empty_like(p))
            srcs.append(src)
            off += n
        dst = [g for g, p in zip(grads, params) if p.dtype != torch.float32]
        if dst:
            _C.multi_copy(dst, [s for s, p in zip(srcs, params) if p.dtype != torch.float32])
        return (None, None) + tuple(grads)


def bo_encoder(bo, loc, params):
    """mean over the 20 tokens of the build-order transformer output, fp32 [B, 64] (params: see
    BeginningBuildOrderEncoder.fused_params)."""
    if bo.dtype not in (torch.int16, torch.int32, torch.int64):
        bo = bo.long()
    if loc.dtype != bo.dtype:
        loc = loc.to(bo.dtype)
    if not torch.is_grad_enabled() or not any(p.requires_grad for p in params):
        return _C.bo_encoder_fwd(bo.contiguous(), loc.contiguous(), list(params), False)[0]
    return _BOEncoder.apply(bo.contiguous(), loc.contiguous(), *params)


# ---------------------------------------------------------------------------- residual MLP stack (value baseline)
class _ResMLP(torch.autograd.Function):
    """n x ResFCBlock2(256) in one forward kernel; backward = weight transpose + one data-gradient kernel +
    one batched MFMA weight-gradient launch + one LayerNorm-affine reduction (resmlp.hip)."""

    @staticmethod
    def forward(ctx, x0, *params):
        out, sx, sh, sxh, srs = _C.resmlp_fwd(x0, list(params), True)
        ctx.save_for_backward(sx, sh, sxh, srs, *params)
        ctx.x_dtype = x0.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        sx, sh, sxh, srs, *params = ctx.saved_tensors
        dx0, gw, gln = _C.resmlp_bwd(dout.float().contiguous(), list(params), sx, sh, sxh, srs)
        n = len(params) // 6
        grads, dst, src = [], [], []
        for k in range(n):
            w1, b1, w2, b2 = params[6 * k:6 * k + 4]
            for j, (w, b) in enumerate(((w1, b1), (w2, b2))):
                row = gw[2 * k + j]
                for p, flat in ((w, row[:65536]), (b, row[65536:])):
                    g = torch.empty_like(p)
                    dst.append(g)
                    src.append(flat.view(p.shape))
                    grads.append(g)
            grads.append(gln[k, :256])
            grads.append(gln[k, 256:])
        _C.multi_copy(dst, src)
        # reorder to the params order (w1, b1, w2, b2, ln_w, ln_b)
        dx = dx0 if ctx.x_dtype == torch.float32 else dx0.to(ctx.x_dtype)
        return (dx,) + tuple(grads)


def resmlp(x0, params):
    """x0 [R, 256] -> fp32 [R, 256] through n ResFCBlock2 blocks (params: 6 per block)."""
    x0 = x0 if x0.dtype in (torch.float32, torch.bfloat16) else x0.float()
    x0 = x0.contiguous()
    if not torch.is_grad_enabled() or not (x0.requires_grad or any(p.requires_grad for p in params)):
        return _C.resmlp_fwd(x0, list(params), False)[0]
    return _ResMLP.apply(x0, *params)


# ---------------------------------------------------------------------------- autograd.Function dispatch
FAST_APPLY = os.environ.get('APPLESTAR_FAST_APPLY', '1') == '1'


def install_fast_apply(namespace: dict, module: str) -> int:
    """Point ``apply`` of the module's autograd Functions straight at the C++ ``_FunctionBase.apply``.  The Python
    ``Function.apply`` wrapper runs functorch's ``unwrap_dead_wrappers`` (a pytree walk over every argument) on each
    call - 141 calls and ~3.9 ms of host time per bf16 learner step (profiles/r6g_host_profile_bf16.txt), a step
    whose host side is its critical path.  The framework never runs these Functions under functorch transforms
    (vmap / grad), which is all that wrapper serves; none uses ``setup_context`` or keyword arguments."""
    if not FAST_APPLY:
        return 0
    n = 0
    base_setup = getattr(torch.autograd.function._SingleLevelFunction, 'setup_context', None)
    for obj in list(namespace.values()):
        if not (isinstance(obj, type) and issubclass(obj, torch.autograd.Function) and obj.__module__ == module):
            continue
        if 'apply' in obj.__dict__ or getattr(obj, 'setup_context', None) is not base_setup:
            continue
        obj.apply = staticmethod(super(torch.autograd.Function, obj).apply)
        n += 1
    return n


install_fast_apply(globals(), __name__)
