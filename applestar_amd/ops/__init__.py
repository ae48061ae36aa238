"""Fused ops used by the AlphaStar policy / learner.

Every op has one definition in :mod:`.reference` (PyTorch, used for CPU tensors and as the golden
oracle in tests) and, for GPU tensors, a hand-written HIP/CDNA4 kernel in ``applestar_amd/csrc``
exposed through :mod:`.native`.  GPU tensors never silently take the reference path for an op that
has a native kernel: if the extension is missing, :func:`._ext.require` raises.

GEMMs and 3x3 convolutions are native too: in fp32 every linear / conv3x3 product (forward, dX, dW) runs on
the bf16x6 split-MFMA kernels (``gemm_f32.hip``, ``conv3x3_f32.hip``, ``wgrad_f32.hip``) or the few-row kernels of
``gemm_small.hip``; the library (hipBLASLt through ``torch.mm``) keeps only the handful of products listed by
``tools/gemm_census.py`` (recurrent LSTM dW, batched pointer logits).  In the bf16 step the entity
transformer's large products stay on hipBLASLt (faster there, docs/OPEN_ISSUES.md).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import reference as ref
from . import _ext

__all__ = ['linear', 'layer_norm', 'conv2d', 'max_pool2x2', 'segment_sum', 'gather_rows', 'embed_relu', 'gated_residual', 'lnlstm_layer', 'varlen_attention',
           'masked_attention', 'scatter_connection', 'sequence_mask', 'native_enabled', 'set_native', 'upsample2x',
           'upsample_conv_out', 'head_sample', 'target_unit_sample']

_NATIVE_ENABLED = True


def set_native(flag: bool) -> None:
    """Globally disable native kernels (used by tests to produce a torch-only GPU baseline)."""
    global _NATIVE_ENABLED
    _NATIVE_ENABLED = bool(flag)


def native_enabled() -> bool:
    return _NATIVE_ENABLED


def _native(t: torch.Tensor):
    """Return the native module when ``t`` lives on a GPU (raising if it is not built), else None."""
    if t.is_cuda and _NATIVE_ENABLED:
        from . import native
        native.ensure_loaded()
        return native
    return None


EMBED_RELU_NATIVE = os.environ.get('APPLESTAR_EMBED_RELU', '1') == '1'
sequence_mask = ref.sequence_mask
masked_attention = ref.masked_attention


def linear(x, w, b=None, act=None, grad_link=None):
    """act(x W^T + b).  GPU: native split-MFMA GEMM (fp32) / ring or library GEMM (bf16) for the forward and dX
    with fused bias / ReLU / residual epilogues, split-R MFMA kernel for dW / db of tall inputs.
    ``grad_link``: native GradLink (residual gradient added in the dX GEMM), ignored elsewhere."""
    n = _native(x)
    if n is not None:
        return n.linear(x, w, b, act, grad_link=grad_link)
    y = F.linear(x, w, b)
    if act is None:
        return y
    return ref.act_fn(y, act)


def layer_norm(x, w, b, residual=None, act=None, eps: float = 1e-5, grad_link=None):
    n = _native(x)
    if n is not None and n.has('layer_norm'):
        # under autocast the normalised activations are stored in bf16 (statistics and affine in fp32):
        # every consumer is a bf16 GEMM, so an fp32 output only bought a cast in forward and an fp32
        # gradient cast + fp32 residual-gradient adds in backward (~0.5 GB per step in the entity encoder)
        out_dtype = torch.bfloat16 if torch.is_autocast_enabled() else None
        return n.layer_norm(x, w, b, residual, act, eps, out_dtype=out_dtype, grad_link=grad_link)
    return ref.layer_norm(x, w, b, residual, act, eps)


def conv2d(x, w, b, stride=1, padding=0, act=None, residual=None):
    """act(conv2d(x, w, b) + residual).  GPU: MFMA implicit-GEMM 3x3 kernel / NHWC GEMM for 1x1 (fused
    bias, residual, ReLU); other shapes go to MIOpen."""
    n = _native(x)
    if n is not None and n.has('conv2d'):
        y = n.conv2d(x, w, b, stride, padding, act, residual)
        if y is not None:
            return y
    return ref.conv2d(x, w, b, stride, padding, act, residual)


def value_spatial_proj(sc, own, enemy, w, b):
    """Fused value-encoder spatial input relu(conv1x1(cat([sc, own, enemy]))) on the GPU; None when it does
    not apply (caller runs the cat path)."""
    n = _native(sc)
    if n is not None and n.has('value_spatial_proj'):
        return n.value_spatial_proj(sc, own, enemy, w, b)
    return None


def rl_loss_tail(alp, ent, kl, v, blp, hm, r, wm, atflag, sc, upgo_f, only_value):
    """Fused RL loss tail (GPU): (total, info vector); callers check _native(...).has('rl_loss') first."""
    return _native(v).rl_loss_tail(alp, ent, kl, v, blp, hm, r, wm, atflag, sc, upgo_f, only_value)


def value_spatial_proj_pool(sc, own, enemy, w, b):
    """max_pool2x2 of the fused value-encoder spatial input on the GPU; None when it does not apply."""
    n = _native(sc)
    if n is not None and n.has('value_spatial_proj_pool'):
        return n.value_spatial_proj_pool(sc, own, enemy, w, b)
    return None


def location_input(pf, skip, w, b):
    """Fused location-head input stage relu(conv1x1(relu(cat([pf as [B,P,H,W], skip])))) on the GPU
    (skip a channels_last ReLU output); None when it does not apply (caller runs the cat path)."""
    n = _native(skip)
    if n is not None and n.has('location_input'):
        return n.location_input(pf, skip, w, b)
    return None


def max_pool2x2(x):
    n = _native(x)
    if n is not None and n.has('maxpool2x2') and x.dim() == 4 and x.shape[1] % 8 == 0:
        return n.maxpool2x2(x)
    return F.max_pool2d(x, 2, 2)


def segment_sum(x, cu_seqlens, seg):
    """Per-segment row sums of packed rows x [T,C] -> fp32 [S,C] (seg [T] = segment id of each row)."""
    n = _native(x)
    if n is not None and n.has('segment_sum') and x.shape[-1] % 4 == 0 and x.shape[-1] <= 1024:
        return n.segment_sum(x, cu_seqlens, seg)
    S = cu_seqlens.numel() - 1
    return x.float().new_zeros(S, x.shape[-1]).index_add(0, seg, x.float())


def embed_relu(table, idx):
    """relu(table[idx.long().clamp(max=V - 1)]): one native launch per direction for the small tables."""
    n = _native(table)
    if n is not None and n.has('embed_relu') and EMBED_RELU_NATIVE:
        out = n.embed_relu(table, idx)
        if out is not None:
            return out
    i = idx.long().clamp(max=table.shape[0] - 1)
    return torch.relu(gather_rows(table, i.reshape(-1)).view(*i.shape, -1))


def gather_rows(table, idx):
    """table[idx] for small lookup tables (native backward: LDS-accumulated row gradients)."""
    n = _native(table)
    if n is not None and n.has('gather_rows') and table.dim() == 2:
        return n.gather_rows(table, idx)
    return table.index_select(0, idx)


def gated_residual(y, g, sp, x):
    n = _native(x)
    if n is not None and n.has('gated_residual'):
        return n.gated_residual(y, g, sp, x)
    return ref.gated_residual(y, g, sp, x)


def lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b):
    n = _native(x)
    if n is not None and n.has('lnlstm_layer'):
        return n.lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b)
    return ref.lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b)


def varlen_attention(qkv, cu_seqlens, max_len: int, num_heads: int, head_dim: int):
    n = _native(qkv)
    if n is not None and n.has('varlen_attention'):
        return n.varlen_attention(qkv, cu_seqlens, max_len, num_heads, head_dim)
    return ref.varlen_attention(qkv, cu_seqlens, max_len, num_heads, head_dim)


def action_logp(logits, actions):
    """{head: log_softmax(logits[head])[actions[head]]} (fp32): one native launch for all heads on the GPU."""
    keys = list(actions)
    n = _native(logits[keys[0]]) if keys else None
    if n is not None and n.has('action_logp') and len(keys) <= 8:
        ls = [logits[k].contiguous() for k in keys]
        if all(t.dtype in (torch.float32, torch.bfloat16) for t in ls):
            outs = n.ensure_loaded().multi_logp(ls, [actions[k].long().contiguous() for k in keys])
            return dict(zip(keys, outs))
    out = {}
    for k in keys:
        lp = torch.log_softmax(logits[k].float(), dim=-1)
        out[k] = lp.gather(-1, actions[k].long().unsqueeze(-1)).squeeze(-1)
    return out


def head_stats(logits, teacher, actions):
    """(logp(action), entropy, KL(teacher || logits)) per distribution row, fp32 (K19 fused kernel on GPU)."""
    n = _native(logits)
    if n is not None and n.has('head_stats'):
        return n.head_stats(logits, teacher, actions)
    return ref.head_stats(logits, teacher, actions)


def scatter_connection(proj, x, y, H: int, W: int):
    return ref.scatter_connection(proj, x, y, H, W)


def upsample2x(x):
    n = _native(x)
    if n is not None and n.has('upsample2x') and x.shape[1] % 4 == 0:
        return n.upsample2x(x)
    return F.interpolate(x, scale_factor=2.0, mode='bilinear', align_corners=False)


def upsample_conv_out(x, w, b):
    """conv3x3(bilinear_x2(x), w, b, padding=1) with ONE output channel, flattened to [B, 4HW] fp32
    (the location head's last stage, action_arg_head.py:445-450).  Fused on the GPU for 32 channels."""
    n = _native(x)
    if n is not None and n.has('upsample_conv_out') and tuple(w.shape) == (1, 32, 3, 3):
        return n.upsample_conv_out(x, w, b)
    y = ref.conv2d(upsample2x(x), w, b, 1, 1)
    return y.reshape(x.shape[0], -1).float()


def head_sample(logits, temperature: float = 1.0, mask=None, lens=None, u=None, table=None, bias=None):
    """Inference sampling tail of an action head (csrc/kernels/heads.hip) on the GPU:
    (logits / T with the head's mask as fp32 [B, C], inverse-CDF sample [B] int64, relu(table[a] + bias) [B, D]
    or None).  ``mask``: bool [C] (shared) or [B, C]; ``lens``: [B] valid prefix length; ``u``: [B] uniforms
    (drawn when None).  None off the GPU / with the native kernels off (callers keep the torch path)."""
    n = _native(logits)
    if n is None or torch.is_grad_enabled():
        return None
    C = n.ensure_loaded()
    B = logits.shape[0]
    if u is None:
        u = torch.rand(B, device=logits.device)
    lg = logits if logits.dtype in (torch.float32, torch.bfloat16) else logits.float()
    if lg.stride(-1) != 1:
        lg = lg.contiguous()
    out, act, emb = C.head_sample(lg, float(temperature), None if mask is None else mask.to(logits.device).contiguous(),
                                  None if lens is None else lens.long().contiguous(), u.float().contiguous(),
                                  table, None if bias is None else bias.float().contiguous())
    return out, act, (emb if table is not None else None)


def target_unit_sample(embedding, q1, q2, key, entity_num, temperature: float = 1.0, u=None):
    """TargetUnitHead inference in one kernel (query MLP, key dot, length mask, 1/T, sample); None when it does not
    apply (CPU, grad mode, native off, non-reference widths)."""
    n = _native(embedding)
    if n is None or torch.is_grad_enabled() or embedding.shape[-1] != 1024 or key.shape[-1] != 32 or \
            q1.weight.shape != (32, 1024) or q2.weight.shape != (32, 32):
        return None
    C = n.ensure_loaded()
    B = embedding.shape[0]
    if u is None:
        u = torch.rand(B, device=embedding.device)
    f = lambda t: t.detach().float().contiguous()  # noqa: E731
    e = embedding if embedding.dtype in (torch.float32, torch.bfloat16) else embedding.float()
    k = key if key.dtype in (torch.float32, torch.bfloat16) else key.float()
    return tuple(C.target_unit_sample(e.contiguous(), f(q1.weight), f(q1.bias), f(q2.weight), f(q2.bias), k.contiguous(),
                                      entity_num.long().contiguous(), float(temperature), u.float().contiguous()))


def grad_link(x):
    """A native residual-gradient link for a block ``LN(f(x) + x)`` on the GPU path, else None."""
    n = _native(x)
    return n.GradLink() if n is not None and hasattr(n, 'GradLink') else None
