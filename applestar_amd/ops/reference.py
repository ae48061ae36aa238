"""Plain-PyTorch definitions of every fused op.

These are (a) the implementation used for CPU tensors (``play.py --cpu``, CPU tests) and (b) the
fp32 golden oracle the HIP kernels are tested against.  Each function documents the reference
op sequence it reproduces.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

_ACTS = {
    None: lambda x: x,
    'relu': F.relu,
    'sigmoid': torch.sigmoid,
    'tanh': torch.tanh,
}


def act_fn(x, act):
    return _ACTS[act](x)


def linear(x, w, b=None, act=None):
    return act_fn(F.linear(x, w, b), act)


def layer_norm(x, w, b, residual=None, act=None, eps: float = 1e-5):
    if residual is not None:
        x = x + residual
    return act_fn(F.layer_norm(x, (x.shape[-1],), w, b, eps), act)


def conv2d(x, w, b, stride=1, padding=0, act=None, residual=None):
    y = F.conv2d(x, w, b, stride, padding)
    if residual is not None:
        y = y + residual
    return act_fn(y, act)


def gated_residual(y, g, sp, x):
    """GatedResBlock tail (module_utils.py:224-231): relu(tanh(y*sigmoid(g))*sp + x)."""
    return F.relu(torch.tanh(y * torch.sigmoid(g)) * sp + x)


def lnlstm_cell(x_proj_ln, h, c, w_hh, lnh_w, lnh_b, lnc_w, lnc_b):
    """One LayerNorm-LSTM step given the already-normalised input projection
    (lstm.py:138-153): gates = LN_i(x W_ih^T) + LN_h(h W_hh^T); (i,f,g,o); c' = LN_c(f c + i g);
    h' = o tanh(c').  The *normalised* c' is carried as state, as in the reference."""
    H = h.shape[-1]
    hg = F.layer_norm(h @ w_hh.t(), (4 * H,), lnh_w, lnh_b)
    gates = x_proj_ln + hg
    i, f, g, o = gates.chunk(4, dim=-1)
    c_new = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    c_new = F.layer_norm(c_new, (H,), lnc_w, lnc_b)
    h_new = torch.sigmoid(o) * torch.tanh(c_new)
    return h_new, c_new


def lnlstm_layer(x, h0, c0, w_ih, w_hh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b):
    """Whole-sequence LN-LSTM layer: x [T,B,I] -> out [T,B,H], (h_T, c_T).

    The input projection and its LayerNorm depend only on x, so they are hoisted out of the time
    loop into one [T*B, I] x [I, 4H] GEMM (the reference runs T small GEMMs).
    """
    T, B, _ = x.shape
    H = h0.shape[-1]
    xp = F.layer_norm(F.linear(x.reshape(T * B, -1), w_ih), (4 * H,), lni_w, lni_b).view(T, B, 4 * H)
    h, c = h0, c0
    outs = []
    for t in range(T):
        h, c = lnlstm_cell(xp[t], h, c, w_hh, lnh_w, lnh_b, lnc_w, lnc_b)
        outs.append(h)
    return torch.stack(outs, 0), h, c


def masked_attention(q, k, v, key_mask: Optional[torch.Tensor]):
    """Dense masked softmax attention (module_utils.py:88-111).
    q,k,v [B,H,N,D]; key_mask [B,N] bool (True = valid key). Scores of masked keys are -1e9."""
    d = q.shape[-1]
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(d)
    if key_mask is not None:
        s = s.masked_fill(~key_mask[:, None, None, :], -1e9)
    p = torch.softmax(s.float(), dim=-1).to(v.dtype)
    return torch.matmul(p, v)


def varlen_attention(qkv, cu_seqlens, max_len: int, num_heads: int, head_dim: int):
    """Packed varlen self-attention.  qkv [T, 3*H*D] laid out [q | k | v], each [H, D];
    cu_seqlens [S+1] int.  Returns [T, H*D].  Equivalent to ``masked_attention`` on the padded
    batch for every valid query row."""
    T = qkv.shape[0]
    HD = num_heads * head_dim
    seqlens = (cu_seqlens[1:] - cu_seqlens[:-1]).long()
    S = seqlens.numel()
    idx, valid = _pack_index(seqlens, max_len)
    pad = torch.zeros(S * max_len, 3 * HD, dtype=qkv.dtype, device=qkv.device)
    pad[valid] = qkv
    pad = pad.view(S, max_len, 3, num_heads, head_dim).permute(2, 0, 3, 1, 4)
    out = masked_attention(pad[0], pad[1], pad[2], valid.view(S, max_len))
    out = out.permute(0, 2, 1, 3).reshape(S * max_len, HD)
    return out[valid]


def _pack_index(seqlens, max_len):
    ar = torch.arange(max_len, device=seqlens.device)
    valid = (ar[None, :] < seqlens[:, None]).reshape(-1)
    return None, valid


def sequence_mask(lengths: torch.Tensor, max_len: Optional[int] = None) -> torch.Tensor:
    if max_len is None:
        max_len = int(lengths.max())
    return torch.arange(max_len, device=lengths.device)[None, :] < lengths.reshape(-1, 1)


def scatter_connection(proj: torch.Tensor, x: torch.Tensor, y: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Scatter-add per-entity features into a map (module_utils.py:11-34, 'add' mode).
    proj [B,N,C] (already masked), x,y [B,N] integer coords -> [B,C,H,W]."""
    B, N, C = proj.shape
    xi = x.long().clamp(0, W - 1)
    yi = y.long().clamp(0, H - 1)
    flat = (yi * W + xi) + (torch.arange(B, device=proj.device) * (H * W))[:, None]
    out = torch.zeros(B * H * W, C, dtype=proj.dtype, device=proj.device)
    out.index_add_(0, flat.reshape(-1), proj.reshape(-1, C))
    return out.view(B, H, W, C).permute(0, 3, 1, 2)


# ----------------------------------------------------------------------------- losses / RL math

def categorical_stats(logits: torch.Tensor, actions: torch.Tensor):
    """log-softmax, logp(action), probs — the quantities every RL loss head needs."""
    logp = torch.log_softmax(logits.float(), dim=-1)
    a_logp = logp.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
    return logp, a_logp


def head_stats(logits: torch.Tensor, teacher: Optional[torch.Tensor], actions: torch.Tensor):
    """Per row of ``logits [..., C]``: (logp(action), entropy, KL(softmax(teacher) || softmax(logits))),
    fp32, shaped like ``actions`` (rl_loss.py:63-90, as_rl_utils.py:52-127).  KL is 0 without a teacher."""
    lp = torch.log_softmax(logits.float(), dim=-1)
    a = actions.long().clamp(0, logits.shape[-1] - 1)
    logp_a = lp.gather(-1, a.unsqueeze(-1)).squeeze(-1)
    ent = -(lp.exp() * lp).sum(-1)
    if teacher is None:
        return logp_a, ent, torch.zeros_like(ent)
    tlp = torch.log_softmax(teacher.float(), dim=-1)
    kl = (tlp.exp() * (tlp - lp)).sum(-1)
    return logp_a, ent, kl


def vtrace_advantages(clipped_rhos, clipped_cs, rewards, values, gamma: float = 1.0, lambda_: float = 1.0):
    """as_rl_utils.py:284-312. rhos/cs/rewards [T,B], values [T+1,B] -> advantages [T,B]."""
    T = rewards.shape[0]
    deltas = clipped_rhos * (rewards + gamma * values[1:] - values[:-1])
    vs = torch.empty_like(values)
    vs[-1] = values[-1]
    for t in range(T - 1, -1, -1):
        vs[t] = values[t] + deltas[t] + gamma * lambda_ * clipped_cs[t] * (vs[t + 1] - values[t + 1])
    return clipped_rhos * (rewards + gamma * vs[1:] - values[:-1])


def lambda_returns(rewards, values, gamma: float, lambdas):
    """generalized_lambda_returns / multistep_forward_view (as_rl_utils.py:157-218).
    rewards [T,B], values [T+1,B], lambdas scalar or [T,B] (last row ignored)."""
    T = rewards.shape[0]
    if not torch.is_tensor(lambdas):
        lambdas = torch.full_like(rewards, float(lambdas))
    boot = values[1:]
    out = torch.empty_like(rewards)
    out[-1] = rewards[-1] + gamma * boot[-1]
    disc = gamma * lambdas
    for t in range(T - 2, -1, -1):
        out[t] = rewards[t] + disc[t] * out[t + 1] + (gamma - disc[t]) * boot[t]
    return out


def upgo_returns(rewards, values):
    """as_rl_utils.py:265-281."""
    lam = (rewards + values[1:]) >= values[:-1]
    lam = torch.cat([lam[1:], torch.ones_like(lam[-1:])], 0).to(rewards.dtype)
    return lambda_returns(rewards, values, 1.0, lam)


def td_lambda_returns(rewards, values, gamma: float = 1.0, lambda_: float = 0.8):
    return lambda_returns(rewards, values, gamma, lambda_)
