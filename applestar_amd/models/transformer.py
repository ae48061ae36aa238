"""Transformer used by the entity encoder (post-LN, packed variable-length entity sets) and the
beginning-build-order encoder (pre-LN, 20 tokens).

Keys follow ``distar/agent/default/model/module_utils.py:71-199`` (``embedding.0``,
``layers.i.attention.attention_pre.0``, ``.project.0``, ``layernorm1``, ``mlp.{0,1}.0``,
``layernorm2``).  Unlike the reference (dense [B,2,N,N] scores over the padded batch), the entity
path runs on *packed* tokens: GEMMs see only real entities and attention is a varlen kernel driven
by ``cu_seqlens`` — identical outputs on every real token, no work on padding.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .blocks import FCBlock


_SEG_BASE = {}


def dense_segments(lengths: torch.Tensor, N: int) -> torch.Tensor:
    """int32 cu_seqlens [2B + 1] of a padded [B, N] token batch as 2B varlen segments: row b's first
    ``lengths[b]`` tokens, then its remaining N - lengths[b] padding tokens.  The row starts [0, 0, N, N, ..., BN]
    are a cached constant; only the clamped lengths are added (3 launches in the actor's graph, was 8)."""
    B = lengths.shape[0]
    key = (B, int(N), str(lengths.device))
    base = _SEG_BASE.get(key)
    if base is None:
        starts = torch.arange(B + 1, dtype=torch.int32) * N
        base = torch.stack([starts[:-1], starts[:-1]], 1).reshape(-1)
        base = _SEG_BASE[key] = torch.cat([base, starts[-1:]]).to(lengths.device)
    lens = lengths.clamp(0, N).to(torch.int32)
    return base.index_add(0, _odd_index(B, lengths.device), lens)


_ODD = {}


def _odd_index(B: int, device):
    key = (B, str(device))
    t = _ODD.get(key)
    if t is None:
        t = _ODD[key] = torch.arange(1, 2 * B, 2, device=device)
    return t


class Attention(nn.Module):
    def __init__(self, input_dim: int, head_dim: int, output_dim: int, head_num: int):
        super().__init__()
        self.head_num = head_num
        self.head_dim = head_dim
        self.attention_pre = FCBlock(input_dim, head_dim * head_num * 3)
        self.project = FCBlock(head_dim * head_num, output_dim)

    def forward_packed(self, x, cu_seqlens, max_len: int):
        qkv = self.attention_pre(x)
        a = ops.varlen_attention(qkv, cu_seqlens, max_len, self.head_num, self.head_dim)
        return self.project(a)

    def forward_dense(self, x, key_mask=None, cu=None):
        """``cu``: the padded batch as 2B varlen segments (each row's real tokens, then its padding rows as a
        segment of their own, :func:`dense_segments`): the native varlen kernel instead of dense masked scores.
        Real rows get the same values; padding rows attend among themselves (finite, discarded downstream)."""
        B, N, _ = x.shape
        if cu is not None:
            a = ops.varlen_attention(self.attention_pre(x).reshape(B * N, -1), cu, N, self.head_num, self.head_dim)
            return self.project(a.view(B, N, -1))
        qkv = self.attention_pre(x).view(B, N, 3, self.head_num, self.head_dim).permute(2, 0, 3, 1, 4)
        a = ops.masked_attention(qkv[0], qkv[1], qkv[2], key_mask)
        a = a.permute(0, 2, 1, 3).reshape(B, N, self.head_num * self.head_dim)
        return self.project(a)


class TransformerLayer(nn.Module):
    def __init__(self, dim: int, head_dim: int, hidden_dim: int, head_num: int, mlp_num: int, ln_type: str):
        super().__init__()
        self.attention = Attention(dim, head_dim, dim, head_num)
        self.layernorm1 = nn.LayerNorm(dim)
        dims = [dim] + [hidden_dim] * (mlp_num - 1) + [dim]
        self.mlp = nn.Sequential(*[FCBlock(dims[i], dims[i + 1], act=True) for i in range(mlp_num)])
        self.layernorm2 = nn.LayerNorm(dim)
        self.ln_type = ln_type

    def _ln(self, ln, x, residual=None):
        return ops.layer_norm(x, ln.weight, ln.bias, residual=residual)

    def forward_packed(self, x, cu_seqlens, max_len: int, act=None):
        """``act``: an activation applied to the layer output inside the closing LayerNorm kernel.  On the GPU
        each residual gradient is added inside the dX GEMM of its branch's first linear (``ops.grad_link``)
        instead of a separate [T, 256] autograd add."""
        assert self.ln_type == 'post'
        link1, link2 = ops.grad_link(x), ops.grad_link(x)
        pre = self.attention.attention_pre[0]
        qkv = ops.linear(x, pre.weight, pre.bias, grad_link=link1)
        a = self.attention.project(ops.varlen_attention(qkv, cu_seqlens, max_len, self.attention.head_num,
                                                        self.attention.head_dim))
        x = ops.layer_norm(a, self.layernorm1.weight, self.layernorm1.bias, residual=x, grad_link=link1)
        fc0 = self.mlp[0]
        m = ops.linear(x, fc0[0].weight, fc0[0].bias, act='relu' if fc0.act else None, grad_link=link2)
        for blk in self.mlp[1:]:
            m = blk(m)
        return ops.layer_norm(m, self.layernorm2.weight, self.layernorm2.bias, residual=x, act=act, grad_link=link2)

    def forward_dense(self, x, key_mask=None, cu=None):
        if self.ln_type == 'post':
            x = self._ln(self.layernorm1, self.attention.forward_dense(x, key_mask, cu), residual=x)
            return self._ln(self.layernorm2, self.mlp(x), residual=x)
        x = x + self.attention.forward_dense(self._ln(self.layernorm1, x), key_mask)
        return x + self.mlp(self._ln(self.layernorm2, x))


class Transformer(nn.Module):
    def __init__(self, input_dim: int, head_dim: int = 128, hidden_dim: int = 1024, output_dim: int = 256,
                 head_num: int = 2, mlp_num: int = 2, layer_num: int = 3, ln_type: str = 'pre'):
        super().__init__()
        self.embedding = FCBlock(input_dim, output_dim, act=True)
        self.layers = nn.ModuleList([TransformerLayer(output_dim, head_dim, hidden_dim, head_num, mlp_num, ln_type)
                                     for _ in range(layer_num)])

    def forward_dense(self, x, key_mask=None):
        x = self.embedding(x)
        for layer in self.layers:
            x = layer.forward_dense(x, key_mask)
        return x

    def forward_packed_embedded(self, x, cu_seqlens, max_len: int, final_act=None):
        """``x`` is the already-embedded packed token matrix [T, output_dim]; ``final_act`` (e.g. the entity
        encoder's ReLU after the transformer) runs inside the last LayerNorm kernel, forward and backward."""
        for i, layer in enumerate(self.layers):
            x = layer.forward_packed(x, cu_seqlens, max_len, act=final_act if i == len(self.layers) - 1 else None)
        return x
