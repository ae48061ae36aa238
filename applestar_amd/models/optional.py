"""Optional / alternative network blocks that the default AlphaStar config does not instantiate but that
reference configs can select (SURVEY §2.4 "Unused/optional blocks", §2.8 "NN blocks").

* :class:`AttentionPool` -- multi-query attention pooling over a token set, used by the selected-units
  head when ``entity_reduce_type`` is ``attention_pool`` / ``attention_pool_add_num``
  (``module_utils.py:37-68``, ``action_arg_head.py:112-115``).
* :class:`FiLM` / :class:`FiLMedResBlock` -- feature-wise linear modulation res-block with the
  reference's conditioning points (``module_utils.py:234-352``).
* :class:`NormLSTM` (``lstm_type='normal'``), :class:`PytorchLSTM` and :func:`get_lstm`
  (``module_utils.py:355-482``).
* :func:`script_lstm` / :func:`script_lnlstm` incl. dropout and bidirectional stacks (``lstm.py:14-297``);
  the LayerNorm variants run every direction through the fused ``ops.lnlstm_layer`` path.
* :func:`build_normalization`, :func:`conv2d_block`, :func:`deconv2d_block`, :func:`fc_block`,
  :func:`fc_block2` (``normalization.py:77-110``, ``nn_module.py:119-314``), producing ``nn.Sequential``
  blocks with the reference's ``.0.weight`` key layout.

State-dict key names follow the reference modules so checkpoints trained with these options load.
"""
from __future__ import annotations

import math
import warnings
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .blocks import FCBlock
from .lstm import LNLSTMCell, StackedLNLSTM, _Layer

__all__ = ['AttentionPool', 'FiLM', 'FiLMedResBlock', 'NormLSTM', 'PytorchLSTM', 'get_lstm', 'LSTMCell',
           'RecurrentStack', 'BidirLayer', 'script_lstm', 'script_lnlstm', 'build_normalization', 'conv2d_block',
           'deconv2d_block', 'fc_block', 'fc_block2', 'GroupSyncBatchNorm', 'SoftArgmax', 'ScatterConnection',
           'Swish', 'build_activation']


# ---------------------------------------------------------------------------------------------- pooling
class AttentionPool(nn.Module):
    """``head_num`` learned queries score every token (dot product over channels); a softmax over the
    (masked) tokens weights them; the ``[C, heads]`` result is flattened and projected to ``output_dim``,
    optionally adding ``relu(num_embed(count))``; ReLU at the end.

    Keys: ``queries`` [1,1,heads,C], ``embed_fc.0.{weight,bias}``, ``num_ebed.weight`` (reference spelling).
    """

    def __init__(self, key_dim: int, head_num: int, output_dim: int, max_num: Optional[int] = None):
        super().__init__()
        self.head_num = head_num
        self.queries = nn.Parameter(torch.zeros(1, 1, head_num, key_dim))
        nn.init.xavier_uniform_(self.queries)
        self.add_num = max_num is not None
        if self.add_num:
            self.num_ebed = nn.Embedding(max_num, output_dim)
        self.embed_fc = FCBlock(key_dim * head_num, output_dim)

    def scores(self, x: torch.Tensor) -> torch.Tensor:
        """[B,T,C] -> [B,T,heads]."""
        return torch.einsum('btc,hc->bth', x.float(), self.queries[0, 0].float())

    def project(self, pooled: torch.Tensor, num: Optional[torch.Tensor] = None) -> torch.Tensor:
        """pooled [..., C, heads] -> [..., output_dim] (flattened C-major like the reference's view)."""
        y = self.embed_fc(pooled.reshape(*pooled.shape[:-2], -1).to(self.embed_fc[0].weight.dtype))
        if self.add_num:
            y = y + F.relu(self.num_ebed(num.long())).to(y.dtype)
        return F.relu(y)

    def forward(self, x: torch.Tensor, num: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None):
        assert x.dim() == 3, 'x: [batch, tokens, channels]'
        s = self.scores(x)
        if mask is not None:
            m = mask.reshape(mask.shape[0], mask.shape[1], 1).bool()
            s = s.masked_fill(~m, -1e9)
        w = torch.softmax(s, dim=1)                                    # [B,T,h]
        pooled = torch.einsum('bth,btc->bch', w, x.float())            # [B,C,h]
        return self.project(pooled, num)

    def prefix(self, key: torch.Tensor, labels: torch.Tensor, new: torch.Tensor,
               num: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Pooled outputs after each step of a growing selection, all steps at once.

        ``key`` [B,N,C]; ``labels`` [B,S] token index selected at step i; ``new`` [B,S] whether that
        selection enters the set.  Step i pools over {labels[j] : j <= i, new[j]} -- a prefix softmax, so
        numerator and denominator are running sums of exp(score) (stabilised by the per-row max).  An
        empty set reproduces the reference's all-masked softmax (uniform over all N tokens).
        Returns [B,S,output_dim].
        """
        B, S = labels.shape
        C = key.shape[-1]
        s = self.scores(key)                                                         # [B,N,h]
        gs = s.gather(1, labels.unsqueeze(-1).expand(B, S, self.head_num))           # [B,S,h]
        gk = key.float().gather(1, labels.unsqueeze(-1).expand(B, S, C))             # [B,S,C]
        newf = new.unsqueeze(-1)
        m = gs.masked_fill(~newf, float('-inf')).amax(1, keepdim=True)
        m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
        e = torch.exp(gs - m) * newf.float()                                         # [B,S,h]
        num_c = torch.cumsum(gk.unsqueeze(-1) * e.unsqueeze(2), 1)                   # [B,S,C,h]
        den = torch.cumsum(e, 1).unsqueeze(2)                                        # [B,S,1,h]
        cnt = torch.cumsum(new.int(), 1)
        uniform = key.float().mean(1)[:, None, :, None].expand(B, S, C, self.head_num)
        pooled = torch.where((cnt > 0)[..., None, None], num_c / den.clamp(min=1e-30), uniform)
        return self.project(pooled, cnt if num is None else num)


# ---------------------------------------------------------------------------------------------- FiLM
class FiLM(nn.Module):
    """gammas * x + betas with [B,C] modulation broadcast over H, W."""

    def forward(self, x, gammas, betas):
        return gammas[:, :, None, None] * x + betas[:, :, None, None]


class FiLMedResBlock(nn.Module):
    """Res-block with FiLM conditioning at one of: block-input, conv (default), bn, relu, block-output.

    input_proj (kxk, ReLU) -> [cond maps / extra channels concat] -> conv1 -> [FiLM] -> [BN] -> [dropout]
    -> relu(x + out) if residual.  Only the single-layer, odd-kernel configuration exists in the reference.
    """

    METHODS = ('block-input-film', 'conv-film', 'bn-film', 'relu-film', 'block-output-film')

    def __init__(self, in_dim, out_dim=None, with_residual=True, with_batchnorm=False, with_cond=(False,),
                 dropout=0.0, num_extra_channels=0, extra_channel_freq=1, with_input_proj=3, num_cond_maps=0,
                 kernel_size=3, batchnorm_affine=False, num_layers=1, condition_method='conv-film'):
        super().__init__()
        out_dim = out_dim or in_dim
        if with_input_proj % 2 == 0 or kernel_size % 2 == 0 or num_layers >= 2:
            raise NotImplementedError('FiLMedResBlock: odd kernels and a single layer only')
        assert condition_method in self.METHODS, condition_method
        self.with_residual = with_residual
        self.cond = bool(with_cond[0])
        self.method = condition_method
        self.extra_channel_freq = 0 if num_extra_channels == 0 else extra_channel_freq
        self.with_input_proj = with_input_proj
        self.film = FiLM() if self.cond else None
        if with_input_proj:
            extra = num_extra_channels if self.extra_channel_freq >= 1 else 0
            self.input_proj = nn.Conv2d(in_dim + extra, in_dim, with_input_proj, padding=with_input_proj // 2)
        extra2 = num_extra_channels if self.extra_channel_freq >= 2 else 0
        self.conv1 = nn.Conv2d(in_dim + num_cond_maps + extra2, out_dim, kernel_size, padding=kernel_size // 2)
        self.bn1 = nn.BatchNorm2d(out_dim, affine=(not self.cond) or batchnorm_affine) if with_batchnorm else None
        self.drop = nn.Dropout2d(dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight)

    def _film(self, point, x, gammas, betas):
        return self.film(x, gammas, betas) if self.film is not None and self.method == point else x

    def forward(self, x, gammas=None, betas=None, extra_channels=None, cond_maps=None):
        x = self._film('block-input-film', x, gammas, betas)
        if self.with_input_proj:
            if extra_channels is not None and self.extra_channel_freq >= 1:
                x = torch.cat([x, extra_channels], 1)
            x = F.relu(self.input_proj(x))
        out = x
        if cond_maps is not None:
            out = torch.cat([out, cond_maps], 1)
        if extra_channels is not None and self.extra_channel_freq >= 2:
            out = torch.cat([out, extra_channels], 1)
        out = self._film('conv-film', self.conv1(out), gammas, betas)
        if self.bn1 is not None:
            out = self.bn1(out)
        out = self._film('bn-film', out, gammas, betas)
        if self.drop is not None:
            out = self.drop(out)
        out = self._film('relu-film', out, gammas, betas)
        if self.with_residual:
            out = F.relu(x + out)
        return self._film('block-output-film', out, gammas, betas)


# ---------------------------------------------------------------------------------------------- normalisation
class GroupSyncBatchNorm(nn.SyncBatchNorm):
    """SyncBatchNorm over a process group (``normalization.py:16-58``); falls back to BatchNorm
    semantics when torch.distributed is not initialised."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, group=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, process_group=group)

    def forward(self, x):
        if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            return F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias,
                                self.training or not self.track_running_stats, self.momentum or 0.0, self.eps)
        return super().forward(x)


def build_normalization(norm_type: str, dim: Optional[int] = None):
    """Normalisation *class* for 'BN' (1/2-d), 'LN', 'IN' (2-d), 'SyncBN' (2-d)."""
    if dim is None:
        key = norm_type
    elif norm_type in ('BN', 'IN', 'SyncBN'):
        key = f'{norm_type}{dim}'
    elif norm_type == 'LN':
        key = 'LN'
    else:
        raise NotImplementedError(f'no dim variant for {norm_type}')
    table = {'BN1': nn.BatchNorm1d, 'BN2': nn.BatchNorm2d, 'LN': nn.LayerNorm, 'IN2': nn.InstanceNorm2d,
             'SyncBN2': GroupSyncBatchNorm}
    if key not in table:
        raise KeyError(f'invalid norm type: {key}')
    return table[key]


def _init_weight(w: torch.Tensor, init_type: str, gain: float = 1.0):
    if init_type == 'xavier':
        nn.init.xavier_normal_(w, gain)
    elif init_type == 'kaiming':
        nn.init.kaiming_normal_(w)
    elif init_type == 'orthogonal':
        nn.init.orthogonal_(w)
    elif init_type != 'default':
        raise KeyError(init_type)


def _act_module(activation):
    if activation is None or isinstance(activation, nn.Module):
        return activation
    return {'relu': nn.ReLU(), 'tanh': nn.Tanh(), 'sigmoid': nn.Sigmoid(), 'prelu': nn.PReLU(init=0.0)}[activation]


def conv2d_block(in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 init_type='xavier', pad_type='zero', activation=None, norm_type=None) -> nn.Sequential:
    """[pad] -> conv -> [norm] -> [act]; ``pad_type`` zero is folded into the conv."""
    layers: List[nn.Module] = []
    if pad_type == 'zero':
        conv_pad = padding
    else:
        layers.append({'reflect': nn.ReflectionPad2d, 'replicate': nn.ReplicationPad2d}[pad_type](padding))
        conv_pad = 0
    conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, conv_pad, dilation, groups)
    _init_weight(conv.weight, init_type)
    layers.append(conv)
    if norm_type is not None:
        layers.append(build_normalization(norm_type, 2)(out_channels))
    act = _act_module(activation)
    if act is not None:
        layers.append(act)
    return nn.Sequential(*layers)


def deconv2d_block(in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                   init_type='xavier', activation=None, norm_type=None) -> nn.Sequential:
    conv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, stride, padding, output_padding, groups)
    _init_weight(conv.weight, init_type)
    layers: List[nn.Module] = [conv]
    if norm_type is not None:
        layers.append(build_normalization(norm_type, 2)(out_channels))
    act = _act_module(activation)
    if act is not None:
        layers.append(act)
    return nn.Sequential(*layers)


def fc_block(in_channels, out_channels, init_type='xavier', activation=None, norm_type=None,
             use_dropout=False, dropout_probability=0.5) -> nn.Sequential:
    lin = nn.Linear(in_channels, out_channels)
    _init_weight(lin.weight, init_type)
    layers: List[nn.Module] = [lin]
    if norm_type is not None:
        layers.append(build_normalization(norm_type, 1 if norm_type != 'LN' else None)(out_channels))
    act = _act_module(activation)
    if act is not None:
        layers.append(act)
    if use_dropout:
        layers.append(nn.Dropout(dropout_probability))
    return nn.Sequential(*layers)


def fc_block2(in_channels, out_channels, init_type='xavier', activation=None, norm_type=None,
              use_dropout=False, gain=1.0, dropout_probability=0.5) -> nn.Sequential:
    """fc_block with xavier_uniform(gain) weights and zero bias (value-head output layer)."""
    blk = fc_block(in_channels, out_channels, 'default', activation, norm_type, use_dropout, dropout_probability)
    if init_type == 'xavier':
        nn.init.xavier_uniform_(blk[0].weight, gain)
    else:
        _init_weight(blk[0].weight, init_type, gain)
    nn.init.zeros_(blk[0].bias)
    return blk


# ---------------------------------------------------------------------------------------------- LSTMs
def _list_state(prev_state, num_layers, batch, hidden, like):
    """Normalise the reference's accepted state formats to (h [L,B,H], c [L,B,H])."""
    if prev_state is None:
        z = like.new_zeros(num_layers, batch, hidden)
        return z, z
    if isinstance(prev_state, (list, tuple)) and len(prev_state) == 2 and torch.is_tensor(prev_state[0]):
        return prev_state[0], prev_state[1]
    if isinstance(prev_state, (list, tuple)) and len(prev_state) == batch:   # per-sample list (None = zeros)
        z = like.new_zeros(num_layers, 1, hidden)
        hs = [z if p is None else p[0] for p in prev_state]
        cs = [z if p is None else p[1] for p in prev_state]
        return torch.cat(hs, 1), torch.cat(cs, 1)
    raise TypeError('unsupported prev_state format')


def _split_state(h, c, list_next_state: bool):
    if not list_next_state:
        return h, c
    return list(zip(torch.chunk(h, h.shape[1], 1), torch.chunk(c, c.shape[1], 1)))


class NormLSTM(nn.Module):
    """``lstm_type='normal'``: gates = norm_A(x Wx) + norm_A'(h Wh) + b; (i, f, o, u) with
    f = sigmoid(f + forget_bias); c' = f c + i tanh(u); h' = o tanh(norm_B(c')).  The un-normalised c'
    is carried as the state.  Keys: ``norm_A.{2l,2l+1}``, ``norm_B.{l}``, ``wx.{l}``, ``wh.{l}``, ``bias``.
    The input projection is one GEMM over all timesteps."""

    def __init__(self, input_size, hidden_size, num_layers, norm_type=None, bias=True, dropout=0.0):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        norm = build_normalization(norm_type) if norm_type else (lambda d: nn.Identity())
        self.norm_A = nn.ModuleList([norm(hidden_size * 4) for _ in range(2 * num_layers)])
        self.norm_B = nn.ModuleList([norm(hidden_size) for _ in range(num_layers)])
        dims = [input_size] + [hidden_size] * num_layers
        self.wx = nn.ParameterList([nn.Parameter(torch.zeros(dims[i], hidden_size * 4)) for i in range(num_layers)])
        self.wh = nn.ParameterList([nn.Parameter(torch.zeros(hidden_size, hidden_size * 4))
                                    for _ in range(num_layers)])
        self.bias = nn.Parameter(torch.zeros(num_layers, hidden_size * 4)) if bias else None
        self.dropout = nn.Dropout(dropout) if dropout > 0 else None
        g = math.sqrt(1.0 / hidden_size)
        for p in list(self.wx) + list(self.wh) + ([self.bias] if bias else []):
            nn.init.uniform_(p, -g, g)

    def forward(self, inputs, prev_state=None, list_next_state: bool = False, forget_bias: float = 1.0):
        T, B = inputs.shape[:2]
        H0, C0 = _list_state(prev_state, self.num_layers, B, self.hidden_size, inputs)
        x = inputs
        hs, cs = [], []
        for l in range(self.num_layers):
            h, c = H0[l], C0[l]
            xin = self.dropout(x) if self.dropout is not None else x
            xg = self.norm_A[2 * l](xin @ self.wx[l])                    # [T,B,4H] all steps at once
            outs = []
            for t in range(T):
                gate = xg[t] + self.norm_A[2 * l + 1](h @ self.wh[l])
                if self.bias is not None:
                    gate = gate + self.bias[l]
                i, f, o, u = gate.chunk(4, 1)
                c = torch.sigmoid(f + forget_bias) * c + torch.sigmoid(i) * torch.tanh(u)
                h = torch.sigmoid(o) * torch.tanh(self.norm_B[l](c))
                outs.append(h)
            x = torch.stack(outs, 0)
            hs.append(h)
            cs.append(c)
        return x, _split_state(torch.stack(hs), torch.stack(cs), list_next_state)


class PytorchLSTM(nn.LSTM):
    """``lstm_type='pytorch'``: nn.LSTM (MIOpen RNN on ROCm) with the reference's state formats."""

    def forward(self, inputs, prev_state=None, list_next_state: bool = False):
        h, c = _list_state(prev_state, self.num_layers, inputs.shape[1], self.hidden_size, inputs)
        out, (h, c) = super().forward(inputs, (h.contiguous(), c.contiguous()))
        return out, _split_state(h, c, list_next_state)


def get_lstm(lstm_type: str, input_size: int, hidden_size: int, num_layers: int, norm_type=None, dropout=0.0):
    assert lstm_type in ('normal', 'pytorch', 'lnlstm'), lstm_type
    if lstm_type == 'normal':
        return NormLSTM(input_size, hidden_size, num_layers, norm_type, dropout=dropout)
    if lstm_type == 'pytorch':
        return PytorchLSTM(input_size, hidden_size, num_layers, dropout=dropout)
    return StackedLNLSTM(input_size, hidden_size, num_layers)


class LSTMCell(nn.Module):
    """Plain LSTM cell (``lstm.py:60-86``): keys weight_ih, weight_hh, bias_ih, bias_hh; gates i, f, g, o."""

    def __init__(self, input_size: int, hidden_size: int):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.weight_ih = nn.Parameter(torch.randn(4 * hidden_size, input_size))
        self.weight_hh = nn.Parameter(torch.randn(4 * hidden_size, hidden_size))
        self.bias_ih = nn.Parameter(torch.randn(4 * hidden_size))
        self.bias_hh = nn.Parameter(torch.randn(4 * hidden_size))

    def run(self, x, h, c):
        """x [T,B,I] -> (out [T,B,H], h, c); the input GEMM is hoisted over all T."""
        xg = F.linear(x, self.weight_ih, self.bias_ih + self.bias_hh)
        outs = []
        for t in range(x.shape[0]):
            i, f, g, o = (xg[t] + h @ self.weight_hh.t()).chunk(4, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            h = torch.sigmoid(o) * torch.tanh(c)
            outs.append(h)
        return torch.stack(outs, 0), h, c


class _PlainLayer(nn.Module):
    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.cell = LSTMCell(input_size, hidden_size)

    def forward(self, x, h0, c0):
        return self.cell.run(x, h0, c0)


class BidirLayer(nn.Module):
    """Forward + time-reversed layer, outputs concatenated on channels (``lstm.py:185-208``).
    Keys ``directions.{0,1}.cell.*``."""

    def __init__(self, layer_cls, input_size, hidden_size):
        super().__init__()
        self.directions = nn.ModuleList([layer_cls(input_size, hidden_size), layer_cls(input_size, hidden_size)])

    def forward(self, x, states):
        (hf, cf), (hb, cb) = states
        of, hf, cf = self.directions[0](x, hf, cf)
        ob, hb, cb = self.directions[1](x.flip(0), hb, cb)
        return torch.cat([of, ob.flip(0)], -1), [(hf, cf), (hb, cb)]


class RecurrentStack(nn.Module):
    """Stack of (optionally bidirectional) recurrent layers with optional inter-layer dropout (p=0.4,
    all but the last layer), matching ``StackedLSTM`` / ``StackedLSTM2`` / ``StackedLSTMWithDropout``.
    ``states``: per layer (h, c), or per layer [(h, c) fwd, (h, c) bwd] when bidirectional."""

    def __init__(self, layer_cls, input_size, hidden_size, num_layers, bidirectional=False, dropout=False):
        super().__init__()
        dirs = 2 if bidirectional else 1
        self.bidirectional = bidirectional
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        sizes = [input_size] + [hidden_size * dirs] * (num_layers - 1)
        if bidirectional:
            self.layers = nn.ModuleList([BidirLayer(layer_cls, s, hidden_size) for s in sizes])
        else:
            self.layers = nn.ModuleList([layer_cls(s, hidden_size) for s in sizes])
        if dropout and num_layers == 1:
            warnings.warn('dropout LSTM applies dropout between layers; num_layers=1 has none')
        self.dropout_layer = nn.Dropout(0.4) if dropout else None

    def zero_state(self, batch, device, dtype=torch.float32):
        z = torch.zeros(batch, self.hidden_size, device=device, dtype=dtype)
        return [[(z, z), (z, z)] if self.bidirectional else (z, z) for _ in range(self.num_layers)]

    def forward(self, x, states):
        out_states = []
        for i, (layer, st) in enumerate(zip(self.layers, states)):
            if self.bidirectional:
                x, st = layer(x, st)
            else:
                x, h, c = layer(x, *st)
                st = (h, c)
            if self.dropout_layer is not None and i < self.num_layers - 1:
                x = self.dropout_layer(x)
            out_states.append(st)
        return x, out_states


def script_lstm(input_size, hidden_size, num_layers, dropout=False, bidirectional=False) -> RecurrentStack:
    """Plain-cell LSTM stack (``lstm.py:14-33``)."""
    return RecurrentStack(_PlainLayer, input_size, hidden_size, num_layers, bidirectional=bidirectional,
                          dropout=dropout and not bidirectional)


def script_lnlstm(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=False,
                  bidirectional=False, decompose_layernorm=False):
    """LayerNorm-LSTM stack (``lstm.py:36-57``).  Unidirectional stacks are :class:`StackedLNLSTM`
    (fused native recurrence); bidirectional stacks run both directions through the same layer op."""
    assert bias and not batch_first and not dropout, 'not implemented in the reference either'
    if not bidirectional:
        return StackedLNLSTM(input_size, hidden_size, num_layers)
    return RecurrentStack(_Layer, input_size, hidden_size, num_layers, bidirectional=True)


# ---------------------------------------------------------------------------------------------- misc
class SoftArgmax(nn.Module):
    """Expected (y, x) location under softmax of a 1-channel heat map [B,1,H,W] -> [B,2]
    (``torch_utils/network/soft_argmax.py``)."""

    def forward(self, x):
        B, C, H, W = x.shape
        assert C == 1
        p = torch.softmax(x.reshape(B, -1).float(), -1).view(B, H, W)
        ys = torch.arange(H, device=x.device, dtype=p.dtype)
        xs = torch.arange(W, device=x.device, dtype=p.dtype)
        return torch.stack([(p.sum(2) * ys).sum(1), (p.sum(1) * xs).sum(1)], 1).to(x.dtype)


class ScatterConnection(nn.Module):
    """Scatter per-entity features [B,M,N] to a [B,N,H,W] map at (y, x) locations [B,M,2]
    (``torch_utils/network/scatter_connection.py``).  'add' sums collisions, 'cover' keeps one."""

    def __init__(self, scatter_type: str):
        super().__init__()
        assert scatter_type in ('cover', 'add')
        self.scatter_type = scatter_type

    def forward(self, x, spatial_size, location):
        B, M, N = x.shape
        H, W = spatial_size
        idx = (location[..., 0].long() * W + location[..., 1].long()) + \
            torch.arange(B, device=x.device)[:, None] * (H * W)
        out = x.new_zeros(B * H * W, N)
        flat = idx.reshape(-1)
        if self.scatter_type == 'add':
            out.index_add_(0, flat, x.reshape(-1, N))
        else:
            out.index_copy_(0, flat, x.reshape(-1, N))
        return out.view(B, H, W, N).permute(0, 3, 1, 2)


class Swish(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(x)


def build_activation(activation: str, inplace: Optional[bool] = None):
    """Activation by name (``torch_utils/network/activation.py:72``); 'glu' returns the GLU class."""
    from .blocks import GLU
    if inplace is not None:
        assert activation == 'relu', f'inplace is not compatible with {activation}'
    table = {'relu': lambda: nn.ReLU(inplace=True if inplace is None else inplace), 'glu': lambda: GLU,
             'prelu': lambda: nn.PReLU(), 'swish': lambda: Swish(), 'tanh': lambda: nn.Tanh(),
             'sigmoid': lambda: nn.Sigmoid()}
    if activation not in table:
        raise KeyError(f'invalid key for activation: {activation}')
    return table[activation]()
