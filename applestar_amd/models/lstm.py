"""Stacked LayerNorm-LSTM (core LSTM and the selected-units query LSTM).

Keys ``layers.{l}.cell.{weight_ih,weight_hh,layernorm_i,layernorm_h,layernorm_c}`` as in
``distar/agent/default/model/lstm.py:114-153,211-234``.  The reference steps a Python loop of
per-timestep cells per layer; here each layer is one ``ops.lnlstm_layer`` call: the input GEMM and
its LayerNorm are hoisted over all T, and the recurrence runs in the fused HIP kernel on GPU.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn as nn

from .. import ops


class LNLSTMCell(nn.Module):
    def __init__(self, input_size: int, hidden_size: int):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.weight_ih = nn.Parameter(torch.randn(4 * hidden_size, input_size))
        self.weight_hh = nn.Parameter(torch.randn(4 * hidden_size, hidden_size))
        self.layernorm_i = nn.LayerNorm(4 * hidden_size)
        self.layernorm_h = nn.LayerNorm(4 * hidden_size)
        self.layernorm_c = nn.LayerNorm(hidden_size)


class _Layer(nn.Module):
    def __init__(self, input_size: int, hidden_size: int):
        super().__init__()
        self.cell = LNLSTMCell(input_size, hidden_size)

    def forward(self, x, h0, c0):
        c = self.cell
        return ops.lnlstm_layer(x, h0, c0, c.weight_ih, c.weight_hh,
                                c.layernorm_i.weight, c.layernorm_i.bias,
                                c.layernorm_h.weight, c.layernorm_h.bias,
                                c.layernorm_c.weight, c.layernorm_c.bias)


class StackedLNLSTM(nn.Module):
    def __init__(self, input_size: int, hidden_size: int, num_layers: int):
        super().__init__()
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.layers = nn.ModuleList([_Layer(input_size if i == 0 else hidden_size, hidden_size)
                                     for i in range(num_layers)])

    def zero_state(self, batch: int, device, dtype=torch.float32) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        z = torch.zeros(batch, self.hidden_size, device=device, dtype=dtype)
        return [(z, z) for _ in range(self.num_layers)]

    def forward(self, x: torch.Tensor, state: Sequence[Tuple[torch.Tensor, torch.Tensor]]):
        """x [T,B,I]; state: per layer (h [B,H], c [B,H]).  Returns (out [T,B,H], new state)."""
        out_state = []
        for layer, (h, c) in zip(self.layers, state):
            x, h, c = layer(x, h, c)
            out_state.append((h, c))
        return x, out_state
