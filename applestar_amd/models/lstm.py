"""Stacked LayerNorm-LSTM (core LSTM and the selected-units query LSTM).

Keys ``layers.{l}.cell.{weight_ih,weight_hh,layernorm_i,layernorm_h,layernorm_c}`` as in
``distar/agent/default/model/lstm.py:114-153,211-234``.  The reference steps a Python loop of
per-timestep cells per layer; here each layer is one ``ops.lnlstm_layer`` call: the input GEMM and
its LayerNorm are hoisted over all T, and the recurrence runs in the fused HIP kernel on GPU.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn as nn

from .. import ops

# Optional wavefront schedule: the stacked layers over time chunks on one HIP stream per layer (layer l,
# chunk c overlaps layer l-1, chunk c+1; autograd replays each node's backward on its forward stream).
# Off by default: measured 37.8 / 45.7 vs 33.5 / 32.8 ms/step (r2bg, A/B/A/B) - three concurrent split
# recurrences (8 co-resident workgroups per row each) compete with the encoders' side streams for CUs
# and their cross-workgroup polls stall.  APPLESTAR_LSTM_PIPELINE=<chunks> turns it on.
PIPELINE_CHUNKS = int(os.environ.get('APPLESTAR_LSTM_PIPELINE', '1'))
_STREAMS: Dict[tuple, 'torch.cuda.Stream'] = {}


def _layer_stream(dev, layer: int):
    key = (dev.index, layer)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(dev)
    return _STREAMS[key]


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
        T = x.shape[0]
        if PIPELINE_CHUNKS > 1 and x.is_cuda and self.num_layers > 1 and T >= 2 * PIPELINE_CHUNKS and \
                not torch.cuda.is_current_stream_capturing():
            return self._forward_pipelined(x, state, PIPELINE_CHUNKS)
        out_state = []
        for layer, (h, c) in zip(self.layers, state):
            x, h, c = layer(x, h, c)
            out_state.append((h, c))
        return x, out_state

    def _forward_pipelined(self, x, state, nchunk: int):
        """Same math as the layer-by-layer pass (the recurrent state is handed from chunk to chunk in fp32,
        the input GEMM + LayerNorm act on row blocks), scheduled as a wavefront over streams."""
        dev = x.device
        main = torch.cuda.current_stream(dev)
        streams = [main] + [_layer_stream(dev, l) for l in range(1, self.num_layers)]
        for st in streams[1:]:
            st.wait_stream(main)
        T = x.shape[0]
        base, extra = divmod(T, nchunk)
        sizes = [base + (1 if i < extra else 0) for i in range(nchunk)]
        hs = [h for h, _ in state]
        cs = [c for _, c in state]
        for l in range(1, self.num_layers):
            for t in (hs[l], cs[l]):
                if t.is_cuda:
                    t.record_stream(streams[l])
        outs = []
        for xc in x.split(sizes, 0):
            inp = xc
            for l, layer in enumerate(self.layers):
                st = streams[l]
                if l > 0:
                    st.wait_stream(streams[l - 1])     # layer l-1 has issued chunks <= this one
                    inp.record_stream(st)
                with torch.cuda.stream(st):
                    inp, hs[l], cs[l] = layer(inp, hs[l], cs[l])
            outs.append(inp)
        for st in streams[1:]:
            main.wait_stream(st)
        for t in outs + hs + cs:
            t.record_stream(main)
        return torch.cat(outs, 0), list(zip(hs, cs))
