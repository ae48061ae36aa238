"""Parameter-holding building blocks.

State-dict key layout is kept identical to the reference so ``rl_model.pth`` / ``sl_model.pth`` load
directly (``distar/ctools/torch_utils/network/nn_module.py:231-314``: a "fc block" is an
``nn.Sequential`` whose index 0 is the Linear, index 1 an optional LayerNorm, then the activation;
``res_block.py:11-140`` for the residual variants; ``model/module_utils.py:204-231,508-524`` for
the gated res-block and GLU).  The forward passes are written for the MI355X path: activations are
computed through :mod:`applestar_amd.ops` (fused bias+act GEMM epilogues, fused LayerNorm), so
the nn.Module objects here are mostly parameter containers.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops

__all__ = ['FCBlock', 'ConvBlock', 'ResFCBlock', 'ResFCBlock2', 'ResBlock', 'MaxPool2x2', 'GLU', 'GatedResBlock',
           'OneHotTable', 'binary_table']


def _xavier_normal(w: torch.Tensor, gain: float = 1.0):
    nn.init.xavier_normal_(w, gain)


class FCBlock(nn.Sequential):
    """Linear (-> LayerNorm) (-> ReLU). Keys: ``0.weight``, ``0.bias`` [, ``1.weight``, ``1.bias``]."""

    def __init__(self, in_dim: int, out_dim: int, act: bool = False, norm: bool = False,
                 init: str = 'xavier_normal', gain: float = 1.0):
        layers = [nn.Linear(in_dim, out_dim)]
        if init == 'xavier_normal':
            _xavier_normal(layers[0].weight)
        else:  # fc_block2 style (value head output): xavier_uniform(gain), zero bias
            nn.init.xavier_uniform_(layers[0].weight, gain)
            nn.init.zeros_(layers[0].bias)
        if norm:
            layers.append(nn.LayerNorm(out_dim))
        if act:
            layers.append(nn.ReLU(inplace=False))
        super().__init__(*layers)
        self.act = act
        self.norm = norm

    @property
    def linear(self) -> nn.Linear:
        return self[0]

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # noqa: D401
        lin = self[0]
        if self.norm:
            y = ops.linear(x, lin.weight, lin.bias)
            return ops.layer_norm(y, self[1].weight, self[1].bias, act='relu' if self.act else None)
        return ops.linear(x, lin.weight, lin.bias, act='relu' if self.act else None)


class ConvBlock(nn.Sequential):
    """Conv2d (-> ReLU). Keys ``0.weight``, ``0.bias``."""

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, pad: int = 0, act: bool = False):
        conv = nn.Conv2d(cin, cout, k, stride, pad)
        _xavier_normal(conv.weight)
        layers = [conv] + ([nn.ReLU(inplace=False)] if act else [])
        super().__init__(*layers)
        self.act = act

    def forward(self, x: torch.Tensor, residual=None) -> torch.Tensor:
        c = self[0]
        return ops.conv2d(x, c.weight, c.bias, stride=c.stride[0], padding=c.padding[0],
                          act='relu' if self.act else None, residual=residual)


class ResFCBlock(nn.Module):
    """x -> fc1(LN,ReLU) -> fc2(LN) -> +x -> ReLU  (res_block.py:71-109)."""

    def __init__(self, dim: int, norm: bool = True):
        super().__init__()
        self.fc1 = FCBlock(dim, dim, act=True, norm=norm)
        self.fc2 = FCBlock(dim, dim, act=False, norm=norm)

    def forward(self, x):
        y = self.fc2(self.fc1(x))
        return F.relu(y + x)


class ResFCBlock2(nn.Module):
    """x -> fc1(ReLU) -> fc2 -> LN(+x)  (res_block.py:111-140); keys fc1.0, fc2.0, norm."""

    def __init__(self, dim: int):
        super().__init__()
        self.fc1 = FCBlock(dim, dim, act=True)
        self.fc2 = FCBlock(dim, dim, act=False)
        self.norm = nn.LayerNorm(dim)

    def forward(self, x):
        y = self.fc2(self.fc1(x))
        return ops.layer_norm(y, self.norm.weight, self.norm.bias, residual=x)


class ResBlock(nn.Module):
    """conv3x3-ReLU-conv3x3 + skip -> ReLU (res_block.py:13-65)."""

    def __init__(self, dim: int):
        super().__init__()
        self.conv1 = ConvBlock(dim, dim, 3, 1, 1, act=True)
        self.conv2 = ConvBlock(dim, dim, 3, 1, 1, act=False)

    def forward(self, x):
        c1, c2 = self.conv1[0], self.conv2[0]
        n = ops._native(x)
        if n is not None and n.has('resblock'):
            y = n.resblock(x, c1.weight, c1.bias, c2.weight, c2.bias)   # one node: skip grad fused in dX
            if y is not None:
                return y
        # relu(conv2(y) + x): residual and ReLU fused into the conv epilogue on the GPU
        return ops.conv2d(self.conv1(x), c2.weight, c2.bias, 1, 1, act='relu', residual=x)


class MaxPool2x2(nn.Module):
    """max_pool2d(x, 2, 2) (parameter-free: keeps the reference's Sequential indices)."""

    def forward(self, x):
        return ops.max_pool2x2(x)


class GLU(nn.Module):
    """out = layer2(sigmoid(layer1(context)) * x)   (module_utils.py:508-524)."""

    def __init__(self, input_dim: int, output_dim: int, context_dim: int):
        super().__init__()
        self.layer1 = FCBlock(context_dim, input_dim)
        self.layer2 = FCBlock(input_dim, output_dim)

    def forward(self, x, context):
        g = ops.linear(context, self.layer1[0].weight, self.layer1[0].bias, act='sigmoid')
        if g.dtype == torch.bfloat16 and x.dtype == torch.float32 and x.is_cuda and not torch.is_grad_enabled():
            # bf16 inference, fp32 x (the core LSTM output): the same fp32 product after an exact upcast of the gate -
            # torch's mixed-dtype (templated) product kernel ran 37 us at B = 1, these are two ~5 us launches.  (x
            # rounded to bf16 first instead moved the selected-units logits: test_full_model_bf16_gpu_vs_cpu_fp32)
            g = g.float()
        return self.layer2(g * x)


FUSED_GATED_RESBLOCK = True


class GatedResBlock(nn.Module):
    """Location-head gated residual block (module_utils.py:204-231)::

        y = conv2(relu(conv1(x)));  g = sigmoid(G4(relu(G3(relu(G2(relu(G1(x))))))))
        out = relu(tanh(y * g) * UpdateSP + x)
    """

    def __init__(self, dim: int):
        super().__init__()
        self.conv1 = ConvBlock(dim, dim, 3, 1, 1, act=True)
        self.conv2 = ConvBlock(dim, dim, 3, 1, 1, act=False)
        self.GateWeightG = nn.Sequential(ConvBlock(dim, dim, 1, act=True), ConvBlock(dim, dim, 1, act=True),
                                         ConvBlock(dim, dim, 1, act=True), ConvBlock(dim, dim, 1, act=False))
        self.UpdateSP = nn.Parameter(torch.full((1,), 0.1))

    def forward(self, x, post=None):
        """``post``: added to the output (the location head's next skip map), in the output pass when fused."""
        n = ops._native(x)
        if n is not None and n.has('gated_resblock') and FUSED_GATED_RESBLOCK:
            out = n.gated_resblock(x, self.conv1[0], self.conv2[0], [m[0] for m in self.GateWeightG], self.UpdateSP,
                                   post)
            if out is not None:
                return out
            if post is not None:
                out = n.gated_resblock(x, self.conv1[0], self.conv2[0], [m[0] for m in self.GateWeightG],
                                       self.UpdateSP)
                if out is not None:
                    return out + post
        y = self.conv2(self.conv1(x))
        g = self.GateWeightG(x)
        out = ops.gated_residual(y, g, self.UpdateSP, x)
        return out if post is None else out + post


class OneHotTable(nn.Module):
    """Frozen lookup table kept only so checkpoints have the reference's ``<name>.weight`` keys
    (``nn.Embedding.from_pretrained(eye(n), freeze=True)``).  Never used in a GEMM: one-hot @ W is
    computed as a row gather by the fused embedding kernels."""

    def __init__(self, table: torch.Tensor):
        super().__init__()
        self.register_buffer('weight', table, persistent=True)

    def forward(self, idx):
        return self.weight[idx.long()]

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        # accept the reference's frozen Parameter under the same key
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


def binary_table(bits: int) -> torch.Tensor:
    """[2**bits, bits] MSB-first binary codes (entity_encoder.py:10-15)."""
    n = torch.arange(2 ** bits).unsqueeze(1)
    shifts = torch.arange(bits - 1, -1, -1).unsqueeze(0)
    return ((n >> shifts) & 1).float()


def eye_table(n: int) -> torch.Tensor:
    return torch.eye(n)


def glorot_uniform_(p: torch.Tensor):
    stdv = 1.0 / math.sqrt(p.shape[-1])
    with torch.no_grad():
        p.uniform_(-stdv, stdv)
