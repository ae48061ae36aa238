"""Fused ``pytorch_norm`` gradient clip + Adam step on the GPU (csrc/kernels/optim.hip).

The RL learner's update (``distar/agent/default/rl_learner.py:114-132``; ``ctools/torch_utils/grad_clip.py``)
is: global L2 norm of every gradient, scale by ``min(1, threshold / (norm + 1e-6))``, then Adam.  As torch ops
that is a ``_foreach_norm`` + stack + pow/sum + clamp + ``_foreach_mul_`` + the fused Adam (~10 launches);
here it is two launches over a (tensor, offset) chunk table that is built once (parameters, gradients and
moments never move).

The moments ARE the wrapped ``torch.optim.Adam``'s own ``exp_avg`` / ``exp_avg_sq`` state tensors and the
step count its ``step``, so ``optimizer.state_dict()`` / ``load_state_dict`` (checkpoints, league resets) are
unchanged and either path can continue the other's run.  Learning rate and weight decay are read from the
optimizer's param group at every step (LR schedulers keep working).  Applies to a single param group of fp32
CUDA tensors with dense fp32 gradients, plain Adam / AdamW without amsgrad and without the reference
optimizer's own clip / ignore options (``utils.optim.Adam`` defaults); anything else keeps the torch path.
"""
from __future__ import annotations

from typing import Optional

import torch


class FusedClipAdam:
    def __init__(self, optimizer: torch.optim.Optimizer, max_norm: Optional[float]):
        self.opt = optimizer
        self.max_norm = float(max_norm) if max_norm else 0.0
        self._table = None
        self._sig = None

    @staticmethod
    def supported(optimizer, clip) -> bool:
        if not isinstance(optimizer, torch.optim.Adam) or len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        if g.get('amsgrad') or g.get('maximize') or g.get('capturable') or g.get('differentiable'):
            return False
        if getattr(optimizer, 'clip_type', None) or getattr(optimizer, 'ignore_type', None):
            return False
        if clip.clip_type not in ('pytorch_norm', 'clip_norm', 'none') or clip.norm_type != 2.0:
            return False
        return all(p.is_cuda and p.dtype == torch.float32 for p in g['params'])

    def _build(self, params):
        from ..ops import native
        C = native.ensure_loaded()
        chunk = C.fused_adam_chunk()
        st = self.opt.state
        rows, chunks = [], []
        for t, p in enumerate(params):
            s = st[p]
            if 'exp_avg' not in s:                       # torch.optim.Adam's lazy state, created the same way
                s['step'] = torch.tensor(0.0, dtype=torch.float32)
                s['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                s['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            for name, x in (('param', p), ('grad', p.grad), ('exp_avg', s['exp_avg']), ('exp_avg_sq', s['exp_avg_sq'])):
                dense = x.is_contiguous() or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last))
                if x.dtype != torch.float32 or not dense or x.stride() != p.stride():
                    raise RuntimeError(f'FusedClipAdam: {name} of a {tuple(p.shape)} parameter is not an fp32 tensor '
                                       f'laid out like its parameter')
            rows += [p.data_ptr(), p.grad.data_ptr(), s['exp_avg'].data_ptr(), s['exp_avg_sq'].data_ptr(), p.numel(), 0]
            for off in range(0, p.numel(), chunk):
                chunks += [t, off]
        dev = params[0].device
        self._table = torch.tensor(rows, dtype=torch.int64, device=dev)
        self._chunks = torch.tensor(chunks, dtype=torch.int64, device=dev)
        self._part = torch.empty(len(chunks) // 2, dtype=torch.float32, device=dev)
        self._C = C

    def _signature(self, params):
        st = self.opt.state
        return tuple((p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0,
                      st[p]['exp_avg'].data_ptr() if 'exp_avg' in st[p] else 0) for p in params)

    @torch.no_grad()
    def step(self, gate: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Clip + Adam in place; returns the pre-clip global gradient norm (0-d device tensor)."""
        g = self.opt.param_groups[0]
        params = [p for p in g['params'] if p.requires_grad]
        if any(p.grad is None for p in params):
            raise RuntimeError('FusedClipAdam: every parameter needs a gradient buffer (the reducer keeps them)')
        sig = self._signature(params)
        if self._table is None or sig != self._sig:
            self._build(params)
            self._sig = self._signature(params)
        st = self.opt.state
        step = float(st[params[0]]['step']) + 1.0
        for p in params:
            st[p]['step'] += 1.0
        b1, b2 = g['betas']
        lr, eps, wd = float(g['lr']), float(g['eps']), float(g['weight_decay'])
        decoupled = bool(getattr(self.opt, '_decoupled_wd', 0.0)) or isinstance(self.opt, torch.optim.AdamW)
        if decoupled:
            wd = lr * float(getattr(self.opt, '_decoupled_wd', 0.0) or g['weight_decay'])
        bc1 = 1.0 - b1 ** step
        bc2 = 1.0 - b2 ** step
        norm = torch.empty((), dtype=torch.float32, device=self._part.device)   # per step: callers may keep it
        self._C.fused_clip_adam(self._table, self._chunks, self._part,
                                gate.reshape(1).float() if gate is not None else None, norm.view(1),
                                self.max_norm, lr / bc1, b1, b2, 1.0 / bc2 ** 0.5, eps, wd, decoupled)
        return norm
