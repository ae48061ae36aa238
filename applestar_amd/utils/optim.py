"""Adam / AdamW with the reference's gradient clip and gradient "ignore" options
(``distar/ctools/torch_utils/optimizer_util.py:43-317``; exported but unused by the default configs).

Options: ``grad_clip_type`` in {None, 'clip_value', 'clip_norm', 'clip_momentum', 'clip_momentum_norm'},
``grad_ignore_type`` in {None, 'ignore_value', 'ignore_norm', 'ignore_momentum', 'ignore_momentum_norm'}.
The "momentum" variants track a separate EMA of the squared (unclipped) gradient per parameter and
compare against ``coef * sqrt(v / bias_correction2)``.

Differences from the reference, by design:
* every decision is made on the device (multipliers instead of ``if tensor:``), so a step issues no
  host synchronisation; the reference calls ``.item()`` per parameter;
* ``ignore_momentum`` tests whether ANY element exceeds its bound (the reference's ``if grad.abs() >
  bound`` raises for non-scalar parameters);
* ``clip_momentum`` keeps the reference's replacement value ``+bound`` for clipped elements (it drops
  the sign); set ``clip_momentum_keep_sign=True`` for a sign-preserving clamp.
The update itself is ``torch.optim.Adam`` (fused / foreach on the GPU).
"""
from __future__ import annotations

import math
from typing import Callable, Iterable, Optional, Tuple

import torch

CLIP_TYPES = (None, 'clip_value', 'clip_norm', 'clip_momentum', 'clip_momentum_norm')
IGNORE_TYPES = (None, 'ignore_value', 'ignore_norm', 'ignore_momentum', 'ignore_momentum_norm')


def _norm(grads, p: float) -> torch.Tensor:
    if not grads:
        return torch.zeros(())
    if p == math.inf:
        return torch.stack([g.abs().max().float() for g in grads]).max()
    return torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g.float(), p) for g in grads]), p)


def grad_ignore_norm(parameters, max_norm: float, norm_type: float = 2.0) -> torch.Tensor:
    """Zero every gradient if the global norm exceeds ``max_norm``; returns the norm (device tensor)."""
    grads = [p.grad for p in parameters if p.grad is not None]
    total = _norm(grads, float(norm_type))
    keep = (total + 1e-6 <= float(max_norm)).to(torch.float32)
    if grads:
        torch._foreach_mul_(grads, keep.to(grads[0].device))
    return total


def grad_ignore_value(parameters, clip_value: float) -> None:
    """Zero every gradient if any element reaches ``clip_value`` in magnitude."""
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return
    peak = torch.stack([g.abs().max().float() for g in grads]).max()
    torch._foreach_mul_(grads, (peak < float(clip_value)).to(torch.float32))


class Adam(torch.optim.Adam):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, amsgrad: bool = False, optim_type: str = 'adam',
                 grad_clip_type: Optional[str] = None, clip_value: Optional[float] = None, clip_coef: float = 5.0,
                 clip_norm_type: float = 2.0, clip_momentum_timestep: int = 100, grad_norm_type=None,
                 grad_ignore_type: Optional[str] = None, ignore_value: Optional[float] = None,
                 ignore_coef: float = 5.0, ignore_norm_type: float = 2.0, ignore_momentum_timestep: int = 100,
                 clip_momentum_keep_sign: bool = False, **torch_kwargs):
        assert optim_type in ('adam', 'adamw'), optim_type
        assert grad_clip_type in CLIP_TYPES, grad_clip_type
        assert grad_ignore_type in IGNORE_TYPES, grad_ignore_type
        assert grad_norm_type is None
        if grad_clip_type:
            assert clip_value is not None, 'grad_clip_type needs clip_value'
        if grad_ignore_type:
            assert ignore_value is not None, 'grad_ignore_type needs ignore_value'
        self.optim_type = optim_type
        self.clip_type, self.clip_value, self.clip_coef = grad_clip_type, clip_value, clip_coef
        self.clip_norm_type, self.clip_momentum_timestep = float(clip_norm_type), clip_momentum_timestep
        self.ignore_type, self.ignore_value, self.ignore_coef = grad_ignore_type, ignore_value, ignore_coef
        self.ignore_norm_type, self.ignore_momentum_timestep = float(ignore_norm_type), ignore_momentum_timestep
        self.keep_sign = clip_momentum_keep_sign
        self._decoupled_wd = weight_decay if optim_type == 'adamw' else 0.0
        super().__init__(params, lr=lr, betas=betas, eps=eps,
                         weight_decay=0.0 if optim_type == 'adamw' else weight_decay, amsgrad=amsgrad,
                         **torch_kwargs)
        self._thre = {}      # param -> EMA of grad^2 for the momentum variants
        self._thre_step = 0  # completed optimizer steps (the reference reads Adam's own step counter)

    # ---------------------------------------------------------------- helpers
    def _params(self):
        return [p for g in self.param_groups for p in g['params'] if p.requires_grad and p.grad is not None]

    def _update_thre(self):
        """EMA of squared gradients (all params with grads); returns {param: bound / coef}."""
        bc2 = 1.0 - self.param_groups[0]['betas'][1] ** self._thre_step
        out = {}
        for group in self.param_groups:
            beta2 = group['betas'][1]
            for p in group['params']:
                if p.grad is None:
                    continue
                v = self._thre.get(p)
                if v is None:
                    v = self._thre[p] = torch.zeros_like(p, dtype=torch.float32)
                g = p.grad.float()
                v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
                out[p] = v.sqrt() / math.sqrt(bc2) if bc2 > 0 else torch.full_like(v, math.inf)
        return out

    # ---------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, closure: Optional[Callable] = None):
        params = self._params()
        ct, it = self.clip_type, self.ignore_type
        momentum = {}
        if ct in ('clip_momentum', 'clip_momentum_norm') or it in ('ignore_momentum', 'ignore_momentum_norm'):
            momentum = self._update_thre()
        if ct == 'clip_value':
            torch.nn.utils.clip_grad_value_(params, self.clip_value)
        elif ct == 'clip_norm':
            torch.nn.utils.clip_grad_norm_(params, self.clip_value, self.clip_norm_type)
        elif ct == 'clip_momentum' and self._thre_step >= self.clip_momentum_timestep:
            for p in params:
                bound = momentum[p] * self.clip_coef
                g = p.grad
                if self.keep_sign:
                    g.copy_(torch.maximum(torch.minimum(g.float(), bound), -bound))
                else:
                    g.copy_(torch.where(g.float().abs() > bound, bound, g.float()))
        elif ct == 'clip_momentum_norm' and self._thre_step > self.clip_momentum_timestep:
            self._scale_by_momentum_norm(momentum, self.clip_coef, self.clip_norm_type, zero=False)
        if it == 'ignore_value':
            grad_ignore_value(params, self.ignore_value)
        elif it == 'ignore_norm':
            grad_ignore_norm(params, self.ignore_value, self.ignore_norm_type)
        elif it == 'ignore_momentum' and self._thre_step >= self.ignore_momentum_timestep and params:
            over = torch.stack([(p.grad.float().abs() > momentum[p] * self.ignore_coef).any() for p in params]).any()
            torch._foreach_mul_([p.grad for p in params], (~over).to(torch.float32))
        elif it == 'ignore_momentum_norm' and self._thre_step > self.ignore_momentum_timestep:
            self._scale_by_momentum_norm(momentum, self.ignore_coef, self.ignore_norm_type, zero=True)
        if self._decoupled_wd:
            for group in self.param_groups:
                ps = [p for p in group['params'] if p.grad is not None]
                if ps:
                    torch._foreach_mul_(ps, 1.0 - self._decoupled_wd * group['lr'])
        self._thre_step += 1
        return super().step(closure)

    def _scale_by_momentum_norm(self, momentum, coef, norm_type, zero: bool):
        """Per group: ratio = ||coef * sqrt(v)|| / ||g||; if ratio < 1 scale grads by it (clip) or zero them."""
        for group in self.param_groups:
            ps = [p for p in group['params'] if p.grad is not None]
            if not ps:
                continue
            gnorm = _norm([p.grad for p in ps], norm_type)
            mnorm = _norm([momentum[p] * coef for p in ps], norm_type)
            ratio = mnorm / (gnorm + 1e-6)
            mult = torch.where(ratio < 1, torch.zeros_like(ratio) if zero else ratio, torch.ones_like(ratio))
            torch._foreach_mul_([p.grad for p in ps], mult)

    def get_grad(self) -> float:
        """Sum over parameters of ||g||^p (the reference returns the un-rooted sum)."""
        return float(sum(torch.linalg.vector_norm(p.grad.float(), self.clip_norm_type) ** self.clip_norm_type
                         for p in self._params()))

    def state_dict(self):
        sd = super().state_dict()
        ids = {id(p): i for i, p in enumerate(p for g in self.param_groups for p in g['params'])}
        sd['thre'] = {ids[id(p)]: v for p, v in self._thre.items()}
        sd['thre_step'] = self._thre_step
        return sd

    def load_state_dict(self, sd):
        sd = dict(sd)
        thre = sd.pop('thre', {})
        self._thre_step = int(sd.pop('thre_step', 0))
        super().load_state_dict(sd)
        plist = [p for g in self.param_groups for p in g['params']]
        self._thre = {plist[int(i)]: v.to(plist[int(i)].device) for i, v in thre.items()}


def build_optimizer(params, lc, betas=(0.9, 0.999), eps: float = 1e-8, device=None,
                    capturable: bool = False) -> torch.optim.Optimizer:
    """Learner optimizer from the config: plain (fused on the GPU) Adam by default; the extended
    :class:`Adam` when ``learner.optimizer`` asks for AdamW or a clip / ignore variant, e.g.
    ``optimizer: {optim_type: adamw, grad_ignore_type: ignore_norm, ignore_value: 50}``."""
    ocfg = dict(lc.get('optimizer') or {})
    fused = device is not None and torch.device(device).type == 'cuda'
    betas = tuple(ocfg.pop('betas', betas))
    eps = float(ocfg.pop('eps', eps))
    kw = dict(lr=lc.learning_rate, betas=betas, eps=eps, weight_decay=lc.get('weight_decay', 0.0))
    if not ocfg or (ocfg.get('optim_type', 'adam') == 'adam' and not ocfg.get('grad_clip_type')
                    and not ocfg.get('grad_ignore_type')):
        # capturable: the step counter stays on the device so the update can be replayed from a HIP graph
        return torch.optim.Adam(params, fused=fused, capturable=bool(capturable and fused), **kw)
    return Adam(params, fused=fused, **kw, **ocfg)
