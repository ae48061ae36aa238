"""Gradient clipping policies (``distar/ctools/torch_utils/grad_clip.py:7-150``):
``none``, ``max_norm`` (EMA-scaled), ``momentum_norm`` (per-parameter norm vs its EMA, used by SL),
``clip_value`` (Adam-like second-moment clamp), ``clip_const`` and ``pytorch_norm`` (RL, threshold 1).

``momentum_norm`` has two modes (``momentum_mode`` in the clip config):

* ``'reference'`` (default): what the reference's code actually does.  Its ``apply`` resets ``norm_mom`` to
  ``[None] * n`` on the first step and then *appends* the new norms (``grad_clip.py:79-106``), so
  ``norm_mom[idx]`` stays ``None`` for every parameter forever and every scale is 1.0: no gradient is ever
  scaled, and the reported norm is the plain global norm.  (The list also grows by n every step; not
  reproduced.)  Pinned by ``tests/test_utils.py::test_momentum_norm_reference_mode_matches_reference_apply``.
* ``'ema'``: the evident intent - each tensor's gradient norm is held to ``threshold`` x the EMA of its past
  clipped norms (``mom = 0.99 mom + 0.01 |g| s``).  The EMA and an "initialised" flag live on the device; a
  gated-off step (timed-out LSTM exchange) changes neither, so a gated FIRST step does not initialise the EMA.

All policies are device-side and sync-free: per-tensor norms come from one ``_foreach_norm`` and the
EMA state lives on the device, so a clip never forces a host round trip (the reference calls
``.item()`` once per parameter).  ``apply`` returns the pre-clip global norm as a 0-d tensor.
"""
from __future__ import annotations

import math
from typing import Optional, Iterable, List

import torch

CLIP_TYPES = ('none', 'max_norm', 'momentum_norm', 'clip_value', 'clip_const', 'pytorch_norm', 'clip_norm')


def build_grad_clip(cfg) -> 'GradClip':
    cfg = cfg or {}
    norm_type = cfg.get('norm_type', 2)
    if norm_type == 'inf':
        norm_type = math.inf
    return GradClip(cfg.get('type', 'none'), cfg.get('threshold', 1.4), norm_type, cfg.get('begin_step', 100),
                    cfg.get('ignore_threshold', 3), momentum_mode=cfg.get('momentum_mode', 'reference'))


def _grads(parameters) -> List[torch.Tensor]:
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    return [p.grad for p in parameters if p.grad is not None]


def _global_norm(norms: List[torch.Tensor], norm_type: float) -> torch.Tensor:
    st = torch.stack(norms)
    if math.isinf(norm_type):
        return st.max()
    return st.pow(norm_type).sum().pow(1.0 / norm_type)


class GradClip:
    def __init__(self, clip_type='none', threshold=1.4, norm_type=2, begin_step=100, ignore_threshold=3,
                 momentum_mode='reference'):
        assert clip_type in CLIP_TYPES, clip_type
        assert momentum_mode in ('reference', 'ema'), momentum_mode
        self.clip_type = clip_type
        self.momentum_mode = momentum_mode
        self.threshold = float(threshold)
        self.norm_type = float(norm_type)
        self.begin_step = begin_step
        self.ignore_threshold = ignore_threshold
        self.beta1, self.beta2 = 0.95, 0.999
        self.step = 0
        self.clip_value = None       # max_norm EMA (device scalar)
        self.norm_mom = None         # momentum_norm ('ema') per-parameter EMA (device vector)
        self.mom_init = None         # 1-element device flag: the EMA holds a kept step's norms
        self.exp_avg_sq = None       # clip_value second moments

    @property
    def ema(self) -> bool:
        """True when this clip scales per tensor against the momentum EMA."""
        return self.clip_type == 'momentum_norm' and self.momentum_mode == 'ema'

    def state_dict(self):
        return {'step': self.step, 'clip_value': self.clip_value, 'norm_mom': self.norm_mom,
                'mom_init': self.mom_init, 'exp_avg_sq': self.exp_avg_sq}

    def load_state_dict(self, sd):
        self.step = sd.get('step', 0)
        self.clip_value = sd.get('clip_value')
        self.norm_mom = sd.get('norm_mom')
        self.mom_init = sd.get('mom_init')
        if self.norm_mom is not None and self.mom_init is None:      # older checkpoints: a stored EMA is live
            self.mom_init = torch.ones(1, dtype=torch.float32, device=self.norm_mom.device)
        self.exp_avg_sq = sd.get('exp_avg_sq')

    def momentum_state(self, n: int, device) -> tuple:
        """(norm_mom, mom_init) as n-vector / 1-flag on ``device``: created as (0, not initialised), moved there
        when a checkpoint brought them in on another device (map_location='cpu') - never re-zeroed."""
        if self.norm_mom is None or self.norm_mom.numel() != n:
            self.norm_mom = torch.zeros(n, dtype=torch.float32, device=device)
            self.mom_init = torch.zeros(1, dtype=torch.float32, device=device)
        if self.norm_mom.device != torch.device(device):
            self.norm_mom = self.norm_mom.to(device)
        if self.mom_init is None:
            self.mom_init = torch.ones(1, dtype=torch.float32, device=device)
        if self.mom_init.device != self.norm_mom.device:
            self.mom_init = self.mom_init.to(self.norm_mom.device)
        self.norm_mom = self.norm_mom.float().contiguous()
        self.mom_init = self.mom_init.float().reshape(1).contiguous()
        return self.norm_mom, self.mom_init

    @torch.no_grad()
    def apply(self, parameters: Iterable[torch.nn.Parameter], gate: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Clip in place and return the global norm.  ``gate``: an optional device scalar (1 = keep, 0 = drop
        the whole step's gradient, e.g. a timed-out LSTM exchange); no host sync either way.  A dropped step's
        gradients are SELECTED away (``torch.where``), not multiplied by 0 - the gradients of a timed-out step
        can be NaN - and the momentum EMA keeps its value.  (The optimizer step that follows still runs on zero
        gradients: with the learners' default beta1 = 0 and no weight decay that leaves the weights unchanged;
        the fused path, utils/fused_optim.py, skips the update altogether.)"""
        self.step += 1
        grads = _grads(list(parameters))
        if not grads:
            return torch.zeros(())
        norms = list(torch._foreach_norm(grads, self.norm_type))
        total = _global_norm(norms, self.norm_type)
        t = self.clip_type
        if t in ('pytorch_norm', 'clip_norm'):
            coef = (self.threshold / (total + 1e-6)).clamp(max=1.0)
            torch._foreach_mul_(grads, coef)
        elif t == 'max_norm':
            bc1 = 1 - self.beta1 ** self.step
            if self.clip_value is None:
                self.clip_value = torch.zeros_like(total)
            if self.step > self.begin_step:
                coef = ((self.clip_value / bc1) * self.threshold / (total + 1e-6)).clamp(max=1.0)
                torch._foreach_mul_(grads, coef)
            self.clip_value = self.beta1 * self.clip_value + (1 - self.beta1) * total
        elif t == 'momentum_norm' and self.momentum_mode == 'ema':
            g = torch.stack(norms)
            mom0, init0 = self.momentum_state(g.numel(), g.device)
            live = init0 > 0
            lim = self.threshold * mom0
            scale = torch.where(live & (g >= lim), lim / (g + 1e-6), torch.ones_like(g))
            torch._foreach_mul_(grads, list(scale.unbind()))
            new = g * scale
            mom = torch.where(live, mom0 * 0.99 + new * 0.01, new)
            init = torch.ones_like(init0)
            if gate is not None:
                keep = gate.reshape(()) > 0
                mom = torch.where(keep, mom, mom0)
                init = torch.where(keep, init, init0)
            self.norm_mom, self.mom_init = mom, init
            total = _global_norm(list(new.unbind()), self.norm_type)
        # momentum_norm in 'reference' mode: no scaling, the plain global norm (see the module docstring)
        elif t == 'clip_value':
            bc2 = 1 - self.beta2 ** self.step
            if self.exp_avg_sq is None:
                self.exp_avg_sq = [torch.zeros_like(g) for g in grads]
            torch._foreach_mul_(self.exp_avg_sq, self.beta2)
            torch._foreach_addcmul_(self.exp_avg_sq, grads, grads, 1 - self.beta2)
            if self.step >= 100:
                for g, s in zip(grads, self.exp_avg_sq):
                    lim = s.sqrt() / math.sqrt(bc2) * 5
                    g.copy_(torch.where(g.abs() > lim, lim, g))
        elif t == 'clip_const':
            for g in grads:
                g.clamp_(-self.threshold, self.threshold)
        if gate is not None:
            keep = gate.reshape(()) > 0
            for g in grads:
                torch.where(keep, g, torch.zeros((), dtype=g.dtype, device=g.device), out=g)
        return total
