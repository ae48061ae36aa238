"""Fused gradient clip + Adam step on the GPU (csrc/kernels/optim.hip).

* RL (``distar/agent/default/rl_learner.py:114-132``): ``pytorch_norm`` - global L2 norm of every gradient,
  scale by ``min(1, threshold / (norm + 1e-6))``, then Adam.  As torch ops that is a ``_foreach_norm`` + stack
  + pow/sum + clamp + ``_foreach_mul_`` + the fused Adam (~10 launches); here two launches over a
  (tensor, offset) chunk table built once (parameters, gradients and moments never move).
* SL (``distar/agent/default/sl_learner.py:46-77``, ``ctools/torch_utils/grad_clip.py:73-106``):
  ``momentum_norm`` - every tensor's norm against the EMA of its past clipped norms (the EMA is the
  :class:`~applestar_amd.utils.grad_clip.GradClip`'s own ``norm_mom`` device vector, so either path can continue
  the other's run) - three launches.

A zero device ``gate`` (timed-out LSTM exchange) skips the update in the kernel: parameters, moments and the
momentum EMA keep their values.  ``device_hparams=True`` reads lr / bias corrections / decay from a 3-float device
buffer refreshed before each step (for HIP-graph replay: the graph keeps the buffer's address, not the values).

The moments ARE the wrapped ``torch.optim.Adam``'s own ``exp_avg`` / ``exp_avg_sq`` state tensors and the
step count its ``step``, so ``optimizer.state_dict()`` / ``load_state_dict`` (checkpoints, league resets) are
unchanged and either path can continue the other's run.  Learning rate and weight decay are read from the
optimizer's param group at every step (LR schedulers keep working).  Applies to a single param group of fp32
CUDA tensors with dense fp32 gradients, plain Adam / AdamW without amsgrad and without the reference
optimizer's own clip / ignore options (``utils.optim.Adam`` defaults); anything else keeps the torch path.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch


def _capturing() -> bool:
    return torch.cuda.is_current_stream_capturing()


class FusedClipAdam:
    """``FusedClipAdam(optimizer, max_norm, clip=None, device_hparams=False, segments=None)``.

    ``segments``: {optimizer param: [(offset, numel), ...]} splits a flat parameter (the bf16 learner's fp32
    master, parallel/mixed.py) into its per-layer pieces, so per-tensor clips (momentum_norm) see the same
    tensors as in the fp32 learner.  ``prepare()`` does the step's host work (step count, bias corrections,
    the hyperparameter upload); :meth:`step` calls it unless a HIP graph is being captured, in which case the
    owner calls it before every replay."""

    HP_RING = 32       # pinned host slots of the device-hyperparameter upload (see prepare)

    def __init__(self, optimizer: torch.optim.Optimizer, max_norm: Optional[float], clip=None,
                 device_hparams: bool = False, segments: Optional[Dict] = None):
        self.opt = optimizer
        self.max_norm = float(max_norm) if max_norm else 0.0
        # only the 'ema' form of momentum_norm scales per tensor; its 'reference' form (the reference's effective
        # behaviour, utils/grad_clip.py) is an unclipped step reporting the global norm
        self.clip = clip if clip is not None and getattr(clip, 'ema', False) else None
        self.device_hparams = device_hparams
        self.segments = segments or {}
        self._hp = None
        self._host_hp = None
        self._table = None
        self._sig = None
        self._steps = None
        self._pending = 0          # steps not yet added to the per-parameter ``step`` tensors (see hparams)
        self._prepared = False
        # the per-parameter counters are written lazily: before anyone reads the optimizer's state dict, and
        # dropped when a state dict is loaded over them
        if hasattr(optimizer, 'register_state_dict_pre_hook'):
            optimizer.register_state_dict_pre_hook(lambda opt: self.sync_steps())
            optimizer.register_load_state_dict_pre_hook(lambda opt, sd: self._drop_pending())

    @staticmethod
    def supported(optimizer, clip) -> bool:
        if not isinstance(optimizer, torch.optim.Adam) or len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        if g.get('amsgrad') or g.get('maximize') or g.get('capturable') or g.get('differentiable'):
            return False
        if getattr(optimizer, 'clip_type', None) or getattr(optimizer, 'ignore_type', None):
            return False
        if clip.clip_type not in ('pytorch_norm', 'clip_norm', 'none', 'momentum_norm') or clip.norm_type != 2.0:
            return False
        return all(p.is_cuda and p.dtype == torch.float32 for p in g['params'])

    def _params(self):
        return [p for p in self.opt.param_groups[0]['params'] if p.requires_grad]

    def sync_steps(self):
        """Write the pending step increments into the optimizer's per-parameter ``step`` tensors."""
        if self._pending and self._steps is not None:
            for t in self._steps:
                t += float(self._pending)
        self._pending = 0

    def _drop_pending(self):
        self._pending = 0

    def _build(self, params):
        self.sync_steps()
        from ..ops import native
        C = native.ensure_loaded()
        chunk = C.fused_adam_chunk()
        st = self.opt.state
        rows, chunks = [], []
        for p in params:
            s = st[p]
            if 'exp_avg' not in s:                       # torch.optim.Adam's lazy state, created the same way
                s['step'] = torch.tensor(0.0, dtype=torch.float32)
                s['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                s['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            xs = (p, p.grad, s['exp_avg'], s['exp_avg_sq'])
            for name, x in zip(('param', 'grad', 'exp_avg', 'exp_avg_sq'), xs):
                dense = x.is_contiguous() or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last))
                if x.dtype != torch.float32 or not dense or x.stride() != p.stride():
                    raise RuntimeError(f'FusedClipAdam: {name} of a {tuple(p.shape)} parameter is not an fp32 tensor '
                                       f'laid out like its parameter')
            for off0, n in self.segments.get(p, [(0, p.numel())]):
                t = len(rows) // 6
                rows += [x.data_ptr() + 4 * off0 for x in xs] + [n, len(chunks) // 2]
                for off in range(0, n, chunk):
                    chunks += [t, off]
        dev = params[0].device
        self.ntensors = len(rows) // 6
        self._table = torch.tensor(rows, dtype=torch.int64, device=dev)
        self._chunks = torch.tensor(chunks, dtype=torch.int64, device=dev)
        self._part = torch.empty(len(chunks) // 2, dtype=torch.float32, device=dev)
        self._scale = torch.ones(self.ntensors, dtype=torch.float32, device=dev)
        self._steps = [st[p]['step'] for p in params]
        self._C = C

    def _signature(self, params):
        st = self.opt.state
        return tuple((p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0,
                      st[p]['exp_avg'].data_ptr() if 'exp_avg' in st[p] else 0) for p in params)

    def _ensure_table(self):
        params = self._params()
        if any(p.grad is None for p in params):
            raise RuntimeError('FusedClipAdam: every parameter needs a gradient buffer (the reducer keeps them)')
        sig = self._signature(params)
        if self._table is None or sig != self._sig:
            self._build(params)
            self._sig = self._signature(params)

    def hparams(self):
        """(lr / bc1, 1 / sqrt(bc2), decay, decoupled) of the NEXT step; advances the step count."""
        g = self.opt.param_groups[0]
        params = self._params()
        st = self.opt.state
        # the per-parameter step counters (torch.optim.Adam's state layout, kept for checkpoints) advance lazily:
        # ~470 scalar CPU tensor adds per step were ~2-4 ms of host time (a foreach add is no faster on the CPU)
        if self._steps is not None and len(self._steps) == len(params) and hasattr(self.opt, 'register_state_dict_pre_hook'):
            step = float(self._steps[0]) + self._pending + 1.0
            self._pending += 1
        else:
            self.sync_steps()
            step = float(st[params[0]]['step']) + 1.0 if 'step' in st[params[0]] else 1.0
            for p in params:
                if 'step' in st[p]:
                    st[p]['step'] += 1.0
        b1, b2 = g['betas']
        lr, wd = float(g['lr']), float(g['weight_decay'])
        decoupled = bool(getattr(self.opt, '_decoupled_wd', 0.0)) or isinstance(self.opt, torch.optim.AdamW)
        if decoupled:
            wd = lr * float(getattr(self.opt, '_decoupled_wd', 0.0) or g['weight_decay'])
        return lr / (1.0 - b1 ** step), 1.0 / (1.0 - b2 ** step) ** 0.5, wd, decoupled

    def prepare(self):
        """Host side of the next step: step counts, bias corrections (uploaded when ``device_hparams``)."""
        self._ensure_table()
        self._host_hp = self.hparams()
        # the fused kernel replaces torch.optim's step: record the call where LRScheduler.step() looks for it (its
        # "lr_scheduler.step() before optimizer.step()" warning otherwise fires on every run)
        self.opt._opt_called = True
        if self.clip is not None:
            self.clip.step += 1
        if self.device_hparams:
            if self._hp is None:
                self._hp = torch.zeros(3, dtype=torch.float32, device=self._part.device)
                # a ring of pinned host slots: the upload is an async DMA on the step's stream (a pageable copy
                # would block the host until the previous step finished - no host / GPU overlap at all).  The ring
                # bounds how far the host may run ahead of the GPU: 32 steps (with 8, a graphed step's host
                # blocked here after 8 replays and its issue time read as ~0.55 of the GPU step instead of ~0.1)
                self._hp_host = torch.empty(self.HP_RING, 3, dtype=torch.float32, pin_memory=True)
                self._hp_events = [None] * self.HP_RING
                self._hp_slot = 0
            i = self._hp_slot
            self._hp_slot = (i + 1) % self.HP_RING
            if self._hp_events[i] is not None:
                self._hp_events[i].synchronize()       # the DMA that last read this slot (HP_RING steps ago) is done
            self._hp_host[i, 0], self._hp_host[i, 1], self._hp_host[i, 2] = self._host_hp[:3]
            self._hp.copy_(self._hp_host[i], non_blocking=True)
            ev = self._hp_events[i] = self._hp_events[i] or torch.cuda.Event()
            ev.record()
        self._prepared = True

    @torch.no_grad()
    def step(self, gate: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Clip + Adam in place; returns the global gradient norm (0-d device tensor): pre-clip for
        pytorch_norm, of the clipped gradients for momentum_norm (as the torch path reports)."""
        capturing = _capturing()
        if capturing:
            if not self.device_hparams or self._host_hp is None:
                raise RuntimeError('FusedClipAdam: capture needs device_hparams and one eager step first')
            self._ensure_table()
        elif not self._prepared:
            self.prepare()
        self._prepared = False
        g = self.opt.param_groups[0]
        lr_bc1, inv_sqrt_bc2, wd, decoupled = self._host_hp
        b1, b2 = g['betas']
        mom = scale = init = None
        if self.clip is not None:
            c = self.clip
            dev = self._part.device
            fresh = c.norm_mom is None or c.norm_mom.numel() != self.ntensors or c.norm_mom.device != dev or \
                c.mom_init is None or c.mom_init.device != dev
            if fresh and capturing:
                raise RuntimeError('FusedClipAdam: momentum state must exist on the device before a capture')
            # created as (0, not initialised) - the kernel initialises the EMA on the first KEPT step - or moved to
            # the device when a checkpoint brought it in elsewhere (never re-zeroed)
            mom, init = c.momentum_state(self.ntensors, dev)
            scale = self._scale
        norm = torch.empty((), dtype=torch.float32, device=self._part.device)   # per step: callers may keep it
        self._C.fused_clip_adam(self._table, self._chunks, self._part,
                                gate.reshape(1).float() if gate is not None else None, norm.view(1),
                                self.clip.threshold if self.clip is not None else self.max_norm, mom, scale, init,
                                self._hp if self.device_hparams else None, lr_bc1, b1, b2, inv_sqrt_bc2,
                                float(g['eps']), wd, decoupled)
        return norm
