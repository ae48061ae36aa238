"""One supervised-learning iteration (``distar/agent/default/sl_learner.py:46-77``): the LSTM state
of each batch slot is carried across consecutive trajectory chunks of the same replay and reset
where a new episode starts; the optimizer is skipped for the first iterations (warm-up of the
carried state); ``momentum_norm`` clip; Adam + optional warm-up/multistep LR schedule."""
from __future__ import annotations

import contextlib
from typing import Dict, Optional

import torch

from ..utils.optim import build_optimizer
from ..models.model import Model
from ..parallel import dist as pdist
from ..parallel.dp import GradientReducer
from ..utils.config import AttrDict, deep_merge_dicts
from ..utils.grad_clip import build_grad_clip
from ..utils.lr_scheduler import build_lr_scheduler
from .loss import SupervisedLoss

DEFAULT_SL_CONFIG = AttrDict({
    'learner': {
        'learning_rate': 1e-3, 'weight_decay': 1e-5, 'ignore_steps': 6,
        'grad_clip': {'type': 'momentum_norm', 'threshold': 1.0},
        'lr_scheduler': {'type': 'none'},
        'data': {'batch_size': 6, 'trajectory_length': 64},
        'bucket_mb': 32, 'amp_dtype': 'bfloat16',
    },
})


class SLTrainer:
    def __init__(self, cfg: Optional[dict] = None, device='cpu', model: Optional[Model] = None):
        self.cfg = deep_merge_dicts(DEFAULT_SL_CONFIG, cfg or {})
        lc = self.cfg.learner
        self.device = torch.device(device)
        self.model = model if model is not None else Model(self.cfg, temperature=1.0)
        self.model.to(self.device)
        if self.device.type == 'cuda':
            # MIOpen find-mode autotuning (cudnn.benchmark) is opt-in: it measured ~10% faster convs on the
            # bench shapes, but two runs that used it left the GPU in a memory-fault state
            torch.backends.cudnn.benchmark = bool(lc.get('conv_autotune', False))
            self.model.to(memory_format=torch.channels_last)
        pdist.broadcast_module(self.model)
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        self.reducer = GradientReducer(self.params, bucket_mb=lc.bucket_mb)
        self.optimizer = build_optimizer(self.params, lc, device=self.device)
        self.lr_scheduler = build_lr_scheduler(self.optimizer, lc.lr_scheduler)
        self.grad_clip = build_grad_clip(lc.grad_clip)
        self.loss = SupervisedLoss(lc)
        self.ignore_steps = int(lc.ignore_steps)
        self.iter = 0
        H = self.model.core_lstm.hidden_size
        B = int(lc.data.batch_size)
        z = torch.zeros(B, H, device=self.device)
        self.hidden_state = [(z.clone(), z.clone()) for _ in range(self.model.core_lstm.num_layers)]
        self.amp_dtype = lc.get('amp_dtype')

    def reset_hidden_state(self, new_episodes):
        mask = torch.as_tensor(new_episodes, dtype=torch.bool, device=self.device)
        self.hidden_state = [(torch.where(mask[:, None], 0.0, h.detach()), torch.where(mask[:, None], 0.0, c.detach()))
                             for h, c in self.hidden_state]

    def step(self, batch: Dict) -> Dict[str, torch.Tensor]:
        if not self.model.training:   # train() walks ~670 modules: ~1 ms of host time per step
            self.model.train()
        batch = dict(batch)
        self.reset_hidden_state(batch.pop('new_episodes'))
        batch.pop('hidden_state', None)
        amp = (torch.autocast('cuda', dtype=getattr(torch, self.amp_dtype))
               if self.device.type == 'cuda' and self.amp_dtype else contextlib.nullcontext())
        with amp:
            logits, infer_action, hidden = self.model.sl_train(**batch, hidden_state=self.hidden_state)
        info = self.loss.compute_loss(logits, batch['action_info'], batch['action_mask'], batch['selected_units_num'],
                                      batch['entity_num'], infer_action)
        if self.iter >= self.ignore_steps:
            self.reducer.zero_grad(buffers=False)    # backward overwrites every slot
            self.reducer.backward(info['total_loss'])
            self.reducer.synchronize()
            gate = None
            if self.device.type == 'cuda':
                from ..ops import native
                gate = info['lstm_exchange_ok'] = native.lstm_exchange_ok(self.device)
            info['gradient'] = self.grad_clip.apply(self.params, gate=gate)
            self.optimizer.step()
            self.lr_scheduler.step()
        self.hidden_state = [(h.detach(), c.detach()) for h, c in hidden]
        self.iter += 1
        return info
