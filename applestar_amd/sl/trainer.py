"""One supervised-learning iteration (``distar/agent/default/sl_learner.py:46-77``): the LSTM state
of each batch slot is carried across consecutive trajectory chunks of the same replay and reset
where a new episode starts; the optimizer is skipped for the first iterations (warm-up of the
carried state); ``momentum_norm`` clip; Adam + optional warm-up/multistep LR schedule.

Everything after the loss is the RL learner's machinery (:class:`~applestar_amd.runtime.train_engine.TrainEngine`):
fp32 by default (bf16 compute weights with fp32 masters on request), derived weight forms, bucketed RCCL
reduction, and the fused momentum_norm clip + Adam (three native launches, optim.hip).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..models.model import Model
from ..runtime.train_engine import TrainEngine, amp_context
from ..utils.config import AttrDict, deep_merge_dicts
from .loss import SupervisedLoss

DEFAULT_SL_CONFIG = AttrDict({
    'learner': {
        'learning_rate': 1e-3, 'weight_decay': 1e-5, 'ignore_steps': 6,
        'grad_clip': {'type': 'momentum_norm', 'threshold': 1.0},
        'lr_scheduler': {'type': 'none'},
        'data': {'batch_size': 6, 'trajectory_length': 64},
        'bucket_mb': 32, 'comm_dtype': None,
        'amp_dtype': None,        # fp32 like the reference; 'bfloat16' = bf16 compute with fp32 masters
    },
})


class SLTrainer(TrainEngine):
    def __init__(self, cfg: Optional[dict] = None, device='cpu', model: Optional[Model] = None):
        self.cfg = deep_merge_dicts(DEFAULT_SL_CONFIG, cfg or {})
        lc = self.cfg.learner
        self.model = model if model is not None else Model(self.cfg, temperature=1.0)
        self.iter = 0
        self._setup_engine(device)
        self.loss = SupervisedLoss(lc)
        self.ignore_steps = int(lc.ignore_steps)
        H = self.model.core_lstm.hidden_size
        B = int(lc.data.batch_size)
        z = torch.zeros(B, H, device=self.device)
        self.hidden_state = [(z.clone(), z.clone()) for _ in range(self.model.core_lstm.num_layers)]

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
        with amp_context(self.device, self.amp_dtype):
            logits, infer_action, hidden = self.model.sl_train(**batch, hidden_state=self.hidden_state)
        info = self.loss.compute_loss(logits, batch['action_info'], batch['action_mask'], batch['selected_units_num'],
                                      batch['entity_num'], infer_action)
        if self.iter >= self.ignore_steps:
            self.backward(info['total_loss'])
            self._reduce()
            info['gradient'] = self._update()
            self.lr_scheduler.step()
            self.step_info(info)
        self.hidden_state = [(h.detach(), c.detach()) for h, c in hidden]
        self.iter += 1
        return info
