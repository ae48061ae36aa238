"""One RL learner iteration (forward -> loss -> backward -> all-reduce -> clip -> Adam).

Step semantics of ``RLLearner._train`` (``distar/agent/default/rl_learner.py:82-145``): Adam with
betas (0, 0.99), eps 1e-5, ``pytorch_norm`` clip at 1.0, value pre-training phase that trains only
the critic for ``value_pretrain_iters`` iterations.  fp32 by default, like the reference (``amp_dtype:
bfloat16`` selects bf16 compute weights with fp32 masters); everything after the loss - bucketed gradient
reduction over RCCL, the fused clip + Adam kernels, derived weight forms, the LSTM health gate, optional
whole-step HIP graphs - is the shared :class:`~applestar_amd.runtime.train_engine.TrainEngine`.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..models.model import Model
from ..runtime.train_engine import TrainEngine, amp_context
from ..utils.config import AttrDict, deep_merge_dicts
from .loss import ReinforcementLoss

DEFAULT_LEARNER_CONFIG = AttrDict({
    'learner': {
        'player_id': 'MP0',
        'learning_rate': 1e-5,
        'weight_decay': 0.0,
        'use_value_feature': True,
        'value_pretrain_iters': -1,
        'grad_clip': {'type': 'pytorch_norm', 'threshold': 1.0},
        'bucket_mb': 32,
        'comm_dtype': None,
        # fp32 like the reference learner (the headline benchmark); 'bfloat16' = bf16 compute, fp32 masters
        'amp_dtype': None,
        # HIP-graph capture of the whole step (runtime/step_graph.py); GPU only.  It pays when the host, not the
        # GPU, is the bottleneck (the bf16 step; many ranks per node contending for CPU)
        'graph_step': False,
    },
    'model': {'enable_baselines': ['winloss']},
})


class RLTrainer(TrainEngine):
    ADAM_BETAS = (0.0, 0.99)
    ADAM_EPS = 1e-5

    def __init__(self, cfg: Optional[dict] = None, device='cpu', model: Optional[Model] = None):
        self.cfg = deep_merge_dicts(DEFAULT_LEARNER_CONFIG, cfg or {})
        lc = self.cfg.learner
        self.model = model if model is not None else Model(self.cfg, use_value_network=True)
        self.iter = 0
        self._setup_engine(device)
        self.loss = ReinforcementLoss(lc, lc.player_id)
        self.remain_value_pretrain = int(lc.get('value_pretrain_iters', -1))
        self.graph = self._make_graph(self._fwd_bwd)

    def _value_pretrain_toggle(self):
        active = self.remain_value_pretrain > 0
        self.model.only_update_baseline = active
        self.loss.only_update_value = active
        if active:
            self.remain_value_pretrain -= 1

    # ------------------------------------------------------------------ one iteration, in three parts
    def _fwd_bwd(self, batch: Dict) -> Dict[str, torch.Tensor]:
        if not self.model.training:   # train() walks ~670 modules: ~1 ms of host time per step
            self.model.train()
        with amp_context(self.device, self.amp_dtype):
            out = self.model.rl_learner_forward(**batch)
        info = self.loss.compute_loss(out)
        self.backward(info['total_loss'])
        # detached: a returned loss must not keep this step's autograd graph (and its AccumulateGrad nodes,
        # bound to the stream they were created on) alive into the next step - or into a graph capture
        return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in info.items()}

    def step(self, batch: Dict) -> Dict[str, torch.Tensor]:
        self._value_pretrain_toggle()
        if self.graph is not None and 'entity_total' in batch:
            from ..models.encoders import entity_pad_for
            b = dict(batch)
            total = b.pop('entity_total')
            b['entity_pad'] = entity_pad_for(total, b['entity_info']['unit_type'].shape[1])
            info = self.graph(b, extra_key=(self.model.only_update_baseline,))
        else:
            info = self._fwd_bwd(batch)
            self._reduce()
            info['gradient'] = self._update()
        self.iter += 1
        return self.step_info(info)
