"""SL learner runtime (``distar/agent/default/sl_learner.py``): carried per-slot LSTM state reset on
``new_episodes``, optimizer skipped for the first ``ignore_steps`` iterations, ``momentum_norm``
clip, optional warm-up LR; data from replay decoding workers, a remote replay actor, or the
synthetic ``FakeSLDataLoader`` when no SC2 / replays are available."""
from __future__ import annotations

from typing import Optional

from ..sl.trainer import SLTrainer
from .base_learner import BaseLearner
from .dataloader import FakeSLDataLoader

DEFAULT_SL_LEARNER_CONFIG = {
    'common': {'type': 'sl'},
    'learner': {'learning_rate': 1e-3, 'weight_decay': 1e-5, 'ignore_steps': 6,
                'grad_clip': {'type': 'momentum_norm', 'threshold': 1.0},
                'data': {'batch_size': 6, 'trajectory_length': 64, 'fake_data': True, 'num_workers': 1,
                         'train_data_file': ''}},
}


class SLLearner(BaseLearner):
    name = 'SLLearner'

    def __init__(self, cfg: Optional[dict] = None):
        super().__init__(cfg, DEFAULT_SL_LEARNER_CONFIG)

    def _setup_trainer(self):
        return SLTrainer(self.cfg, device=self.device)

    def _setup_dataloader(self):
        d = self.cfg.learner.data
        if d.get('fake_data', False) or not d.get('train_data_file'):
            return FakeSLDataLoader(d.batch_size, d.trajectory_length, self.device,
                                    max_entities=int(d.get('fake_max_entities', 512)))
        from .replay_dataloader import ReplayDataLoader
        return ReplayDataLoader(self.cfg, self.device, rank=self.rank, world_size=self.world_size)
