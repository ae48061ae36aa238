"""BaseLearner: the learner runtime around a trainer step (``distar/ctools/worker/learner/base_learner.py``).

* merges defaults, initialises distributed state (one process per GPU, RCCL) when launched under
  ``torch.distributed.run`` or with ``use_distributed``;
* builds the trainer (model + optimizer + bucketed gradient reducer + clip), dataloader, hooks;
* ``run()``: ``before_run`` hooks, then ``max_iterations`` x (data -> ``before_iter`` -> trainer step ->
  ``after_iter``), then ``after_run``; wrapped in :func:`auto_checkpoint` so an exception or
  SIGINT/SIGTERM/SIGUSR1 saves a checkpoint first (``base_learner.py:248-272``).
Subclasses override ``_setup_trainer`` / ``_setup_dataloader`` and may add hooks.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Iterator, Optional

import torch

from ..parallel import dist as pdist
from ..utils import faults
from ..utils.checkpoint import CheckpointHelper, CountVar, auto_checkpoint
from ..utils.config import AttrDict, deep_merge_dicts
from ..utils.log import LogDict, ScalarLogger, TextLogger, VariableRecord
from .hooks import DEFAULT_HOOK_CONFIG, build_learner_hooks

DEFAULT_BASE_LEARNER_CONFIG = {
    'common': {'experiment_name': 'test', 'type': 'rl'},
    'learner': {'load_path': '', 'use_cuda': True, 'use_distributed': False, 'max_iterations': int(1e8),
                'learning_rate': 1e-3, 'weight_decay': 1e-4, 'data': {'batch_size': 1, 'trajectory_length': 64},
                'grad_clip': {'type': 'none', 'threshold': 1.4}, 'hook': DEFAULT_HOOK_CONFIG,
                'player_id': 'MP0', 'log_to_stdout': True},
}


class BaseLearner:
    name = 'BaseLearner'

    def __init__(self, cfg: Optional[dict] = None, defaults: Optional[dict] = None):
        base = deep_merge_dicts(DEFAULT_BASE_LEARNER_CONFIG, defaults or {})
        self.cfg = self._whole_cfg = deep_merge_dicts(base, cfg or {})
        lc = self.cfg.learner
        if lc.get('use_distributed') or int(os.environ.get('WORLD_SIZE', '1')) > 1:
            pdist.init()
        self.rank = pdist.get_rank()
        self.world_size = pdist.get_world_size()
        use_cuda = bool(lc.use_cuda) and torch.cuda.is_available()
        self.device = torch.device(f'cuda:{pdist.local_device_index()}' if use_cuda else 'cpu')
        if use_cuda:
            torch.cuda.set_device(self.device)
        self.experiment_name = self.cfg.common.experiment_name
        self.exp_dir = os.path.join(os.getcwd(), 'experiments', self.experiment_name)
        log_dir = os.path.join(self.exp_dir, 'log') if self.cfg.common.type != 'rl' else \
            os.path.join(self.exp_dir, lc.player_id, 'log')
        self.logger = TextLogger(log_dir, name=f'learner_rank{self.rank}', to_stdout=bool(lc.log_to_stdout))
        self.scalar_logger = ScalarLogger(log_dir) if self.rank == 0 else None
        self.record = VariableRecord(length=int(lc.hook.get('log_show', {}).get('ext_args', {}).get('freq', 10)))
        self.log_buffer = LogDict()
        self.last_iter = CountVar(0)
        self.checkpoint_helper = CheckpointHelper()
        self.last_checkpoint_path = ''
        # a supervisor restart passes the newest checkpoint (runtime/supervisor.py)
        self.load_path = os.environ.get('APPLESTAR_RESUME_PATH') or lc.get('load_path', '')
        self.trainer = self._setup_trainer()
        self.dataloader: Optional[Iterator] = self._setup_dataloader()
        self.hooks = build_learner_hooks(lc.hook)
        self._max_iterations = int(lc.max_iterations)
        self.samples_per_iter = int(lc.data.batch_size) * int(lc.data.trajectory_length)

    # ------------------------------------------------------------------ overridables
    def _setup_trainer(self):
        raise NotImplementedError

    def _setup_dataloader(self) -> Optional[Iterator]:
        return None

    def _train(self, data: Dict) -> Dict:
        return self.trainer.step(data)

    # ------------------------------------------------------------------ properties used by hooks
    @property
    def model(self):
        return self.trainer.model

    @property
    def optimizer(self):
        return self.trainer.optimizer

    @property
    def lr_scheduler(self):
        return getattr(self.trainer, 'lr_scheduler', None)

    def info(self, msg: str):
        if self.rank == 0:
            self.logger.info(msg)

    def checkpoint_path(self, it: int) -> str:
        if self.cfg.common.type == 'rl':
            pid = self.cfg.learner.player_id
            d = os.path.join(self.exp_dir, pid, 'checkpoint')
            return os.path.join(d, f'{self.experiment_name}_{pid}_iteration_{it}.pth.tar')
        return os.path.join(self.exp_dir, 'checkpoint', f'{self.experiment_name}_iteration_{it}.pth.tar')

    def model_state_dict(self):
        f = getattr(self.trainer, 'model_state_dict', None)
        return f() if f else self.model.state_dict()

    def model_loader(self):
        return getattr(self.trainer, 'load_model_state_dict', None)

    def save_checkpoint(self):
        if self.rank == 0:
            path = self.checkpoint_path(self.last_iter.val)
            self.checkpoint_helper.save(path, self.model, self.optimizer, last_iter=self.last_iter.val,
                                        state_dict=self.model_state_dict())
            self.last_checkpoint_path = path

    def call_hooks(self, position: str):
        for h in self.hooks[position]:
            h(self)

    # ------------------------------------------------------------------ loop
    def _next_data(self):
        return next(self.dataloader)

    @auto_checkpoint('save_checkpoint')
    def run(self, max_iterations: Optional[int] = None):
        self.call_hooks('before_run')
        # config max_iterations is the run's total (resumes continue to it); an explicit argument is relative
        end = self._max_iterations if max_iterations is None else self.last_iter.val + int(max_iterations)
        while self.last_iter.val < end:
            t0 = time.time()
            data = self._next_data()
            t1 = time.time()
            self.call_hooks('before_iter')
            info = self._train(data)
            self.last_iter.add(1)
            self._log_info(info)
            self.log_buffer['data_time'] = t1 - t0
            self.log_buffer['train_time'] = time.time() - t1
            self.call_hooks('after_iter')
            faults.inject('learner_iter')
        self.call_hooks('after_run')
        self._write_fingerprint()

    def _write_fingerprint(self):
        """``learner.fingerprint_path`` (a directory): after the run each rank writes {rank, world, iter,
        weight_hash} there - the data-parallel replica check of tools/rl_train_dp_rehearsal.py."""
        d = self.cfg.learner.get('fingerprint_path')
        if not d:
            return
        import json
        os.makedirs(d, exist_ok=True)
        with torch.no_grad():
            h = 0
            for k, v in sorted(self.model.state_dict().items()):
                if v.is_floating_point():
                    x = v.detach().float().reshape(-1).cpu()
                    h = (h * 1000003 + int((x.view(torch.int32).long() * 2654435761 % (1 << 31)).sum())) % (1 << 61)
        rec = {'rank': self.rank, 'world': self.world_size, 'iter': self.last_iter.val, 'weight_hash': h}
        with open(os.path.join(d, f'rank{self.rank}.json'), 'w') as f:
            json.dump(rec, f)

    def _log_info(self, info: Dict):
        # one device->host transfer for every logged scalar
        keys = [k for k, v in info.items() if torch.is_tensor(v) and v.numel() == 1]
        if keys:
            vals = torch.stack([info[k].detach().float().reshape(()) for k in keys]).cpu().tolist()
            self.log_buffer.update(dict(zip(keys, vals)))
            if self.log_buffer.get('lstm_exchange_ok', 1.0) == 0.0:
                # the split LSTM recurrence's cross-workgroup exchange timed out: this step's update was gated
                # to zero on the device (trainer._lstm_gate); stop rather than train on garbage
                raise RuntimeError('LSTM split-recurrence exchange timed out (lstm.hip kSplitPollLimit); '
                                   'the update of this iteration was dropped')
        for k, v in info.items():
            if isinstance(v, (int, float)):
                self.log_buffer[k] = float(v)

    def close(self):
        pass
