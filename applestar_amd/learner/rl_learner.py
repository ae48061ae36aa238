"""RL learner runtime: league registration, model push, train-info / reset, replay dataloader.

Behaviour of ``distar/agent/default/rl_learner.py`` + ``ctools/worker/learner/learner_comm.py``:
* registers with the league (``league/register_learner``) and takes the returned checkpoint path as
  load path unless one was given (``learner_comm.py:41-51``);
* every ``learner_send_model_freq`` iterations (after value pre-training) the *policy* weights
  (no value nets) are published as the ``<player>model`` broadcast with ``model_last_iter`` and
  ``reset_flag`` (``:53-99``) — here as ONE flat fp32 snapshot with a version counter
  (``runtime/flat_model.py``): one native multi-tensor copy into a flat device buffer, one D2H DMA on a side
  stream into a pinned ``/dev/shm`` slot that co-located inference servers read directly (H2D + one D2D
  multi-copy into their resident model), and the same flat tensor pushed as a one-tensor frame for actors on
  other hosts by a background thread - the training loop never blocks on the network;
* every ``learner_send_train_info_freq`` iterations rank 0 posts the frames trained; a returned
  ``reset_checkpoint_path`` reloads the model, resets the value networks and value pre-training, and
  re-broadcasts (``:101-137``) — the reset flag is broadcast as a *device* tensor (the reference
  broadcasts a CPU tensor over NCCL, which fails);
* staleness (current iter - trajectory ``model_last_iter``) is logged (``rl_learner.py:85-101``);
* hot-reload / reset through ``update_config`` / ``reset_value`` admin routes (``:203-287``).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional

import torch

from ..comm.adapter import Adapter
from ..league.api import HttpClient
from ..parallel import dist as pdist
from ..rl.trainer import RLTrainer
from ..utils.config import deep_update
from .base_learner import BaseLearner
from .dataloader import RLDataLoader, SyntheticRLDataLoader
from .hooks import LearnerHook, add_learner_hook

DEFAULT_RL_LEARNER_CONFIG = {
    'common': {'type': 'rl'},
    'learner': {'job_type': 'train', 'player_id': 'MP0', 'learning_rate': 1e-5, 'use_value_feature': True,
                'value_pretrain_iters': -1, 'grad_clip': {'type': 'pytorch_norm', 'threshold': 1.0},
                'data': {'batch_size': 6, 'trajectory_length': 64, 'buffer_size': 12, 'synthetic': False}},
    'communication': {'coordinator_ip': '127.0.0.1', 'coordinator_port': 0, 'league_ip': '127.0.0.1',
                      'league_port': 0, 'learner_send_model_freq': 4, 'learner_send_train_info_freq': 100},
}


def model_slot_name(player_id: str, experiment: str = '') -> str:
    """The /dev/shm slot of a player's published policy (runtime/flat_model.SharedModelSlot): per experiment, player
    and user, so two experiments on one host that both train ``MP0`` never share a slot."""
    exp = ''.join(ch if ch.isalnum() or ch in '-_.' else '_' for ch in str(experiment)) or 'default'
    return f'applestar_model_{exp}_{player_id}_{os.getuid()}'


class LearnerComm:
    def __init__(self, cfg, learner: 'RLLearner'):
        c = cfg.communication
        self.cfg = cfg
        self.player_id = cfg.learner.player_id
        self._league = HttpClient(c.league_ip, c.league_port) if c.league_port else None
        self._adapter = Adapter(c.coordinator_ip, c.coordinator_port) if c.coordinator_port else None
        self._send_model_freq = int(c.learner_send_model_freq)
        self._send_info_freq = int(c.learner_send_train_info_freq)
        self._model_count = 0
        self._info_count = 0
        self._publisher = None          # runtime.flat_model.ModelPublisher, built at the first push
        self._pending = threading.Event()
        self._lock = threading.Lock()
        self._meta = (0, False)
        self._stop = False
        if self._adapter is not None:
            threading.Thread(target=self._publish_loop, daemon=True, name='model-publisher').start()
        self._heartbeat = None
        if self._league is not None:
            from ..runtime.health import HeartbeatSender
            self._heartbeat = HeartbeatSender(self._league, 'learner', f'{self.player_id}/rank{learner.rank}',
                                              float(c.get('heartbeat_interval', 10.0)),
                                              info_fn=lambda: {'iter': learner.last_iter.val})

    def register(self, learner) -> None:
        if self._league is None:
            return
        info = self._league.post('/league/register_learner', {
            'player_id': self.player_id, 'ip': '127.0.0.1', 'port': 0, 'rank': learner.rank,
            'world_size': learner.world_size})
        if not (learner.load_path and os.path.exists(learner.load_path)):
            learner.load_path = info.get('ckpt_path', '')

    # ---------------------------------------------------------------- model push
    def send_model(self, learner, ignore_freq: bool = False, reset_flag: bool = False) -> None:
        due = ignore_freq or (self._model_count % self._send_model_freq == 0 and
                              learner.trainer.remain_value_pretrain <= 0)
        if not ignore_freq:
            self._model_count += 1
        if not due or self._adapter is None or learner.rank != 0:
            return
        sd = {k: v for k, v in learner.model_state_dict().items()
              if 'value_networks' not in k and 'value_encoder' not in k}
        with self._lock:
            if self._publisher is None:
                from ..runtime.flat_model import ModelPublisher
                shm = (model_slot_name(self.player_id, self.cfg.common.get('experiment_name', ''))
                       if learner.device.type == 'cuda' else None)
                self._publisher = ModelPublisher(sd, shm_name=shm)
            self._publisher.publish(sd, learner.last_iter.val, reset_flag)
        self._pending.set()

    def _publish_loop(self):
        while not self._stop:
            if not self._pending.wait(timeout=0.5):
                continue
            self._pending.clear()
            with self._lock:
                payload = self._publisher.payload()      # waits for the D2H; stamps the shared slot's version
            self._adapter.push(payload, self.player_id + 'model', broadcast=True)

    # ---------------------------------------------------------------- train info / reset
    def send_train_info(self, learner) -> None:
        self._info_count += 1
        if self._info_count % self._send_info_freq != 0:
            return
        reset_path = 'none'
        if learner.rank == 0 and self._league is not None:
            frames = self._send_info_freq * learner.world_size * learner.samples_per_iter
            try:
                out = self._league.post('/league/learner_send_train_info', {
                    'player_id': self.player_id, 'train_steps': frames,
                    'checkpoint_path': os.path.abspath(learner.last_checkpoint_path or '')})
                reset_path = out.get('reset_checkpoint_path', 'none')
            except (ConnectionError, RuntimeError) as e:
                learner.logger.warning(f'send_train_info failed: {e}')
        flag = torch.tensor([1 if reset_path != 'none' else 0], device=learner.device)
        if learner.world_size > 1:
            torch.distributed.broadcast(flag, 0)
        if int(flag.item()):
            path = pdist.broadcast_object(reset_path)
            learner.reset_from_checkpoint(path)
            self.send_model(learner, ignore_freq=True, reset_flag=True)

    def close(self):
        self._stop = True
        if self._heartbeat is not None:
            self._heartbeat.stop()
        if self._adapter is not None:
            self._adapter.close()
        with self._lock:
            if self._publisher is not None:
                self._publisher.close(unlink=True)
                self._publisher = None


class SendModelHook(LearnerHook):
    def __call__(self, engine):
        engine.comm.send_model(engine, ignore_freq=self.position == 'before_run')


class SendTrainInfoHook(LearnerHook):
    def __call__(self, engine):
        engine.comm.send_train_info(engine)


class RLLearner(BaseLearner):
    name = 'RLLearner'

    def __init__(self, cfg: Optional[dict] = None):
        super().__init__(cfg, DEFAULT_RL_LEARNER_CONFIG)
        self.comm = LearnerComm(self.cfg, self)
        if self.cfg.learner.job_type == 'train':
            self.comm.register(self)
            add_learner_hook(self.hooks, SendModelHook('send_model_before_run', 30, 'before_run'))
            add_learner_hook(self.hooks, SendModelHook('send_model', 30, 'after_iter'))
            add_learner_hook(self.hooks, SendTrainInfoHook('send_train_info', 35, 'after_iter'))
        self._admin_flags = {}
        if self.cfg.learner.get('var_record_type', 'alphastar') == 'alphastar':
            from ..utils.log import AlphaStarVarRecord
            self.record = AlphaStarVarRecord(self.record.length)

    def _setup_trainer(self):
        return RLTrainer(self.cfg, device=self.device)

    def _setup_dataloader(self, ring_bytes: Optional[int] = None):
        lc = self.cfg.learner
        c = self.cfg.communication
        if lc.data.get('synthetic') or not c.coordinator_port:
            return SyntheticRLDataLoader(lc.data.batch_size, lc.data.trajectory_length, self.device,
                                         use_value_feature=lc.use_value_feature)
        return RLDataLoader(Adapter(c.coordinator_ip, c.coordinator_port), lc.player_id, lc.data.batch_size,
                            lc.data.get('buffer_size'), self.device,
                            ring_bytes=ring_bytes or self._ring_bytes(),
                            max_reuse=int(lc.data.get('max_reuse', 2)))

    def _ring_bytes(self) -> int:
        """``learner.data.ring_gb``: a number of GB, or 'auto' (default) = sized from the free HBM minus the
        step's peak (runtime/traj_ring.py auto_ring_bytes; ``ring_fraction`` of it, default 0.75)."""
        d = self.cfg.learner.data
        gb = d.get('ring_gb', 'auto')
        if gb in (None, 'auto'):
            from ..runtime.traj_ring import auto_ring_bytes
            return auto_ring_bytes(self.device, step_peak_gb=float(d.get('step_peak_gb', 20.0)),
                                   fraction=float(d.get('ring_fraction', 0.75)))
        return int(float(gb) * (1 << 30))

    def _train(self, data: Dict) -> Dict:
        mli = data.pop('model_last_iter', None)
        info = self.trainer.step(data)
        if mli is not None and self.trainer.remain_value_pretrain <= 0:
            diff = self.last_iter.val - torch.as_tensor(mli, dtype=torch.float32).reshape(-1).cpu()
            info['staleness/mean'] = float(diff.mean())
            info['staleness/std'] = float(diff.std()) if diff.numel() > 1 else 0.0
            info['staleness/max'] = float(diff.max())
        for k in list(self._admin_flags):
            self._apply_admin(k, self._admin_flags.pop(k))
        return info

    # ---------------------------------------------------------------- resets / admin
    def reset_value(self) -> None:
        """Re-initialise the value networks (``rl_learner.py:_reset_value``)."""
        from ..models.model import ValueBaseline
        if hasattr(self.model, 'value_networks'):
            for name, net in self.model.value_networks.items():
                fresh = ValueBaseline(net.input_dim, net.res_dim, net.res_num, atan=net.atan).to(
                    next(net.parameters()).device)
                net.load_state_dict(fresh.state_dict())
        pdist.broadcast_module(self.model)
        self.trainer.on_model_changed()

    def reset_from_checkpoint(self, path: str) -> None:
        self.checkpoint_helper.load(path, self.model, None, load_optimizer=False, logger=self.logger,
                                    loader=self.model_loader())
        self.reset_value()
        self.trainer.remain_value_pretrain = int(self.cfg.learner.get('value_pretrain_iters', -1))
        self.trainer.reset_optimizer()
        self.info(f'{self.comm.player_id} reset from {path}')

    def request_admin(self, kind: str, payload=None) -> None:
        """Thread-safe: applied between iterations (admin HTTP routes call this)."""
        self._admin_flags[kind] = payload

    def reset_comm_setting(self) -> None:
        """Re-create the league / data-plane links from the (possibly hot-updated) communication config
        (``rl_learner.py:244-261``): close the old LearnerComm and dataloader, register again, rebuild the
        dataloader (its HBM trajectory ring is re-allocated on the new coordinator)."""
        self.comm.close()
        # the old loader's ring is released (ingest thread joined, arena freed and returned to the driver) before
        # the new one is sized, and the new ring keeps the old capacity: sizing it from mem_get_info while the old
        # ~hundreds-of-GB arena is still allocated would shrink it to the floor
        keep_bytes = getattr(self.dataloader, 'ring_bytes', None)
        if hasattr(self.dataloader, 'close') and self.dataloader.close() is False:
            self.dataloader.close(timeout=30.0)   # the ingest thread was mid-frame: its ring must go first
        self.dataloader = None
        if self.device.type == 'cuda':
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()
        self.comm = LearnerComm(self.cfg, self)
        if self.cfg.learner.job_type == 'train':
            self.comm.register(self)
        self.dataloader = self._setup_dataloader(ring_bytes=keep_bytes)
        self.info(f'{self.comm.player_id} communication reset')

    def _apply_admin(self, kind: str, payload):
        if kind == 'reset_comm_setting':
            deep_update(self.cfg, payload or {})
            self.reset_comm_setting()
        elif kind == 'update_config':
            deep_update(self.cfg, payload or {})
            for g in self.optimizer.param_groups:
                g['lr'] = self.cfg.learner.learning_rate
            sched = getattr(self.trainer, 'lr_scheduler', None)
            if sched is not None and hasattr(sched, 'base_lrs'):
                sched.base_lrs = [self.cfg.learner.learning_rate for _ in sched.base_lrs]
        elif kind == 'reset_value':
            self.reset_value()
            self.trainer.remain_value_pretrain = int((payload or {}).get(
                'value_pretrain_iters', self.cfg.learner.get('value_pretrain_iters', -1)))

    def close(self):
        self.comm.close()
        if hasattr(self.dataloader, 'close'):
            self.dataloader.close()


def create_learner_app(learner: RLLearner):
    """Flask admin routes ``/rl_learner/{update_config,reset_value,reset_comm_setting}`` (``rl_learner.py:263-287``)."""
    from flask import Flask, jsonify, request
    app = Flask('applestar_learner')

    @app.route('/rl_learner/update_config', methods=['POST'])
    def update_config():
        learner.request_admin('update_config', request.json)
        return jsonify({'code': 0, 'info': True})

    @app.route('/rl_learner/reset_value', methods=['POST'])
    def reset_value():
        learner.request_admin('reset_value', request.json or {})
        return jsonify({'code': 0, 'info': True})

    @app.route('/rl_learner/reset_comm_setting', methods=['GET', 'POST'])
    def reset_comm_setting():
        learner.request_admin('reset_comm_setting', request.get_json(silent=True) or {})
        return jsonify({'code': 0, 'info': True})

    @app.route('/rl_learner/status', methods=['GET'])
    def status():
        return jsonify({'code': 0, 'info': {'iter': learner.last_iter.val,
                                             'checkpoint': learner.last_checkpoint_path}})
    return app
