"""Actor <-> league / learner communication (``distar/ctools/worker/actor/actor_comm.py``).

* ``ask_for_job``: POST ``league/actor_ask_for_job`` until a job is returned (retry with back-off);
* ``update_model``: every ``actor_model_update_interval`` seconds pull each trained player's newest
  ``<player>model`` broadcast from the data plane and hot-load it (into the GPU inference server's
  resident model when batching, else into the local models); a ``reset_flag`` edge restarts envs.  A learner on
  the same host is read from its ``/dev/shm`` slot instead; a slot that went stale (replaced by another
  publisher) is re-attached, and one that stopped advancing for ``actor.shared_model_slot_stale_s`` seconds is
  checked against the broadcast, which wins when it is newer;
* ``send_result``: POST ``league/actor_send_result``.
Trajectories are pushed by the env workers themselves (see :mod:`applestar_amd.actor.actor`).
"""
from __future__ import annotations

import time
from collections import deque

from ..comm.adapter import Adapter
from ..league.api import HttpClient


class ActorComm:
    def __init__(self, cfg, actor_uid: str, logger=None):
        c = cfg.communication
        self._cfg = cfg
        self._uid = actor_uid
        self._logger = logger
        self._league = HttpClient(c.league_ip, c.league_port)
        self._adapter = Adapter(c.coordinator_ip, c.coordinator_port)
        self._interval = float(c.actor_model_update_interval)
        self._last_update = -1.0
        self._last_reset = {}
        self.update_times = deque(maxlen=100)
        self.job = None
        self._attached = {}       # player id -> reading its learner's /dev/shm slot
        self._attach_t = 0.0
        self._slot_seen = {}      # player id -> when its slot last advanced
        from ..runtime.health import HeartbeatSender
        self._heartbeat = HeartbeatSender(self._league, 'actor', actor_uid, float(c.get('heartbeat_interval', 10.0)))

    def ask_for_job(self, actor=None) -> dict:
        delay = 1.0
        while True:
            try:
                job = self._league.post('/league/actor_ask_for_job', {'job_type': self._cfg.actor.league_job_type,
                                                                   'actor_id': self._uid})
                if job:
                    self.job = job
                    return job
            except (ConnectionError, RuntimeError) as e:
                if self._logger:
                    self._logger.warning(f'ask_for_job failed: {e}')
            time.sleep(delay)
            delay = min(delay * 2, 30.0)

    def update_model(self, actor) -> None:
        if not self.job or not self.job.get('update_players'):
            return
        now = time.time()
        if self._last_update > 0 and now - self._last_update < self._interval:
            return
        self._last_update = now
        reset = False
        server = getattr(actor, '_server', None)
        slot_wait = float(self._cfg.actor.get('shared_model_slot_stale_s', 60.0))
        for pid in self.job['update_players']:
            t0 = time.time()
            if server is not None and pid in server.models and self._colocated(server, pid):
                # the learner shares this host: its /dev/shm snapshot slot, no network (runtime/flat_model.py)
                if pid in server.poll_model_slots():
                    self._slot_seen[pid] = now
                    self.update_times.append(time.time() - t0)
                    flag = bool(server._subscribers[pid].reset_flag)
                    if flag and not self._last_reset.get(pid, False):
                        reset = True
                    self._last_reset[pid] = flag
                    continue
                if server.model_slot_state(pid) == 'stale':
                    # the path names another publisher's slot now (restarted learner, reset_comm_setting):
                    # re-attach at the next update, take the network broadcast meanwhile
                    server.detach_model_slot(pid)
                    self._attached[pid] = False
                    self._attach_t = 0.0
                elif now - self._slot_seen.get(pid, now) < slot_wait:
                    continue
                # else: the slot has not advanced for slot_wait seconds - check the broadcast below
            got = self._adapter.pull(pid + 'model', size=1, block=False)
            if not got:
                continue
            sd = got[0]
            it = int(sd.get('model_last_iter', 0))
            if server is not None and pid in server.models:
                if self._attached.get(pid) and it <= server.model_iter.get(pid, -1):
                    continue                  # the slot is up to date with the broadcast: keep reading it
                if self._attached.get(pid):
                    # the broadcast moved past a slot that stopped advancing (its learner died or moved): drop it
                    server.detach_model_slot(pid)
                    self._attached[pid] = False
                    self._attach_t = time.time()
                if 'flat_model' in sd:        # the learner's flat snapshot (runtime/flat_model.py)
                    server.load_flat(pid, sd['flat_model'], sd['names'], sd['shapes'], last_iter=it)
                else:
                    server.load_state_dict(pid, sd['model'], last_iter=it)
            self.update_times.append(time.time() - t0)
            flag = bool(sd.get('reset_flag', False))
            if flag and not self._last_reset.get(pid, False):
                reset = True
            self._last_reset[pid] = flag
        if reset:
            actor.reset_env()

    def _colocated(self, server, pid: str) -> bool:
        """Attach to the player's shared model slot when its learner runs on this host (retried every 30 s while
        detached)."""
        att = self._attached
        if pid not in att or (not att[pid] and time.time() - self._attach_t > 30.0):
            from ..learner.rl_learner import model_slot_name
            self._attach_t = time.time()
            try:
                att[pid] = bool(self._cfg.actor.get('shared_model_slot', True)) and server.attach_model_slot(
                    pid, model_slot_name(pid, self._cfg.common.get('experiment_name', '')))
            except (OSError, ValueError, RuntimeError):
                att[pid] = False
            if att[pid]:
                self._slot_seen[pid] = time.time()
        return att[pid]

    def send_result(self, result: dict) -> None:
        try:
            self._league.post('/league/actor_send_result', result)
        except (ConnectionError, RuntimeError) as e:
            if self._logger:
                self._logger.error(f'send_result failed: {e}')

    def close(self):
        self._heartbeat.stop()
        self._adapter.close()
