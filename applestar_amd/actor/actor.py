"""Actor runtime: env loop, job handling, multi-process envs, batched GPU inference, data/result send.

Behaviour of ``distar/actor/actor.py`` (``Actor :23``):
* job types ``eval_test`` / ``train_test`` run one in-process env loop; ``train`` asks the league
  for a job, runs ``env_num`` env processes, streams trajectories to the learner and results to
  the league, and restarts with a new job after ``actor_ask_for_job_interval`` x U(0.7, 1.3);
  ``eval`` runs the multi-process envs without sending anything;
* agent setup loads ``state_dict['model']`` minus value networks, non-strict, and reads the optional
  ``map_name`` / ``fake_reward_prob`` / ``z_path`` / ``z_idx`` keys (``actor.py:40-103``);
* episode loop: agent.step for every player that got an observation -> env.step -> collect_data ->
  send -> on game end send_result (``actor.py:105-266``).

MI355X structure:
* env workers are *spawned* processes (the parent owns the GPU; forking after HIP init is unsafe);
* with ``gpu_batch_inference`` the parent runs one :class:`InferenceServer` that batches every
  worker's policy and teacher requests (dynamic batching, no polling); workers hold no model;
* trajectories go worker -> learner directly through each worker's own :class:`Adapter`
  (producer-side payload server), never through the parent;
* model refresh: the parent pulls ``<player>model`` broadcasts every ``actor_model_update_interval``
  seconds and hot-loads them into the server's resident models.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import random
import time
import traceback
import uuid
from collections import defaultdict
from typing import Dict, List, Optional

import torch

from ..agent.agent import Agent
from ..league.players import FRAC_ID
from ..utils import faults
from ..utils.config import AttrDict, deep_merge_dicts
from ..utils.log import TextLogger, VariableRecord

DEFAULT_ACTOR_CONFIG = {
    'common': {'experiment_name': 'test', 'type': 'rl'},
    'actor': {'job_type': 'eval_test', 'league_job_type': 'train', 'gpu_batch_inference': False,
              'env_num': 1, 'episode_num': 1, 'print_freq': 100, 'traj_len': 64, 'use_cuda': False,
              'fake_model': True, 'player_ids': ['model1'], 'agents': {}, 'model_paths': {},
              'teacher_player_ids': ['none'], 'teacher_model_paths': {}, 'max_wait_ms': 2.0,
              # env workers run at this nice level: on a box shared with a learner / inference server the host
              # threads that feed the GPU keep their CPU (0: unchanged)
              'env_nice': 5},
    'env': {'map_name': 'KairosJunction', 'player_ids': ['agent1', 'bot7'], 'races': ['zerg', 'zerg'],
            'realtime': False, 'game_steps_per_episode': 100000, 'fake': None},
    'communication': {'coordinator_ip': '127.0.0.1', 'coordinator_port': 0, 'league_ip': '127.0.0.1',
                      'league_port': 0, 'actor_ask_for_job_interval': 1800, 'actor_model_update_interval': 10},
    'learner': {'use_value_feature': False, 'use_dapo': False},
}

_NO_CKPT = ('', 'none', 'default', 'fake', None)


def load_policy_weights(model: torch.nn.Module, path: str, agent: Optional[Agent] = None) -> int:
    """Load a checkpoint's policy weights (value networks dropped, non-strict); returns last_iter."""
    if path in _NO_CKPT or not os.path.exists(str(path)):
        return 0
    from ..utils.checkpoint import load_file, load_state_dict_matched
    sd = load_file(path)
    load_state_dict_matched(model, sd.get('model', sd), drop=('value_networks', 'value_encoder'))
    if agent is not None and 'map_name' in sd:
        agent._fake_reward_prob = sd.get('fake_reward_prob', agent._fake_reward_prob)
        agent._z_path = sd.get('z_path', agent._z_path)
        agent.z_idx = sd.get('z_idx')
    return int(sd.get('last_iter', 0))


def make_env(cfg):
    """Real SC2 when available and not forced fake, else :class:`FakeSC2Env`."""
    from ..envs import make_env as _make
    return _make(cfg)


def _job_from_config(cfg) -> dict:
    """An actor ``*_test`` / ``eval`` run described as a league-style job."""
    a, e = cfg.actor, cfg.env
    ids = list(e.player_ids)
    teacher_ids = list(a.get('teacher_player_ids', ['none'] * len(ids)))
    teacher_ids += ['none'] * (len(ids) - len(teacher_ids))
    model_ids = list(a.player_ids) + ['none'] * len(ids)
    return {'player_ids': [model_ids[i] if 'bot' not in ids[i] else ids[i] for i in range(len(ids))],
            'side_ids': list(range(len(ids))),
            'pipelines': ['bot' if 'bot' in p else a.agents.get(model_ids[i], 'default') for i, p in enumerate(ids)],
            'checkpoint_paths': [a.model_paths.get(model_ids[i], 'none') for i in range(len(ids))],
            'teacher_player_ids': teacher_ids,
            'teacher_checkpoint_paths': [a.teacher_model_paths.get(t, 'none') for t in teacher_ids],
            'z_path': [cfg.get('agent', {}).get('z_path', '7map_filter_spine.json')] * len(ids),
            'z_prob': [cfg.get('agent', {}).get('fake_reward_prob', 1.0)] * len(ids),
            'send_data_players': [], 'update_players': [], 'successive_ids': ['none'] * len(ids),
            'env_info': {'player_ids': ids}}


def build_agents(cfg, job: dict, clients: Optional[Dict] = None) -> List[Agent]:
    """One Agent per non-bot seat; models shared per player id (or remote through ``clients``)."""
    agents, models, teachers = [], {}, {}
    for idx, pid in enumerate(job['player_ids']):
        if 'bot' in job['pipelines'][idx]:
            continue
        acfg = deep_merge_dicts(cfg, {'agent': {'z_path': job['z_path'][idx]}})
        tid = job['teacher_player_ids'][idx]
        pipeline = job['pipelines'][idx]
        if pipeline != 'default':  # plugin agent (registry name / module path)
            from ..agent.registry import import_agent
            agent = import_agent(pipeline)(acfg)
            agent.player_id, agent.side_id, agent.slot = pid, job['side_ids'][idx], idx
            agent.opponent_id = job.get('bot_id') or 'none'
            agent._fake_reward_prob = job['z_prob'][idx]
            agents.append(agent)
            continue
        tkey = tid if tid != 'none' else pid  # no teacher configured: KL against the player's own policy
        if clients is not None:
            agent = Agent(acfg, inference_client=clients.get((pid, 'policy')),
                          teacher_client=clients.get((tkey, 'teacher')), model=None, teacher_model=None)
        else:
            if pid not in models:
                from ..models.model import Model
                models[pid] = Model(acfg).eval()
                if not cfg.actor.fake_model:
                    load_policy_weights(models[pid], job['checkpoint_paths'][idx])
            teacher = None
            if 'train' in cfg.actor.job_type and tid != 'none':
                if tid not in teachers:
                    from ..models.model import Model
                    teachers[tid] = Model(acfg).eval()
                    if not cfg.actor.fake_model:
                        load_policy_weights(teachers[tid], job['teacher_checkpoint_paths'][idx])
                teacher = teachers[tid]
            agent = Agent(acfg, model=models[pid], teacher_model=teacher or (models[pid]
                                                                             if 'train' in cfg.actor.job_type else None))
        agent.player_id = pid
        agent.side_id = job['side_ids'][idx]
        agent._fake_reward_prob = job['z_prob'][idx]
        others = [p for j, p in enumerate(job['env_info']['player_ids']) if j != idx]
        agent.opponent_id = job.get('bot_id') or (others[0] if others else 'none')
        agent.slot = idx
        agents.append(agent)
    return agents


def run_episodes(cfg, job: dict, env_id: int = 0, clients=None, send_traj=None, send_result=None,
                 ctrl=None, logger=None, episode_num: Optional[int] = None) -> List[dict]:
    """The env loop (``actor.py:105-266``). Returns the per-episode result dicts."""
    races = [random.choice(FRAC_ID[f]) for f in job.get('frac_ids', [])]
    env_info = dict(job.get('env_info', {}))
    if races:
        env_info['races'] = races
    cfg = deep_merge_dicts(cfg, {'env': env_info})
    env = make_env(cfg)
    agents = build_agents(cfg, job, clients)
    by_slot = {}
    train = 'train' in cfg.actor.job_type
    results = []
    record = VariableRecord(cfg.actor.print_freq)
    n_ep = episode_num if episode_num is not None else cfg.actor.episode_num
    iters = 0
    try:
        for ep in range(n_ep):
            t_game = time.time()
            faults.inject('env_reset')
            obs, game_info, map_name = env.reset()
            # env observation index == agent order among non-bot seats
            by_slot = {i: a for i, a in enumerate(agents)}
            for i, o in obs.items():
                by_slot[i].reset(map_name, cfg.env.races[by_slot[i].slot], game_info[i], o)
            game_iters = 0
            while True:
                if ctrl is not None and ctrl.poll():
                    cmd = ctrl.recv()
                    if cmd in ('reset', 'close'):
                        return results
                faults.inject('actor_step')
                faults.inject(f'actor_step@{env_id}')
                t0 = time.time()
                actions = {i: by_slot[i].step(o) for i, o in obs.items()}
                t1 = time.time()
                nobs, reward, done = env.step(actions)
                t2 = time.time()
                if train:
                    for i, o in nobs.items():
                        a = by_slot[i]
                        if not hasattr(a, 'collect_data'):
                            continue
                        if cfg.actor.job_type == 'train_test' or a.player_id in job['send_data_players']:
                            traj = a.collect_data(o, reward[i], done, i)
                            if traj is not None and send_traj is not None:
                                send_traj(traj, a.player_id)
                        else:
                            a._update_fake_reward(a._last_action_type, a._last_location, o)
                iters += 1
                game_iters += 1
                record.update_var({'agent_time': t1 - t0, 'env_time': t2 - t1,
                                   'agent_time_per_agent': (t1 - t0) / max(1, len(obs))})
                if logger is not None and env_id == 0 and iters % cfg.actor.print_freq == 0:
                    logger.info(f'actor env {env_id} iter {iters}\n{record.get_vars_text()}')
                if not done:
                    obs = nobs
                    continue
                info = {'game_steps': env._game_loop if hasattr(env, '_game_loop') else game_iters,
                        'game_iters': game_iters, 'game_duration': time.time() - t_game}
                for i, a in by_slot.items():
                    side = {'race': getattr(a, 'race', None), 'player_id': a.player_id,
                            'opponent_id': a.opponent_id, 'winloss': reward[i],
                            'agent_iters': getattr(a, 'iter_count', game_iters)}
                    if hasattr(a, 'get_stat_data'):
                        side.update(a.get_stat_data())
                    info[str(a.side_id)] = side
                results.append(info)
                if send_result is not None:
                    send_result(info)
                break
    finally:
        env.close()
    return results


# ----------------------------------------------------------------------------- worker process
def _worker_main(cfg_dict, job, env_id, req_conns, ctrl, result_q, coord):
    """Spawned env worker: CPU featurization + env; model calls go to the parent's server."""
    torch.set_num_threads(1)
    cfg = AttrDict(cfg_dict)
    nice = int(cfg.actor.get('env_nice', 0) or 0)
    if nice > 0:
        try:
            os.nice(nice)
        except OSError:
            pass
    from .inference import InferenceClient
    clients = None
    if req_conns is not None:
        clients = {}
        for (pid, key_kind), (conn, kind, tkey) in req_conns.items():
            clients[(pid, key_kind)] = InferenceClient(conn, pid, kind, teacher_id=tkey)
    adapter = None
    if coord is not None and cfg.actor.job_type == 'train':
        from ..comm.adapter import Adapter
        adapter = Adapter(coord[0], coord[1])

    def send_traj(traj, player_id):
        if adapter is not None:
            adapter.push(traj, token=player_id + 'traj')

    def send_result(info):
        result_q.put(('result', info))
    try:
        run_episodes(cfg, job, env_id, clients, send_traj, send_result, ctrl)
    except Exception as e:  # noqa: BLE001 - report and exit; the parent restarts the job
        result_q.put(('error', f'{e}\n{traceback.format_exc()}'))
    result_q.put(('done', env_id))


class Actor:
    def __init__(self, cfg):
        self._whole_cfg = deep_merge_dicts(DEFAULT_ACTOR_CONFIG, cfg or {})
        self._cfg = self._whole_cfg.actor
        self._job_type = self._cfg.job_type
        self._uid = str(uuid.uuid1())
        self._logger = TextLogger(os.path.join(os.getcwd(), 'experiments', self._whole_cfg.common.experiment_name,
                                               'actor_log'), name=self._uid)
        self._processes: List[mp.Process] = []
        self._ctrl: List = []
        self._server = None
        self._comm = None
        if self._job_type == 'train':
            from .comm import ActorComm
            self._comm = ActorComm(self._whole_cfg, self._uid, self._logger)
        self.results: List[dict] = []

    # ------------------------------------------------------------------ single process
    def _run_test(self):
        job = _job_from_config(self._whole_cfg)
        self.results = run_episodes(self._whole_cfg, job, 0, logger=self._logger)
        return self.results

    # ------------------------------------------------------------------ multi process
    def _start_workers(self, job: dict):
        self._close_workers()
        ctx = mp.get_context('spawn')
        self._result_q = ctx.Queue()
        gpu = bool(self._cfg.gpu_batch_inference)
        if gpu:
            from .inference import InferenceServer
            from ..models.model import Model
            dev = 'cuda' if torch.cuda.is_available() else 'cpu'
            self._server = InferenceServer(dev, max_wait_ms=self._cfg.max_wait_ms)
            for idx, pid in enumerate(job['player_ids']):
                if 'bot' in job['pipelines'][idx]:
                    continue
                if pid not in self._server.models:
                    m = Model(self._whole_cfg).eval()
                    it = 0 if self._cfg.fake_model else load_policy_weights(m, job['checkpoint_paths'][idx])
                    self._server.set_model(pid, m)
                    self._server.model_iter[pid] = it
                tid = job['teacher_player_ids'][idx]
                tkey = tid if tid != 'none' else pid
                if 'train' in self._job_type and tkey not in self._server.teachers:
                    if tid == 'none':
                        self._server.set_model(pid, self._server.models[pid], teacher=True)
                    else:
                        t = Model(self._whole_cfg).eval()
                        if not self._cfg.fake_model:
                            load_policy_weights(t, job['teacher_checkpoint_paths'][idx])
                        self._server.set_model(tid, t, teacher=True)
        coord = None
        if self._comm is not None:
            coord = (self._whole_cfg.communication.coordinator_ip, self._whole_cfg.communication.coordinator_port)
        for env_id in range(self._cfg.env_num):
            req = None
            if gpu:
                # one pipe per (player, kind): a training agent's policy sample and its teacher's logits for that
                # action are ONE request ('policy+teacher', served by one graph); eval agents ask the policy only
                req = {}
                for idx, pid in enumerate(job['player_ids']):
                    if 'bot' in job['pipelines'][idx]:
                        continue
                    tid = job['teacher_player_ids'][idx]
                    tkey = tid if tid != 'none' else pid
                    kind = 'policy+teacher' if 'train' in self._job_type else 'policy'
                    if (pid, 'policy') in req:
                        continue
                    parent, child = ctx.Pipe()
                    self._server.add_connection(parent, route=(pid, kind, tkey if kind != 'policy' else None))
                    req[(pid, 'policy')] = (child, kind, tkey)
            p_ctrl, c_ctrl = ctx.Pipe()
            p = ctx.Process(target=_worker_main, daemon=True,
                            args=(dict(self._whole_cfg), job, env_id, req, c_ctrl, self._result_q, coord))
            p.start()
            self._processes.append(p)
            self._ctrl.append(p_ctrl)

    def _close_workers(self):
        for c in self._ctrl:
            try:
                c.send('close')
            except (BrokenPipeError, OSError):
                pass
        for p in self._processes:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
        self._processes, self._ctrl = [], []
        if self._server is not None:
            self._server.stop()
            self._server = None

    def _drain(self, deadline: float) -> bool:
        """Serve inference + forward results until all workers finish or the deadline passes."""
        done = 0
        finished = set()
        while done < len(self._processes) and time.time() < deadline:
            # a worker that died without reporting (crash, OOM kill, injected fault) counts as finished
            for i, p in enumerate(self._processes):
                if i not in finished and not p.is_alive() and p.exitcode not in (0, None):
                    finished.add(i)
                    done += 1
                    self._logger.error(f'env worker {i} died with exit code {p.exitcode}')
            if self._server is not None:
                self._server.serve_once(timeout=0.01)
            else:
                time.sleep(0.01)
            if self._comm is not None:
                self._comm.update_model(self)
            while True:
                try:
                    kind, payload = self._result_q.get_nowait()
                except queue.Empty:
                    break
                if kind == 'result':
                    self.results.append(payload)
                    if self._comm is not None:
                        self._comm.send_result(payload)
                elif kind == 'error':
                    self._logger.error(f'env worker error: {payload}')
                elif kind == 'done':
                    if payload not in finished:
                        finished.add(payload)
                        done += 1
        return done >= len(self._processes)

    def run(self, max_jobs: Optional[int] = None):
        if 'test' in self._job_type:
            return self._run_test()
        jobs = 0
        while max_jobs is None or jobs < max_jobs:
            if self._comm is not None:
                job = self._comm.ask_for_job(self)
            else:
                job = _job_from_config(self._whole_cfg)
            self.job = job
            self._start_workers(job)
            dur = self._whole_cfg.communication.actor_ask_for_job_interval * random.uniform(0.7, 1.3)
            self._drain(time.time() + dur)
            self._close_workers()
            jobs += 1
            if self._job_type == 'eval':
                break
        return self.results

    def reset_env(self):
        for c in self._ctrl:
            c.send('reset')

    def close(self):
        self._close_workers()
        if self._comm is not None:
            self._comm.close()
