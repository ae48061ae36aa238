"""Per-agent-step cost breakdown of ONE env worker process (the 44 ms/agent-step).

Runs the actor env loop (``actor/actor.py run_episodes``) on FakeSC2Env with the training job's data path
(featurize -> policy request -> env step -> collect_data with the teacher request -> trajectory push), but
with the GPU inference server replaced by an in-process stub that returns a canned model output of the right
shapes after serializing / deserializing the request exactly as the pipe transport does.  So the numbers are
the env worker's own CPU cost per agent step, which bounds agent-steps/s per CPU core.

    python tools/actor_step_profile.py --steps 300 [--cprofile]
Prints one JSON line: per-phase ms / agent step (featurize, request encode/decode, post-process, collect_data,
trajectory serialize, env step) and the total.
"""
from __future__ import annotations

import argparse
import cProfile
import json
import os
import pstats
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

torch.set_num_threads(1)


class StubClient:
    """Serializes the request like InferenceClient, answers from a canned output of the real model."""

    def __init__(self, kind, model, times):
        self.kind, self.model, self.t = kind, model, times
        self._canned = {}

    def infer(self, model_input):
        from applestar_amd.utils import serialize
        from applestar_amd.agent.collate import collate_obs, decollate_output
        t0 = time.perf_counter()
        buf = serialize.dumps({'player_id': 'p', 'kind': self.kind, 'input': model_input})
        t1 = time.perf_counter()
        req = serialize.loads(buf)['input']
        t2 = time.perf_counter()
        self.t['request_codec'] += t1 - t0
        self.t['server_side_decode'] += t2 - t1
        key = self.kind          # one canned answer per kind: the model's own cost is the server's, not ours
        if key not in self._canned:
            with torch.no_grad():
                b = collate_obs([req])
                out = self.model.compute_logp_action(**b) if self.kind == 'policy' else \
                    self.model.compute_teacher_logit(**b)
            self._canned[key] = serialize.dumps(decollate_output(out, 0))
        t3 = time.perf_counter()
        out = serialize.loads(self._canned[key])
        self.t['reply_decode'] += time.perf_counter() - t3
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--traj-len', type=int, default=64)
    ap.add_argument('--cprofile', action='store_true')
    args = ap.parse_args()
    from applestar_amd.actor.actor import DEFAULT_ACTOR_CONFIG, _job_from_config, run_episodes
    from applestar_amd.models.model import Model
    from applestar_amd.utils.config import deep_merge_dicts
    from applestar_amd.utils import serialize
    from applestar_amd.utils.stopwatch import sw
    cfg = deep_merge_dicts(DEFAULT_ACTOR_CONFIG, {
        'actor': {'job_type': 'train_test', 'traj_len': args.traj_len, 'player_ids': ['p'], 'print_freq': 10 ** 9},
        'env': {'player_ids': ['agent1', 'agent2'], 'races': ['zerg', 'zerg'], 'fake': True,
                'game_steps_per_episode': 10 ** 9, 'max_agent_steps': args.steps},
        'learner': {'use_value_feature': True}})
    job = _job_from_config(cfg)
    job['player_ids'] = ['p', 'p']
    job['pipelines'] = ['default', 'default']
    times = defaultdict(float)
    model = Model(cfg).eval()
    clients = {('p', 'policy'): StubClient('policy', model, times), ('p', 'teacher'): StubClient('teacher', model, times)}
    n_steps = [0]
    ser = [0.0]

    def send_traj(traj, pid):
        t0 = time.perf_counter()
        serialize.dumps(traj)
        ser[0] += time.perf_counter() - t0

    from applestar_amd.agent import agent as agent_mod
    orig_step, orig_collect, orig_pre = agent_mod.Agent.step, agent_mod.Agent.collect_data, agent_mod.Agent._pre_process

    def step(self, obs):
        n_steps[0] += 1
        t0 = time.perf_counter()
        r = orig_step(self, obs)
        times['agent_step_total'] += time.perf_counter() - t0
        if n_steps[0] >= args.steps:
            raise KeyboardInterrupt
        return r

    def collect(self, *a, **k):
        t0 = time.perf_counter()
        r = orig_collect(self, *a, **k)
        times['collect_data_total'] += time.perf_counter() - t0
        return r

    def pre(self, obs):
        t0 = time.perf_counter()
        r = orig_pre(self, obs)
        times['featurize'] += time.perf_counter() - t0
        return r
    agent_mod.Agent.step, agent_mod.Agent.collect_data, agent_mod.Agent._pre_process = step, collect, pre
    from applestar_amd.envs import fake_env
    orig_env_step = fake_env.FakeSC2Env.step

    def env_step(self, actions):
        t0 = time.perf_counter()
        r = orig_env_step(self, actions)
        times['fake_env_step'] += time.perf_counter() - t0
        return r
    fake_env.FakeSC2Env.step = env_step
    prof = cProfile.Profile() if args.cprofile else None
    t0, c0 = time.perf_counter(), time.process_time()
    if prof:
        prof.enable()
    try:
        run_episodes(cfg, job, 0, clients=clients, send_traj=send_traj, episode_num=1000)
    except KeyboardInterrupt:
        pass
    if prof:
        prof.disable()
    wall, cpu = time.perf_counter() - t0, time.process_time() - c0
    n = max(n_steps[0], 1)
    res = {k: round(1000 * v / n, 3) for k, v in sorted(times.items())}
    res['traj_serialize'] = round(1000 * ser[0] / n, 3)
    res['wall_per_agent_step_ms'] = round(1000 * wall / n, 3)
    # process CPU time (one torch thread): insensitive to other tenants of the host, unlike the wall clock
    res['cpu_per_agent_step_ms'] = round(1000 * cpu / n, 3)
    # the stub decodes each request as the GPU server would: that decode is the server's cost, not the actor's
    # ... nor is the stand-in game's own step (SC2 runs in its own process)
    res['actor_cpu_per_agent_step_ms'] = round(1000 * cpu / n - res.get('server_side_decode', 0.0)
                                               - res.get('fake_env_step', 0.0), 3)
    res['agent_steps'] = n
    print(json.dumps(res))
    if prof:
        pstats.Stats(prof).sort_stats('cumulative').print_stats(45)


if __name__ == '__main__':
    main()
