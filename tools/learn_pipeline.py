"""Does the production RL pipeline learn?  

    python tools/learn_pipeline.py --envs 24 --seconds 300 --precision fp32 --out gpurun_out/learn_fp32.json

The whole stack of a run on one host, as ``tools/bench_pipeline.py`` wires it (``distar/actor/actor.py:105-266``,
``distar/ctools/worker/learner/learner_comm.py:53-99``): league HTTP server (vs-bot jobs), coordinator (data
plane), an Actor whose env-worker processes run the agent (featurisation, pseudo-rewards, trajectory packing) on
the LEARNABLE FakeSC2Env (``env.fake_learnable``: a fixed quarter of the action types is rewarded and the game
result is drawn from the agent's rewarded-action rate against the bot's chance rate, ``envs/fake_env.py``),
every policy + teacher call served by the GPU batched inference server (HIP graphs), trajectories pushed over the
data plane into the learner's HBM trajectory ring, the RL learner (V-trace / UPGO / TD(lambda) / entropy / KL,
clip + Adam) training in its own process on the same GPU, and its weights coming back to the inference server
through the flat model push (``/dev/shm`` slot, ``runtime/flat_model.py``).

The curve is the ACTOR side: every finished episode's rewarded-action rate and result (written by the env
processes to a JSONL file), binned over wall time, next to the learner's iteration count.  One progress line every
``--report`` seconds; one JSON line at the end (``--out`` also writes it to a file), with the first and the last
bins' rate and win rate.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _learner_main(comm, B, T, precision, lr, iq, stop_ev, exp):
    import torch
    from applestar_amd.learner.rl_learner import RLLearner
    gpu = torch.cuda.is_available()
    if not gpu:
        torch.set_num_threads(2)
    lrn = RLLearner({'common': {'experiment_name': exp},
                     'learner': {'use_cuda': gpu, 'player_id': 'MP0', 'use_value_feature': False,
                                 'learning_rate': lr,
                                 'amp_dtype': 'bfloat16' if precision == 'bf16' else None,
                                 'data': {'batch_size': B, 'trajectory_length': T, 'buffer_size': 2 * B,
                                          'max_reuse': 2},
                                 'log_to_stdout': False},
                     'communication': comm})
    orig = lrn._train
    state = {'n': 0}

    def timed(data):
        if stop_ev.is_set():
            raise SystemExit(0)
        out = orig(data)
        state['n'] += 1
        if state['n'] % 10 == 0:        # a few scalars (each a device sync) every 10 iterations
            rec = {k: float(out[k]) for k in ('total_loss', 'pg/total', 'entropy/action_type', 'kl/total')
                   if k in out and torch.is_tensor(out[k])}
            iq.put((time.time(), lrn.last_iter.val + 1, rec))
        return out
    lrn._train = timed
    lrn.run(max_iterations=10 ** 9)


def _bins(episodes, t0, width):
    out = {}
    for e in episodes:
        k = int((e['t'] - t0) // width)
        b = out.setdefault(k, {'episodes': 0, 'rate_sum': 0.0, 'wins': 0})
        b['episodes'] += 1
        b['rate_sum'] += e['rate'][0]
        b['wins'] += e['win'][0]
    rows = []
    for k in sorted(out):
        b = out[k]
        rows.append({'t_s': round((k + 1) * width, 1), 'episodes': b['episodes'],
                     'rewarded_rate': round(b['rate_sum'] / b['episodes'], 4),
                     'win_rate': round(b['wins'] / b['episodes'], 4)})
    return rows


def _read(path):
    try:
        with open(path) as f:
            return [json.loads(x) for x in f if x.strip()]
    except (OSError, ValueError):
        return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=24)
    ap.add_argument('--seconds', type=float, default=300.0)
    ap.add_argument('--batch', type=int, default=6)
    ap.add_argument('--traj-len', type=int, default=16)
    ap.add_argument('--episode-steps', type=int, default=16, help='agent steps per fake episode')
    ap.add_argument('--lr', type=float, default=1e-4)
    ap.add_argument('--precision', choices=['bf16', 'fp32'], default='fp32')
    ap.add_argument('--bin', type=float, default=30.0, help='curve bin width (s)')
    ap.add_argument('--report', type=float, default=30.0)
    ap.add_argument('--workdir', default='/tmp/applestar_learn')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    if args.out:
        args.out = os.path.abspath(args.out)      # before the chdir below
    os.makedirs(args.workdir, exist_ok=True)
    os.chdir(args.workdir)
    stats_path = os.path.join(args.workdir, f'episodes_{os.getpid()}.jsonl')
    import torch
    from werkzeug.serving import make_server
    from applestar_amd.comm.adapter import Coordinator, serve_coordinator
    from applestar_amd.league.league import League
    from applestar_amd.league.api import create_league_app
    from applestar_amd.actor.actor import Actor
    from applestar_amd.envs.fake_env import REWARDED_ACTION_TYPES
    from applestar_amd.lib.game_data import ACTIONS

    coord = serve_coordinator(Coordinator(), '127.0.0.1', 0)
    cport = coord.server_address[1]
    league = League({'league': {'active_players': {'checkpoint_path': ['none'], 'player_id': ['MP0'],
                                                   'pipeline': ['default'], 'frac_id': [1], 'z_prob': [0.0],
                                                   'teacher_id': ['none'], 'teacher_path': ['none'],
                                                   'z_path': ['3map.json'], 'one_phase_step': [1e9],
                                                   'chosen_weight': [1]},
                                'vs_bot': True, 'bot_probs': [0, 0, 0, 0, 0, 0, 0, 1.0, 0, 0, 0]}},
                    root=args.workdir)
    lport = _free_port()
    srv = make_server('127.0.0.1', lport, create_league_app(league), threaded=True)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    comm = {'coordinator_ip': '127.0.0.1', 'coordinator_port': cport, 'league_ip': '127.0.0.1',
            'league_port': lport, 'learner_send_model_freq': 10, 'learner_send_train_info_freq': 1000,
            'actor_ask_for_job_interval': 3600, 'actor_model_update_interval': 2}
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    iq = ctx.Queue()
    stop_ev = ctx.Event()
    exp = f'learn_pipeline_{os.getpid()}'     # this run's own model slot (runtime/flat_model.py)
    lp = ctx.Process(target=_learner_main, args=(comm, args.batch, args.traj_len, args.precision, args.lr, iq,
                                                 stop_ev, exp), daemon=True)
    lp.start()
    iters = []

    def drain():
        while True:
            iters.append(iq.get())
    threading.Thread(target=drain, daemon=True).start()
    actor = Actor({'common': {'experiment_name': exp},
                   'actor': {'job_type': 'train', 'env_num': args.envs, 'gpu_batch_inference': True,
                             'traj_len': args.traj_len, 'episode_num': 10 ** 9, 'print_freq': 10 ** 9},
                   'env': {'game_steps_per_episode': 10 ** 9, 'fake': True, 'fake_learnable': True,
                           'fake_episode_agent_steps': args.episode_steps, 'fake_stats_path': stats_path},
                   'communication': comm})
    threading.Thread(target=lambda: actor.run(max_jobs=1), daemon=True).start()
    t_start = time.time()
    while not iters and time.time() - t_start < 900:      # the first logged learner iterations
        time.sleep(1.0)
    t0 = time.time()
    print(json.dumps({'progress': 'learner running', 'startup_s': round(t0 - t_start, 1)}), flush=True)
    next_report = t0 + args.report
    while time.time() - t0 < args.seconds:
        time.sleep(1.0)
        if time.time() >= next_report:
            next_report += args.report
            eps = [e for e in _read(stats_path) if e['t'] >= t0]
            recent = [e for e in eps if e['t'] >= time.time() - args.report]
            print(json.dumps({'progress': round(time.time() - t0, 1), 'learner_iter': iters[-1][1] if iters else 0,
                              'episodes': len(eps),
                              'recent_rate': round(sum(e['rate'][0] for e in recent) / max(len(recent), 1), 4),
                              'recent_win': round(sum(e['win'][0] for e in recent) / max(len(recent), 1), 4),
                              'loss': iters[-1][2] if iters else None}), flush=True)
    t1 = time.time()
    eps_all = _read(stats_path)
    before = [e for e in eps_all if e['t'] < t0]
    eps = [e for e in eps_all if t0 <= e['t'] <= t1]
    curve = _bins(eps, t0, args.bin)
    if len(curve) > 2 and curve[-1]['episodes'] < 0.5 * curve[-2]['episodes']:
        curve = curve[:-1]               # the partial bin after the window
    it_curve = [{'t_s': round(t - t0, 1), 'iter': it, **rec} for t, it, rec in iters if t >= t0]
    first = curve[0] if curve else {}
    last = curve[-1] if curve else {}
    out = {'metric': 'end-to-end RL learning on the learnable FakeSC2Env (actor-side curve)',
           'precision': args.precision, 'envs': args.envs, 'seconds': round(t1 - t0, 1), 'lr': args.lr,
           'batch': args.batch, 'traj_len': args.traj_len, 'episode_agent_steps': args.episode_steps,
           'rewarded_action_types': len(REWARDED_ACTION_TYPES), 'action_types': len(ACTIONS),
           'chance_rate': round(len(REWARDED_ACTION_TYPES) / len(ACTIONS), 4),
           'episodes_before_first_iteration': len(before),
           'rate_before_training': round(sum(e['rate'][0] for e in before) / max(len(before), 1), 4) if before else None,
           'episodes': len(eps), 'learner_iterations': (iters[-1][1] if iters else 0),
           'first_bin': first, 'last_bin': last,
           'rate_gain': round(last.get('rewarded_rate', 0) - first.get('rewarded_rate', 0), 4) if curve else None,
           'win_gain': round(last.get('win_rate', 0) - first.get('win_rate', 0), 4) if curve else None,
           'curve': curve, 'learner_curve': it_curve[::5],
           'path': 'league -> actor env workers (agent) -> GPU inference server -> data plane -> HBM ring -> '
                   'learner -> flat model push (/dev/shm slot) -> inference server'}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(line + '\n')
    stop_ev.set()
    lp.join(timeout=30)
    if lp.is_alive():
        lp.terminate()
    try:
        actor.close()
    except Exception:   # noqa: BLE001 - best-effort teardown of the worker processes
        pass
    srv.shutdown()
    coord.shutdown()
    os._exit(0)


if __name__ == '__main__':
    main()
