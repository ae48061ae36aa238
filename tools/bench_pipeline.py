"""End-to-end single-GPU RL pipeline throughput.

    python tools/bench_pipeline.py --envs 12 --seconds 90 --batch 6 --traj-len 64 [--precision bf16]

Wires the whole stack the way a run does (tests/test_pipeline.py on the CPU): league HTTP server, coordinator
(data plane), an Actor with ``--envs`` spawned env-worker processes on FakeSC2Env (CPU featurization, agent
logic, trajectory packing) whose policy + teacher calls go to the GPU batched inference server (HIP graphs per
batch bucket), trajectories pushed over the data plane into the learner's HBM trajectory ring, and the RL learner
training on the same GPU (``distar/actor/actor.py:268-299``, ``distar/agent/default/agent.py:781-805``,
``rl_dataloader.py:79-127``).

Reports, over the measured window after the learner's first iteration: actor agent-steps/s (total and per env
process = per CPU core), trajectories/s and fresh samples/s reaching the data plane, learner iterations/s and
learner samples/s as fed by the actors (a batch of B trajectories x T steps; each trajectory is trained on
``max_reuse`` = 2 times, as the reference).  One JSON line on stdout.  The fake env makes no game
simulation cost: the numbers bound the framework's own actor / inference / data-plane cost.
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


def _learner_main(comm, B, T, gpu, precision, iq, graph_step=False):
    import torch
    if not gpu:
        torch.set_num_threads(2)      # CPU rehearsal: leave cores to the env workers and the inference server
    from applestar_amd.learner.rl_learner import RLLearner
    lrn = RLLearner({'common': {'experiment_name': 'pipeline'},
                     'learner': {'use_cuda': gpu, 'player_id': 'MP0', 'use_value_feature': False,
                                 'amp_dtype': 'bfloat16' if precision == 'bf16' else None,
                                 'data': {'batch_size': B, 'trajectory_length': T, 'buffer_size': 2 * B},
                                 'graph_step': bool(graph_step),
                                 'log_to_stdout': False},
                     'communication': comm})
    orig = lrn._train

    def timed(data):
        t0 = time.time()
        out = orig(data)
        th = time.time()                 # the step's host side (launches, Python) is done
        if gpu:
            torch.cuda.synchronize()
        t1 = time.time()
        iq.put((t1, lrn.last_iter.val + 1, t1 - t0, th - t0))
        return out
    lrn._train = timed
    lrn.run(max_iterations=1000000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=8)
    ap.add_argument('--seconds', type=float, default=60.0)
    ap.add_argument('--batch', type=int, default=6)
    ap.add_argument('--traj-len', type=int, default=64)
    ap.add_argument('--precision', choices=['bf16', 'fp32'], default='bf16')
    ap.add_argument('--workdir', default='/tmp/applestar_pipeline')
    ap.add_argument('--graph-step', action='store_true', help='the learner replays its whole step as one HIP graph')
    args = ap.parse_args()
    os.makedirs(args.workdir, exist_ok=True)
    os.chdir(args.workdir)
    import torch
    from werkzeug.serving import make_server
    from applestar_amd.comm.adapter import Coordinator, serve_coordinator, Adapter
    from applestar_amd.league.league import League
    from applestar_amd.league.api import create_league_app
    from applestar_amd.actor.actor import Actor

    gpu = torch.cuda.is_available()
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
            'league_port': lport, 'learner_send_model_freq': 50, 'learner_send_train_info_freq': 50,
            'actor_ask_for_job_interval': 3600, 'actor_model_update_interval': 30}
    T, B = args.traj_len, args.batch
    # the learner runs in its own process, as in a deployment: in a thread of the actor process its ~25 ms of
    # Python per step would hold the GIL the inference server's batching loop needs
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    iq = ctx.Queue()
    lp = ctx.Process(target=_learner_main, args=(comm, B, T, gpu, args.precision, iq, args.graph_step), daemon=True)
    lp.start()
    iters = []          # (wall time, iteration) after each learner iteration

    def drain():
        while True:
            iters.append(iq.get())
    threading.Thread(target=drain, daemon=True).start()
    actor = Actor({'common': {'experiment_name': 'pipeline'},
                   'actor': {'job_type': 'train', 'env_num': args.envs, 'gpu_batch_inference': True, 'traj_len': T,
                             'episode_num': 100000, 'print_freq': 1000000},
                   'env': {'game_steps_per_episode': 100000, 'fake': True},
                   'communication': comm})
    at = threading.Thread(target=lambda: actor.run(max_jobs=1), daemon=True)
    at.start()
    probe = Adapter('127.0.0.1', cport)
    t_start = time.time()
    # wait for the first learner iteration (actors warmed up, graphs captured), then measure
    while not iters and time.time() - t_start < 600:
        time.sleep(0.5)
    t0 = time.time()
    st0 = probe.stats()
    it0 = iters[-1][1] if iters else 0
    n_rec0 = len(iters)
    srv_stats = lambda: dict(actor._server.stats) if getattr(actor, '_server', None) is not None else {}
    ss0 = srv_stats()
    time.sleep(args.seconds)
    t1 = time.time()
    st1 = probe.stats()
    it1 = iters[-1][1] if iters else 0
    win = iters[n_rec0:]
    ss1 = srv_stats()
    sd = {k: ss1.get(k, 0.0) - ss0.get(k, 0.0) for k in ss1}
    pushed = st1.get('push', {}).get('MP0traj', 0) - st0.get('push', {}).get('MP0traj', 0)
    dt = t1 - t0
    n_it = it1 - it0
    out = {'metric': 'end-to-end single-GPU RL pipeline', 'envs': args.envs, 'precision': args.precision,
           'graph_step': bool(args.graph_step),
           'seconds': round(dt, 1), 'traj_len': T, 'batch': B,
           'trajectories_per_s': round(pushed / dt, 2),
           'actor_agent_steps_per_s': round(pushed * T / dt, 1),
           'actor_agent_steps_per_s_per_env_process': round(pushed * T / dt / max(args.envs, 1), 1),
           'learner_iters_per_s': round(n_it / dt, 3),
           'learner_samples_per_s_fed': round(n_it * B * T / dt, 1),
           # time inside the learner's train step (incl. the GPU finishing it) vs the whole iteration: the rest is
           # the learner waiting for / assembling data
           'learner_train_ms_mean': round(1e3 * sum(r[2] for r in win) / max(len(win), 1), 1),
           'learner_train_host_ms_mean': round(1e3 * sum(r[3] for r in win) / max(len(win), 1), 1),
           'learner_iter_ms_mean': round(1e3 * dt / max(n_it, 1), 1),
           'fresh_samples_per_s': round(pushed * T / dt, 1),
           'startup_s': round(t0 - t_start, 1),
           'inference_server': {
               'groups_per_s': round(sd.get('batches', 0) / dt, 1),
               'mean_group_rows': round(sd.get('requests', 0) / max(sd.get('batches', 0), 1), 2),
               'ms_per_group': {k[:-2]: round(1e3 * sd.get(k, 0) / max(sd.get('batches', 0), 1), 3)
                                for k in ('collate_h2d_s', 'launch_s', 'd2h_wait_s', 'decollate_s', 'reply_s',
                                          'served_s')},
               'host_busy_fraction': round(sum(sd.get(k, 0) for k in ('collate_h2d_s', 'launch_s', 'decollate_s',
                                                                       'reply_s')) / dt, 3)},
           'cpus': os.cpu_count(),
           'data': 'FakeSC2Env observations, random-init policy; learner reuses each trajectory 2x (reference)'}
    print(json.dumps(out), flush=True)
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
