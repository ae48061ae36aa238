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


def _cgroup_cpu():
    """cgroup v2 cpu.stat of this job (usage / throttling under a CPU quota), {} when not readable."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            d = dict(line.split() for line in f if line.strip())
        with open('/sys/fs/cgroup/cpu.max') as f:
            d['max'] = f.read().strip()
        return d
    except OSError:
        return {}


def _cg_delta(a, b, dt):
    if not a or not b:
        return {}
    out = {'cpu.max': b.get('max')}
    for k in ('usage_usec', 'throttled_usec', 'nr_throttled', 'nr_periods'):
        if k in a and k in b:
            out[k] = int(b[k]) - int(a[k])
    if 'usage_usec' in out:
        out['cpus_used'] = round(out['usage_usec'] / 1e6 / dt, 2)
    return out


def _learner_main(comm, B, T, gpu, precision, iq, graph_step=False, max_reuse=2, stop_ev=None):
    import torch
    sw = os.environ.get('APPLESTAR_PIPE_SWITCH')
    if sw:
        sys.setswitchinterval(float(sw))     # the GIL hand-over interval of the learner process (default 5 ms)
    if not gpu:
        torch.set_num_threads(2)      # CPU rehearsal: leave cores to the env workers and the inference server
    from applestar_amd.learner.rl_learner import RLLearner
    lrn = RLLearner({'common': {'experiment_name': 'pipeline'},
                     'learner': {'use_cuda': gpu, 'player_id': 'MP0', 'use_value_feature': False,
                                 'amp_dtype': 'bfloat16' if precision == 'bf16' else None,
                                 'data': {'batch_size': B, 'trajectory_length': T, 'buffer_size': 2 * B,
                                          'max_reuse': max_reuse},
                                 'graph_step': bool(graph_step),
                                 'log_to_stdout': False},
                     'communication': comm})
    orig = lrn._train

    prof_at = int(os.environ.get('APPLESTAR_PIPE_PROFILE_AT', '0'))     # cProfile the learner's main thread
    prof_n = int(os.environ.get('APPLESTAR_PIPE_PROFILE_N', '5'))
    prof_out = os.environ.get('APPLESTAR_PIPE_PROFILE_OUT', 'learner_profile.txt')
    state = {'n': 0, 'prof': None}

    def thread_cpu():
        """{thread id: (name, cpu seconds)} from /proc (Linux)."""
        out = {}
        try:
            for tid in os.listdir('/proc/self/task'):
                with open(f'/proc/self/task/{tid}/stat') as f:
                    parts = f.read().rsplit(')', 1)[1].split()
                with open(f'/proc/self/task/{tid}/comm') as f:
                    name = f.read().strip()
                out[int(tid)] = (name, (int(parts[11]) + int(parts[12])) / os.sysconf('SC_CLK_TCK'))
        except OSError:
            pass
        return out

    def sampler(stop, hist):
        """Every 2 ms: the innermost frame of every Python thread (sampled while this thread holds the GIL)."""
        import sys as _sys
        import traceback as _tb
        names = {}
        while not stop.is_set():
            for t in threading.enumerate():
                names[t.ident] = t.name
            for ident, fr in _sys._current_frames().items():
                if ident == threading.get_ident():
                    continue
                st = _tb.extract_stack(fr)[-3:]
                key = (names.get(ident, str(ident)),
                       ' < '.join(f'{os.path.basename(x.filename)}:{x.lineno}:{x.name}' for x in st[::-1]))
                hist[key] = hist.get(key, 0) + 1
            time.sleep(0.002)

    def timed(data):
        if stop_ev is not None and stop_ev.is_set():
            raise SystemExit(0)         # a normal interpreter exit (atexit handlers run: profiler traces flush)
        state['n'] += 1
        if prof_at and state['n'] == prof_at:
            import cProfile
            state['prof'] = cProfile.Profile()
            state['cpu0'] = thread_cpu()
            state['wall0'] = time.time()
            state['hist'] = {}
            state['stop'] = threading.Event()
            if os.environ.get('APPLESTAR_PIPE_SAMPLER', '0') == '1':     # perturbs: it takes the GIL every 2 ms
                threading.Thread(target=sampler, args=(state['stop'], state['hist']), daemon=True,
                                 name='stack-sampler').start()
            state['prof'].enable()
        t0, c0, tc0 = time.time(), time.process_time(), time.thread_time()
        if gpu:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        out = orig(data)
        th = time.time()                 # the step's host side (launches, Python) is done
        if gpu:
            e1.record()
            torch.cuda.synchronize()
        t1, c1, tc1 = time.time(), time.process_time(), time.thread_time()
        if state['prof'] is not None and state['n'] == prof_at + prof_n - 1:
            import io
            import pstats
            state['prof'].disable()
            state['stop'].set()
            cpu1, wall = thread_cpu(), time.time() - state['wall0']
            buf = io.StringIO()
            buf.write(f'per-thread CPU over the window ({wall:.2f} s wall):\n')
            rows = sorted(((c - state['cpu0'].get(t, (n, 0.0))[1], n, t) for t, (n, c) in cpu1.items()), reverse=True)
            pynames = {t.native_id: t.name for t in threading.enumerate()}
            for c, n, t in rows[:20]:
                buf.write(f'  {c:7.3f} s  {n} ({t}) {pynames.get(t, "")}\n')
            buf.write('\nstack samples of the other Python threads (thread, innermost frames):\n')
            for (tn, st), c in sorted(state['hist'].items(), key=lambda kv: -kv[1])[:40]:
                buf.write(f'  {c:6d}  {tn}: {st}\n')
            buf.write('\n')
            st = pstats.Stats(state['prof'], stream=buf)
            st.sort_stats('tottime').print_stats(45)
            st.sort_stats('cumulative').print_stats(45)
            with open(prof_out, 'w') as f:
                f.write(f'{prof_n} learner iterations; cProfile of the main thread below\n' + buf.getvalue())
            state['prof'] = None
        # CPU seconds the learner process got during the step (all its threads) and the stream's span between
        # the step's first and last launch: wall >> cpu and >> gpu = the process waited to be scheduled
        iq.put((t1, lrn.last_iter.val + 1, t1 - t0, th - t0, c1 - c0,
                e0.elapsed_time(e1) / 1e3 if gpu else 0.0, tc1 - tc0))
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
    ap.add_argument('--max-reuse', type=int, default=2,
                    help='trainings per trajectory (reference: 2); huge = the ring fills once and ingest stops')
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
    stop_ev = ctx.Event()
    lp = ctx.Process(target=_learner_main, args=(comm, B, T, gpu, args.precision, iq, args.graph_step, args.max_reuse, stop_ev), daemon=True)
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
    cg0 = _cgroup_cpu()
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
           'graph_step': bool(args.graph_step), 'max_reuse': args.max_reuse,
           'switch_interval': os.environ.get('APPLESTAR_PIPE_SWITCH'),
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
           'learner_train_cpu_ms_mean': round(1e3 * sum(r[4] for r in win) / max(len(win), 1), 1),
           'learner_train_main_thread_cpu_ms_mean': round(1e3 * sum(r[6] for r in win) / max(len(win), 1), 1),
           'learner_train_stream_ms_mean': round(1e3 * sum(r[5] for r in win) / max(len(win), 1), 1),
           'learner_iter_ms_mean': round(1e3 * dt / max(n_it, 1), 1),
           'cgroup_cpu': _cg_delta(cg0, _cgroup_cpu(), dt),
           'affinity_cpus': len(os.sched_getaffinity(0)),
           'loadavg': open('/proc/loadavg').read().split()[:3],
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
    stop_ev.set()
    lp.join(timeout=30)        # the learner leaves at its next step (a clean exit: traced runs keep their data)
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
