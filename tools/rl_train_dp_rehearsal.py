"""Multi-rank rehearsal of the whole RL training system on ONE GPU: ``rl_train`` itself -
coordinator, league, the learner role under ``torch.distributed.run --nproc-per-node 2`` (gloo between the two
ranks, both on the one GPU: RCCL refuses two ranks on one device), and an actor with fake-env workers feeding the
GPU inference server - runs N learner iterations; each learner rank then writes a weight fingerprint
(learner.fingerprint_path) and the replicas must be identical (the data-parallel invariant: every rank pulled its
own trajectories, the gradients were all-reduced, the updates match).

    python tools/rl_train_dp_rehearsal.py [--iters 6] [--ranks 2] [--out gpurun_out/rl_train_dp2]

Prints one JSON line (ranks, iterations, identical, wall seconds); exit code 1 if the replicas differ.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=6)
    ap.add_argument('--ranks', type=int, default=2)
    ap.add_argument('--out', default=os.path.join(ROOT, 'gpurun_out', 'rl_train_dp2'))
    ap.add_argument('--timeout', type=float, default=420)
    args = ap.parse_args()
    from applestar_amd.utils.config import read_config, save_config
    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)
    cfg = read_config(os.path.join(ROOT, 'applestar_amd', 'bin', 'rl_user_config.yaml'))
    c = cfg.communication
    c.coordinator_port, c.league_port = free_port(), free_port()
    c.learner_send_model_freq = 2
    c.actor_model_update_interval = 2
    cfg.common.experiment_name = 'dp_rehearsal'
    lc = cfg.learner
    lc.max_iterations = args.iters
    lc.value_pretrain_iters = 0
    lc.fingerprint_path = os.path.join(out, 'fingerprints')
    lc.data.batch_size, lc.data.trajectory_length, lc.data.buffer_size = 2, 8, 4
    lc.data.ring_gb = 2                      # two learner ranks + the inference server share the one GPU
    lc.hook = {}
    cfg.actor.env_num = 6
    cfg.actor.traj_len = 8
    cfg.env.game_steps_per_episode = 2000
    cfg.env.fake = True
    # no released checkpoints on the boxes: random-init players / teacher (the league's 'none' path)
    lg = cfg.league
    lg.active_players.checkpoint_path = ['none']
    lg.active_players.teacher_path = ['none']
    lg.active_players.teacher_id = ['none']
    lg.historical_players.checkpoint_path = ['none']
    lg.use_historical_players = False
    lg.fake_model = True
    cfg.actor.fake_model = True
    cfg_path = os.path.join(out, 'rl_user_config.yaml')
    save_config(cfg, cfg_path)
    fp = lc.fingerprint_path
    if os.path.isdir(fp):
        for f in os.listdir(fp):
            os.unlink(os.path.join(fp, f))
    env = dict(os.environ, APPLESTAR_DIST_BACKEND='gloo', PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''))
    base = [sys.executable, '-m', 'applestar_amd.bin.rl_train', '--config', cfg_path, '--task', 'bot']
    logs = {r: open(os.path.join(out, f'{r}.log'), 'w') for r in ('coordinator', 'league', 'learner', 'actor')}
    procs = {}
    t0 = time.time()
    try:
        procs['coordinator'] = subprocess.Popen(base + ['--type', 'coordinator'], cwd=out, env=env,
                                                stdout=logs['coordinator'], stderr=subprocess.STDOUT)
        procs['league'] = subprocess.Popen(base + ['--type', 'league'], cwd=out, env=env, stdout=logs['league'],
                                           stderr=subprocess.STDOUT)
        time.sleep(5)
        learner = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.ranks),
                   '--master-addr', '127.0.0.1', '--master-port', str(free_port()), '-m', 'applestar_amd.bin.rl_train',
                   '--config', cfg_path, '--task', 'bot', '--type', 'learner']
        procs['learner'] = subprocess.Popen(learner, cwd=out, env=env, stdout=logs['learner'], stderr=subprocess.STDOUT)
        time.sleep(5)
        procs['actor'] = subprocess.Popen(base + ['--type', 'actor', '--fake-env'], cwd=out, env=env,
                                          stdout=logs['actor'], stderr=subprocess.STDOUT)
        rc = None
        while time.time() - t0 < args.timeout:
            rc = procs['learner'].poll()
            if rc is not None:
                break
            for r in ('coordinator', 'league', 'actor'):
                if procs[r].poll() is not None:
                    raise RuntimeError(f'{r} exited early with {procs[r].returncode} (see {out}/{r}.log)')
            time.sleep(2)
        if rc is None:
            raise RuntimeError(f'learners did not finish {args.iters} iterations in {args.timeout} s')
        if rc != 0:
            raise RuntimeError(f'learner ranks failed with {rc} (see {out}/learner.log)')
    finally:
        for r in ('actor', 'learner', 'league', 'coordinator'):
            p = procs.get(r)
            if p is not None and p.poll() is None:
                p.terminate()
                try:
                    p.wait(20)
                except subprocess.TimeoutExpired:
                    p.kill()
        for f in logs.values():
            f.close()
    recs = []
    for f in sorted(os.listdir(fp)):
        with open(os.path.join(fp, f)) as fh:
            recs.append(json.load(fh))
    same = len(recs) == args.ranks and len({(r['iter'], r['weight_hash']) for r in recs}) == 1
    res = {'ranks': args.ranks, 'iterations': [r['iter'] for r in recs], 'weight_hashes': [r['weight_hash'] for r in recs],
           'replicas_identical': same, 'wall_s': round(time.time() - t0, 1), 'backend': 'gloo (ranks share one GPU)'}
    print(json.dumps(res), flush=True)
    with open(os.path.join(out, 'result.json'), 'w') as f:
        json.dump(res, f)
    sys.exit(0 if same else 1)


if __name__ == '__main__':
    main()
