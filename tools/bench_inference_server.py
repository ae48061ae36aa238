"""Synthetic-client throughput of the actor inference server (>= 4,000 agent-steps/s of
policy + teacher on one GPU).

    python tools/bench_inference_server.py --procs 8 --envs-per-proc 16 --seconds 20 [--kind policy+teacher]

``--procs`` client processes each drive ``--envs-per-proc`` routed pipes (one per simulated env, every pipe with
one request in flight, as an env worker blocks on its reply), so the server sees procs x envs outstanding
requests.  Requests are pre-encoded frames of the agent's exact schema with entity counts drawn from U[20, 320]
(the fake env's range); the server runs the training-actor path (policy sample + teacher logits in one graph per
(batch bucket, entity bucket)).  Reports agent-steps/s after a warm-up (graph captures), the per-batch host phases
and the mean batch size.  One JSON line on stdout.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _frames(n, seed, kind):
    import torch
    from applestar_amd.lib.features import random_obs
    from applestar_amd.utils import serialize
    g = torch.Generator().manual_seed(seed)
    ents = torch.randint(20, 321, (n,), generator=g)
    obs = random_obs(n, entity_num=ents, generator=g)
    out = []
    for i in range(n):
        k = int(ents[i])
        r = {key: ({kk: (vv[i, :k] if key == 'entity_info' else vv[i]) for kk, vv in v.items()}
                   if isinstance(v, dict) else v[i]) for key, v in obs.items()}
        r['hidden_state'] = [(torch.zeros(384), torch.zeros(384)) for _ in range(3)]
        if kind == 'policy+teacher':
            r['teacher_hidden_state'] = [(torch.zeros(384), torch.zeros(384)) for _ in range(3)]
        out.append(serialize.dumps(r))
    return out


def _client(conns, seed, kind, t_stop, q):
    import torch
    torch.set_num_threads(1)
    frames = _frames(len(conns), seed, kind)
    from multiprocessing.connection import wait
    n = 0
    for c, f in zip(conns, frames):
        c.send_bytes(f)
    idx = {id(c): i for i, c in enumerate(conns)}
    while time.time() < t_stop:
        for c in wait(conns, timeout=0.5):
            c.recv_bytes()
            n += 1
            c.send_bytes(frames[idx[id(c)]])
    q.put(n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=8)
    ap.add_argument('--envs-per-proc', type=int, default=16)
    ap.add_argument('--seconds', type=float, default=20.0)
    ap.add_argument('--warmup', type=float, default=25.0, help='seconds of serving before the timed window')
    ap.add_argument('--kind', default='policy+teacher', choices=['policy', 'policy+teacher'])
    ap.add_argument('--max-batch', type=int, default=64)
    args = ap.parse_args()
    import torch
    from applestar_amd.actor.inference import InferenceServer
    from applestar_amd.models.model import Model
    dev = 'cuda' if torch.cuda.is_available() else 'cpu'
    srv = InferenceServer(dev, max_wait_ms=1.0, max_batch=args.max_batch)
    torch.manual_seed(0)
    srv.set_model('p', Model().eval())
    srv.set_model('t', Model().eval(), teacher=True)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    t_start = time.time() + 5.0
    t_stop = t_start + args.warmup + args.seconds + 5.0
    procs = []
    route = ('p', args.kind, 't' if args.kind != 'policy' else None)
    for p in range(args.procs):
        kids = []
        for _ in range(args.envs_per_proc):
            a, b = ctx.Pipe()
            srv.add_connection(a, route=route)
            kids.append(b)
        pr = ctx.Process(target=_client, args=(kids, 100 + p, args.kind, t_stop, q), daemon=True)
        pr.start()
        procs.append(pr)
    t_warm_end = time.time() + args.warmup
    last_print = time.time()
    while time.time() < t_warm_end:
        srv.serve_once(timeout=0.05)
        if time.time() - last_print > 10:
            print(f'warm-up: {int(srv.stats["requests"])} requests, {len(srv._graphed)} graphs', file=sys.stderr,
                  flush=True)
            last_print = time.time()
    base = dict(srv.stats)
    t0 = time.time()
    while time.time() < t0 + args.seconds:
        srv.serve_once(timeout=0.05)
    dt = time.time() - t0
    st = {k: srv.stats[k] - base.get(k, 0.0) for k in srv.stats}
    while any(p.is_alive() for p in procs) and time.time() < t_stop + 10:
        srv.serve_once(timeout=0.05)
    srv.drain()
    nb = max(st.get('batches', 0), 1)
    res = {'metric': 'inference_server_agent_steps_per_s', 'kind': args.kind, 'device': dev,
           'value': round(st['requests'] / dt, 1), 'clients': args.procs * args.envs_per_proc,
           'mean_batch': round(st['requests'] / nb, 2), 'seconds': round(dt, 2),
           'graphs': len(srv._graphed),
           'per_batch_ms': {k[:-2]: round(1000 * st.get(k, 0.0) / nb, 3)
                            for k in ('collate_h2d_s', 'launch_s', 'd2h_wait_s', 'decollate_s', 'reply_s', 'served_s')}}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
