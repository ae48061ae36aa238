"""Trajectory ring throughput on the GPU: ingest of realistic RL trajectories (T=64, entity counts
up to 500, teacher logits incl. 24320 location logits) and on-device batch assembly (B=6), vs the
host deserialize + collate path.  Usage: python tools/bench_ring.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.agent.collate import collate_trajectories  # noqa: E402
from applestar_amd.lib.features import random_obs, random_actions, actions_mask  # noqa: E402
from applestar_amd.runtime.traj_ring import TrajectoryRing  # noqa: E402
from applestar_amd.utils import serialize  # noqa: E402


def traj(g, T=64):
    steps = []
    for t in range(T + 1):
        o = random_obs(1, max_entities=500, generator=g)
        n = int(o['entity_num'][0])
        s = {'spatial_info': {k: v[0] for k, v in o['spatial_info'].items()},
             'entity_info': {k: v[0][:n] for k, v in o['entity_info'].items()},
             'scalar_info': {k: v[0] for k, v in o['scalar_info'].items()},
             'entity_num': o['entity_num'][0], 'hidden_state': [(torch.zeros(384), torch.zeros(384))] * 3}
        if t < T:
            a, su = random_actions(1, o['entity_num'], generator=g)
            k = int(su[0])
            s['action_info'] = {kk: (v[0][:k] if kk == 'selected_units' else v[0]) for kk, v in a.items()}
            s['selected_units_num'] = su[0]
            s['behaviour_logp'] = {kk: torch.zeros(()) for kk in a}
            s['behaviour_logp']['selected_units'] = torch.zeros(k)
            s['teacher_logit'] = {'action_type': torch.randn(327), 'delay': torch.randn(128), 'queued': torch.randn(2),
                                  'selected_units': torch.randn(k, n + 1), 'target_unit': torch.randn(n),
                                  'target_location': torch.randn(24320)}
            s['mask'] = {'actions_mask': {kk: v[0] for kk, v in actions_mask(a['action_type']).items()},
                         'cum_action_mask': torch.tensor(1.), 'build_order_mask': torch.tensor(1.),
                         'built_unit_mask': torch.tensor(1.)}
            s['reward'] = {kk: torch.zeros(()) for kk in ('winloss', 'build_order', 'built_unit', 'battle')}
            s['step'] = torch.tensor(1.)
            s['model_last_iter'] = torch.tensor(0.)
        steps.append(s)
    return steps


def main():
    g = torch.Generator().manual_seed(0)
    trajs = [traj(g) for _ in range(6)]
    frames = [serialize.dumps(t) for t in trajs]
    mb = sum(len(f) for f in frames) / len(frames) / 1e6
    ring = TrajectoryRing(4 << 30, device='cuda')
    ids = [ring.put(f) for f in frames]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        ids = [ring.put(f) for f in frames]
    torch.cuda.synchronize()
    ingest = (time.perf_counter() - t) / 18 * 1000
    b = ring.batch(ids)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        b = ring.batch(ids)
    torch.cuda.synchronize()
    assemble = (time.perf_counter() - t) / 5 * 1000
    t = time.perf_counter()
    host = collate_trajectories([serialize.loads(f) for f in frames])
    host_ms = (time.perf_counter() - t) * 1000
    print(json.dumps({'traj_mb': round(mb, 1), 'ring_ingest_ms_per_traj': round(ingest, 2),
                      'ring_batch_ms_B6': round(assemble, 2), 'host_deserialize_collate_ms_B6': round(host_ms, 1)}))


if __name__ == '__main__':
    main()
