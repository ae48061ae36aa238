"""Actor-side inference latency: policy step (compute_logp_action, sampling incl. the SU pointer loop)
and teacher forward, bf16 on one GPU, at batch sizes B (one row per env).  Reference figure:
batched GPU inference ~0.16 s per step for 16 envs.  Prints p50/p99 per B as JSON lines.
Usage: python tools/bench_inference.py [--batches 1,16,64] [--iters 30]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.models.model import Model  # noqa: E402
from applestar_amd.lib.features import random_obs, random_actions  # noqa: E402
from applestar_amd.rl.synthetic import to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', default='1,16,64')
    ap.add_argument('--iters', type=int, default=30)
    ap.add_argument('--entities', type=int, default=300)
    ap.add_argument('--graphs', type=int, default=1, help='also time the HIP-graph replay (runtime.graphs.GraphedPolicy)')
    ap.add_argument('--modes', default='', help='comma list of policy,teacher,policy_graph,teacher_graph (default all)')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    m = Model({'agent': {'extra_units': True}}).to(dev).eval().to(memory_format=torch.channels_last)
    if os.environ.get('APPLESTAR_INFERENCE_FORMS', '1') == '1':
        from applestar_amd.ops import native
        native.ensure_loaded()
        native.attach_inference_forms(m)       # as the inference server does (actor/inference.py set_model)
    for B in [int(x) for x in args.batches.split(',')]:
        g = torch.Generator().manual_seed(B)
        en = torch.randint(args.entities // 2, args.entities, (B,), generator=g)
        obs = random_obs(B, entity_num=en, generator=g)
        obs['hidden_state'] = [(torch.zeros(B, 384), torch.zeros(B, 384)) for _ in range(3)]
        obs = to_device(obs, dev)
        act, su_num = random_actions(B, en, generator=g)
        res = {}
        from applestar_amd.runtime.graphs import GraphedPolicy
        gp = GraphedPolicy(m, 'compute_logp_action')
        gt = GraphedPolicy(m, 'compute_teacher_logit')
        act_d = {k: v.to(dev) for k, v in act.items()}
        modes = [('policy', False), ('teacher', False)] + ([('policy_graph', True), ('teacher_graph', True)]
                                                           if args.graphs else [])
        if args.modes:
            modes = [m for m in modes if m[0] in args.modes.split(',')]
        for name, graphed in modes:
            times = []
            for i in range(args.iters + 3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                if graphed:
                    if name.startswith('policy'):
                        out = gp(**obs)
                    else:
                        out = gt(**obs, selected_units_num=su_num.to(dev), action_info=act_d)
                else:
                    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
                        if name == 'policy':
                            out = m.compute_logp_action(**obs)
                        else:
                            out = m.compute_teacher_logit(**obs, selected_units_num=su_num.to(dev), action_info=act_d)
                torch.cuda.synchronize()
                if i >= 3:
                    times.append((time.perf_counter() - t) * 1000)
            times.sort()
            res[name] = {'p50_ms': round(times[len(times) // 2], 2), 'p99_ms': round(times[-1], 2)}
        su = int(out['selected_units_num'].max()) if 'selected_units_num' in out else None
        pol = res.get('policy', res.get('policy_graph', {'p50_ms': float('nan')}))
        print(json.dumps({'batch': B, **res, 'per_env_policy_ms': round(pol['p50_ms'] / B, 3),
                          'reference_16env_ms': 160.0}), flush=True)


if __name__ == '__main__':
    main()
