"""Attribute the GPU time of small torch ops (casts, copies, adds, masks, reductions) to their source:
forward ops by the innermost applestar_amd stack frame, backward ops by their autograd node.
Usage: python tools/elementwise_attrib.py [--steps 2] [--top 70]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--top', type=int, default=70)
    ap.add_argument('--out', default='gpurun_out/elementwise_attrib.txt')
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='bf16')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    amp = 'bfloat16' if args.precision == 'bf16' else None
    tr = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': amp}, 'model': {'enable_baselines': ['winloss']}},
                   device=dev)
    b = to_device(rl_batch(6, 64, seed=0), dev)
    for _ in range(2):
        tr.step(dict(b))
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step(dict(b))
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0.0, 0])
    for e in prof.events():
        t = e.self_device_time_total
        if t <= 0 or not e.name.startswith('aten::'):
            continue
        where = None
        for fr in (e.stack or []):
            if 'applestar_amd' in fr and 'trainer.py' not in fr:
                where = fr.split('applestar_amd/')[-1]
                break
        if where is None:
            p = e.cpu_parent
            while p is not None and 'evaluate_function' not in p.name and 'Optimizer' not in p.name:
                p = p.cpu_parent
            where = p.name.replace('autograd::engine::evaluate_function: ', 'bwd ') if p is not None else '?'
        a = agg[(e.name, where)]
        a[0] += t
        a[1] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.top]
    tot = sum(v[0] for v in agg.values()) / args.steps / 1000
    lines = [f'aten-op self device time per iter: {tot:.2f} ms']
    for (name, where), (t, n) in rows:
        lines.append(f'{t / args.steps / 1000:8.3f} ms {n // args.steps:5d}  {name:32s} {where[:120]}')
    txt = '\n'.join(lines)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, 'w').write(txt)
    print(txt)


if __name__ == '__main__':
    main()
