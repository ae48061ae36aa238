"""Op-level GPU time breakdown of RL learner iterations with torch.profiler (aten ops incl. backward,
and native kernels), grouped by top-level op.  Usage: python tools/op_profile.py [--steps 3] [--top 60]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--out', default='gpurun_out/op_profile.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    b = to_device(rl_batch(6, 64, seed=0), dev)
    for _ in range(2):
        tr.step(dict(b))
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=False) as prof:
        for _ in range(args.steps):
            tr.step(dict(b))
        torch.cuda.synchronize()
    ka = prof.key_averages()
    lines = []
    tot = sum(e.self_device_time_total for e in ka) / args.steps / 1000
    lines.append(f'total self device time per iter: {tot:.2f} ms')
    rows = sorted(ka, key=lambda e: -e.self_device_time_total)[:args.top]
    for e in rows:
        lines.append(f'{e.self_device_time_total / args.steps / 1000:8.3f} ms  {e.count // args.steps:6d}  {e.key[:110]}')
    lines.append('\n--- by total device time (incl. children), top ops ---')
    rows = sorted([e for e in ka if not e.key.startswith('void') and 'kernel' not in e.key.lower()],
                  key=lambda e: -e.device_time_total)[:args.top]
    for e in rows:
        lines.append(f'{e.device_time_total / args.steps / 1000:8.3f} ms  {e.count // args.steps:6d}  {e.key[:110]}')
    txt = '\n'.join(lines)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, 'w').write(txt)
    print(txt[:6000])


if __name__ == '__main__':
    main()
