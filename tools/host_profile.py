"""Host (Python) time of the learner step: cProfile over K steps after W warm-up steps, top functions by
cumulative and by own time.  Shows what the host does per step when the GPU work is graphed or fast.

    python tools/host_profile.py [--precision fp32|bf16] [--graph] [--steps 10] [--top 40]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='bf16')
    ap.add_argument('--graph', action='store_true')
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--top', type=int, default=40)
    args = ap.parse_args()
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree
    device = torch.device('cuda', 0)
    amp = 'bfloat16' if args.precision == 'bf16' else None
    trainer = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': args.graph, 'amp_dtype': amp},
                         'model': {'enable_baselines': ['winloss']}}, device=device)
    batches = [pin_tree(rl_batch(6, 64, seed=i)) for i in range(2)]

    def source():
        i = 0
        while True:
            yield batches[i % 2]
            i += 1

    it = DevicePrefetcher(source(), device)
    for _ in range(args.warmup):
        trainer.step(next(it))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        trainer.step(next(it))
    pr.disable()
    torch.cuda.synchronize()
    for key in ('cumulative', 'tottime'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(args.top)
        print(f'==== by {key} ({args.steps} steps)')
        print(s.getvalue())


if __name__ == '__main__':
    main()
