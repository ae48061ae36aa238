"""Find host <-> GPU synchronisations inside one learner step (the bench's fp32 RL step by default).

A synchronising call (``.item()``, a pageable H2D/D2H copy, ``nonzero``, ...) makes the host wait for the GPU
to drain its queue; afterwards the GPU idles while the host issues the next kernels.  torch's sync debug mode
reports every such call; this tool records the Python stack of each report during W+1 steps and prints the
call sites of the last step, most frequent first.

    python tools/sync_audit.py [--precision fp32|bf16] [--mode rl|sl] [--warmup 3] [--depth 6]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    ap.add_argument('--mode', choices=['rl', 'sl'], default='rl')
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--depth', type=int, default=6)
    ap.add_argument('--graph', action='store_true')
    args = ap.parse_args()
    from applestar_amd.rl.synthetic import rl_batch, sl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher
    from applestar_amd.runtime.prefetch import pin_tree
    device = torch.device('cuda', 0)
    amp = 'bfloat16' if args.precision == 'bf16' else None
    if args.mode == 'rl':
        from applestar_amd.rl.trainer import RLTrainer
        trainer = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': args.graph, 'amp_dtype': amp},
                             'model': {'enable_baselines': ['winloss']}}, device=device)
        batches = [pin_tree(rl_batch(6, 64, seed=i)) for i in range(2)]
    else:
        from applestar_amd.sl.trainer import SLTrainer
        trainer = SLTrainer({'learner': {'ignore_steps': 0, 'amp_dtype': amp,
                                         'data': {'batch_size': 6, 'trajectory_length': 64}}}, device=device)
        batches = [pin_tree(sl_batch(6, 64, seed=i)) for i in range(2)]

    def source():
        i = 0
        while True:
            yield batches[i % 2]
            i += 1

    it = DevicePrefetcher(source(), device)
    for _ in range(args.warmup):
        trainer.step(next(it))
    torch.cuda.synchronize()

    sites = collections.Counter()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def record(message, category, filename, lineno, file=None, line=None):
        if 'synchroniz' not in str(message):
            return
        st = [f for f in traceback.extract_stack()[:-1] if 'warnings.py' not in f.filename]
        own = [f for f in st if f.filename.startswith(here) and 'sync_audit' not in f.filename]
        key = ' <- '.join(f'{os.path.relpath(f.filename, here)}:{f.lineno} {f.name}' for f in reversed(own[-args.depth:]))
        sites[(str(message).split('\n')[0][:60], key)] += 1

    old = warnings.showwarning
    warnings.showwarning = record
    warnings.simplefilter('always')
    torch.cuda.set_sync_debug_mode('warn')
    b = next(it)
    trainer.step(b)
    torch.cuda.set_sync_debug_mode('default')
    warnings.showwarning = old
    torch.cuda.synchronize()
    total = sum(sites.values())
    print(f'{total} synchronising calls in one {args.mode} {args.precision} step')
    for (msg, key), n in sites.most_common():
        print(f'{n:5d}  {msg}\n       {key}')


if __name__ == '__main__':
    main()
