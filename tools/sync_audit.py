"""Host <-> device synchronisations inside one learner step: every op that makes the host wait for the GPU
(``torch.cuda.set_sync_debug_mode``) with the framework call site that issued it, counted per site.

    python tools/sync_audit.py [--precision fp32|bf16] [--mode rl|sl] [--steps 2]

A sync in the middle of the step drains the launch queue: the GPU idles while the host catches up (the largest
idle gaps of ``tools/prof_gaps.py``).  Run after warm-up, so one-off syncs (allocation, autotuning) are excluded.
"""
import argparse
import collections
import json
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
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=3)
    args = ap.parse_args()
    import bench
    from applestar_amd.rl.synthetic import rl_batch, sl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree
    device = torch.device('cuda', 0)
    mk = rl_batch if args.mode == 'rl' else sl_batch
    batches = [pin_tree(mk(6, 64, max_entities=512, seed=i)) for i in range(2)]
    ns = argparse.Namespace(mode=args.mode, graph=False, batch=6, unroll=64)
    trainer = bench._make_trainer(ns, args.precision, device, args.mode)

    def source():
        i = 0
        while True:
            yield batches[i % 2]
            i += 1
    it = DevicePrefetcher(source(), device)
    for _ in range(args.warmup):
        trainer.step(next(it))
    torch.cuda.synchronize()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sites = collections.Counter()
    examples = {}

    def show(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1] if f.filename.startswith(root) and 'sync_audit' not in f.filename]
        key = ' <- '.join(f'{os.path.relpath(f.filename, root)}:{f.lineno}' for f in reversed(stack[-4:]))
        sites[key] += 1
        examples.setdefault(key, str(message)[:120])
    warnings.showwarning = show
    warnings.simplefilter('always')
    torch.cuda.set_sync_debug_mode('warn')
    for _ in range(args.steps):
        trainer.step(next(it))
    torch.cuda.set_sync_debug_mode('default')
    torch.cuda.synchronize()
    print(json.dumps({'precision': args.precision, 'mode': args.mode, 'steps': args.steps,
                      'syncs_per_step': sum(sites.values()) / args.steps}))
    for k, n in sites.most_common():
        print(f'{n / args.steps:6.1f}/step  {k}\n         {examples[k]}')


if __name__ == '__main__':
    main()
