"""Host (launch-side) time of the learner step's phases: model forward, loss, backward, update.

With a tiny batch the GPU never holds the host back, so these are the host floors of each phase
(dispatch, autograd bookkeeping, Python wrappers); with the bench batch they show where the host
waits.  No device syncs inside a step.

    python tools/host_phases.py [--batch 1 --unroll 2 --max-entities 16] [--steps 10]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer, _amp  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1)
    ap.add_argument('--unroll', type=int, default=2)
    ap.add_argument('--max-entities', type=int, default=16)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--no-sync', action='store_true', help='pipelined steps (no device sync between them): shows where the host blocks')
    ap.add_argument('--fp32', action='store_true', help='the fp32 step (no autocast, fp32 weights)')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    amp = None if args.fp32 else 'bfloat16'
    tr = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': amp}, 'model': {'enable_baselines': ['winloss']}},
                   device=dev)
    h = rl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    tot = {}
    for i in range(args.steps + 3):
        if not args.no_sync:
            torch.cuda.synchronize()
        t = [time.perf_counter()]
        if not tr.model.training:
            tr.model.train()
        with _amp(dev, amp):
            out = tr.model.rl_learner_forward(**b)
        t.append(time.perf_counter())
        info = tr.loss.compute_loss(out)
        t.append(time.perf_counter())
        tr.reducer.zero_grad(buffers=False)
        if tr.master is not None:
            tr.master.backward(info['total_loss'])
        else:
            tr.reducer.backward(info['total_loss'])
        t.append(time.perf_counter())
        tr._reduce()
        tr._update()
        t.append(time.perf_counter())
        if not args.no_sync:
            torch.cuda.synchronize()
        t.append(time.perf_counter())
        if i >= 3:
            for k, a, z in (('forward', 0, 1), ('loss', 1, 2), ('backward', 2, 3), ('update', 3, 4), ('gpu_tail', 4, 5),
                            ('total', 0, 5)):
                tot[k] = tot.get(k, 0.0) + (t[z] - t[a])
    n = args.steps
    print(f'batch {args.batch} x unroll {args.unroll}, max entities {args.max_entities}: host ms per phase ' +
          ', '.join(f'{k} {1000 * v / n:.2f}' for k, v in tot.items()))


if __name__ == '__main__':
    main()
