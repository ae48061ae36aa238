"""Per-step loss / gradient-norm trace of the RL learner step (finiteness debugging).

    python tools/loss_probe.py --steps 8 --seed-base 1000          # one process, rank-1 data
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/loss_probe.py --steps 8   # every rank prints

Prints one JSON line per step and rank: total loss, clipped-gradient norm and, on the first step with a
non-finite gradient, the parameter names that carry it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=8)
    ap.add_argument('--batch', type=int, default=6)
    ap.add_argument('--unroll', type=int, default=64)
    ap.add_argument('--seed-base', type=int, default=-1, help='batch seed base (default: 1000 * rank, as bench.py)')
    ap.add_argument('--n-batches', type=int, default=2)
    ap.add_argument('--loss-parts', action='store_true')
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    args = ap.parse_args()

    from applestar_amd.parallel import dist as pdist
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher

    rank, world = pdist.init()
    gpu = torch.cuda.is_available()
    device = torch.device('cuda', torch.cuda.current_device()) if gpu else torch.device('cpu')
    torch.manual_seed(1234 + rank)
    trainer = RLTrainer({'learner': {'use_value_feature': True,
                                     'amp_dtype': 'bfloat16' if args.precision == 'bf16' else None},
                         'model': {'enable_baselines': ['winloss']}}, device=device)
    base = 1000 * rank if args.seed_base < 0 else args.seed_base
    batches = [rl_batch(args.batch, args.unroll, seed=base + i) for i in range(args.n_batches)]

    def source():
        i = 0
        while True:
            yield batches[i % len(batches)]
            i += 1

    it = DevicePrefetcher(source(), device)
    reported = False
    for s in range(args.steps):
        info = trainer.step(next(it))
        rec = {'rank': rank, 'world': world, 'step': s, 'loss': float(info['total_loss']),
               'grad_norm': float(info['gradient'])}
        # bit-level fingerprint of the weights after the update: identical on every rank iff the ranks hold
        # the same replica (the fp32 masters in the bf16 step)
        with torch.no_grad():
            flat = trainer.master.master.detach() if trainer.master is not None else \
                torch.cat([p.detach().reshape(-1) for p in trainer.params])
            rec['weight_sum'] = float(flat.double().sum())
            rec['weight_hash'] = int((flat.view(torch.int32).long() * 2654435761 % (1 << 31)).sum().item())
        if args.loss_parts:
            rec['parts'] = {k: float(v) for k, v in info.items()
                            if torch.is_tensor(v) and v.numel() == 1 and k not in ('total_loss', 'gradient')}
        bad = trainer.nonfinite_grads()
        if bad and not reported:
            rec['nonfinite_grads'] = bad[:40]
            rec['n_nonfinite'] = len(bad)
            reported = True
        sys.stdout.write(json.dumps(rec) + '\n')   # one write per record: ranks share the launcher's stdout
        sys.stdout.flush()
    pdist.finalize()


if __name__ == '__main__':
    main()
