#!/usr/bin/env python
"""Headline benchmark: RL learner samples/sec of the AlphaStar policy (BASELINE.json).

Config: per GPU 6 trajectories x 64 steps (= 384 learner samples / iteration), the
reference RL learner model (policy 29.1 M + value encoder + winloss baseline, ``use_value_feature``),
full iteration timed: H2D of the next batch (overlapped), encoder over (T+1)*B observations, core
LSTM, teacher-forced heads, V-trace/UPGO/TD(lambda)/entropy/KL loss, backward, RCCL gradient
all-reduce, grad clip, Adam.  Synthetic observations with the reference fake-data distribution
(entity_num ~ U[1,512), padded to the batch max), random-init weights, bf16 compute.

Run:  python bench.py --gpus 1 --steps 10 --warmup 3
      torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_PER_GPU = 256.0  # samples/s/GPU, 32xA100 learner, docs/guidance_to_small_scale_training.md:280-284
SL_BASELINE_PER_GPU = 384.0  # samples/s/GPU, 56xA100 SL learner, docs/guidance_to_small_scale_training.md:178-184


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=6, help='trajectories per GPU')
    ap.add_argument('--unroll', type=int, default=64)
    ap.add_argument('--max-entities', type=int, default=512)
    ap.add_argument('--n-batches', type=int, default=2, help='distinct synthetic batches cycled')
    ap.add_argument('--no-native', action='store_true', help='disable HIP kernels (torch-only baseline)')
    ap.add_argument('--profile-steps', type=int, default=0)
    ap.add_argument('--mode', choices=['rl', 'sl'], default='rl',
                    help='rl: the headline RL learner step; sl: supervised learner step (reference 384 samples/s/GPU)')
    ap.add_argument('--graph', action='store_true', help='replay the learner step from HIP graphs (runtime/step_graph.py)')
    ap.add_argument('--conv-benchmark', type=int, default=-1,
                    help='1/0: force MIOpen find-mode autotuning of convolutions on/off (-1: trainer default)')
    args = ap.parse_args()

    from applestar_amd.parallel import dist as pdist
    from applestar_amd import ops
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree

    rank, world = pdist.init()
    if world != args.gpus and rank == 0:
        print(f'warning: --gpus {args.gpus} but WORLD_SIZE={world}', file=sys.stderr)
    gpu = torch.cuda.is_available()
    device = torch.device('cuda', torch.cuda.current_device()) if gpu else torch.device('cpu')
    if args.no_native:
        ops.set_native(False)
    if args.conv_benchmark >= 0:
        torch.backends.cudnn.benchmark = bool(args.conv_benchmark)
    torch.manual_seed(1234 + rank)

    if args.mode == 'rl':
        trainer = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': args.graph},
                             'model': {'enable_baselines': ['winloss']}}, device=device)
        make = lambda i: rl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i)  # noqa
    else:
        from applestar_amd.sl.trainer import SLTrainer
        from applestar_amd.rl.synthetic import sl_batch
        trainer = SLTrainer({'learner': {'ignore_steps': 0, 'data': {'batch_size': args.batch,
                                                                       'trajectory_length': args.unroll}}},
                            device=device)
        make = lambda i: sl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i)  # noqa
    host_batches = [pin_tree(make(i)) if gpu else make(i) for i in range(args.n_batches)]

    def source():
        i = 0
        while True:
            yield host_batches[i % len(host_batches)]
            i += 1

    it = DevicePrefetcher(source(), device)

    def sync():
        if gpu:
            torch.cuda.synchronize()
        pdist.barrier()
        if gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        info = trainer.step(next(it))
    sync()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        info = trainer.step(next(it))
        host += time.perf_counter() - h0
    sync()
    elapsed = time.perf_counter() - t0
    loss = float(info['total_loss'].detach())
    t = torch.tensor([elapsed], dtype=torch.float64, device=device if gpu else 'cpu')
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = 1000.0 * elapsed / max(args.steps, 1)
    samples = args.batch * args.unroll * world * args.steps
    value = samples / elapsed
    if rank == 0:
        out = {
            'metric': 'learner samples/sec (AlphaStar policy)' if args.mode == 'rl' else
                      'SL learner samples/sec (AlphaStar policy)',
            'value': round(value, 2),
            'unit': 'samples/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': round(value / ((BASELINE_PER_GPU if args.mode == 'rl' else SL_BASELINE_PER_GPU) * world), 3),
            'dtype': 'bf16',
            'data': 'synthetic (reference fake-data distribution, entity_num~U[1,512)), random-init weights',
            'config': {
                'model': 'AlphaStar policy + value encoder + winloss baseline (DI-star rl_model arch)' if args.mode == 'rl'
                         else 'AlphaStar policy (DI-star sl_model arch)',
                'global_batch': args.batch * world,
                'seq_len': args.unroll,
                'parallelism': f'dp{world}',
                'samples_per_step': args.batch * args.unroll * world,
                'baseline_note': 'vs_baseline = per-GPU samples/s / 256 (reference RL learner, A100)' if args.mode == 'rl'
                                 else 'vs_baseline = per-GPU samples/s / 384 (reference SL learner, A100)',
                'native_kernels': (not args.no_native) and gpu,
                'final_loss': loss,
                'host_ms_per_step': round(1000.0 * host / max(args.steps, 1), 3),
                'graph_step': ({'captures': trainer.graph.captures, 'replays': trainer.graph.replays,
                                'eager_steps': trainer.graph.eager_steps,
                                'host_ms_per_replay': {k: round(1000.0 * v / max(trainer.graph.replays, 1), 3)
                                                       for k, v in trainer.graph.host_time.items()}}
                               if getattr(trainer, 'graph', None) is not None else None),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.finalize()


if __name__ == '__main__':
    main()
