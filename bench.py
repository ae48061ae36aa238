#!/usr/bin/env python
"""Headline benchmark: RL learner samples/sec of the AlphaStar policy (BASELINE.json).

Config: per GPU 6 trajectories x 64 steps (= 384 learner samples / iteration), the
reference RL learner model (policy 29.1 M + value encoder + winloss baseline, ``use_value_feature``),
full iteration timed: H2D of the next batch (overlapped), encoder over (T+1)*B observations, core
LSTM, teacher-forced heads, V-trace/UPGO/TD(lambda)/entropy/KL loss, backward, RCCL gradient
all-reduce, grad clip, Adam.  Synthetic observations with the reference fake-data distribution
(entity_num ~ U[1,512), padded to the batch max), random-init weights.

Precision.  The reference learner is fp32 end to end (``distar/agent/default/rl_learner.py:82-145``:
no autocast / AMP anywhere in ``distar/``).  ``--precision fp32`` runs the like-for-like step: fp32
weights, fp32 activations, every GEMM / conv / attention on fp32 operands.  gfx950 has no TF32/xf32 mode;
the native conv / GEMM / weight-gradient products run as fp32-accurate bf16x6 split MFMAs
(``applestar_amd/csrc/split_mfma.h``: exact three-way bf16 split of each fp32 operand, six partial products,
fp32 accumulation; error vs float64 equal to or below the exact-f32 MFMA's), ``APPLESTAR_F32_MFMA=exact``
runs them on the exact-f32 MFMA instead; the JSON's ``config.fp32_products`` names the mode.  ``--precision bf16`` is the mixed-precision step: bf16
compute weights over fp32 master weights, fp32 LayerNorm statistics / softmax / losses / optimizer;
its training parity against fp32 is pinned by
``tests/test_model_parity_gpu.py::test_bf16_training_tracks_fp32``.
``--precision both`` (default) measures both, fp32 first; the headline ``value`` / ``dtype`` are the
fp32 run, the bf16 run is reported under ``"mixed_bf16"``.

After the learner, ``--inference`` (default on, rank 0) times the actor's agent step
(``compute_logp_action``: full policy forward + sampling including the selected-units pointer loop,
HIP-graph replay) at B = 1 and B = 16 -> ``inference_p50_ms``.  Per-step wall / GPU times of the timed
steps go to stderr.

Run:  python bench.py --gpus 1 --steps 10 --warmup 3
      torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch

BASELINE_PER_GPU = 256.0  # samples/s/GPU, 32xA100 learner, docs/guidance_to_small_scale_training.md:280-284
SL_BASELINE_PER_GPU = 384.0  # samples/s/GPU, 56xA100 SL learner, docs/guidance_to_small_scale_training.md:178-184
INFERENCE_BASELINE_16ENV_MS = 160.0  # batched GPU inference, 16 envs (guidance_to_small_scale_training.md:230-232)


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def _fp32_products():
    from applestar_amd.ops import native
    mode = native.ensure_loaded().f32_mfma_mode()
    return ('exact-f32 MFMA (v_mfma_f32_32x32x2_f32)' if mode == 0 else
            'fp32-accurate bf16x6 split MFMA (exact 3-way bf16 split, 6 partial products, fp32 accumulation)')


def _make_trainer(args, precision, device, mode=None):
    amp = 'bfloat16' if precision == 'bf16' else None
    if (mode or args.mode) == 'rl':
        from applestar_amd.rl.trainer import RLTrainer
        return RLTrainer({'learner': {'use_value_feature': True, 'graph_step': args.graph, 'amp_dtype': amp},
                          'model': {'enable_baselines': ['winloss']}}, device=device)
    from applestar_amd.sl.trainer import SLTrainer
    return SLTrainer({'learner': {'ignore_steps': 0, 'amp_dtype': amp,
                                  'data': {'batch_size': args.batch, 'trajectory_length': args.unroll}}},
                     device=device)


def run_learner(args, precision, rank, world, device, host_batches, mode=None):
    """W untimed warm-up steps, then exactly K timed steps between barrier + synchronize pairs."""
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.runtime.prefetch import DevicePrefetcher
    gpu = device.type == 'cuda'
    torch.manual_seed(1234 + rank)
    t_build = time.perf_counter()
    trainer = _make_trainer(args, precision, device, mode)
    if rank == 0:
        _log(f'[{precision}] trainer built in {time.perf_counter() - t_build:.1f} s')

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

    for w in range(args.warmup):
        tw = time.perf_counter()
        info = trainer.step(next(it))
        if gpu:
            torch.cuda.synchronize()
        if rank == 0:     # progress (first steps include MIOpen / hipBLASLt kernel selection)
            _log(f'[{precision}] warm-up step {w}: {1000 * (time.perf_counter() - tw):.1f} ms')
    sync()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if gpu else None
    host_t = []
    t0 = time.perf_counter()
    if gpu:
        ev[0].record()
    for i in range(args.steps):
        h0 = time.perf_counter()
        info = trainer.step(next(it))
        if gpu:
            ev[i + 1].record()
        host_t.append(time.perf_counter() - h0)
    sync()
    elapsed = time.perf_counter() - t0
    loss = float(info['total_loss'].detach())
    t = torch.tensor([elapsed], dtype=torch.float64, device=device if gpu else 'cpu')
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    replicas = None
    if world > 1:
        # after the timed region: every rank's weights (fp32 masters in the bf16 step) and last gradient norm
        # must be bit-identical - the data-parallel invariant - checked with one small all-gather
        with torch.no_grad():
            flat = trainer.master.master.detach() if trainer.master is not None else \
                torch.cat([p.detach().reshape(-1) for p in trainer.params])
            fp = torch.stack([(flat.view(torch.int32).long() * 2654435761 % (1 << 31)).sum(),
                              info['gradient'].detach().reshape(()).double().view(torch.int64)]).to(device)
        allfp = [torch.zeros_like(fp) for _ in range(world)]
        torch.distributed.all_gather(allfp, fp)
        replicas = all(torch.equal(allfp[0], f) for f in allfp[1:])
    gpu_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)] if gpu else []
    host_ms = [1000.0 * h for h in host_t]
    if rank == 0:
        _log(f'[{precision}] per-step wall between events (ms): ' + ' '.join(f'{x:.2f}' for x in gpu_ms))
        _log(f'[{precision}] per-step host issue time (ms): ' + ' '.join(f'{x:.2f}' for x in host_ms))
    res = {
        'ms_per_step': 1000.0 * elapsed / max(args.steps, 1),
        'elapsed_s': elapsed,
        'host_ms_per_step': sum(host_ms) / max(len(host_ms), 1),
        'step_ms_min': min(gpu_ms) if gpu_ms else None,
        'step_ms_max': max(gpu_ms) if gpu_ms else None,
        'step_ms_median': sorted(gpu_ms)[len(gpu_ms) // 2] if gpu_ms else None,
        'final_loss': loss,
        'replicas_identical': replicas,
        'peak_mem_gb': (torch.cuda.max_memory_allocated(device) / 2 ** 30) if gpu else None,
        'graph_step': ({'captures': trainer.graph.captures, 'replays': trainer.graph.replays,
                        'eager_steps': trainer.graph.eager_steps}
                       if getattr(trainer, 'graph', None) is not None else None),
    }
    del trainer, it, info
    gc.collect()
    if gpu:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(device)
    return res


def run_inference(device, batches=(1, 16), iters=20, entities=300):
    """p50 latency of one actor agent step (compute_logp_action, HIP-graph replay) per batch size."""
    from applestar_amd.models.model import Model
    from applestar_amd.lib.features import random_obs
    from applestar_amd.rl.synthetic import to_device
    from applestar_amd.runtime.graphs import GraphedPolicy
    out = {}
    m = Model({'agent': {'extra_units': True}}).to(device).eval().to(memory_format=torch.channels_last)
    # the inference server's configuration (actor/inference.py set_model): the model's parameters carry their cached
    # bf16 / channels-last compute forms, so the graph reads them instead of casting every weight per call
    from applestar_amd.ops import native
    native.ensure_loaded()
    native.attach_inference_forms(m)
    gp = GraphedPolicy(m, 'compute_logp_action')
    for B in batches:
        g = torch.Generator().manual_seed(B)
        en = torch.randint(entities // 2, entities, (B,), generator=g)
        obs = random_obs(B, entity_num=en, generator=g)
        obs['hidden_state'] = [(torch.zeros(B, 384), torch.zeros(B, 384)) for _ in range(3)]
        obs = to_device(obs, device)
        times = []
        for i in range(iters + 3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            gp(**obs)
            torch.cuda.synchronize()
            if i >= 3:
                times.append((time.perf_counter() - t) * 1000)
        times.sort()
        out[f'b{B}'] = round(times[len(times) // 2], 3)
    del gp, m
    gc.collect()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=6, help='trajectories per GPU')
    ap.add_argument('--unroll', type=int, default=64)
    ap.add_argument('--max-entities', type=int, default=512)
    ap.add_argument('--n-batches', type=int, default=2, help='distinct synthetic batches cycled')
    ap.add_argument('--precision', choices=['fp32', 'bf16', 'both'], default='both',
                    help='fp32: like-for-like with the fp32 reference learner; bf16: mixed precision; both: fp32 '
                         'headline + bf16 reported under "mixed_bf16"')
    ap.add_argument('--no-native', action='store_true', help='disable HIP kernels (torch-only baseline)')
    ap.add_argument('--mode', choices=['rl', 'sl'], default='rl',
                    help='rl: the headline RL learner step; sl: supervised learner step (reference 384 samples/s/GPU)')
    ap.add_argument('--graph', action='store_true', help='replay the learner step from HIP graphs (runtime/step_graph.py)')
    ap.add_argument('--inference', type=int, default=1, help='1: also time the actor agent step at B=1 and B=16')
    ap.add_argument('--sl', type=int, default=1,
                    help='1 (rl mode): also time the fp32 SL learner step on the same config -> "sl_fp32" '
                         '(reference 384 samples/s/GPU)')
    ap.add_argument('--conv-benchmark', type=int, default=-1,
                    help='1/0: force MIOpen find-mode autotuning of convolutions on/off (-1: trainer default)')
    args = ap.parse_args()

    from applestar_amd.parallel import dist as pdist
    from applestar_amd import ops
    from applestar_amd.rl.synthetic import rl_batch, sl_batch
    from applestar_amd.runtime.prefetch import pin_tree

    rank, world = pdist.init()
    if world != args.gpus and rank == 0:
        _log(f'warning: --gpus {args.gpus} but WORLD_SIZE={world}')
    gpu = torch.cuda.is_available()
    device = torch.device('cuda', torch.cuda.current_device()) if gpu else torch.device('cpu')
    if args.no_native:
        ops.set_native(False)
    if args.conv_benchmark >= 0:
        torch.backends.cudnn.benchmark = bool(args.conv_benchmark)

    make = (lambda i: rl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i)) \
        if args.mode == 'rl' else \
        (lambda i: sl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i))
    host_batches = [pin_tree(make(i)) if gpu else make(i) for i in range(args.n_batches)]

    precisions = ['fp32', 'bf16'] if args.precision == 'both' else [args.precision]
    results = {p: run_learner(args, p, rank, world, device, host_batches) for p in precisions}
    if args.sl and args.mode == 'rl':
        # the supervised learner step (distar/agent/default/sl_learner.py) on the same per-GPU batch, fp32 like the
        # reference's, reported beside the headline so the 384 samples/s/GPU comparison is observed by the driver
        sl_batches = [pin_tree(sl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i))
                      if gpu else sl_batch(args.batch, args.unroll, max_entities=args.max_entities, seed=1000 * rank + i)
                      for i in range(args.n_batches)]
        results['sl_fp32'] = run_learner(args, 'fp32', rank, world, device, sl_batches, mode='sl')
        del sl_batches
    inference = None
    if args.inference and gpu and rank == 0 and args.mode == 'rl':
        try:
            inference = run_inference(device)
        except Exception as e:   # the learner number stands on its own; say why the latency is missing
            inference = {'error': repr(e)[:200]}
    pdist.barrier()

    if rank == 0:
        samples_per_step = args.batch * args.unroll * world
        base = (BASELINE_PER_GPU if args.mode == 'rl' else SL_BASELINE_PER_GPU) * world

        def summary(p, base=base):
            r = results[p]
            v = samples_per_step * args.steps / r['elapsed_s']
            return v, {'value': round(v, 2), 'ms_per_step': round(r['ms_per_step'], 3),
                       'vs_baseline': round(v / base, 3), 'host_ms_per_step': round(r['host_ms_per_step'], 3),
                       'step_ms_min': r['step_ms_min'] and round(r['step_ms_min'], 3),
                       'step_ms_median': r['step_ms_median'] and round(r['step_ms_median'], 3),
                       'step_ms_max': r['step_ms_max'] and round(r['step_ms_max'], 3),
                       'final_loss': r['final_loss'], 'replicas_identical': r['replicas_identical'],
                       'peak_mem_gb': r['peak_mem_gb'] and round(r['peak_mem_gb'], 2)}

        head = precisions[0]
        value, hs = summary(head)
        out = {
            'metric': 'learner samples/sec (AlphaStar policy)' if args.mode == 'rl' else
                      'SL learner samples/sec (AlphaStar policy)',
            'value': hs['value'],
            'unit': 'samples/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': hs['ms_per_step'],
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': hs['vs_baseline'],
            'dtype': head,
            'data': 'synthetic (reference fake-data distribution, entity_num~U[1,512)), random-init weights',
            'config': {
                'model': 'AlphaStar policy + value encoder + winloss baseline (DI-star rl_model arch)' if args.mode == 'rl'
                         else 'AlphaStar policy (DI-star sl_model arch)',
                'global_batch': args.batch * world,
                'seq_len': args.unroll,
                'parallelism': f'dp{world}',
                'samples_per_step': samples_per_step,
                'baseline_note': ('vs_baseline = per-GPU samples/s / 256 (reference RL learner, fp32, A100)'
                                  if args.mode == 'rl' else
                                  'vs_baseline = per-GPU samples/s / 384 (reference SL learner, fp32, A100)'),
                'precision': ('fp32 weights / activations / GEMM operands (like-for-like with the reference)'
                              if head == 'fp32' else 'bf16 compute over fp32 master weights'),
                'native_kernels': (not args.no_native) and gpu,
                'fp32_products': (_fp32_products() if head == 'fp32' and gpu and not args.no_native else None),
                **{k: v for k, v in hs.items() if k not in ('value', 'ms_per_step', 'vs_baseline')},
                'graph_step': results[head]['graph_step'],
            },
        }
        if len(precisions) > 1:
            out['mixed_bf16'] = summary('bf16')[1]
        if 'sl_fp32' in results:
            out['sl_fp32'] = {'metric': 'SL learner samples/sec (AlphaStar policy, fp32)',
                              **summary('sl_fp32', base=SL_BASELINE_PER_GPU * world)[1],
                              'baseline_note': 'vs_baseline = per-GPU samples/s / 384 (reference SL learner, fp32, A100)'}
        if inference is not None:
            out['inference_p50_ms'] = inference
            out['inference_note'] = ('actor agent step (compute_logp_action incl. sampling), bf16, HIP-graph replay; '
                                     f'reference: {INFERENCE_BASELINE_16ENV_MS:.0f} ms per 16-env batched step')
        print(json.dumps(out), flush=True)
    pdist.finalize()


if __name__ == '__main__':
    main()
