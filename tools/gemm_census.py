"""Every library GEMM (aten mm / addmm / bmm / baddbmm / addmv ...) issued by one learner step, with shapes,
dtypes and the Python call site: the list of products still on hipBLASLt / rocBLAS.

    python tools/gemm_census.py [--precision fp32|bf16] [--mode rl|sl]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEMMS = {'mm', 'addmm', 'bmm', 'baddbmm', 'addmv', 'mv', '_addmm_activation', 'addbmm', 'matmul', 'linear',
         '_scaled_mm'}


class Census(TorchDispatchMode):
    def __init__(self, all_ops=False):
        super().__init__()
        self.calls = collections.Counter()
        self.all_ops = all_ops

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split('.')[0]
        if self.all_ops and name not in GEMMS and name not in ('detach', 'view', '_unsafe_view', 'as_strided', 't',
                                                                'transpose', 'permute', 'expand', 'slice', 'select',
                                                                'unsqueeze', 'squeeze', 'alias', 'split', 'narrow',
                                                                'empty', 'empty_strided', 'empty_like', 'lift_fresh',
                                                                'set_', 'unbind', 'split_with_sizes', 'chunk'):
            out = func(*args, **(kwargs or {}))
            big = max([a.numel() for a in args if torch.is_tensor(a)] + [0])
            st = [f for f in traceback.extract_stack() if f.filename.startswith(HERE) and 'gemm_census' not in f.filename]
            site = ' <- '.join(f'{os.path.relpath(f.filename, HERE)}:{f.lineno}' for f in reversed(st[-3:]))
            self.calls[('*' + name, big, '', site)] += 1
            return out
        if name in GEMMS:
            shapes = tuple(tuple(a.shape) for a in args if torch.is_tensor(a))
            dt = next((str(a.dtype).replace('torch.', '') for a in args if torch.is_tensor(a)), '')
            st = [f for f in traceback.extract_stack() if f.filename.startswith(HERE) and 'gemm_census' not in f.filename]
            site = ' <- '.join(f'{os.path.relpath(f.filename, HERE)}:{f.lineno}' for f in reversed(st[-3:]))
            self.calls[(name, shapes, dt, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    ap.add_argument('--mode', choices=['rl', 'sl'], default='rl')
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--all', action='store_true', help='every aten op (not only GEMMs): op, largest operand numel, site')
    args = ap.parse_args()
    from applestar_amd.rl.synthetic import rl_batch, sl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree
    device = torch.device('cuda', 0)
    amp = 'bfloat16' if args.precision == 'bf16' else None
    if args.mode == 'rl':
        from applestar_amd.rl.trainer import RLTrainer
        trainer = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': amp},
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
    b = next(it)
    census = Census(args.all)
    # native few-row / split-K products too: wrap the extension's entry points for this step
    from applestar_amd.ops import native as NN
    C = NN.ensure_loaded()
    native_calls = collections.Counter()

    class _Wrap:
        def __getattr__(self, k):
            f = getattr(C, k)
            if k not in ('small_gemm', 'small_wgrad', 'small_gemm_splitk', 'gemm_f32', 'gemm_bf16', 'gemm_bf16_small',
                         'wgrad_f32', 'wgrad', 'mm_k32'):
                return f

            def g(*a):
                native_calls[(k, tuple(tuple(t.shape) for t in a if torch.is_tensor(t)))] += 1
                return f(*a)
            return g
    NN._C = _Wrap()
    try:
        with census:
            trainer.step(b)
        torch.cuda.synchronize()
    finally:
        NN._C = C
    print(f'{sum(native_calls.values())} native GEMM-family calls')
    for (k, shapes), n in sorted(native_calls.items(), key=lambda kv: -kv[1]):
        print(f'  native {n:3d} {k:18s} {shapes}')
    print(f'{sum(census.calls.values())} library GEMM calls in one {args.mode} {args.precision} step')
    key = (lambda kv: -kv[1] * (kv[0][1] if isinstance(kv[0][1], int) else 1)) if args.all else (lambda kv: -kv[1])
    for (name, shapes, dt, site), n in sorted(census.calls.items(), key=key):
        print(f'{n:4d} {name:10s} {dt:9s} {shapes}  {site}')


if __name__ == '__main__':
    main()
