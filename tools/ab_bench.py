"""In-process A/B timing of runtime switches on the RL learner step (box-to-box variance is larger than
most single optimisations, so compare within one process, interleaved).
Usage: python tools/ab_bench.py --variant graphs --rounds 4 --steps 10"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch  # noqa: E402
from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree  # noqa: E402
from applestar_amd.ops import native  # noqa: E402


def set_variant(name, on):
    if name == 'graphs':
        os.environ['APPLESTAR_GRAPHS'] = '1' if on else '0'
    elif name == 'wgrad_small':
        native._WGRAD_MIN_ROWS = 256 if on else 4096
    elif name == 'wgrad_bf16':
        native.WGRAD_BF16_OUT = on
    elif name == 'gated_fused':
        from applestar_amd.models import blocks
        blocks.FUSED_GATED_RESBLOCK = on
    elif name == 'critic_side':
        from applestar_amd.models import model
        model.CRITIC_SIDE_STREAM = on
        model.CRITIC_SIDE_STREAM_FP32 = on
    elif name == 'scalar_side':
        from applestar_amd.models import encoders
        encoders.SCALAR_SIDE_STREAM = on
    elif name == 'side_stream':
        from applestar_amd.models import model
        model.SIDE_STREAMS_ENABLED = on
    elif name == 'f32_small_gemm':
        native.F32_SMALL = on
    elif name == 'f32_kpad':
        native.F32_KPAD = on
    else:
        raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variant', required=True)
    ap.add_argument('--rounds', type=int, default=4)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--precision', choices=['bf16', 'fp32'], default='bf16')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True,
                                'amp_dtype': 'bfloat16' if args.precision == 'bf16' else None}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    hb = [pin_tree(rl_batch(6, 64, max_entities=512, seed=i)) for i in range(2)]

    def src():
        i = 0
        while True:
            yield hb[i % 2]
            i += 1
    it = DevicePrefetcher(src(), dev)
    res = {False: [], True: []}
    for on in (False, True):
        set_variant(args.variant, on)
        for _ in range(4):
            tr.step(next(it))
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for on in ((False, True) if r % 2 == 0 else (True, False)):
            set_variant(args.variant, on)
            tr.step(next(it))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step(next(it))
            torch.cuda.synchronize()
            res[on].append(1000 * (time.perf_counter() - t0) / args.steps)
    out = {'variant': args.variant, 'precision': args.precision, 'off_ms': [round(x, 2) for x in res[False]],
           'on_ms': [round(x, 2) for x in res[True]],
           'off_mean': round(sum(res[False]) / len(res[False]), 2), 'on_mean': round(sum(res[True]) / len(res[True]), 2)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
