"""Learning curves of the production trainers on one GPU ("show that training learns").

    python tools/learn_curves.py [--sl-steps 300] [--rl-iters 150] [--out gpurun_out/learn_curves.json]

Runs applestar_amd.runtime.learning_checks twice each: native HIP kernels, and the torch fp32 path on the same GPU
as the control curve.  Writes one JSON with the four curves and a per-run summary line to stdout."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from applestar_amd.runtime.learning_checks import sl_overfit_curve, rl_bandit_curve  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sl-steps', type=int, default=300)
    ap.add_argument('--rl-iters', type=int, default=150)
    ap.add_argument('--rl-lr', type=float, default=3e-4)
    ap.add_argument('--out', default='gpurun_out/learn_curves.json')
    ap.add_argument('--no-control', action='store_true')
    ap.add_argument('--rl-only', action='store_true')
    ap.add_argument('--rl-lrs', default='', help='comma list: RL learning-rate sweep (native only)')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    res = {}
    if args.rl_lrs:
        for lr in [float(x) for x in args.rl_lrs.split(',')]:
            rl = rl_bandit_curve(dev, iters=args.rl_iters, native=True, lr=lr)
            res[f'rl_native_lr{lr:g}'] = rl
            print(json.dumps({'run': f'rl_native_lr{lr:g}', 'first': rl[0], 'mid': rl[len(rl) // 2], 'last': rl[-1]}),
                  flush=True)
    for native in ([True] if args.no_control else [True, False]):
        tag = 'native' if native else 'torch_control'
        if not args.rl_only:
            sl = sl_overfit_curve(dev, steps=args.sl_steps, native=native)
            res['sl_' + tag] = sl
            print(json.dumps({'run': 'sl_' + tag, 'first': sl[0], 'last': sl[-1]}), flush=True)
        rl = rl_bandit_curve(dev, iters=args.rl_iters, native=native, lr=args.rl_lr)
        res['rl_' + tag] = rl
        print(json.dumps({'run': 'rl_' + tag, 'first': rl[0], 'last': rl[-1]}), flush=True)
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(res, f)


if __name__ == '__main__':
    main()
