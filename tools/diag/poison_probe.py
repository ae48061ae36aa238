"""Uninitialised-memory probe of the learner forward: the caching allocator's free blocks are filled with a poison
value (0, NaN, 1e30, -7) before each forward, and every head's logits and the value are compared with the run after
the zero poison.  A deterministic forward that reads only what it wrote gives bit-identical outputs whatever the
free memory held; any difference names a read of unwritten memory (the selected-units bf16 logit error moved from
box to box).

    python tools/diag/poison_probe.py [--precision bf16|fp32|both] [--backward]
"""
import argparse
import copy
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from applestar_amd.models.model import Model  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402


def poison(val):
    """Fill (then free) blocks of every size class of the caching allocator with val."""
    torch.cuda.synchronize()
    held = []
    for k in range(8, 28):                       # 256 B .. 128 MB
        for _ in range(6 if k < 21 else 2):
            held.append(torch.full((1 << (k - 2),), val, device='cuda'))
    del held
    torch.cuda.synchronize()


def outputs(tr, batches, amp, backward):
    res = []
    for b in batches:
        bd = to_device(copy.deepcopy(b), 'cuda')
        ctx = torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False) if amp else torch.autocast('cuda', enabled=False)
        if backward:
            with ctx:
                out = tr.model.rl_learner_forward(**bd)
            loss = sum(v.float().clamp(-1e4, 1e4).sum() for v in out['target_logit'].values()) + \
                sum(v.float().sum() for v in out['value'].values())
            tr.model.zero_grad(set_to_none=True)
            loss.backward()
            res.append({'grad.' + n: p.grad.detach().float().clone() for n, p in tr.model.named_parameters()
                        if p.grad is not None})
        else:
            with ctx, torch.no_grad():
                out = tr.model.rl_learner_forward(**bd)
        d = {('logit.' + k): v.detach().float().clone() for k, v in out['target_logit'].items()}
        d.update({('value.' + k): v.detach().float().clone() for k, v in out['value'].items()})
        res.append(d)
    torch.cuda.synchronize()
    return res


def diff(a, b):
    worst = {}
    for ra, rb in zip(a, b):
        for k in ra:
            x, y = ra[k], rb[k]
            keep = (y > -1e8) & torch.isfinite(y) & (x > -1e8)
            nan_mismatch = int((torch.isnan(x) != torch.isnan(y)).sum())
            d = float((x[keep] - y[keep]).abs().max()) if keep.any() else 0.0
            w = worst.get(k, (0.0, 0))
            worst[k] = (max(w[0], d), w[1] + nan_mismatch)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', default='both')
    ap.add_argument('--backward', action='store_true')
    args = ap.parse_args()
    torch.manual_seed(0)
    cpu = Model({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}},
                use_value_network=True)
    batches = [rl_batch(2, 4, max_entities=48, seed=s) for s in (3, 0, 1, 2)]
    clean = True
    for prec in (['bf16', 'fp32'] if args.precision == 'both' else [args.precision]):
        cfg = {'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16' if prec == 'bf16' else None},
               'model': {'enable_baselines': ['winloss']}}
        tr = RLTrainer(cfg, device='cuda')
        tr.load_model_state_dict(cpu.state_dict())
        outputs(tr, batches, prec == 'bf16', args.backward)            # warm-up (derived weights, graphs)
        runs = {}
        for val in (0.0, float('nan'), 1e30, -7.0):
            poison(val)
            runs[val] = outputs(tr, batches, prec == 'bf16', args.backward)
        base = runs[0.0]
        for val, r in runs.items():
            if val == 0.0:
                continue
            w = diff(r, base)
            bad = {k: v for k, v in w.items() if v[0] > 0 or v[1]}
            clean &= not bad
            print(f'[{prec}] poison {val}: {"identical" if not bad else "DIFFERS"}', flush=True)
            for k, (d, n) in sorted(bad.items(), key=lambda kv: -kv[1][0])[:12]:
                print(f'    {k:40s} max|diff| {d:.3g}  nan-mismatch {n}', flush=True)
        again = outputs(tr, batches, prec == 'bf16', args.backward)
        w = diff(again, base)
        rep = {k: v for k, v in w.items() if v[0] > 0 or v[1]}
        print(f'[{prec}] rerun without poison: {"identical" if not rep else "DIFFERS (run-to-run nondeterminism)"}')
        for k, (d, n) in sorted(rep.items(), key=lambda kv: -kv[1][0])[:8]:
            print(f'    {k:40s} max|diff| {d:.3g}  nan-mismatch {n}')
    print('CLEAN' if clean else 'UNINITIALISED READS FOUND')


if __name__ == '__main__':
    main()
