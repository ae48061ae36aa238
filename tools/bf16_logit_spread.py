"""Spread of the bf16 trainer's head-logit errors against the fp32 CPU oracle over several batches, with the
native kernels on and off (PyTorch's own bf16 autocast path: the control).  One batch of B=2 x T=4 puts only a
few hundred selected-units logits behind each number, so a single seed says little about whether a change
moved the bf16 error; this prints per-seed errors and their mean for both paths.

    python tools/bf16_logit_spread.py [--seeds 8] > gpurun_out/bf16_logit_spread.json
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HEADS = ['action_type', 'delay', 'queued', 'selected_units', 'target_unit', 'target_location']


def _masked_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    keep = b > -1e8
    return float((a[keep] - b[keep]).norm() / b[keep].norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seeds', type=int, default=8)
    args = ap.parse_args()
    from applestar_amd import ops
    from applestar_amd.models.model import Model
    from applestar_amd.rl.synthetic import rl_batch, to_device
    from applestar_amd.rl.trainer import RLTrainer
    cfg = {'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16'}, 'model': {'enable_baselines': ['winloss']}}
    torch.manual_seed(0)
    cpu = Model(cfg, use_value_network=True).train()
    trainers = {}
    for native in (True, False):
        ops.set_native(native)
        tr = RLTrainer(cfg, device='cuda')
        tr.load_model_state_dict(cpu.state_dict())
        trainers[native] = tr
    ops.set_native(True)
    rows = []
    for s in range(args.seeds):
        batch = rl_batch(2, 4, max_entities=48, seed=s)
        with torch.no_grad():
            ref = cpu.rl_learner_forward(**copy.deepcopy(batch))['target_logit']
        rec = {'seed': s}
        for native, tr in trainers.items():
            ops.set_native(native)
            with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False), torch.no_grad():
                out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))['target_logit']
            rec['native' if native else 'torch'] = {h: round(_masked_rel(out[h].float(), ref[h]), 5) for h in HEADS}
        ops.set_native(True)
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    mean = {k: {h: sum(r[k][h] for r in rows) / len(rows) for h in HEADS} for k in ('native', 'torch')}
    print(json.dumps({'mean': mean}), flush=True)


if __name__ == '__main__':
    main()
