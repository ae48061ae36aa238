"""Probe: the gradient -> bucket copy of the RL model's 475 parameters (parallel/dp.py copy_into: one multi-tensor
launch per 64 tensors) against one flat device copy of the same bytes.

    python tools/probe_grad_copy.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    from applestar_amd.models.model import Model
    from applestar_amd.parallel.dp import copy_into
    m = Model({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}},
              use_value_network=True).cuda()
    ps = list(m.parameters())
    total = sum(p.numel() for p in ps)
    flat = torch.empty(total, device='cuda')
    views, off = [], 0
    for p in ps:
        views.append(flat[off:off + p.numel()].view(p.shape))
        off += p.numel()
    grads = [torch.randn_like(p) for p in ps]
    src_flat = torch.randn(total, device='cuda')
    rec = {'tensors': len(ps), 'MB': round(total * 4 / 2 ** 20, 1),
           'copy_into_us': round(timed(lambda: copy_into(views, grads)), 1),
           'flat_copy_us': round(timed(lambda: flat.copy_(src_flat)), 1)}
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
