"""Which ops of one RL learner step issue device-to-device hipMemcpyAsync calls (each one is a
``__amd_rocclr_copyBuffer`` blit kernel on the GPU, ~290 per step in r2bo): torch.profiler runtime events
grouped by the aten op that enclosed them and its shapes.

    python tools/memcpy_sources.py [--out gpurun_out/memcpy_sources.txt]
"""
import argparse
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/memcpy_sources.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(2):
        tr.step(dict(b))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        tr.step(dict(b))
        torch.cuda.synchronize()
    events = prof.events()
    # parent chain: runtime event -> enclosing cpu op (by time containment on the same thread)
    ops = [e for e in events if e.device_type == torch.autograd.DeviceType.CPU and not e.name.startswith(('hip', 'cuda'))]
    ops.sort(key=lambda e: e.time_range.start)
    hits = collections.Counter()
    total = 0
    for e in events:
        if 'Memcpy' not in e.name and 'memcpy' not in e.name:
            continue
        total += 1
        best = None
        for o in ops:
            if o.thread == e.thread and o.time_range.start <= e.time_range.start and o.time_range.end >= e.time_range.end:
                if best is None or o.time_range.start >= best.time_range.start:
                    best = o
        if best is None:
            hits[(e.name, '?', '')] += 1
            continue
        stack = [s for s in (best.stack or []) if 'applestar_amd' in s][:2]
        shapes = str(best.input_shapes)[:90] if best.input_shapes else ''
        hits[(e.name, best.name, ' <- '.join(s.split('applestar_amd/')[-1] for s in stack) + ' ' + shapes)] += 1
    with open(args.out, 'w') as f:
        f.write(f'{total} memcpy runtime calls in one step\n')
        for (name, op, where), n in hits.most_common():
            f.write(f'{n:4d}  {name:24s} {op:36s} {where}\n')
    print(open(args.out).read()[:4000])


if __name__ == '__main__':
    main()
