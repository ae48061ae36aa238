"""Which Python lines launch a given kind of kernel in one RL learner step (forward; backward kernels
are attributed to their autograd node).  Example: where do the ~290 D2D copyBuffer kernels come from?

    python tools/kernel_sources.py --pattern copyBuffer --pattern elementwise [--out gpurun_out/ksrc.txt]
"""
import argparse
import collections
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--pattern', action='append', default=[])
    ap.add_argument('--out', default='gpurun_out/kernel_sources.txt')
    args = ap.parse_args()
    pats = [re.compile(p) for p in (args.pattern or ['copyBuffer'])]
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(3):
        tr.step(dict(b))
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        tr.step(dict(b))
        torch.cuda.synchronize()
    cnt = collections.Counter()
    tm = collections.Counter()
    for ev in prof.events():
        ks = [k for k in (getattr(ev, 'kernels', None) or []) if any(p.search(k.name) for p in pats)]
        if not ks:
            continue
        where = None
        p = ev
        while p is not None and where is None:
            st = [f for f in (getattr(p, 'stack', None) or []) if 'applestar_amd' in f or 'bench' in f]
            if st:
                where = ' | '.join(s.split('applestar_amd/')[-1] for s in st[:3])
            elif 'Backward' in p.name:
                where = 'backward: ' + p.name
            p = p.cpu_parent
        key = (ks[0].name[:40], ev.name, where or '?')
        for k in ks:
            cnt[key] += 1
            tm[key] += k.duration
    lines = []
    for key, n in sorted(cnt.items(), key=lambda kv: -tm[kv[0]]):
        lines.append(f'{n:5d} {tm[key] / 1e3:7.3f} ms  {key[0]:40s} {key[1][:28]:28s} {key[2][:200]}')
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    open(args.out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:80]))


if __name__ == '__main__':
    main()
