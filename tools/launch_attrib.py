"""Which autograd nodes / forward ops launch the small aten kernels (fill_, copy_, add_, cat, cast) in
one RL learner step: counts aten leaf ops by their outermost autograd-node / module-level parent.
Usage: python tools/launch_attrib.py [--out gpurun_out/launch_attrib.txt]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402

LEAVES = ('aten::fill_', 'aten::zero_', 'aten::copy_', 'aten::add_', 'aten::add', 'aten::cat', 'aten::mul',
          'aten::_to_copy', 'aten::index_select', 'aten::sum')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/launch_attrib.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    b = to_device(rl_batch(6, 64, seed=0), dev)
    for _ in range(3):
        tr.step(dict(b))
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        tr.step(dict(b))
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name not in LEAVES:
            continue
        p, chain = ev.cpu_parent, []
        while p is not None:
            chain.append(p.name)
            p = p.cpu_parent
        node = next((c for c in chain if 'autograd::engine' in c or 'Backward' in c), None)
        top = [c for c in chain if not c.startswith('aten::')][:2]
        cnt[(ev.name, node or 'forward', ' <- '.join(top)[:110])] += 1
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, 'w') as f:
        for k, v in cnt.most_common(80):
            f.write(f'{v:5d}  {k[0]:18s} {k[1][:70]:70s} {k[2]}\n')
    print(open(args.out).read()[:3000])


if __name__ == '__main__':
    main()
