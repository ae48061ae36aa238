"""Library GEMM calls of one learner step by (op, input shapes): count and device time, forward and
backward (torch.profiler with record_shapes).  Usage: python tools/gemm_profile.py [--out F]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402

OPS = ('aten::mm', 'aten::addmm', 'aten::_addmm_activation', 'aten::bmm', 'aten::linear', 'aten::matmul')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/gemm_profile.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(3):
        tr.step(dict(b))
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        tr.step(dict(b))
        torch.cuda.synchronize()
    cnt, tm = collections.Counter(), collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        ks = getattr(ev, 'kernels', None) or []
        if not ks:
            continue
        key = (ev.name, str(ev.input_shapes)[:120])
        cnt[key] += 1
        tm[key] += sum(k.duration for k in ks)
    lines = [f'{cnt[k]:4d} {tm[k] / 1e3:8.3f} ms  {k[0]:24s} {k[1]}' for k in sorted(tm, key=lambda k: -tm[k])]
    lines.insert(0, f'total {sum(tm.values()) / 1e3:.3f} ms in {sum(cnt.values())} calls')
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    open(args.out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:60]))


if __name__ == '__main__':
    main()
