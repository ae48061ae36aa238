"""Per-shape device time of the native 3x3 conv launches (forward and input-gradient calls) and of the
native weight-gradient launches in one learner step: the extension entry points are wrapped with CUDA
events.  Usage: python tools/conv_shapes.py [--out F]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.ops import native  # noqa: E402
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402


class Timed:
    def __init__(self, C, names):
        self.C, self.rec, self.on = C, [], False
        self.orig = {n: getattr(C, n) for n in names}

    def wrap(self, name):
        fn = self.orig[name]

        def inner(*a, **k):
            if not self.on:
                return fn(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn(*a, **k)
            e.record()
            shapes = tuple(tuple(t.shape) for t in a if isinstance(t, torch.Tensor))[:2]
            self.rec.append((name, shapes, s, e))
            return r
        return inner


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/conv_shapes.txt')
    ap.add_argument('--names', default='conv3x3_fwd,wgrad,act_grad_nhwc,maxpool2_fwd,maxpool2_bwd,conv3x3_f32,'
                    'conv3x3_f32_v2,conv3x3_f32_psb,conv3x3_f32_epi2,wgrad_f32,gemm_f32,gemm_f32_psb')
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    args = ap.parse_args()
    C = native.ensure_loaded()
    names = [n for n in args.names.split(',') if hasattr(C, n)]

    class Proxy:
        pass
    t = Timed(C, names)
    proxy = Proxy()
    for n in dir(C):
        if not n.startswith('__'):
            setattr(proxy, n, getattr(C, n))
    for n in names:
        setattr(proxy, n, t.wrap(n))
    native._C = proxy
    dev = torch.device('cuda', 0)
    lcfg = {'use_value_feature': True}
    if args.precision == 'bf16':
        lcfg['amp_dtype'] = 'bfloat16'
    tr = RLTrainer({'learner': lcfg, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(3):
        tr.step(dict(b))
    torch.cuda.synchronize()
    t.on = True
    tr.step(dict(b))
    torch.cuda.synchronize()
    cnt, tm = collections.Counter(), collections.Counter()
    for name, shapes, s, e in t.rec:
        cnt[(name, shapes)] += 1
        tm[(name, shapes)] += s.elapsed_time(e)
    lines = [f'{cnt[k]:4d} {tm[k]:8.3f} ms  {k[0]:14s} {k[1]}' for k in sorted(tm, key=lambda k: -tm[k])]
    lines.insert(0, f'total {sum(tm.values()):.3f} ms')
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    open(args.out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:50]))


if __name__ == '__main__':
    main()
