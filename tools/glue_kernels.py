"""Which framework lines launch the glue kernels (fills, copies, ReLU-backward thresholds, adds) of one learner step:
torch.profiler with Python stacks, every GPU kernel attributed to the innermost applestar_amd frame of the CPU
op that launched it (autograd-engine ops: the backward node's name), counted and timed per site.

    python tools/glue_kernels.py [--precision fp32] [--match Fill,copy,threshold,CUDAFunctor_add,copyBuffer]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    ap.add_argument('--match', default='Fill,copy,threshold,CUDAFunctor_add,copyBuffer,CatArray,where,Mul')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--shapes', action='store_true', help='key the sites by the launching op\'s input shapes too')
    args = ap.parse_args()
    import bench
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree
    dev = torch.device('cuda', 0)
    batches = [pin_tree(rl_batch(6, 64, max_entities=512, seed=i)) for i in range(2)]
    tr = bench._make_trainer(argparse.Namespace(mode='rl', graph=False, batch=6, unroll=64), args.precision, dev, 'rl')

    def source():
        i = 0
        while True:
            yield batches[i % 2]
            i += 1
    it = DevicePrefetcher(source(), dev)
    for _ in range(3):
        tr.step(next(it))
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=args.shapes) as prof:
        tr.step(next(it))
        torch.cuda.synchronize()
    keys = [k for k in args.match.split(',') if k]
    sites = collections.defaultdict(lambda: [0, 0.0])
    kinds = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA or not getattr(e, 'kernels', None):
            continue
        site, p = None, e
        while p is not None and site is None:
            for fr in (p.stack or []):
                if ROOT in fr and 'glue_kernels' not in fr and 'bench.py' not in fr:
                    site = fr.replace(ROOT + '/', '')
                    break
            if site is None and ('Backward' in p.name or p.name.startswith('autograd::')):
                site = p.name
            p = p.cpu_parent
        for k in e.kernels:
            kind = next((c for c in keys if c in k.name), None)
            if kind is None:
                continue
            dur = getattr(k, 'duration', 0)
            if site is None:     # no framework frame: name the CPU op chain (and any stack frame at all)
                chain, p = [], e
                while p is not None and len(chain) < 5:
                    chain.append(p.name)
                    p = p.cpu_parent
                fr = next((f for f in (e.stack or []) if 'torch/' not in f), None)
                site = '(no frame) ' + ' < '.join(chain[1:]) + (f' @ {fr}' if fr else '')
            key = f'{kind:16s} {e.name:28s} {site}'
            if args.shapes:
                key += f'  {[tuple(x) for x in (e.input_shapes or []) if x][:2]}'
            sites[key][0] += 1
            sites[key][1] += dur
            kinds[kind][0] += 1
            kinds[kind][1] += dur
    print({k: (v[0], round(v[1] / 1e3, 3)) for k, v in kinds.items()})
    for k, (n, t) in sorted(sites.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f'{t / 1e3:7.3f} ms {n:4d}x  {k}')


if __name__ == '__main__':
    main()
