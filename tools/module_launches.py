"""Kernel launches and device time of one RL learner step, attributed to model components, forward
and backward separately (backward kernels are mapped to the component whose forward op created the
autograd node, via the profiler's sequence numbers).

    python tools/module_launches.py [--depth 2] [--out gpurun_out/module_launches.txt]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402


def install_hooks(model, depth):
    ranges = {}

    def pre(name):
        def f(m, args, kwargs=None):
            r = torch.profiler.record_function('mod:' + name)
            r.__enter__()
            ranges.setdefault(name, []).append(r)
        return f

    def post(name):
        def f(m, args, out):
            ranges[name].pop().__exit__(None, None, None)
        return f

    for name, m in model.named_modules():
        if not name or name.count('.') >= depth:
            continue
        m.register_forward_pre_hook(pre(name))
        m.register_forward_hook(post(name))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--depth', type=int, default=2)
    ap.add_argument('--out', default='gpurun_out/module_launches.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': False},
                    'model': {'enable_baselines': ['winloss']}}, device=dev)
    install_hooks(tr.model, args.depth)
    loss_fn = tr.loss.compute_loss

    def wrapped_loss(out):
        with torch.profiler.record_function('mod:loss'):
            return loss_fn(out)
    tr.loss.compute_loss = wrapped_loss
    upd = tr._update

    def wrapped_update():
        with torch.profiler.record_function('mod:update'):
            return upd()
    tr._update = wrapped_update
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(3):
        tr.step(dict(b))
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts) as prof:
        tr.step(dict(b))
        torch.cuda.synchronize()
    evs = prof.events()
    seqmap = {}

    def module_of(ev):
        p = ev
        while p is not None:
            if p.name.startswith('mod:'):
                return p.name[4:]
            p = p.cpu_parent
        return None

    for ev in evs:
        if getattr(ev, 'sequence_nr', -1) >= 0 and not ev.name.startswith('autograd'):
            m = module_of(ev)
            if m is not None and ev.sequence_nr not in seqmap:
                seqmap[ev.sequence_nr] = m
    cnt = collections.Counter()
    tm = collections.Counter()
    for ev in evs:
        ks = getattr(ev, 'kernels', None) or []
        if not ks:
            continue
        m = module_of(ev)
        if m is not None:
            key = ('fwd', m)
        else:
            p, key = ev, None
            while p is not None:
                if 'Backward' in p.name and getattr(p, 'sequence_nr', -1) >= 0:
                    key = ('bwd', seqmap.get(p.sequence_nr, '?' + p.name[:40]))
                    break
                p = p.cpu_parent
            if key is None:
                top = ev
                while top.cpu_parent is not None:
                    top = top.cpu_parent
                key = ('other', top.name[:50])
        for k in ks:
            cnt[key] += 1
            tm[key] += k.duration
    total_n, total_t = sum(cnt.values()), sum(tm.values())
    lines = [f'one RL step (B=6, T=64): {total_n} kernels, {total_t / 1e3:.2f} ms device time (profiled)',
             f'{"phase":6s} {"component":48s} {"kernels":>8s} {"ms":>8s}']
    for key, n in sorted(cnt.items(), key=lambda kv: -tm[kv[0]]):
        lines.append(f'{key[0]:6s} {key[1][:48]:48s} {n:8d} {tm[key] / 1e3:8.3f}')
    by = collections.Counter()
    byt = collections.Counter()
    for (ph, m), n in cnt.items():
        by[ph] += n
        byt[ph] += tm[(ph, m)]
    lines.append('totals: ' + ', '.join(f'{ph} {by[ph]} kernels {byt[ph] / 1e3:.2f} ms' for ph in by))
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    with open(args.out, 'w') as f:
        f.write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:70]))


if __name__ == '__main__':
    main()
