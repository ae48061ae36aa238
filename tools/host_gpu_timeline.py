"""Host issue time vs GPU completion time through one learner step, per phase: where the GPU waits for the host.

    python tools/host_gpu_timeline.py [--precision fp32|bf16] [--steps 3]

A CUDA event is recorded at every phase boundary (model submodules' forward entry / exit, loss, backward,
reduce, optimizer) together with the host clock.  For each mark: ``host_ms`` = when the host issued it,
``gpu_ms`` = when the GPU reached it (both from the step start).  Where ``gpu_ms - host_ms`` is near zero the GPU
had drained its queue and was waiting for the host (host-bound stretch); the growth of ``gpu_ms - host_ms``
across a phase is GPU-bound time.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='fp32')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=3)
    args = ap.parse_args()
    import bench
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree
    device = torch.device('cuda', 0)
    batches = [pin_tree(rl_batch(6, 64, max_entities=512, seed=i)) for i in range(2)]
    ns = argparse.Namespace(mode='rl', graph=False, batch=6, unroll=64)
    tr = bench._make_trainer(ns, args.precision, device, 'rl')
    marks = []
    on = {'v': False}

    def mark(name):
        if on['v']:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append((name, time.perf_counter(), e))

    def wrap(obj, attr, name):
        f = getattr(obj, attr)

        def g(*a, **k):
            mark(name + '>')
            r = f(*a, **k)
            mark(name + '<')
            return r
        setattr(obj, attr, g)
    for n, m in tr.model.named_modules():
        if not n or n.count('.') > 1 or (n.count('.') == 1 and not n.startswith('policy.')):
            continue        # the model's children and the policy heads
        m.register_forward_pre_hook(lambda mod, inp, n=n: mark('fwd:' + n + '>'))
        m.register_forward_hook(lambda mod, inp, out, n=n: mark('fwd:' + n + '<'))
    wrap(tr.model.policy.selected_units_head, 'forward_teacher', 'fwd:policy.selected_units_head.teacher')
    wrap(tr.loss, 'compute_loss', 'loss')
    wrap(tr, 'backward', 'backward')
    wrap(tr, '_reduce', 'reduce')
    wrap(tr, '_update', 'update')

    def source():
        i = 0
        while True:
            yield batches[i % 2]
            i += 1
    it = DevicePrefetcher(source(), device)
    for _ in range(args.warmup):
        tr.step(next(it))
    torch.cuda.synchronize()
    rows = []
    for s in range(args.steps):
        marks.clear()
        batch = next(it)
        torch.cuda.synchronize()
        on['v'] = True
        mark('start')
        tr.step(batch)
        mark('end')
        on['v'] = False
        torch.cuda.synchronize()
        h0, e0 = marks[0][1], marks[0][2]
        rows.append([(n, (h - h0) * 1e3, e0.elapsed_time(e)) for n, h, e in marks])
    # the last step's table; the mean over steps for the totals
    print(json.dumps({'precision': args.precision,
                      'host_ms': [round(r[-1][1], 2) for r in rows], 'gpu_ms': [round(r[-1][2], 2) for r in rows]}))
    print(f'{"mark":40s} {"host_ms":>8s} {"gpu_ms":>8s} {"lag":>7s}  d_host  d_gpu')
    prev = None
    for n, h, g in rows[-1]:
        dh = h - prev[1] if prev else 0.0
        dg = g - prev[2] if prev else 0.0
        print(f'{n:40s} {h:8.2f} {g:8.2f} {g - h:7.2f}  {dh:6.2f} {dg:6.2f}')
        prev = (n, h, g)


if __name__ == '__main__':
    main()
