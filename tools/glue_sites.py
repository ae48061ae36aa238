"""Where the fp32 learner step's torch glue launches come from: torch.profiler with Python stacks over a few RL
learner iterations, device time of the aten ops that launch torch's own kernels (elementwise, copies, fills,
reductions, cat / index), grouped by their innermost applestar_amd call sites.

    python tools/glue_sites.py [--steps 2] [--precision fp32|bf16] [--shapes] > gpurun_out/glue_sites.txt
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--precision', default='fp32')
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--shapes', action='store_true', help='key the call sites by the first two tensor shapes too')
    ap.add_argument('--timed', action='store_true',
                    help='also time every dispatched aten op with stream events and attribute backward ops to their '
                         'autograd node and its forward call site (anomaly mode keeps the forward stacks)')
    ap.add_argument('--premask', action='store_true',
                    help='count the ReLU backward passes not folded into a consumer epilogue, by forward site')
    args = ap.parse_args()
    if args.premask:
        os.environ['APPLESTAR_DEBUG_PREMASK'] = '1'
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch, to_device
    dev = torch.device('cuda', 0)
    learner = {'use_value_feature': True}
    if args.precision == 'bf16':
        learner['amp_dtype'] = 'bfloat16'
    tr = RLTrainer({'learner': learner, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    b = to_device(rl_batch(6, 64, seed=0), dev)
    for _ in range(2):
        tr.step(dict(b))
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step(dict(b))
        torch.cuda.synchronize()
    glue = ('aten::add', 'aten::add_', 'aten::mul', 'aten::mul_', 'aten::copy_', 'aten::fill_', 'aten::zero_',
            'aten::threshold_backward', 'aten::sum', 'aten::cat', 'aten::index', 'aten::index_put_', 'aten::where',
            'aten::sub', 'aten::div', 'aten::clamp', 'aten::relu', 'aten::masked_fill_', 'aten::scatter_add_',
            'aten::gather', 'aten::to', 'aten::_to_copy', 'aten::contiguous', 'aten::neg', 'aten::exp', 'aten::log',
            'aten::max', 'aten::mean', 'aten::addcmul_', 'aten::lerp_', 'aten::sigmoid', 'aten::tanh')
    by_site = collections.defaultdict(lambda: [0.0, 0])
    for ev in prof.events():
        if ev.name not in glue:
            continue
        dt = getattr(ev, 'device_time_total', None)
        if dt is None:
            dt = ev.cuda_time_total
        if dt <= 0:
            continue
        frames = [f for f in (ev.stack or []) if 'applestar_amd' in f]
        site = frames[0].split('applestar_amd/')[-1] if frames else '(autograd / no python frame)'
        key = (ev.name, site)
        by_site[key][0] += dt / args.steps
        by_site[key][1] += 1.0 / args.steps
    rows = sorted(by_site.items(), key=lambda kv: -kv[1][0])
    total = sum(v[0] for _, v in rows)
    print(f'glue device time {total / 1e3:.2f} ms / iteration over {sum(v[1] for _, v in rows):.0f} ops')
    for (name, site), (t, n) in rows[:args.top]:
        print(f'{t / 1e3:8.3f} ms {n:6.1f}x  {name:26s} {site}')
    # call sites of the aten ops one iteration dispatches: the innermost three applestar_amd frames (a backward op of a
    # built-in autograd formula has none)
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    sites = collections.Counter()
    META = {'view', 'slice', 'empty', 'detach', 'permute', 'select', 't', 'transpose', 'expand', 'record_stream',
            'empty_like', 'alias', 'as_strided', 'unsqueeze', 'squeeze', '_unsafe_view', 'reshape', 'split',
            'split_with_sizes', 'unbind', 'narrow', 'new_empty', 'set_', 'lift_fresh', '_reshape_alias', 'diagonal',
            'unfold', 'chunk', 'is_same_size', '_local_scalar_dense', 'resize_', 'new_empty_strided', 'empty_strided',
            'clone_meta', 'is_nonzero', 'size', 'stride', 'dim'}

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, a=(), kw=None):
            name = str(func.overloadpacket.__name__)
            if name not in META:
                fr = [f for f in traceback.extract_stack() if 'applestar_amd' in f.filename][-3:]
                site = ' < '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in fr[::-1]) \
                    if fr else '(autograd formula)'
                if args.shapes:
                    site += '  ' + str([tuple(t.shape) for t in a if isinstance(t, torch.Tensor)][:2])
                sites[(name, site)] += 1
            return func(*a, **(kw or {}))
    with Rec():
        tr.step(dict(b))
    torch.cuda.synchronize()
    print()
    print('kernel-launching aten calls per iteration by site (TorchDispatchMode; metadata-only ops skipped):')
    for (name, site), n in sorted(sites.items(), key=lambda kv: -kv[1]):
        print(f'{n:6d}  {name:28s} {site}')
    if args.timed:
        timed_sites(tr, b, META, args)
    if args.premask:
        from applestar_amd.ops import native
        native.PREMASK_MISSES.clear()
        tr.step(dict(b))
        torch.cuda.synchronize()
        print()
        print('ReLU backward passes not folded into a consumer epilogue (one iteration):')
        for (kind, shape, site), n in sorted(native.PREMASK_MISSES.items(), key=lambda kv: -kv[1]):
            print(f'{n:4d}  {kind:9s} {str(shape):24s} {site}')


def _fwd_site(node):
    """innermost applestar_amd frames of the forward call that created autograd node ``node``"""
    tb = (getattr(node, 'metadata', None) or {}).get('traceback_')
    if not tb:
        return '?'
    lines = [ln for ln in ''.join(tb).splitlines() if 'applestar_amd/' in ln and 'File' in ln][-2:]
    out = []
    for ln in lines[::-1]:
        f = ln.split('applestar_amd/')[-1]
        out.append(f.split('"')[0] + ':' + f.split('line ')[-1].split(',')[0])
    return ' < '.join(out)


def timed_sites(tr, b, META, args):
    """device time of each dispatched aten op (a start / end event pair on the current stream around it),
    grouped by op and site; ops inside backward carry their autograd node and the node's forward site"""
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    recs = []

    class Timed(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, a=(), kw=None):
            name = str(func.overloadpacket.__name__)
            if name in META:
                return func(*a, **(kw or {}))
            fr = [f for f in traceback.extract_stack() if 'applestar_amd' in f.filename][-2:]
            if fr:
                site = ' < '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in fr[::-1])
            else:
                node = torch._C._current_autograd_node()
                site = f'[{node.name()}] fwd {_fwd_site(node)}' if node is not None else '(no frame)'
            if args.shapes:
                site += '  ' + str([tuple(t.shape) for t in a if isinstance(t, torch.Tensor)][:2])
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            out = func(*a, **(kw or {}))
            e1.record(st)
            recs.append((name, site, e0, e1))
            return out
    with torch.autograd.set_detect_anomaly(True, check_nan=False):
        tr.step(dict(b))             # anomaly mode records forward stacks of the nodes
        torch.cuda.synchronize()
        with Timed():
            tr.step(dict(b))
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0.0, 0])
    for name, site, e0, e1 in recs:
        agg[(name, site)][0] += e0.elapsed_time(e1)
        agg[(name, site)][1] += 1
    total = sum(v[0] for v in agg.values())
    print()
    print(f'event-timed aten ops, one iteration: {total:.2f} ms over {len(recs)} ops (includes any stall on the '
          f'stream between the two events)')
    for (name, site), (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.top * 2]:
        print(f'{t:8.3f} ms {n:5d}x  {name:24s} {site}')


if __name__ == '__main__':
    main()
