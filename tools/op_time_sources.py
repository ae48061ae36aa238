"""Device time of the aten ops issued by the learner's forward + loss + backward, by (op, source line):
a TorchDispatchMode brackets every non-view op with CUDA events (timed on the current stream; ops on side
streams are attributed but their times include any queueing).  Usage:
    python tools/op_time_sources.py [--out gpurun_out/op_time_sources.txt]"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer, _amp  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402
from applestar_amd.runtime.prefetch import entity_total_hint  # noqa: E402

# metadata-only ops, matched on the op's base name (a substring match on 'aten.cat.default' would hit 't.default')
SKIP = ('view', 'reshape', 'permute', 'transpose', 't', 'expand', 'slice', 'select', 'unsqueeze', 'squeeze',
        'as_strided', 'detach', 'alias', 'split', 'split_with_sizes', 'chunk', 'unbind', '_unsafe_view', 'narrow',
        'size', 'stride', 'lift_fresh', 'dim', '_local_scalar_dense', 'item', 'record_stream', 'expand_as', 'view_as')
SKIP_PREFIX = ('is_', 'empty', 'sym_')


def _skip(name: str) -> bool:
    base = name.split('.')[1] if name.count('.') >= 1 else name
    return base in SKIP or base.startswith(SKIP_PREFIX)


class Timer(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rec = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if _skip(name):
            return func(*args, **(kwargs or {}))
        frames = [f for f in traceback.extract_stack()[:-1] if 'applestar_amd' in f.filename]
        depth = int(os.environ.get('OP_FRAMES', '2'))
        where = ' <- '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in frames[-depth:][::-1])
        if os.environ.get('OP_SHAPES'):
            where += ' ' + ' '.join(f'{tuple(a.shape)}{str(a.dtype)[6:]}' for a in args if isinstance(a, torch.Tensor))[:60]
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = func(*args, **(kwargs or {}))
        e.record()
        if not where:   # autograd-engine ops: identify them by operand shapes / dtypes
            shapes = [f'{tuple(a.shape)}{str(a.dtype)[6:]}' for a in args if isinstance(a, torch.Tensor)][:2]
            where = '(autograd engine) ' + ' '.join(shapes)
        self.rec.append((name, where, s, e))
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/op_time_sources.txt')
    ap.add_argument('--precision', choices=['fp32', 'bf16'], default='bf16')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    amp = 'bfloat16' if args.precision == 'bf16' else None
    tr = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': amp},
                    'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    for _ in range(2):
        tr.step(dict(b))
    torch.cuda.synchronize()
    mode = Timer()
    with mode:
        with _amp(dev, amp):
            out = tr.model.rl_learner_forward(**b)
        info = tr.loss.compute_loss(out)
        loss = info['total_loss']
        params = [p for p in tr.model.parameters() if p.requires_grad]
        torch.autograd.grad(loss, params, allow_unused=True)   # as the trainer (no .grad accumulation)
    torch.cuda.synchronize()
    cnt, tm = collections.Counter(), collections.Counter()
    for name, where, s, e in mode.rec:
        cnt[(name, where)] += 1
        tm[(name, where)] += s.elapsed_time(e)
    lines = [f'{cnt[k]:5d} {tm[k]:8.3f} ms  {k[0][:34]:34s} {k[1]}' for k in sorted(tm, key=lambda k: -tm[k])]
    lines.insert(0, f'total {sum(tm.values()):.3f} ms over {sum(cnt.values())} ops')
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    open(args.out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:80]))


if __name__ == '__main__':
    main()
