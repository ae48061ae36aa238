"""Which source lines issue the small aten ops (copies, casts, cat, fills, elementwise) in the learner's
forward + loss, counted with a TorchDispatchMode (host-side; the backward of these ops follows the
same lines).  Usage: python tools/op_sources.py [--out gpurun_out/op_sources.txt]"""
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

SKIP = ('view', 'reshape', 'permute', 'transpose', 't.default', 'expand', 'slice', 'select', 'unsqueeze', 'squeeze',
        'as_strided', 'detach', 'alias', 'split', 'chunk', 'unbind', '_unsafe_view', 'narrow', 'is_', 'size', 'stride',
        'lift_fresh', 'empty', 'sym_', 'dim', '_local_scalar_dense', 'item')


class Counter(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not any(s in name for s in SKIP):
            frames = [f for f in traceback.extract_stack()[:-1] if 'applestar_amd' in f.filename]
            where = ' <- '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in frames[-2:][::-1])
            self.cnt[(name, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default='gpurun_out/op_sources.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    h = rl_batch(6, 64, seed=0)
    b = to_device(h, dev)
    b['entity_total'] = entity_total_hint(h)
    tr.step(dict(b))
    torch.cuda.synchronize()
    mode = Counter()
    with mode:
        with _amp(dev, 'bfloat16'):
            out = tr.model.rl_learner_forward(**b)
        tr.loss.compute_loss(out)
    lines = [f'{n:5d}  {k[0][:40]:40s} {k[1]}' for k, n in mode.cnt.most_common(150)]
    lines.insert(0, f'total dispatched (non-view) ops in forward + loss: {sum(mode.cnt.values())}')
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    open(args.out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:120]))


if __name__ == '__main__':
    main()
