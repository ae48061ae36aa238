"""Find where dtype casts / copies / small elementwise ops come from in one RL learner step: a
TorchDispatchMode records every aten op with the innermost applestar_amd Python frame (forward) and
groups by (op, frame); backward ops are grouped under '<backward>' (they run on autograd's thread).
Usage: python tools/cast_sources.py [--ops _to_copy,copy_,add,mul,...]"""
import argparse
import collections
import os
import sys
import threading
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402


class Rec(TorchDispatchMode):
    def __init__(self, ops):
        super().__init__()
        self.ops = ops
        self.agg = collections.defaultdict(lambda: [0, 0])
        self.main = threading.get_ident()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split('.')[0]
        if name in self.ops:
            where = '<backward>'
            if threading.get_ident() == self.main:
                where = '?'
                for fr in reversed(traceback.extract_stack()[:-2]):
                    if 'applestar_amd' in fr.filename and 'trainer.py' not in fr.filename:
                        where = f"{fr.filename.split('applestar_amd/')[-1]}:{fr.lineno} {fr.name}"
                        break
            numel = out.numel() if torch.is_tensor(out) else 0
            if torch.is_tensor(out) and (where == '<backward>' or name == '_to_copy'):
                ins = [f"{tuple(a.shape)}:{str(a.dtype)[6:]}" + ('' if a.is_contiguous() else '(nc)')
                       for a in args if torch.is_tensor(a)]
                where = f"{where} out {tuple(out.shape)}:{str(out.dtype)[6:]} in {' '.join(ins)}"
            a = self.agg[(name, where)]
            a[0] += 1
            a[1] += numel
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ops', default='_to_copy,copy_,clone,contiguous,add,add_,mul,cat,sum,relu,threshold_backward')
    ap.add_argument('--out', default='gpurun_out/cast_sources.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    b = to_device(rl_batch(6, 64, seed=0), dev)
    tr.step(dict(b))
    torch.cuda.synchronize()
    rec = Rec(set(args.ops.split(',')))
    with rec:
        tr.step(dict(b))
    torch.cuda.synchronize()
    rows = sorted(rec.agg.items(), key=lambda kv: -kv[1][1])
    lines = [f'{n:6d} calls {e / 1e6:9.2f} Melem  {op:20s} {w}' for (op, w), (n, e) in rows[:150]]
    txt = '\n'.join(lines)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, 'w').write(txt)
    print(txt)


if __name__ == '__main__':
    main()
