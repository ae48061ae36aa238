"""Attribute the learner step's autograd nodes to their forward call sites (which torch-level ops are left
between the native nodes, and where).

Builds the bench's RL trainer (``--precision fp32|bf16``), runs one forward + loss under anomaly mode (each
node records its forward traceback), walks the graph from ``total_loss`` and prints, per (node type, innermost
package frame): node count and summed output elements.  One backward launch (or more) per node, so this is the
map of the step's torch elementwise / copy / cat work.

    python tools/diag/autograd_nodes.py --precision fp32 > gpurun_out/autograd_nodes_fp32.txt
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def _site(node):
    tb = node.metadata.get('traceback_') if hasattr(node, 'metadata') else None
    if not tb:
        return '?'
    frames = [ln for ln in ''.join(tb).splitlines() if 'File "' in ln and 'applestar_amd' in ln]
    if not frames:
        return '?'
    out = []
    for f in frames[-2:]:
        f = f.strip()
        path = f.split('"')[1]
        path = path[path.index('applestar_amd') + len('applestar_amd/'):]
        line = f.split('line ')[1].split(',')[0]
        fn = f.split(' in ')[-1] if ' in ' in f else ''
        out.append(f'{path}:{line} {fn}')
    return ' <- '.join(reversed(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--batch', type=int, default=6)
    ap.add_argument('--unroll', type=int, default=64)
    args = ap.parse_args()
    from applestar_amd.rl.synthetic import rl_batch, to_device
    from applestar_amd.rl.trainer import RLTrainer, _amp
    dev = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    tr = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16' if args.precision == 'bf16' else None},
                    'model': {'enable_baselines': ['winloss']}}, device=dev)
    batch = to_device(rl_batch(args.batch, args.unroll, max_entities=512, seed=7), dev)
    tr.step(batch)              # warm caches (derived weights, workspaces) like a steady step
    tr.model.train()
    with torch.autograd.set_detect_anomaly(True, check_nan=False):
        with _amp(dev, tr.amp_dtype):
            out = tr.model.rl_learner_forward(**batch)
        info = tr.loss.compute_loss(out)
    root = info['total_loss'].grad_fn
    seen, stack = set(), [root]
    count = collections.Counter()
    elems = collections.Counter()
    types = collections.Counter()
    while stack:
        n = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        name = type(n).__name__
        types[name] += 1
        key = (name, _site(n))
        count[key] += 1
        try:
            elems[key] += sum(int(t.numel()) for t in getattr(n, '_saved_result', None) and [n._saved_result] or [])
        except Exception:       # noqa: BLE001 - best effort size
            pass
        for nxt, _ in n.next_functions:
            if nxt is not None:
                stack.append(nxt)
    print(f'# {len(seen)} autograd nodes ({args.precision}, B={args.batch}, T={args.unroll})')
    print('# by type:')
    for name, c in types.most_common():
        print(f'{c:6d}  {name}')
    print('# by (type, forward site), AccumulateGrad omitted:')
    for (name, site), c in count.most_common():
        if name == 'AccumulateGrad':
            continue
        print(f'{c:6d}  {name:40s} {site}')


if __name__ == '__main__':
    main()
