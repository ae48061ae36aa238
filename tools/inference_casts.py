"""Where the actor inference forward's dtype casts and other glue launches come from: one eager
compute_logp_action / compute_teacher_logit under bf16 autocast (the GraphedPolicy's captured sequence), every
dispatched aten op counted by op and innermost applestar_amd call sites (TorchDispatchMode).

    python tools/inference_casts.py [--batch 1] [--top 60]
"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

META = {'view', 'slice', 'empty', 'detach', 'permute', 'select', 't', 'transpose', 'expand', 'record_stream',
        'empty_like', 'alias', 'as_strided', 'unsqueeze', 'squeeze', '_unsafe_view', 'reshape', 'split',
        'split_with_sizes', 'unbind', 'narrow', 'new_empty', 'set_', 'lift_fresh', '_reshape_alias', 'diagonal',
        'unfold', 'chunk', 'is_same_size', '_local_scalar_dense', 'resize_', 'new_empty_strided', 'empty_strided',
        'size', 'stride', 'dim'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1)
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--method', default='compute_logp_action')
    args = ap.parse_args()
    from applestar_amd.models.model import Model
    from applestar_amd.lib.features import random_obs, random_actions
    from applestar_amd.rl.synthetic import to_device
    from applestar_amd.models import encoders, model as model_mod
    dev = torch.device('cuda', 0)
    m = Model({'agent': {'extra_units': True}}).to(dev).eval().to(memory_format=torch.channels_last)
    if os.environ.get('APPLESTAR_INFERENCE_FORMS', '1') == '1':
        from applestar_amd.ops import native
        native.ensure_loaded()
        native.attach_inference_forms(m)       # as the inference server does (actor/inference.py set_model)
    B = args.batch
    g = torch.Generator().manual_seed(B)
    en = torch.randint(150, 300, (B,), generator=g)
    obs = random_obs(B, entity_num=en, generator=g)
    obs['hidden_state'] = [(torch.zeros(B, 384), torch.zeros(B, 384)) for _ in range(3)]
    obs = to_device(obs, dev)
    kw = dict(obs)
    if args.method == 'compute_teacher_logit':
        act, su_num = random_actions(B, en, generator=g)
        kw.update(selected_units_num=su_num.to(dev), action_info={k: v.to(dev) for k, v in act.items()})
    fn = getattr(m, args.method)
    # the graph-capture configuration (runtime/graphs.py GraphedPolicy)
    encoders.STATIC_SHAPES, encoders.SCALAR_SIDE_STREAM, model_mod.SIDE_STREAMS_ENABLED = True, False, False
    for _ in range(2):
        with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
            fn(**kw)
    torch.cuda.synchronize()
    sites = collections.Counter()
    ops = collections.Counter()

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, a=(), k=None):
            name = str(func.overloadpacket.__name__)
            if name not in META:
                fr = [f for f in traceback.extract_stack() if 'applestar_amd' in f.filename][-2:]
                site = ' < '.join(f'{f.filename.split("applestar_amd/")[-1]}:{f.lineno}' for f in fr[::-1]) \
                    if fr else '(no frame)'
                shp = [tuple(t.shape) for t in a if isinstance(t, torch.Tensor)][:1]
                dt = [str(t.dtype).replace('torch.', '') for t in a if isinstance(t, torch.Tensor)][:1]
                if name in ('_to_copy', 'to', 'copy_'):
                    site += f'  {shp} {dt}->{k.get("dtype") if k else ""}'
                sites[(name, site)] += 1
                ops[name] += 1
            return func(*a, **(k or {}))
    with Rec(), torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False):
        fn(**kw)
    torch.cuda.synchronize()
    print(f'aten ops dispatched (non-metadata): {sum(ops.values())}')
    for n, c in ops.most_common(25):
        print(f'{c:6d}  {n}')
    print()
    for (n, s), c in sorted(sites.items(), key=lambda kv: -kv[1])[:args.top]:
        print(f'{c:5d}  {n:22s} {s}')


if __name__ == '__main__':
    main()
