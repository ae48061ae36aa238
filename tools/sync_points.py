"""List the host<->device synchronisations of one RL learner step (torch.cuda.set_sync_debug_mode),
with the applestar_amd source line that triggered each.  Usage: python tools/sync_points.py [--fp32 | --infer]"""
import collections
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch, to_device  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    infer = '--infer' in sys.argv
    if infer:
        from applestar_amd.models.model import Model
        from applestar_amd.lib.features import random_obs
        m = Model({'agent': {'extra_units': True}}).to(dev).eval().to(memory_format=torch.channels_last)
        g = torch.Generator().manual_seed(0)
        obs = to_device(random_obs(1, entity_num=torch.tensor([300]), generator=g), dev)
        hs = [(torch.zeros(1, 384, device=dev), torch.zeros(1, 384, device=dev)) for _ in range(3)]

        def run():
            with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
                m.compute_logp_action(**obs, hidden_state=hs)

        class _T:
            def step(self, _):
                run()
        tr = _T()
        b = {}
    else:
        amp = None if '--fp32' in sys.argv else 'bfloat16'
        tr = RLTrainer({'learner': {'use_value_feature': True, 'amp_dtype': amp}, 'model': {'enable_baselines': ['winloss']}},
                       device=dev)
        from applestar_amd.runtime.prefetch import entity_total_hint
        h = rl_batch(6, 64, seed=0)
        b = to_device(h, dev)
        b['entity_total'] = entity_total_hint(h)   # as the bench's prefetcher supplies it
    tr.step(dict(b))
    torch.cuda.synchronize()
    hits = collections.Counter()

    def showwarning(message, category, filename, lineno, file=None, line=None):
        where = '?'
        for fr in reversed(traceback.extract_stack()[:-1]):
            if 'applestar_amd' in fr.filename:
                where = f"{fr.filename.split('applestar_amd/')[-1]}:{fr.lineno} {fr.name}: {fr.line}"
                break
        hits[where] += 1

    warnings.showwarning = showwarning
    warnings.simplefilter('always')
    torch.cuda.set_sync_debug_mode('warn')
    tr.step(dict(b))
    torch.cuda.set_sync_debug_mode('default')
    torch.cuda.synchronize()
    for where, n in hits.most_common():
        print(f'{n:4d}  {where}')


if __name__ == '__main__':
    main()
