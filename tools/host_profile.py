"""cProfile of the host side of RL learner steps (where the per-step Python / dispatch time goes).
Usage: python tools/host_profile.py [--steps 10]"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.trainer import RLTrainer  # noqa: E402
from applestar_amd.rl.synthetic import rl_batch  # noqa: E402
from applestar_amd.runtime.prefetch import DevicePrefetcher, pin_tree  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--out', default='gpurun_out/host_profile.txt')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
    hb = [pin_tree(rl_batch(6, 64, max_entities=512, seed=i)) for i in range(2)]

    def src():
        i = 0
        while True:
            yield hb[i % 2]
            i += 1
    it = DevicePrefetcher(src(), dev)
    for _ in range(5):
        tr.step(next(it))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        tr.step(next(it))
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats('tottime').print_stats(45)
    st.sort_stats('cumulative').print_stats(60)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, 'w').write(s.getvalue())
    print(s.getvalue()[:20000])


if __name__ == '__main__':
    main()
