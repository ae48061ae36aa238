"""Microbenchmark of the fused value-baseline residual MLP kernels (resmlp.hip): forward without and
with the saved activations, and the data-gradient backward, over a few row counts (R = 390 is the
learner's (T + 1) * B).  One JSON line per case: us / call.

    python tools/bench_resmlp.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.ops import native  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    C = native.ensure_loaded()
    torch.manual_seed(0)
    dev = 'cuda'
    for nblk in (16, 4):
        params = []
        for _ in range(nblk):
            params += [(torch.randn(256, 256, device=dev) / 16).to(torch.bfloat16),
                       (torch.randn(256, device=dev) / 10).to(torch.bfloat16),
                       (torch.randn(256, 256, device=dev) / 16).to(torch.bfloat16),
                       (torch.randn(256, device=dev) / 10).to(torch.bfloat16),
                       1 + torch.randn(256, device=dev) / 10, torch.randn(256, device=dev) / 10]
        for R in (16, 390, 4096):
            x = torch.randn(R, 256, device=dev)
            f0 = timed(lambda: C.resmlp_fwd(x, params, False))
            f1 = timed(lambda: C.resmlp_fwd(x, params, True))
            out, sx, sh, sxh, srs = C.resmlp_fwd(x, params, True)
            d = torch.randn_like(out)
            b = timed(lambda: C.resmlp_bwd(d, params, sx, sh, sxh, srs))
            print(json.dumps({'nblk': nblk, 'R': R, 'fwd_us': round(f0, 1), 'fwd_save_us': round(f1, 1),
                              'bwd_us': round(b, 1)}), flush=True)


if __name__ == '__main__':
    main()
