"""Few-row, long-K products on gemm_small.hip (small_gemm_splitk / small_gemm) vs torch.mm: the actor's B = 1..16
spatial-encoder fc (48,640 -> 256) and the learner's 390-row form.  Prints one JSON line per shape / dtype.

    python tools/bench_small_gemm.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    from applestar_amd.ops import native as N
    C = N.ensure_loaded()
    dev = torch.device('cuda', 0)
    for (M, Nn, K) in [(1, 256, 48640), (16, 256, 48640), (390, 256, 48640), (1, 128, 12160), (16, 128, 12160)]:
        for dt in (torch.bfloat16, torch.float32):
            a = torch.randn(M, K, device=dev).to(dt)
            w = (torch.randn(Nn, K, device=dev) * 0.01).to(dt)
            b = torch.randn(Nn, device=dev)
            med, mn = _time(lambda: C.small_gemm_splitk(a, w, b, 1))
            tmed, tmn = _time(lambda: torch.relu(torch.nn.functional.linear(a, w, b.to(dt))))
            ref = torch.relu(a.double() @ w.double().t() + b.double())
            err = (C.small_gemm_splitk(a, w, b, 1).double() - ref).abs().max().item()
            print(json.dumps({'shape': [M, Nn, K], 'dtype': str(dt).replace('torch.', ''),
                              'splits': C.small_nt_splits(M, Nn, K) if hasattr(C, 'small_nt_splits') else None,
                              'us_med': round(med, 1), 'us_min': round(mn, 1), 'torch_us_med': round(tmed, 1),
                              'gbps': round((M * K + Nn * K) * a.element_size() / med / 1e3, 1),
                              'err_max': err}), flush=True)


if __name__ == '__main__':
    main()
