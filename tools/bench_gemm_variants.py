"""A/B of the fp32 split-MFMA GEMM tile / ring variants (``set_f32_pipe_variant``) on the learner's GEMM shapes,
interleaved rounds in one process; per (shape, variant): median / min us, TF/s, max and relative-Frobenius error
against float64 on a row subsample.

    python tools/bench_gemm_variants.py [variants=0,3,4] [rounds=5]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (M, N, K): entity transformer forward (QKV, proj, FFN1, FFN2) and dX (N = input width, K = output width)
SHAPES = [(99526, 768, 256), (99526, 256, 256), (99526, 1024, 256), (99526, 256, 1024), (99526, 256, 768)]


def timed(fn, n=10):
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
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '0,3,4').split(',')]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.manual_seed(0)
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device='cuda')
        b = torch.randn(N, K, device='cuda')
        bias = torch.randn(N, device='cuda')
        rows = torch.arange(0, M, 97, device='cuda')
        ref = a[rows].double() @ b.double().t() + bias.double()
        times = {v: [] for v in variants}
        errs = {}
        for r in range(rounds):
            for v in variants:
                C.set_f32_pipe_variant(v)
                times[v].append(timed(lambda: C.gemm_f32(a, b, bias, None, 0)))
                if r == 0:
                    out = C.gemm_f32(a, b, bias, None, 0)[rows].double()
                    d = (out - ref).abs()
                    errs[v] = (float(d.max() / ref.abs().max()), float(d.norm() / ref.norm()))
        for v in variants:
            t = sorted(times[v])
            print(json.dumps({'shape': [M, N, K], 'variant': v, 'us_med': round(t[len(t) // 2], 1),
                              'us_min': round(t[0], 1), 'tflops': round(2.0 * M * N * K / t[len(t) // 2] / 1e6, 1),
                              'err_max': errs[v][0], 'err_fro': errs[v][1]}), flush=True)
    C.set_f32_pipe_variant(0)


if __name__ == '__main__':
    main()
