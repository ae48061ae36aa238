"""Pre-split-weight fp32 GEMM (gemm_f32_psb.hip) vs the split ring GEMM (gemm_f32.hip) on the learner's shapes:
time per call, TF/s of fp32 products, and max / Frobenius error against float64.

    python tools/bench_gemm_psb.py [iters]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from applestar_amd.ops import native as N
    C = N.ensure_loaded()
    torch.manual_seed(0)
    shapes = [(99526, 768, 256), (99526, 256, 256), (99526, 1024, 256), (99526, 256, 1024), (145920, 128, 128)]
    for M, Nn, K in shapes:
        a = torch.randn(M, K, device='cuda')
        b = torch.randn(Nn, K, device='cuda') / K ** 0.5
        bias = torch.randn(Nn, device='cuda')
        bs = C.presplit_b(b)
        ref = (a[:4096].double() @ b.double().t() + bias.double()).relu()
        res = {}
        for name, fn in (('ring', lambda: C.gemm_f32(a, b, bias, None, 1)),
                         ('psb_db2w', lambda: C.gemm_f32_psb(a, bs, Nn, K, bias, None, 1, 0)),
                         ('psb_sb', lambda: C.gemm_f32_psb(a, bs, Nn, K, bias, None, 1, 1)),
                         ('v2_ns3', lambda: C.gemm_f32_psb(a, bs, Nn, K, bias, None, 1, 10)),
                         ('v2_ns2', lambda: C.gemm_f32_psb(a, bs, Nn, K, bias, None, 1, 12)),
                         ('v2_k32', lambda: C.gemm_f32_psb(a, bs, Nn, K, bias, None, 1, 14))):
            out = fn()
            err = (out[:4096].double() - ref).abs()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ts = []
            for _ in range(iters):
                ev[0].record()
                fn()
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
            ts.sort()
            us = ts[len(ts) // 2]
            res[name] = us
            print(json.dumps({'shape': [M, Nn, K], 'kernel': name, 'us_med': round(us, 1), 'us_min': round(ts[0], 1),
                              'tflops': round(2 * M * Nn * K / us / 1e6, 1), 'err_max': float(err.max()),
                              'err_fro': float(err.norm() / ref.norm())}), flush=True)
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(iters):
            C.presplit_b(b)
        t1.record()
        torch.cuda.synchronize()
        print(json.dumps({'shape': [Nn, K], 'presplit_us': round(t0.elapsed_time(t1) * 1e3 / iters, 1),
                          'speedup_db2w': round(res['ring'] / res['psb_db2w'], 3),
                          'speedup_sb': round(res['ring'] / res['psb_sb'], 3),
                          'best_v2_vs_psb': round(min(res['psb_db2w'], res['psb_sb']) /
                                                  min(res['v2_ns3'], res['v2_ns2'], res['v2_k32']), 3)}), flush=True)


if __name__ == '__main__':
    main()
