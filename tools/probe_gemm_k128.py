"""Probe: the fp32 split GEMM at small K (the location head's gate layers, K = N = 128 over 145,920 rows; the
entity transformer's K = 256 products) against a plain device copy of the same bytes (the memory floor).

    python tools/probe_gemm_k128.py      (APPLESTAR_GEMM_F32_STAGED=0|1 selects the epilogue)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    staged = os.environ.get('APPLESTAR_GEMM_F32_STAGED', '1')
    for M, N, K in [(145920, 128, 128), (99526, 1024, 256), (99526, 768, 256), (99526, 256, 1024)]:
        a = torch.randn(M, K, device='cuda')
        b = torch.randn(N, K, device='cuda') / K ** 0.5
        bias = torch.randn(N, device='cuda')
        out = torch.empty(M, N, device='cuda')
        us = timed(lambda: C.gemm_f32(a, b, bias, None, 1))
        cp = timed(lambda: out.copy_(a[:, :1].expand(M, N)) if N != K else out.copy_(a))
        print(json.dumps({'M': M, 'N': N, 'K': K, 'staged': staged, 'gemm_us': round(us, 1),
                          'tflops': round(2.0 * M * N * K / us / 1e6, 1), 'copy_us': round(cp, 1)}), flush=True)


if __name__ == '__main__':
    main()
