"""hipBLASLt (torch.mm) on the GEMM shapes of the learner's 3x3 convs, as a library reference for the
native implicit-GEMM conv and its weight gradient: conv fwd = [M, 9 Cin] x [9 Cin, Cout] with
M = B*H*W pixels; wgrad = [Cout, M] x [M, 9 Cin].  One JSON line per shape.

    python tools/bench_gemm_shapes.py
"""
import json

import torch


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
    for M, cin, cout in [(390 * 380, 128, 128), (390 * 1520, 64, 128), (390 * 1520, 128, 64)]:
        K = 9 * cin
        a = torch.randn(M, K, device='cuda').to(torch.bfloat16)
        b = torch.randn(K, cout, device='cuda').to(torch.bfloat16)
        dy = torch.randn(M, cout, device='cuda').to(torch.bfloat16)
        f = timed(lambda: torch.mm(a, b))
        w = timed(lambda: torch.mm(dy.t(), a))
        flop = 2.0 * M * K * cout
        print(json.dumps({'M': M, 'K': K, 'N': cout, 'fwd_us': round(f, 1), 'fwd_tflops': round(flop / f / 1e6, 1),
                          'wgrad_us': round(w, 1), 'wgrad_tflops': round(flop / w / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()
