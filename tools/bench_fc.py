"""Microbenchmark of the skinny-M / huge-K linears (spatial fc 48640->256, value spatial fc 12160->128):
hipBLASLt vs rocBLAS vs the split-K formulations.  Usage: python tools/bench_fc.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    dev = 'cuda'
    for (M, K, N) in [(390, 48640, 256), (390, 12160, 128), (384, 1024, 1520)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        res = {'shape': [M, K, N]}
        for lib in ('cublaslt', 'cublas'):
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as e:  # noqa: BLE001
                res[lib] = str(e)[:60]
                continue
            res[f'{lib}_fwd_us'] = timeit(lambda: torch.nn.functional.linear(x, w))
            res[f'{lib}_dx_us'] = timeit(lambda: dy @ w)
            res[f'{lib}_dw_us'] = timeit(lambda: dy.t() @ x)
        torch.backends.cuda.preferred_blas_library('cublaslt')
        for S in (16, 64):
            xs = x.view(M, S, K // S).transpose(0, 1)
            ws = w.view(N, S, K // S).permute(1, 2, 0)
            try:
                res[f'bmm_splitk{S}_fp32out_us'] = timeit(lambda: torch.bmm(xs, ws, out_dtype=torch.float32).sum(0))
            except Exception as e:  # noqa: BLE001
                res[f'bmm_splitk{S}_fp32out_us'] = str(e)[:80]
            res[f'bmm_splitk{S}_us'] = timeit(lambda: torch.bmm(xs, ws).float().sum(0))
        wt = w.t().contiguous()
        res['dx_via_wT_us'] = timeit(lambda: torch.nn.functional.linear(dy, wt))
        from applestar_amd.ops import native
        C = native.ensure_loaded()
        res['native_wgrad_dw_us'] = timeit(lambda: C.wgrad(dy, x, 0, False))
        print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
