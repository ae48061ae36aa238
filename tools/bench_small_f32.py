"""Small fp32 linears of the learner step (a few hundred to a few thousand rows, the shapes the RL model issues
per step: core/heads/value MLPs at 390 / 384 rows, the 7800-row scalar-context MLPs): library forward
(addmm / _addmm_activation) and dX (mm) vs the f32-MFMA GEMM (gemm_f32.hip) at any tile count, time per call
from GPU events over 50 back-to-back calls, max error of each against float64.

    python tools/bench_small_f32.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_f32_kernels import timed  # noqa: E402

# (R, N, K): forward x[R, K] W[N, K]^T; dX = dY[R, N] W[N, K] -> the [R, K] x [K, N]^T product
SHAPES = [(390, 256, 256), (384, 256, 256), (384, 1024, 256), (384, 256, 1024), (384, 1520, 1024),
          (390, 256, 1440), (390, 64, 260), (390, 128, 260), (384, 256, 384), (384, 1024, 384), (384, 128, 256),
          (7800, 128, 64), (7800, 64, 128), (7800, 48, 64), (7800, 64, 16)]


def rel(out, ref):
    return float((out.double() - ref).abs().max() / ref.abs().max())


def main():
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(0)
    for R, N, K in SHAPES:
        x = torch.randn(R, K, device='cuda')
        w = torch.randn(N, K, device='cuda') / K ** 0.5
        b = torch.randn(N, device='cuda')
        dy = torch.randn(R, N, device='cuda')
        wt = w.t().contiguous()
        ref_f = torch.relu(x.double() @ w.double().t() + b.double())
        ref_d = dy.double() @ w.double()
        row = {'shape': [R, N, K]}
        row['lib_fwd_us'] = round(timed(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False), 50), 1)
        row['lib_dx_us'] = round(timed(lambda: torch.mm(dy, w), 50), 1)
        row['lib_fwd_err'] = rel(torch._addmm_activation(b, x, w.t(), use_gelu=False), ref_f)
        if K % 4 == 0:
            row['mfma_fwd_us'] = round(timed(lambda: C.gemm_f32(x, w, b, None, 1), 50), 1)
            row['mfma_fwd_err'] = rel(C.gemm_f32(x, w, b, None, 1), ref_f)
        if N % 4 == 0:
            row['mfma_dx_us'] = round(timed(lambda: C.gemm_f32(dy, wt, None, None, 0), 50), 1)
            row['mfma_dx_err'] = rel(C.gemm_f32(dy, wt, None, None, 0), ref_d)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
