"""Exact-f32 MFMA vs bf16x6 split MFMA (csrc/split_mfma.h) on the fp32 learner's GEMM / conv / wgrad shapes: time
per call and max / relative-Frobenius error of each against a float64 reference on a row subsample.

    python tools/bench_split_f32.py [gemm|conv|wgrad|all]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_f32_kernels import CONV, GEMM, timed  # noqa: E402


def err(out, ref):
    d = (out.double() - ref).abs()
    return float(d.max() / ref.abs().max()), float(d.norm() / ref.norm())


def run(C, kind, shape, flop, fn, ref_fn, acc_fn=None):
    """times fn; checks acc_fn (default fn) against ref_fn"""
    row = {'kernel': kind, 'shape': shape}
    ref = ref_fn()
    acc_fn = acc_fn or fn
    for mode, tag in ((0, 'exact'), (1, 'split'), (2, 'regsplit')):
        C.set_f32_mfma_mode(mode)
        us = timed(fn)
        out = acc_fn()
        row[tag + '_us'] = round(us, 1)
        row[tag + '_tflops'] = round(flop / us / 1e6, 1)
        row[tag + '_err_max'], row[tag + '_err_fro'] = err(out, ref)
    row['speedup'] = round(row['exact_us'] / row['split_us'], 3)
    print(json.dumps(row), flush=True)


def main():
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    torch.manual_seed(0)
    if which in ('gemm', 'all'):
        for M, N, K in GEMM:
            a = torch.randn(M, K, device='cuda')
            b = torch.randn(N, K, device='cuda')
            bias = torch.randn(N, device='cuda')
            rows = slice(0, 4096)
            run(C, 'gemm_f32', [M, N, K], 2.0 * M * N * K, lambda: C.gemm_f32(a, b, bias, None, 0)[rows],
                lambda: a[rows].double() @ b.double().t() + bias.double())
    if which in ('conv', 'all'):
        for B, H, W, cin, cout in CONV:
            x = torch.randn(B, H, W, cin, device='cuda')
            w = torch.randn(cout, 3, 3, cin, device='cuda') / 30
            bias = torch.randn(cout, device='cuda')
            xs = x[:4].contiguous()     # accuracy on 4 images (float64 reference on the CPU)
            ref = lambda: torch.nn.functional.conv2d(xs.cpu().double().permute(0, 3, 1, 2),
                                                     w.cpu().double().permute(0, 3, 1, 2), bias.cpu().double(),
                                                     padding=1).permute(0, 2, 3, 1).cuda()
            run(C, 'conv3x3_f32', [B, H, W, cin, cout], 2.0 * B * H * W * cout * 9 * cin,
                lambda: C.conv3x3_f32(x, w, bias, None, 0), ref, lambda: C.conv3x3_f32(xs, w, bias, None, 0))
    if which in ('wgrad', 'all'):
        for M, N, K in GEMM:
            x = torch.randn(M, K, device='cuda')
            dy = torch.randn(M, N, device='cuda')
            run(C, 'wgrad_f32_dense', [M, N, K], 2.0 * M * N * K, lambda: C.wgrad_f32(dy, x, 0, False)[0],
                lambda: dy.double().t() @ x.double())
        for B, H, W, cin, cout in CONV:
            x = torch.randn(B, H, W, cin, device='cuda')
            dy = torch.randn(B * H * W, cout, device='cuda')
            xs, dys = x[:4].contiguous(), dy[:4 * H * W].contiguous()

            def ref():
                xd = xs.cpu().double().permute(0, 3, 1, 2)
                dyd = dys.cpu().double().view(4, H, W, cout).permute(0, 3, 1, 2)
                g = torch.nn.grad.conv2d_weight(xd, (cout, cin, 3, 3), dyd, padding=1)
                return g.permute(0, 2, 3, 1).reshape(cout, -1).cuda()
            run(C, 'wgrad_f32_conv', [B, H, W, cin, cout], 2.0 * B * H * W * cout * 9 * cin,
                lambda: C.wgrad_f32(dy, x, cin, False)[0], ref, lambda: C.wgrad_f32(dys, xs, cin, False)[0])

if __name__ == '__main__':
    main()
