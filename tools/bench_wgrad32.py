"""fp32 weight gradients with a <= 32-wide output (N tile 32): time per call and error vs float64 on a row
subsample, for the A/B of the 32-wide LDS-DMA ring kernel (run once with APPLESTAR_WGRAD32_PIPE=0 for the
register-staged kernel, APPLESTAR_WGRAD32_PIPE=1 for the ring; the switch is read once per process).
Round 6: the split-once staging kernel for 32 / 64-wide N tiles is the default (APPLESTAR_WGRAD_STG_NARROW=0: off).

    python tools/bench_wgrad32.py > out.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_f32_kernels import timed  # noqa: E402

# learner shapes whose Cout / N <= 32: location-head 76x80 64->32 and 16->16 convs, the 19x20 32->32 conv, a
# 32-wide dense product and a 16-wide one
CONV = [(384, 76, 80, 64, 32), (390, 76, 80, 16, 16), (390, 19, 20, 32, 32), (384, 152, 160, 32, 16),
        (390, 76, 80, 32, 64), (384, 38, 40, 128, 64), (390, 38, 40, 16, 32)]
DENSE = [(100000, 32, 256), (199680, 16, 64), (100000, 64, 256)]


def err(out, ref):
    d = (out.double().cpu() - ref).abs()
    return float(d.max() / ref.abs().max())


def main():
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    C.set_f32_mfma_mode(1)
    mode = 'ring' if os.environ.get('APPLESTAR_WGRAD32_PIPE', '0') == '1' else 'regstaged'
    if os.environ.get('APPLESTAR_WGRAD_STG_NARROW', '1') != '0':
        mode = 'stg_narrow'
    if os.environ.get('APPLESTAR_WGRAD32_BK', '128') == '256':
        mode += '_bk256'
    torch.manual_seed(0)
    for B, H, W, cin, cout in CONV:
        x = torch.randn(B, H, W, cin, device='cuda')
        dy = torch.randn(B * H * W, cout, device='cuda')
        xs, dys = x[:4].contiguous(), dy[:4 * H * W].contiguous()
        xd = xs.cpu().double().permute(0, 3, 1, 2)
        dyd = dys.cpu().double().view(4, H, W, cout).permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xd, (cout, cin, 3, 3), dyd, padding=1).permute(0, 2, 3, 1).reshape(cout, -1)
        us = timed(lambda: C.wgrad_f32(dy, x, cin, False)[0])
        flop = 2.0 * B * H * W * cout * 9 * cin
        print(json.dumps({'kernel': 'wgrad_f32_conv', 'mode': mode, 'shape': [B, H, W, cin, cout], 'us': round(us, 1),
                          'tflops': round(flop / us / 1e6, 1),
                          'err_max': err(C.wgrad_f32(dys, xs, cin, False)[0], ref)}), flush=True)
    for M, N, K in DENSE:
        x = torch.randn(M, K, device='cuda')
        dy = torch.randn(M, N, device='cuda')
        ref = dy[:8192].cpu().double().t() @ x[:8192].cpu().double()
        us = timed(lambda: C.wgrad_f32(dy, x, 0, False)[0])
        print(json.dumps({'kernel': 'wgrad_f32_dense', 'mode': mode, 'shape': [M, N, K], 'us': round(us, 1),
                          'tflops': round(2.0 * M * N * K / us / 1e6, 1),
                          'err_max': err(C.wgrad_f32(dy[:8192].contiguous(), x[:8192].contiguous(), 0, False)[0],
                                         ref)}), flush=True)


if __name__ == '__main__':
    main()
