"""Microbenchmark: native conv3x3 fwd / split-R wgrad vs MIOpen / hipBLASLt on the model's shapes.

Run on a GPU box: ``python tools/bench_conv.py`` -> one JSON line per (op, shape)."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.ops import native  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    C = native.ensure_loaded()
    dev = 'cuda'
    cl = torch.channels_last
    B = 390
    for (H, W, cin, cout) in [(19, 20, 128, 128), (38, 40, 64, 128), (76, 80, 32, 64), (38, 40, 128, 64),
                              (76, 80, 64, 32), (152, 160, 32, 32)]:
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, 3, 3, cin, device=dev) / 30).to(torch.bfloat16)
        dy = torch.randn(B, H, W, cout, device=dev).to(torch.bfloat16)
        bias = torch.zeros(cout, device=dev)
        flop = 2.0 * B * H * W * cin * cout * 9
        t_nat = timeit(lambda: C.conv3x3_fwd(x, w, bias, None, 1))
        xm = x.permute(0, 3, 1, 2)
        wm = w.permute(0, 3, 1, 2)
        t_mio = timeit(lambda: torch.nn.functional.conv2d(xm, wm, None, 1, 1))
        t_wg = timeit(lambda: C.wgrad(dy.view(-1, cout), x, cin, True))
        dym = dy.permute(0, 3, 1, 2)
        t_wrw = timeit(lambda: torch.ops.aten.convolution_backward(dym, xm, wm, None, [1, 1], [1, 1], [1, 1], False,
                                                                   [0, 0], 1, [False, True, False]))
        print(json.dumps({'op': 'conv3x3', 'shape': [B, H, W, cin, cout], 'fwd_native_us': round(t_nat, 1),
                          'fwd_miopen_us': round(t_mio, 1), 'fwd_native_tflops': round(flop / t_nat / 1e6, 1),
                          'wgrad_native_us': round(t_wg, 1), 'wgrad_miopen_us': round(t_wrw, 1),
                          'wgrad_native_tflops': round(flop / t_wg / 1e6, 1)}), flush=True)
    for (R, N, K) in [(B * 380, 128, 128), (B * 380, 128, 132 // 4 * 4 + 4), (100000, 768, 256), (100000, 256, 1024),
                      (B * 24320, 32, 56), (B, 256, 48640)]:
        if N % 8 or K % 8:
            continue
        dy = torch.randn(R, N, device=dev).to(torch.bfloat16)
        x = torch.randn(R, K, device=dev).to(torch.bfloat16)
        flop = 2.0 * R * N * K
        t_wg = timeit(lambda: C.wgrad(dy, x, 0, True))
        t_lt = timeit(lambda: (dy.t() @ x, dy.sum(0)))
        print(json.dumps({'op': 'linear_wgrad', 'shape': [R, N, K], 'native_us': round(t_wg, 1),
                          'hipblaslt_us': round(t_lt, 1), 'native_tflops': round(flop / t_wg / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()
