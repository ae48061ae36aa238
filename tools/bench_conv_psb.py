"""The fp32 split-MFMA 3x3 conv on the ResBlock shape (19 x 20 x 128 -> 128, 390 observations): time per call,
TF/s of fp32 products and max error against float64 (a row subsample), per kernel variant.

    python tools/bench_conv_psb.py [iters] [variants...]      # variants: psb (shipped), v2 ... (experimental)

Under ``rocprofv3 --pmc`` run with ITERS small: every launch is a dispatch in the counter table.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    names = sys.argv[2:] or ['psb']
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(0)
    shapes = [(390, 19, 20, 128, 128), (384, 19, 20, 128, 128)]
    if os.environ.get('CONV_SHAPES'):          # e.g. "384,38,40,128,64;384,76,80,64,32"
        shapes = [tuple(int(v) for v in t.split(',')) for t in os.environ['CONV_SHAPES'].split(';')]
    for B, H, W, Ci, Co in shapes:
        x = torch.randn(B, H, W, Ci, device='cuda').relu()
        w = torch.randn(Co, 3, 3, Ci, device='cuda') / (9 * Ci) ** 0.5
        bias = torch.randn(Co, device='cuda')
        ws = C.presplit_b(w.reshape(Co, -1).contiguous(), False, None)
        xs = x[:4].double().cpu().permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xs, w.double().cpu().permute(0, 3, 1, 2), bias.double().cpu(),
                                         padding=1).permute(0, 2, 3, 1)
        flop = 2.0 * B * H * W * Ci * Co * 9
        for name in names:
            if name == 'psb':
                fn = lambda: C.conv3x3_f32_psb(x, ws, Co, bias, None, None, None, 1)   # noqa: E731
            else:
                v = int(name[1:]) if name[1:].isdigit() else 0
                fn = lambda v=v: C.conv3x3_f32_v2(x, ws, Co, bias, None, None, None, 1, v)      # noqa: E731
            out = fn()
            err = float((out[:4].double().cpu() - ref.relu()).abs().max() / ref.abs().max())
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
            print(json.dumps({'shape': [B, H, W, Ci, Co], 'kernel': name, 'us_med': round(us, 1),
                              'us_min': round(ts[0], 1), 'tflops': round(flop / us / 1e6, 1), 'err_max_rel': err}),
                  flush=True)


if __name__ == '__main__':
    main()
