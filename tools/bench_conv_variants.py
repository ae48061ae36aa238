"""A/B of the fp32 split-MFMA conv3x3 tile variants (``set_f32_conv_variant``: 0 = 128-pixel tiles on 4 waves,
1 = 256-pixel tiles on 8 waves / 4-stage ring, 2 = the same with the LDS-staged epilogue) on the learner's
128-channel shapes, interleaved rounds in one process; median / min us, TF/s and error against float64 on 4 images.

    python tools/bench_conv_variants.py [variants=0,1,2] [rounds=5]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gemm_variants import timed  # noqa: E402

SHAPES = [(390, 19, 20, 128, 128), (390, 38, 40, 64, 128), (384, 19, 20, 128, 128)]


def main():
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '0,1,2').split(',')]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    torch.manual_seed(0)
    for B, H, W, cin, cout in SHAPES:
        x = torch.randn(B, H, W, cin, device='cuda')
        w = torch.randn(cout, 3, 3, cin, device='cuda') / 30
        bias = torch.randn(cout, device='cuda')
        res = torch.randn(B, H, W, cout, device='cuda')
        ref = torch.nn.functional.conv2d(x[:4].cpu().double().permute(0, 3, 1, 2), w.cpu().double().permute(0, 3, 1, 2),
                                         bias.cpu().double(), padding=1).permute(0, 2, 3, 1) + res[:4].cpu().double()
        flop = 2.0 * B * H * W * cout * 9 * cin
        times = {v: [] for v in variants}
        errs = {}
        for r in range(rounds):
            for v in variants:
                C.set_f32_conv_variant(v)
                times[v].append(timed(lambda: C.conv3x3_f32(x, w, bias, res, 0)))
                if r == 0:
                    out = C.conv3x3_f32(x, w, bias, res, 0)[:4].cpu().double()
                    d = (out - ref).abs()
                    errs[v] = (float(d.max() / ref.abs().max()), float(d.norm() / ref.norm()))
        for v in variants:
            t = sorted(times[v])
            print(json.dumps({'shape': [B, H, W, cin, cout], 'variant': v, 'us_med': round(t[len(t) // 2], 1),
                              'us_min': round(t[0], 1), 'tflops': round(flop / t[len(t) // 2] / 1e6, 1),
                              'err_max': errs[v][0], 'err_fro': errs[v][1]}), flush=True)
    C.set_f32_conv_variant(0)


if __name__ == '__main__':
    main()
