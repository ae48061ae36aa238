"""Microbenchmark of the packed varlen attention kernels on the learner's shape: 390 observations with
entity counts U[1, 512) (LENS=max: 130 x 511), 2 heads x 128.  One JSON line with fwd / bwd us and the
achieved TFLOP/s.

    python tools/bench_attention.py
"""
import json
import os
import subprocess
import sys

import torch


def run():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    g = torch.Generator().manual_seed(0)
    dist = os.environ.get('LENS', 'uniform')
    lens = torch.randint(1, 512, (390,), generator=g) if dist == 'uniform' else torch.full((130,), 511)
    H, Dh = 2, 128
    T = int(lens.sum())
    cu = torch.cat([torch.zeros(1, dtype=torch.int64), lens.cumsum(0)]).to(torch.int32).cuda()
    prec = os.environ.get('PREC', 'bf16')          # bf16: attention.hip, fp32: attention_f32.hip
    qkv = torch.randn(T, 3 * H * Dh, device='cuda') * 0.5
    if prec == 'bf16':
        qkv = qkv.to(torch.bfloat16)
    fwd = C.varlen_attn_fwd if prec == 'bf16' else C.varlen_attn_fwd_f32
    bwd = C.varlen_attn_bwd if prec == 'bf16' else C.varlen_attn_bwd_f32
    mx = int(lens.max())
    out, lse = fwd(qkv, cu, mx, H)
    dout = torch.randn_like(out)

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

    f = timed(lambda: fwd(qkv, cu, mx, H))
    b = timed(lambda: bwd(qkv, out, dout, lse, cu, mx, H))
    flop = float((lens.double() ** 2).sum()) * H * Dh * 4        # QK^T + PV
    print(json.dumps({'prec': prec, 'lens': dist, 'fwd_us': round(f, 1),
                      'bwd_us': round(b, 1), 'fwd_tflops': round(flop / f / 1e6, 1),
                      'bwd_tflops': round(2.5 * flop / b / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        run()
    else:
        subprocess.run([sys.executable, __file__, 'child'], check=True)
