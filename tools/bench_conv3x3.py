"""Microbenchmark of the native 3x3 conv forward on the learner's shapes: halo-window kernel vs the
per-tap implicit GEMM (the same binary; APPLESTAR_CONV_HALO is read once per process, so the script
runs itself once per variant).  r2z also measured a whole-window variant with the weight fragments
loaded straight from L2 into registers and no loop barriers: 30-100 % SLOWER than the halo kernel
(profiles/r2z_conv3x3_variants_microbench.jsonl), so it was dropped.  Prints one JSON line per shape with
us / call and TFLOP/s.

    python tools/bench_conv_halo.py
"""
import json
import os
import subprocess
import sys

SHAPES = [(390, 19, 20, 128, 128), (384, 19, 20, 128, 128), (390, 38, 40, 64, 128), (384, 38, 40, 128, 64),
          (384, 76, 80, 64, 32)]


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    for B, H, W, cin, cout in SHAPES:
        x = torch.randn(B, H, W, cin, device='cuda').to(torch.bfloat16)
        w = (torch.randn(cout, 3, 3, cin, device='cuda') / 30).to(torch.bfloat16)
        b = torch.randn(cout, device='cuda')
        for _ in range(3):
            C.conv3x3_fwd(x, w, b, None, 1)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        s.record()
        for _ in range(n):
            y = C.conv3x3_fwd(x, w, b, None, 1)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / n * 1e3
        flop = 2.0 * B * H * W * cout * 9 * cin
        print(json.dumps({'variant': os.environ.get('VARIANT', 'win'), 'shape': [B, H, W, cin, cout],
                          'us': round(us, 1), 'tflops': round(flop / us / 1e6, 1),
                          'checksum': float(y.float().abs().mean())}), flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        run()
    else:
        for name, halo in (('implicit', '0'), ('halo', '1')):
            env = dict(os.environ, APPLESTAR_CONV_HALO=halo, VARIANT=name)
            subprocess.run([sys.executable, __file__, 'child'], env=env, check=True)
