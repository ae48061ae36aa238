"""Microbenchmarks of the fp32 learner step's f32-MFMA kernels on the learner's shapes: conv3x3_f32 (forward /
dX), wgrad_f32 (conv + dense dW), gemm_f32, against the exact-f32 MFMA peak (157.3 TFLOP/s, MI355X).  One JSON
line per (kernel, shape) with us / call and TFLOP/s.  Also the child process of PMC passes (tools/gpu_pmc.sh).

    python tools/bench_f32_kernels.py [conv|narrow|wgrad|gemm|small|smallnative|bf16|attn|gate|all]
"""
import json
import os
import sys

import torch

CONV = [(390, 19, 20, 128, 128), (390, 38, 40, 64, 128), (384, 38, 40, 128, 64), (384, 76, 80, 64, 32),
        (390, 76, 80, 16, 16), (390, 19, 20, 32, 32)]
GEMM = [(100000, 768, 256), (100000, 256, 256), (100000, 1024, 256), (100000, 256, 1024), (24576, 1536, 384)]


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def emit(kind, shape, us, flop):
    print(json.dumps({'kernel': kind, 'shape': shape, 'us': round(us, 1), 'tflops': round(flop / us / 1e6, 1),
                      'pct_f32_peak': round(100 * flop / us / 1e6 / 157.3, 1)}), flush=True)


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    if which in ('narrow', 'all'):
        # the value encoder's narrow convs: direct split-MFMA kernel vs the ring kernel (APPLESTAR_CONV_F32_NARROW)
        for B, H, W, cin, cout in [(390, 76, 80, 16, 16), (390, 38, 40, 16, 32), (390, 38, 40, 32, 16),
                                   (390, 19, 20, 32, 32)]:
            x = torch.randn(B, H, W, cin, device='cuda')
            w = torch.randn(cout, 3, 3, cin, device='cuda') / 30
            b = torch.randn(cout, device='cuda')
            flop = 2.0 * B * H * W * cout * 9 * cin
            emit('conv3x3_f32', [B, H, W, cin, cout], timed(lambda: C.conv3x3_f32(x, w, b, None, 1)), flop)
    if which in ('conv', 'all'):
        for B, H, W, cin, cout in CONV:
            x = torch.randn(B, H, W, cin, device='cuda')
            w = torch.randn(cout, 3, 3, cin, device='cuda') / 30
            b = torch.randn(cout, device='cuda')
            flop = 2.0 * B * H * W * cout * 9 * cin
            emit('conv3x3_f32', [B, H, W, cin, cout], timed(lambda: C.conv3x3_f32(x, w, b, None, 1)), flop)
    if which in ('wgrad', 'all'):
        for B, H, W, cin, cout in CONV:
            x = torch.randn(B, H, W, cin, device='cuda')
            dy = torch.randn(B * H * W, cout, device='cuda')
            flop = 2.0 * B * H * W * cout * 9 * cin
            emit('wgrad_f32_conv', [B, H, W, cin, cout], timed(lambda: C.wgrad_f32(dy, x, cin, True)), flop)
        for M, N, K in GEMM:
            x = torch.randn(M, K, device='cuda')
            dy = torch.randn(M, N, device='cuda')
            emit('wgrad_f32_dense', [M, N, K], timed(lambda: C.wgrad_f32(dy, x, 0, True)), 2.0 * M * N * K)
    if which == 'tail':
        # wave quantization probe: 768 resident 128x128 tiles (3 per CU); time should step at whole rounds
        for M in (49000, 50000, 98000, 99000, 100000, 147000, 148000):
            a = torch.randn(M, 256, device='cuda')
            b = torch.randn(256, 256, device='cuda')
            emit('gemm_f32_tail', [M, 256, 256, (M + 127) // 128 * 2], timed(lambda: C.gemm_f32(a, b, None, None, 0)),
                 2.0 * M * 256 * 256)
        for B in (130, 200, 259, 260, 390):
            x = torch.randn(B, 19, 20, 128, device='cuda')
            w = torch.randn(128, 3, 3, 128, device='cuda') / 30
            emit('conv3x3_f32_tail', [B, 19, 20, 128, 128, (B * 380 + 127) // 128],
                 timed(lambda: C.conv3x3_f32(x, w, None, None, 0)), 2.0 * B * 380 * 128 * 9 * 128)
    if which in ('small', 'all'):
        # few-row products of the fp32 step (heads / scalar encoder / value projections): native small-tile
        # kernel vs the library
        for M, N, K in [(384, 256, 384), (384, 1024, 448), (390, 256, 256), (384, 256, 1024), (390, 1024, 64),
                        (384, 128, 256), (390, 64, 320)]:
            a = torch.randn(M, K, device='cuda')
            b = torch.randn(N, K, device='cuda')
            bias = torch.randn(N, device='cuda')
            emit('gemm_f32_small', [M, N, K], timed(lambda: C.gemm_f32(a, b, bias, None, 1), 50), 2.0 * M * N * K)
            emit('torch_fp32_addmm_relu', [M, N, K],
                 timed(lambda: torch._addmm_activation(bias, a, b.t(), use_gelu=False), 50), 2.0 * M * N * K)
    if which in ('smallnative', 'all'):
        # the any-shape few-row kernels (gemm_small.hip) on the step's shapes vs the library
        for R, N, K in [(390, 64, 10), (390, 128, 167), (384, 256, 448), (390, 64, 269), (390, 1, 256),
                        (384, 327, 256), (390, 32, 90)]:
            for dt in (torch.float32, torch.bfloat16):
                x = torch.randn(R, K, device='cuda').to(dt)
                w = torch.randn(N, K, device='cuda').to(dt)
                dy = torch.randn(R, N, device='cuda').to(dt)
                y = torch.randn(R, N, device='cuda').to(dt)
                bias = torch.randn(N, device='cuda')
                tag = 'f32' if dt == torch.float32 else 'bf16'
                emit(f'small_nt_{tag}', [R, N, K], timed(lambda: C.small_gemm(x, w, bias, None, None, 0, 1), 50),
                     2.0 * R * N * K)
                emit(f'small_tn_{tag}', [R, N, K], timed(lambda: C.small_wgrad(dy, x, y, 1, True, dt == torch.bfloat16), 50),
                     2.0 * R * N * K)
                emit(f'torch_dw_{tag}', [R, N, K], timed(lambda: dy.t() @ x, 50), 2.0 * R * N * K)
    if which in ('bf16', 'all'):
        # the bf16 step's large products (tools/gemm_census.py): native LDS-DMA ring kernel vs hipBLASLt
        for M, N, K in [(99526, 768, 256), (99526, 256, 256), (99526, 1024, 256), (99526, 256, 1024),
                        (99526, 256, 768), (199290, 64, 256), (24576, 1024, 256), (145920, 128, 128),
                        (390, 12160, 128), (199290, 256, 64)]:
            a = torch.randn(M, K, device='cuda').bfloat16()
            b = (torch.randn(N, K, device='cuda') / K ** 0.5).bfloat16()
            bias = torch.randn(N, device='cuda')
            bb = bias.bfloat16()
            emit('gemm_bf16', [M, N, K], timed(lambda: C.gemm_bf16(a, b, bias, None, 1), 20), 2.0 * M * N * K)
            emit('torch_bf16_addmm_relu', [M, N, K],
                 timed(lambda: torch._addmm_activation(bb, a, b.t(), use_gelu=False), 20), 2.0 * M * N * K)
    if which in ('attn', 'all'):
        # the entity transformer's fp32 attention at the learner's shape (384 observations, 2 heads x 128, lengths
        # up to 512, mean ~260): forward and backward per split-path variant (attention_f32.hip)
        g = torch.Generator().manual_seed(0)
        lens = torch.randint(1, 513, (384,), generator=g)
        cu = torch.zeros(385, dtype=torch.int32)
        cu[1:] = lens.cumsum(0)
        cu = cu.cuda()
        T, H = int(lens.sum()), 2
        qkv = torch.randn(T, 3 * H * 128, device='cuda')
        flop_f = 4.0 * H * 128 * float((lens.double() ** 2).sum())
        ref = None
        for v in (0, 1, 7, 17, 23):
            old = C.attn_f32_variant(v)
            out, lse = C.varlen_attn_fwd_f32(qkv, cu, 512, H)
            dout = torch.randn(out.shape, device='cuda') if ref is None else ref[2]
            dq = C.varlen_attn_bwd_f32(qkv, out, dout, lse, cu, 512, H)
            if ref is None:
                ref = (out, dq, dout)
            err_f = float((out - ref[0]).abs().max())
            err_b = float((dq - ref[1]).abs().max() / ref[1].abs().max())
            emit(f'attn_f32_fwd_v{v}', [T, H, err_f], timed(lambda: C.varlen_attn_fwd_f32(qkv, cu, 512, H)), flop_f)
            emit(f'attn_f32_bwd_v{v}', [T, H, err_b],
                 timed(lambda: C.varlen_attn_bwd_f32(qkv, out, dout, lse, cu, 512, H)), 2.5 * flop_f)
            C.attn_f32_variant(old)
    if which in ('gate', 'all'):
        # the location head's gate chain (four 128 x 128 layers over 145,920 pixels): one launch vs four GEMMs
        P = 145920
        x = torch.randn(P, 128, device='cuda')
        ms = [torch.randn(128, 128, device='cuda') / 11 for _ in range(4)]
        bs = [torch.randn(128, device='cuda') for _ in range(4)]
        flop = 4 * 2.0 * P * 128 * 128

        def four():
            h = x
            for i in range(4):
                h = C.gemm_f32(h, ms[i], bs[i], None, 1 if i < 3 else 0)
            return h
        emit('gate_chain_f32', [P, 128, 4], timed(lambda: C.gate_chain_f32(x, ms, bs, [None] * 4, [None] * 4, 7)), flop)
        emit('gemm_f32_x4', [P, 128, 4], timed(four), flop)
        d = torch.randn(P, 128, device='cuda')
        acts = C.gate_chain_f32(x, ms, bs, [None] * 4, [None] * 4, 7)
        emit('gate_chain_f32_bwd', [P, 128, 4],
             timed(lambda: C.gate_chain_f32(d, [m.t().contiguous() for m in ms[::-1]], [None] * 4,
                                            [acts[2], acts[1], acts[0], None], [None, None, None, x], 0)), flop)
    if which in ('gemm', 'all'):
        for M, N, K in GEMM:
            a = torch.randn(M, K, device='cuda')
            b = torch.randn(N, K, device='cuda')
            bias = torch.randn(N, device='cuda')
            emit('gemm_f32', [M, N, K], timed(lambda: C.gemm_f32(a, b, bias, None, 1)), 2.0 * M * N * K)
            emit('torch_fp32_linear', [M, N, K], timed(lambda: torch.nn.functional.linear(a, b, bias)), 2.0 * M * N * K)


if __name__ == '__main__':
    main()
