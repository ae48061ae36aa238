"""Library GEMM shapes from the learner step that hipBLASLt runs far below its rate (r2ax gemm profile),
timed against reformulations: split-K batched GEMM for the K = 48640 spatial fc, transposed-operand
forms of the dX products.  Prints one JSON line per (case, variant) with us per call.

    python tools/bench_gemm_alts.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / n


def rep(case, variant, us, ref=None, out=None):
    d = {'case': case, 'variant': variant, 'us': round(us, 1)}
    if ref is not None and out is not None:
        d['max_rel_err'] = float((out.float() - ref.float()).abs().max() / ref.float().abs().max().clamp(min=1e-6))
    print(json.dumps(d), flush=True)


def main():
    dev = 'cuda'
    bf = torch.bfloat16
    torch.manual_seed(0)
    # 1. spatial fc forward: relu(x W^T + b), x [390, 48640], W [256, 48640]
    x = torch.randn(390, 48640, device=dev).to(bf)
    w = (torch.randn(256, 48640, device=dev) / 200).to(bf)
    b = torch.randn(256, device=dev).to(bf)
    ref = torch._addmm_activation(b, x, w.t())
    rep('fc48640_fwd', 'addmm_relu', timeit(lambda: torch._addmm_activation(b, x, w.t())))
    for S in (16, 32, 64, 128):
        kc = 48640 // S

        def f(S=S, kc=kc):
            p = torch.bmm(x.view(390, S, kc).transpose(0, 1), w.view(256, S, kc).permute(1, 2, 0))
            return torch.relu(p.sum(0, dtype=torch.float32) + b.float()).to(bf)
        rep('fc48640_fwd', f'splitk_bmm_S{S}', timeit(f), ref, f())
    # 2. dX of the value spatial fc: dy [390, 128] @ W [128, 12160]
    dy = torch.randn(390, 128, device=dev).to(bf)
    w2 = (torch.randn(128, 12160, device=dev) / 30).to(bf)
    ref2 = torch.mm(dy, w2)
    rep('dx12160', 'mm', timeit(lambda: torch.mm(dy, w2)))
    w2t = w2.t().contiguous()
    rep('dx12160', 'linear_pretransposed', timeit(lambda: F.linear(dy, w2t)), ref2, F.linear(dy, w2t))
    rep('dx12160', 'mm_t_then_copy', timeit(lambda: torch.mm(w2t, dy.t()).t().contiguous()), ref2,
        torch.mm(w2t, dy.t()).t().contiguous())
    # 3. dX of the transformer FFN2: dy [99526, 256] @ W2 [256, 1024]
    dy3 = torch.randn(99526, 256, device=dev).to(bf)
    w3 = (torch.randn(256, 1024, device=dev) / 30).to(bf)
    ref3 = torch.mm(dy3, w3)
    rep('dx_ffn2', 'mm', timeit(lambda: torch.mm(dy3, w3)))
    w3t = w3.t().contiguous()
    rep('dx_ffn2', 'linear_pretransposed', timeit(lambda: F.linear(dy3, w3t)), ref3, F.linear(dy3, w3t))
    rep('ffn1_fwd', 'addmm_relu', timeit(lambda: torch._addmm_activation(b.new_zeros(1024), dy3, w3t.t())))
    # 4. small dW with K = 260: dy^T [64, 390] @ x [390, 260]
    dy4 = torch.randn(390, 64, device=dev).to(bf)
    x4 = torch.randn(390, 260, device=dev).to(bf)
    ref4 = dy4.float().t() @ x4.float()
    rep('dw_k260', 'mm_bf16', timeit(lambda: torch.mm(dy4.t(), x4)), ref4, torch.mm(dy4.t(), x4))
    rep('dw_k260', 'mm_fp32', timeit(lambda: torch.mm(dy4.t().float(), x4.float())), ref4,
        torch.mm(dy4.t().float(), x4.float()))
    x4p = F.pad(x4, (0, 4))
    rep('dw_k260', 'mm_bf16_padded264', timeit(lambda: torch.mm(dy4.t(), x4p)[:, :260]), ref4, torch.mm(dy4.t(), x4p)[:, :260])
    # 5. wgrad through the library: [128, 24576] @ [24576, 32]
    a5 = torch.randn(24576, 128, device=dev).to(bf)
    b5 = torch.randn(24576, 32, device=dev).to(bf)
    rep('dw_24576', 'mm', timeit(lambda: torch.mm(a5.t(), b5)))
    rep('dw_24576', 'splitk_bmm_S32', timeit(lambda: torch.bmm(a5.view(32, 768, 128).transpose(1, 2),
                                                               b5.view(32, 768, 32)).sum(0)))


if __name__ == '__main__':
    main()
