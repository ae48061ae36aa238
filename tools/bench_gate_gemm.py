"""GatedResBlock gate-chain GEMM shape ([145920 x 128] x [128 x 128], bias + ReLU) under the library's
layout choices; prints us per call.  (r2cs: the addmm form took ~48 us per call inside the step.)"""
import json
import torch
import torch.nn.functional as F


def timeit(fn, n=30):
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


x = torch.randn(145920, 128, device='cuda').bfloat16()
w = (torch.randn(128, 128, device='cuda') / 11).bfloat16()
b = torch.randn(128, device='cuda').bfloat16()
wt = w.t().contiguous()
cases = {
    'addmm_act_NT': lambda: torch._addmm_activation(b, x, w.t()),
    'addmm_act_NN': lambda: torch._addmm_activation(b, x, wt),
    'linear_NT': lambda: F.linear(x, w, b),
    'mm_NN': lambda: torch.mm(x, wt),
    'mm_NT': lambda: torch.mm(x, w.t()),
    'bmm_4chunks_NT': lambda: torch.baddbmm(b.view(1, 1, 128), x.view(4, -1, 128), w.t().expand(4, 128, 128)),
    'copy_only': lambda: x.clone(),
}
for k, f in cases.items():
    print(json.dumps({'case': k, 'us': round(timeit(f), 1)}), flush=True)
