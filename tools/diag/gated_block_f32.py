"""fp32 GatedResBlock gradients vs float64 at a size where the gate layers take the f32 GEMM: per parameter the
fraction of entries off by > 3e-5 of the max and the relative Frobenius error, for (split | exact MFMA) x (gate layers
on gemm_f32 | on the library GEMM)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from applestar_amd.models.blocks import GatedResBlock  # noqa: E402
from applestar_amd.ops import native as N  # noqa: E402


def main():
    C = N.ensure_loaded()
    torch.manual_seed(8)
    blk0 = GatedResBlock(128)
    ref = copy.deepcopy(blk0).double()
    x = torch.randn(12, 128, 38, 40)
    xr = x.double().requires_grad_()
    g = torch.randn(12, 128, 38, 40, dtype=torch.float64)
    ref(xr).backward(g)
    ok = N._gemm_f32_ok
    for mode in (1, 0):
        for lib in (False, True):
            C.set_f32_mfma_mode(mode)
            N._gemm_f32_ok = (lambda *a: False) if lib else ok
            blk = copy.deepcopy(blk0).cuda().to(memory_format=torch.channels_last)
            xg = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_()
            blk(xg).backward(g.float().cuda().contiguous(memory_format=torch.channels_last))
            rows = [('dx', xg.grad, xr.grad)] + [(n, p.grad, pr.grad) for (n, p), (_, pr) in
                                                 zip(blk.named_parameters(), ref.named_parameters())]
            for n, a, r in rows:
                d = (a.detach().cpu().double() - r).abs()
                b = 3e-5 * max(1.0, r.abs().max().item())
                print(f'mode={mode} lib={int(lib)} {n:28s} frac {(d > b).double().mean().item():.2e} '
                      f'fro {(d.norm() / r.norm()).item():.2e}', flush=True)
    N._gemm_f32_ok = ok


if __name__ == '__main__':
    main()
