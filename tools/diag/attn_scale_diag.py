"""Varlen attention backward vs an fp32 torch reference as the score scale grows (diagnostic)."""
import torch
from applestar_amd.ops import native as N, reference as R
N.ensure_loaded()

DEV = torch.device('cuda', 0)
lens = [1, 37, 200, 511, 64, 300]
H, Dh = 2, 128
T = sum(lens)
cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
for scale in (0.5, 1.0, 2.0, 4.0):
    torch.manual_seed(7)
    base = torch.randn(T, 3 * H * Dh, device=DEV) * scale
    qkv = base.to(torch.bfloat16).requires_grad_()
    ref_in = qkv.detach().float().requires_grad_()
    out = N.varlen_attention(qkv, cu, max(lens), H, Dh)
    ref = R.varlen_attention(ref_in, cu, max(lens), H, Dh)
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    d = (qkv.grad.float() - ref_in.grad).abs()
    parts = [d[:, i * H * Dh:(i + 1) * H * Dh].max().item() for i in range(3)]
    sc = [ref_in.grad[:, i * H * Dh:(i + 1) * H * Dh].abs().max().item() for i in range(3)]
    print(f'scale {scale}: fwd err {(out.float() - ref).abs().max().item():.4f}  '
          f'dq/dk/dv err {parts[0]:.4f}/{parts[1]:.4f}/{parts[2]:.4f}  of max {sc[0]:.3f}/{sc[1]:.3f}/{sc[2]:.3f}',
          flush=True)
