"""Packed post-LN transformer layer on the GPU vs a float64 CPU reference: native bf16 path, torch bf16
autocast path (native off) and fp32 (diagnostic for tests/test_resid_link_gpu.py)."""
import torch
from applestar_amd import ops
from applestar_amd.models.transformer import TransformerLayer
from applestar_amd.ops import native

native.ensure_loaded()
dev = torch.device('cuda', 0)
torch.manual_seed(0)
lens = [1, 37, 200, 511, 64, 300]
cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device=dev)
T = int(cu[-1])
layer = TransformerLayer(256, 128, 1024, 2, 2, 'post').to(dev)
x0 = torch.randn(T, 256, device=dev).to(torch.bfloat16)
dy = torch.randn(T, 256, device=dev)
ref = TransformerLayer(256, 128, 1024, 2, 2, 'post').double()
ref.load_state_dict({k: v.double().cpu() for k, v in layer.state_dict().items()})
xr = x0.double().cpu().requires_grad_(True)
cuc = cu.cpu()
yr = ref.forward_packed(xr, cuc, max(lens), act='relu')
yr.backward(dy.double().cpu())


def run(name, native_on, autocast, xdtype):
    ops.set_native(native_on)
    x = x0.to(xdtype).clone().requires_grad_(True)
    layer.zero_grad(set_to_none=True)
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        y = layer.forward_packed(x, cu, max(lens), act='relu')
    y.float().backward(dy)
    torch.cuda.synchronize()
    ey = (y.double().cpu() - yr).abs().max().item()
    eg = (x.grad.double().cpu() - xr.grad).abs().max().item()
    gw = {n: ((p.grad.double().cpu() - dict(ref.named_parameters())[n].grad).abs().max().item(),
              dict(ref.named_parameters())[n].grad.abs().max().item()) for n, p in layer.named_parameters()}
    worst = max(gw.items(), key=lambda kv: kv[1][0] / (kv[1][1] + 1e-9))
    print(f'{name:28s} y err {ey:.4f}  dx err {eg:.4f} (max {xr.grad.abs().max().item():.3f})  worst dW {worst[0]} '
          f'{worst[1][0]:.4f} of {worst[1][1]:.4f}', flush=True)
    ops.set_native(True)


run('native bf16 autocast', True, True, torch.bfloat16)
run('torch bf16 autocast', False, True, torch.bfloat16)
run('torch fp32', False, False, torch.float32)
run('native fp32 (no autocast)', True, False, torch.float32)
