"""Which op puts the fp32 layer's one off row (r3a/r3b layer_grad_diag: native fp32 dx row 138 off by 0.0038
while torch fp32 is exact)?  Runs the post-LN layer in fp32 with native on / off, twice each, and compares
x.grad and every parameter gradient: run-to-run (determinism) and native-vs-torch (per tensor, worst row)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from applestar_amd import ops  # noqa: E402
from applestar_amd.models.transformer import TransformerLayer  # noqa: E402

dev = torch.device('cuda', 0)
torch.manual_seed(0)
lens = [1, 37, 200, 511, 64, 300]
cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device=dev)
base = TransformerLayer(256, 128, 1024, 2, 2, 'post')
x0 = torch.randn(int(cu[-1]), 256).to(torch.bfloat16).float()
dy = torch.randn(int(cu[-1]), 256)


def run(native, hook_qkv=False):
    ops.set_native(native)
    layer = TransformerLayer(256, 128, 1024, 2, 2, 'post').to(dev)
    layer.load_state_dict(base.state_dict())
    x = x0.to(dev).requires_grad_(True)
    inter = {}
    orig_lin, orig_ln = ops.linear, ops.layer_norm

    def lin(xx, w, b=None, act=None, grad_link=None):
        y = orig_lin(xx, w, b, act, grad_link=grad_link)
        if y.requires_grad:
            k = f'linear{len(inter)}[{w.shape[0]}x{w.shape[1]}]'
            inter[k] = y
            y.retain_grad()
        return y
    ops.linear = lin
    try:
        y = layer.forward_packed(x, cu, max(lens), act=None)
        y.backward(dy.to(dev))
    finally:
        ops.linear, ops.layer_norm = orig_lin, orig_ln
        ops.set_native(True)
    torch.cuda.synchronize()
    out = {'x.grad': x.grad.detach().cpu(), 'y': y.detach().cpu()}
    for n, p in layer.named_parameters():
        out[n + '.grad'] = p.grad.detach().cpu()
    for k, t in inter.items():
        out[k] = t.detach().cpu()
        out[k + '.grad'] = t.grad.detach().cpu()
    return out


def cmp(a, b, label):
    print(label)
    for k in a:
        d = (a[k] - b[k]).abs()
        if d.max() == 0:
            continue
        row = int(d.reshape(d.shape[0], -1).max(1).values.argmax()) if d.dim() > 1 else int(d.argmax())
        print(f'  {k:40s} max {float(d.max()):.3e} (of {float(b[k].abs().max()):.3e}) worst row {row}')


n1, n2, t1, t2 = run(True), run(True), run(False), run(False)
cmp(n1, n2, 'native fp32 run 1 vs run 2 (determinism)')
cmp(t1, t2, 'torch fp32 run 1 vs run 2 (determinism)')
cmp(n1, t1, 'native fp32 vs torch fp32')
