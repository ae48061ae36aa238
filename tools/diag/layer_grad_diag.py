"""Where does the post-LN entity-transformer layer's input-gradient error come from?  

One random-init layer (module_utils.py:130-139 shape: 256 wide, 2 heads x 128, FFN 1024) on packed
sequences of lengths ``lens``, run four ways against a float64 CPU reference of the same weights:
native bf16 autocast, torch bf16 autocast (native off), native fp32 (fp32 weights, no autocast: the fp32
kernels) and torch fp32.  For each, with and without the entity encoder's final ReLU (``act``):

* y / dx max-abs error and RELATIVE FROBENIUS error (the max-abs of one element is what r2 quoted);
* the ReLU decision flips: elements whose pre-activation sign differs from float64's (a flipped element
  passes (or drops) a whole upstream gradient element: an O(|dy|) change of that row's dx, whatever the
  precision of the arithmetic), and the dx error over rows WITHOUT a flip;
* the worst rows.

Run on the GPU box: ``python tools/diag/layer_grad_diag.py > profiles/r3_layer_grad_diag.txt``."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from applestar_amd import ops  # noqa: E402
from applestar_amd.models.transformer import TransformerLayer  # noqa: E402
from applestar_amd.ops import native  # noqa: E402

native.ensure_loaded()
dev = torch.device('cuda', 0)
torch.manual_seed(0)
lens = [1, 37, 200, 511, 64, 300]
cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device=dev)
T = int(cu[-1])
base = TransformerLayer(256, 128, 1024, 2, 2, 'post')
x0 = torch.randn(T, 256).to(torch.bfloat16).float()      # bf16-representable input: same x for every variant
dy = torch.randn(T, 256)


def reference(act):
    ref = TransformerLayer(256, 128, 1024, 2, 2, 'post').double()
    ref.load_state_dict({k: v.double() for k, v in base.state_dict().items()})
    xr = x0.double().requires_grad_(True)
    # the pre-activation of the final ReLU (= the act=None output) for the flip count
    pre = ref.forward_packed(xr, cu.cpu(), max(lens), act=None)
    y = torch.relu(pre) if act == 'relu' else pre
    y.backward(dy.double())
    return y.detach(), xr.grad.detach(), pre.detach()


def run(native_on, bf16, act, ref_op=None):
    """``ref_op``: 'attention' / 'layer_norm' runs that one op on the plain PyTorch path (per-op isolation)."""
    ops.set_native(native_on)
    saved = None
    if ref_op is not None:
        from applestar_amd.ops import reference
        saved = getattr(ops, ref_op if ref_op != 'attention' else 'varlen_attention')
        if ref_op == 'attention':
            ops.varlen_attention = reference.varlen_attention
        else:
            ops.layer_norm = lambda x, w, b, residual=None, act=None, eps=1e-5, grad_link=None: \
                reference.layer_norm(x if residual is None else x.float(),
                                     w, b, None if residual is None else residual.float(), act, eps)
    layer = TransformerLayer(256, 128, 1024, 2, 2, 'post').to(dev)
    layer.load_state_dict(base.state_dict())
    x = x0.to(dev).to(torch.bfloat16 if bf16 else torch.float32).requires_grad_(True)
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
        pre = layer.forward_packed(x, cu, max(lens), act=None)
        y = layer.forward_packed(x, cu, max(lens), act=act) if act else pre
    y.float().backward(dy.to(dev))
    torch.cuda.synchronize()
    ops.set_native(True)
    if ref_op == 'attention':
        ops.varlen_attention = saved
    elif ref_op is not None:
        ops.layer_norm = saved
    return y.detach().double().cpu(), x.grad.double().cpu(), pre.detach().double().cpu()


def report(name, got, ref):
    y, g, pre = got
    yr, gr, prer = ref
    err = (g - gr).abs()
    rel = float((g - gr).norm() / gr.norm())
    yrel = float((y - yr).norm() / yr.norm())
    flips = (pre > 0) != (prer > 0)
    nflip = int(flips.sum())
    rows_flip = flips.any(1)
    clean = err[~rows_flip]
    clean_max = float(clean.max()) if clean.numel() else 0.0
    clean_rel = float((g - gr)[~rows_flip].norm() / gr[~rows_flip].norm()) if clean.numel() else 0.0
    row_err = err.max(1).values
    worst = torch.topk(row_err, 3)
    print(f'  {name:30s} y rel {yrel:.2e}  dx: max {float(err.max()):.4f} (of {float(gr.abs().max()):.3f}), '
          f'rel-Frobenius {rel:.2e} | ReLU flips {nflip:5d} in {int(rows_flip.sum()):4d}/{T} rows | '
          f'rows without a flip: max {clean_max:.4f}, rel {clean_rel:.2e} | worst rows '
          + ', '.join(f'{int(i)}:{float(v):.3f}{"*" if bool(rows_flip[i]) else ""}'
                      for v, i in zip(worst.values, worst.indices)), flush=True)


for act in (None, 'relu'):
    ref = reference(act)
    print(f'act={act}  (T={T}, lens={lens}; * = row with a ReLU flip; flips counted on the final pre-activation)')
    report('native bf16 autocast', run(True, True, act), ref)
    report('torch bf16 autocast', run(False, True, act), ref)
    report('native fp32', run(True, False, act), ref)
    report('native fp32, torch attention', run(True, False, act, 'attention'), ref)
    report('native fp32, torch LN', run(True, False, act, 'layer_norm'), ref)
    report('torch fp32', run(False, False, act), ref)
