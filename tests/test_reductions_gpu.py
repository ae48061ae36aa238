"""Column-sum kernels used in backward passes, against fp32/fp64 torch references."""
import pytest
import torch

from applestar_amd.ops import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('shape', [(65, 6, 1536), (65, 6, 384), (390, 7), (24576, 128), (3, 1, 100)])
def test_ln_affine_grads_matches_torch(shape):
    C = native.ensure_loaded()
    g = torch.Generator(device='cuda').manual_seed(1)
    dy = torch.randn(shape, device='cuda', generator=g)
    xh = torch.randn(shape, device='cuda', generator=g)
    out = C.ln_affine_grads(dy, xh)
    torch.cuda.synchronize()
    red = tuple(range(len(shape) - 1))
    ref_w = (dy.double() * xh.double()).sum(red)
    ref_b = dy.double().sum(red)
    rows = dy.numel() // shape[-1]
    tol = 1e-5 * rows ** 0.5 + 1e-5
    assert out.shape == (2, shape[-1])
    assert (out[0].double() - ref_w).abs().max().item() < tol
    assert (out[1].double() - ref_b).abs().max().item() < tol


@pytest.mark.parametrize('R,K,N,act', [(390, 10, 64, 'relu'), (390, 269, 64, 'relu'), (384, 256, 2, None),
                                       (60, 64, 64, 'relu'), (390, 256, 1, None)])
def test_small_linear_matches_fp32(R, K, N, act):
    """native.linear's few-row / odd-width path (_SmallLinear) vs an fp32 torch linear: output and the
    x / W / b gradients (bias gradient from the ones-row GEMV)."""
    native.ensure_loaded()
    g = torch.Generator(device='cuda').manual_seed(2)
    x = torch.randn(R, K, device='cuda', generator=g)
    w = (0.1 * torch.randn(N, K, device='cuda', generator=g)).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(N, device='cuda', generator=g)).to(torch.bfloat16).requires_grad_()
    xg = x.to(torch.bfloat16).requires_grad_()
    dy = torch.randn(R, N, device='cuda', generator=g)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = native.linear(xg, w, b, act)
    assert 'SmallLinear' in type(y.grad_fn.next_functions[0][0]).__name__      # (the output is a view)
    y.float().backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (xg, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    if act == 'relu':
        yr = torch.relu(yr)
    yr.backward(dy)
    for got, ref in ((y, yr), (xg.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        scale = ref.abs().max().item()
        assert (got.float() - ref).abs().max().item() <= 2e-2 * max(1.0, scale), (got.shape, scale)
