"""Extended Adam (utils/optim.py): clip / ignore variants, AdamW, state round trip; parity with the
reference optimizer for the variants whose reference code runs on this torch version."""
import copy
import math

import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.utils.optim import Adam


def _params(seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(5, 4, generator=g)), torch.nn.Parameter(torch.randn(7, generator=g))]
    for p in ps:
        p.grad = torch.randn(p.shape, generator=g) * scale
    return ps


def _ref_adam():
    import_reference()
    from distar.ctools.torch_utils.optimizer_util import Adam as RefAdam
    return RefAdam


@pytest.mark.skipif(not reference_available(), reason='reference tree not available')
@pytest.mark.parametrize('kw', [dict(grad_clip_type='clip_value', clip_value=0.5),
                                dict(grad_clip_type='clip_norm', clip_value=1.0),
                                dict(grad_ignore_type='ignore_value', ignore_value=1.5),
                                dict(grad_ignore_type='ignore_value', ignore_value=50.0),
                                dict(grad_ignore_type='ignore_norm', ignore_value=2.0),
                                dict(grad_ignore_type='ignore_norm', ignore_value=100.0)])
def test_matches_reference_optimizer(kw):
    RefAdam = _ref_adam()
    a, b = _params(1), _params(1)
    ra = RefAdam(a, lr=0.01, betas=(0.0, 0.99), eps=1e-5, **kw)
    ob = Adam(b, lr=0.01, betas=(0.0, 0.99), eps=1e-5, **kw)
    ra.step()
    ob.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x.grad, y.grad)
        torch.testing.assert_close(x.data, y.data)


def test_adamw_matches_torch():
    a, b = _params(2), _params(2)
    ours = Adam(a, lr=0.1, weight_decay=0.3, optim_type='adamw')
    ref = torch.optim.AdamW(b, lr=0.1, weight_decay=0.3)
    for _ in range(3):
        ours.step()
        ref.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x.data, y.data)


def _manual_bound(vs, grads, beta2, step, coef):
    bc2 = 1 - beta2 ** step
    out = []
    for v, g in zip(vs, grads):
        v.mul_(beta2).add_((1 - beta2) * g * g)
        out.append(v.sqrt() / math.sqrt(bc2) * coef)
    return out


@pytest.mark.parametrize('keep_sign', [False, True])
def test_clip_momentum(keep_sign):
    ps = _params(3)
    opt = Adam(ps, lr=0.0, grad_clip_type='clip_momentum', clip_value=1.0, clip_coef=0.5,
               clip_momentum_timestep=2, clip_momentum_keep_sign=keep_sign)
    vs = [torch.zeros_like(p) for p in ps]
    g = torch.Generator().manual_seed(7)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=g) * (1 + 5 * (step == 3)) for p in ps]
        for p, gr in zip(ps, grads):
            p.grad = gr.clone()
        bounds = _manual_bound(vs, grads, 0.999, step, 0.5)
        opt.step()
        for p, gr, bd in zip(ps, grads, bounds):
            if step >= 2:
                if keep_sign:
                    exp = torch.maximum(torch.minimum(gr, bd), -bd)
                else:
                    exp = torch.where(gr.abs() > bd, bd, gr)
            else:
                exp = gr
            torch.testing.assert_close(p.grad, exp)


def test_ignore_momentum_and_norm_variants():
    ps = _params(4)
    opt = Adam(ps, lr=0.0, grad_ignore_type='ignore_momentum', ignore_value=1.0, ignore_coef=3.0,
               ignore_momentum_timestep=1)
    for step in range(21):
        for p in ps:
            p.grad = torch.ones_like(p) * (1000.0 if step == 20 else 1.0)
        opt.step()
        if step == 19:
            assert all(float(p.grad.abs().sum()) > 0.0 for p in ps)
    assert all(float(p.grad.abs().sum()) == 0.0 for p in ps)  # spike at the last step -> all zeroed
    ps = _params(5)
    opt = Adam(ps, lr=0.0, grad_clip_type='clip_momentum_norm', clip_value=1.0, clip_coef=1.0,
               clip_momentum_timestep=1)
    for step in range(3):
        for p in ps:
            p.grad = torch.ones_like(p) * (10.0 if step == 2 else 1.0)
        opt.step()
    n = math.sqrt(sum(float((p.grad ** 2).sum()) for p in ps))
    v = 0.999 * (0.999 * 0.001 + 0.001) + 0.001 * 100.0  # EMA of g^2 after the three steps
    expected = math.sqrt(v / (1 - 0.999 ** 2)) * math.sqrt(27)  # grads rescaled to the momentum norm
    assert abs(n - expected) < 1e-3 * expected


def test_state_dict_round_trip():
    ps = _params(6)
    opt = Adam(ps, lr=0.01, grad_clip_type='clip_momentum', clip_value=1.0)
    opt.step()
    sd = copy.deepcopy(opt.state_dict())
    qs = _params(6)
    opt2 = Adam(qs, lr=0.01, grad_clip_type='clip_momentum', clip_value=1.0)
    opt2.load_state_dict(sd)
    assert opt2._thre_step == 1
    for p, q in zip(ps, qs):
        torch.testing.assert_close(opt._thre[p], opt2._thre[q])
