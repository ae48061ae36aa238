"""Derived weight forms (ops/native.py DerivedWeights): the strided multi-tensor copy that rebuilds them,
and a learner whose forms are cached across steps producing exactly the losses, gradient norms and weights
of a learner that rebuilds every form per call."""
import pytest
import torch

from applestar_amd.ops import native
from applestar_amd.rl.synthetic import rl_batch, to_device
from applestar_amd.rl.trainer import RLTrainer

pytestmark = pytest.mark.gpu

CFG = {'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16'}, 'model': {'enable_baselines': ['winloss']}}


def test_multi_strided_copy_forms_match_torch():
    C = native.ensure_loaded()
    g = torch.Generator(device='cuda').manual_seed(0)
    w_cl = torch.randn(64, 32, 3, 3, device='cuda', generator=g).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w_c = torch.randn(48, 40, 3, 3, device='cuda', generator=g).to(torch.bfloat16)
    lin = torch.randn(96, 200, device='cuda', generator=g).to(torch.bfloat16)
    gate = torch.randn(128, 128, 1, 1, device='cuda', generator=g).to(torch.bfloat16)
    bias = torch.randn(77, device='cuda', generator=g).to(torch.bfloat16)
    w32 = torch.randn(16, 24, device='cuda', generator=g)
    forms = []
    for w in (w_cl, w_c):
        s0, s1, s2, s3 = w.stride()
        forms.append((w, torch.empty(w.shape[1], 3, 3, w.shape[0], dtype=torch.bfloat16, device='cuda'),
                      [w.shape[1], 3, 3, w.shape[0], s1, -s2, -s3, s0, 2 * s2 + 2 * s3],
                      w.flip(2, 3).permute(1, 2, 3, 0)))
    big = torch.randn(250, 1003, device='cuda', generator=g).to(torch.bfloat16)      # tiled transpose path (>= 64 K)
    big32 = torch.randn(130, 700, device='cuda', generator=g)
    for t, dt in ((lin, torch.bfloat16), (gate, torch.bfloat16), (w32, torch.bfloat16), (lin, torch.float32),
                  (big, torch.bfloat16), (big32, torch.bfloat16), (big32, torch.float32)):
        v = t.view(t.shape[0], -1).t()
        forms.append((t, torch.empty(v.shape, dtype=dt, device='cuda'), native._view_spec(v, t), v.to(dt)))
    forms.append((bias, torch.empty(77, dtype=torch.float32, device='cuda'), native._view_spec(bias, bias), bias.float()))
    # more forms than one launch carries (24): several launches
    forms = forms * 4
    spec = []
    for f in forms:
        spec += f[2]
    C.multi_strided_copy([f[1] for f in forms], [f[0] for f in forms], spec)
    torch.cuda.synchronize()
    for src, out, _, ref in forms:
        assert torch.equal(out, ref.contiguous()), (tuple(src.shape), out.dtype)
    # a spec that reaches past the source is refused before anything is launched
    with pytest.raises(RuntimeError):
        C.multi_strided_copy([torch.empty(78, device='cuda')], [bias], [1, 1, 1, 78, 0, 0, 0, 1, 0])


def test_cached_forms_match_per_call_forms_over_steps():
    """lr 1e-2 so every step moves the bf16 weights (at the default 1e-5 most bf16 values would not change and
    a stale form would go unnoticed).  After every step each cached form equals a fresh per-call rebuild from
    the current parameter, and the learner's loss / gradient norm track the uncached learner's (the BO
    encoder's fp32 gradient atomics make the two runs differ in the last bits, so not bitwise)."""
    cfg = {'learner': dict(CFG['learner'], learning_rate=1e-2), 'model': CFG['model']}
    torch.manual_seed(0)
    a = RLTrainer(cfg, device='cuda')
    torch.manual_seed(0)
    b = RLTrainer(cfg, device='cuda')
    b.master.derived.enabled = False
    batches = [to_device(rl_batch(2, 4, max_entities=64, seed=s), 'cuda') for s in (1, 2, 3)]
    reg = a.master.derived
    moved = 0
    for i, batch in enumerate(batches):
        before = {k: f[1].clone() for k, f in reg.forms.items()}
        ia, ib = a.step(dict(batch)), b.step(dict(batch))
        torch.cuda.synchronize()
        la, lb = float(ia['total_loss']), float(ib['total_loss'])
        assert abs(la - lb) <= 1e-3 * max(1.0, abs(lb)), (i, la, lb)
        ga, gb = float(ia['gradient']), float(ib['gradient'])
        assert abs(ga - gb) <= 1e-2 * max(1.0, abs(gb)), (i, ga, gb)
        for fk, (p, out, spec, epoch, version) in reg.forms.items():
            k = fk[1]
            assert epoch == reg.epoch and version == p._version
            if callable(spec):
                assert torch.equal(out, spec()), (i, k, tuple(p.shape))
                continue
            fresh = {'convwt': lambda: native.ensure_loaded().conv_wt(p.detach())}.get(k)
            if fresh is not None:
                ref = fresh()
            elif k == 'f32':
                ref = p.detach().float().contiguous()
            else:
                ref = p.detach().reshape(p.shape[0], -1).t().to(k[1]).contiguous()
            assert torch.equal(out, ref), (i, k, tuple(p.shape))
            moved += int(fk in before and not torch.equal(before[fk], out))
    assert len(reg.forms) > 50 and len(b.master.derived.forms) == 0
    assert moved > 50          # the refreshed forms did change between steps


def test_fp32_trainer_cached_forms_match_per_call_forms():
    """The fp32 learner (no master weights) caches the same derived forms (transposed GEMM weights, flipped conv
    weights), rebuilt after every optimizer step: each cached form equals a fresh rebuild from the current fp32
    parameter, and loss / gradient norm equal those of a learner that rebuilds every form per call."""
    cfg = {'learner': dict(CFG['learner'], learning_rate=1e-2, amp_dtype=None), 'model': CFG['model']}
    torch.manual_seed(0)
    a = RLTrainer(cfg, device='cuda')
    torch.manual_seed(0)
    b = RLTrainer(cfg, device='cuda')
    assert a.master is None and a.derived is not None
    b.derived.enabled = False
    batches = [to_device(rl_batch(2, 4, max_entities=64, seed=s), 'cuda') for s in (1, 2, 3)]
    reg = a.derived
    for i, batch in enumerate(batches):
        ia, ib = a.step(dict(batch)), b.step(dict(batch))
        torch.cuda.synchronize()
        la, lb = float(ia['total_loss']), float(ib['total_loss'])
        assert abs(la - lb) <= 1e-4 * max(1.0, abs(lb)), (i, la, lb)
        for fk, (p, out, spec, epoch, version) in reg.forms.items():
            if callable(spec):
                # built forms (pre-split weight planes): a fresh build from the current parameter
                assert torch.equal(out, spec()), (i, fk[1], tuple(p.shape))
                continue
            if fk[1] == 'convwt':
                ref = p.detach().flip(2, 3).permute(1, 2, 3, 0).contiguous()
            else:
                ref = p.detach().reshape(p.shape[0], -1).t().contiguous()
            assert torch.equal(out, ref), (i, fk[1], tuple(p.shape))
    assert len(reg.forms) > 20 and len(b.derived.forms) == 0
