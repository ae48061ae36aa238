"""Whole-model precision parity on the MI355X (SURVEY §4 "numerics vs an fp32 oracle", extended to the full
learner).

* fp32 path: the GPU learner forward over all six heads + the winloss value and the backward of the RL
  total loss, with fp32 weights and no autocast (every native op on fp32 operands), against the fp32 CPU
  model with the same weights and batch: per-output and per-parameter-group relative errors.
* bf16 path: the same comparison for the mixed-precision trainer (bf16 compute weights over fp32 masters,
  autocast), with bounds that state how far bf16 compute moves each gradient group.
* training parity: fp32 and bf16 trainers from the same initial weights on the same batches for 30 steps:
  loss / gradient-norm trajectories and the direction of the accumulated update.

Reference semantics: ``distar/agent/default/rl_learner.py:82-145`` (fp32 end to end)."""
import copy
import json
import os

import pytest
import torch

from applestar_amd.models.model import Model
from applestar_amd.rl.loss import ReinforcementLoss
from applestar_amd.rl.synthetic import rl_batch, to_device
from applestar_amd.rl.trainer import RLTrainer

pytestmark = pytest.mark.gpu
CFG = {'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}
HEADS = ['action_type', 'delay', 'queued', 'selected_units', 'target_unit', 'target_location']
OUT_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')


def _group(name: str) -> str:
    return '.'.join(name.split('.')[:2])


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _masked_rel(a, b):
    """Relative error over finite reference entries (masked logits carry -1e9 on both sides)."""
    a, b = a.double().cpu(), b.double().cpu()
    keep = b > -1e8
    return _rel(a[keep], b[keep])


def _cpu_reference(batch):
    torch.manual_seed(0)
    cpu = Model(CFG, use_value_network=True).train()
    loss_fn = ReinforcementLoss(RLTrainer(CFG).cfg.learner, 'MP0')
    out = cpu.rl_learner_forward(**copy.deepcopy(batch))
    info = loss_fn.compute_loss(out)
    info['total_loss'].backward()
    grads = {n: p.grad.detach().clone() for n, p in cpu.named_parameters() if p.grad is not None}
    return cpu, out, info, grads


def _group_errors(got: dict, ref: dict):
    groups = {}
    for n, g in ref.items():
        k = _group(n)
        e = groups.setdefault(k, [0.0, 0.0])
        d = got[n].double().cpu() - g.double()
        e[0] += float(d.square().sum())
        e[1] += float(g.double().square().sum())
    return {k: (v[0] / max(v[1], 1e-60)) ** 0.5 for k, v in groups.items()}


@pytest.fixture(scope='module')
def reference():
    batch = rl_batch(2, 4, max_entities=48, seed=3)
    return batch, _cpu_reference(batch)


def test_full_model_fp32_gpu_matches_cpu_fp32(reference):
    """fp32 learner step on the GPU (fp32 weights, no autocast: native fp32 kernels + fp32 library GEMMs)
    == the fp32 CPU model: every head's logits, the value, the loss terms and every parameter-group
    gradient within fp32 reassociation error."""
    batch, (cpu, ref_out, ref_info, ref_grads) = reference
    tr = RLTrainer({**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None}}, device='cuda')
    assert tr.master is None
    tr.model.load_state_dict(cpu.state_dict())
    assert all(p.dtype == torch.float32 for p in tr.model.parameters())
    out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
    for h in HEADS:
        a, b = out['target_logit'][h], ref_out['target_logit'][h]
        assert a.dtype == torch.float32, h
        assert _masked_rel(a, b) < 1e-4, (h, _masked_rel(a, b))
    assert _rel(out['value']['winloss'], ref_out['value']['winloss']) < 1e-4
    info = tr.loss.compute_loss(out)
    for k in ('total_loss', 'pg/winloss', 'value/winloss', 'entropy/action_type', 'kl/action_type'):
        if k in ref_info:
            a, r = float(info[k]), float(ref_info[k])
            assert abs(a - r) <= 1e-4 * max(1.0, abs(r)), (k, a, r)
    info['total_loss'].backward()
    got = {n: p.grad for n, p in tr.model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref_grads)
    errs = _group_errors(got, ref_grads)
    bad = {k: v for k, v in errs.items() if v > 2e-3}
    assert not bad, bad


def test_full_model_bf16_gpu_vs_cpu_fp32(reference):
    """The mixed-precision trainer (bf16 compute weights + autocast) against the same fp32 oracle: all six
    heads' logits and the value within bf16 rounding, and every parameter-group gradient (read from the fp32
    master gradient) within a stated relative Frobenius bound."""
    batch, (cpu, ref_out, ref_info, ref_grads) = reference
    tr = RLTrainer(CFG, device='cuda')
    assert tr.master is not None
    tr.load_model_state_dict(cpu.state_dict())
    info = tr._fwd_bwd(to_device(copy.deepcopy(batch), 'cuda'))
    tr._reduce()
    with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False), torch.no_grad():
        out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
    for h in HEADS:
        e = _masked_rel(out['target_logit'][h].float(), ref_out['target_logit'][h])
        assert e < 3e-2, (h, e)
    assert _rel(out['value']['winloss'].float(), ref_out['value']['winloss']) < 3e-2
    a, r = float(info['total_loss']), float(ref_info['total_loss'])
    assert abs(a - r) <= 2e-2 * max(1.0, abs(r)), (a, r)
    views = tr.master._master_grad_views()
    names = tr.master.names
    got = {}
    for p in tr.master.reducer.params:
        g = views.get(p, p.grad)
        if g is not None:
            got[names[p]] = g.float()
    errs = _group_errors(got, ref_grads)
    with open(os.path.join(OUT_DIR, 'bf16_grad_group_errors.json'), 'w') if os.path.isdir(OUT_DIR) else \
            open(os.devnull, 'w') as f:
        json.dump(errs, f, indent=1, sort_keys=True)
    bad = {k: v for k, v in errs.items() if v > 0.1}
    assert not bad, (bad, errs)


def test_bf16_training_tracks_fp32():
    """30 learner steps of the fp32 and the bf16 trainer from the same weights on the same 4 batches
    (lr 1e-4, Adam betas (0, 0.99), pytorch_norm clip 1.0 as the reference): the total-loss and gradient-norm
    trajectories agree step by step, and the accumulated parameter update points the same way."""
    steps = 30
    cfg32 = {**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None, 'learning_rate': 1e-4}}
    cfg16 = {**CFG, 'learner': {**CFG['learner'], 'learning_rate': 1e-4}}
    torch.manual_seed(0)
    t32 = RLTrainer(cfg32, device='cuda')
    torch.manual_seed(0)
    t16 = RLTrainer(cfg16, device='cuda')
    t16.load_model_state_dict(t32.model.state_dict())
    w0 = {k: v.detach().clone() for k, v in t32.model_state_dict().items()}
    batches = [to_device(rl_batch(2, 8, max_entities=64, seed=100 + i), 'cuda') for i in range(4)]
    rec = []
    for s in range(steps):
        b = batches[s % len(batches)]
        i32 = t32.step(copy.deepcopy(b))
        i16 = t16.step(copy.deepcopy(b))
        rec.append({'step': s, 'loss_fp32': float(i32['total_loss']), 'loss_bf16': float(i16['total_loss']),
                    'gnorm_fp32': float(i32['gradient']), 'gnorm_bf16': float(i16['gradient'])})
    w32, w16 = t32.model_state_dict(), t16.model_state_dict()
    num = den32 = den16 = 0.0
    for k, v0 in w0.items():
        if not v0.is_floating_point():
            continue
        d32 = (w32[k].double() - v0.double()).flatten()
        d16 = (w16[k].double() - v0.double()).flatten()
        num += float((d32 * d16).sum())
        den32 += float(d32.square().sum())
        den16 += float(d16.square().sum())
    cos = num / max((den32 * den16) ** 0.5, 1e-60)
    rel_loss = [abs(r['loss_bf16'] - r['loss_fp32']) / max(abs(r['loss_fp32']), 1e-3) for r in rec]
    rel_gn = [abs(r['gnorm_bf16'] - r['gnorm_fp32']) / max(r['gnorm_fp32'], 1e-6) for r in rec]
    summary = {'update_cosine': cos, 'update_norm_ratio': (den16 / max(den32, 1e-60)) ** 0.5,
               'max_rel_loss': max(rel_loss), 'median_rel_loss': sorted(rel_loss)[len(rel_loss) // 2],
               'max_rel_gnorm': max(rel_gn), 'median_rel_gnorm': sorted(rel_gn)[len(rel_gn) // 2], 'steps': rec}
    if os.path.isdir(OUT_DIR):
        with open(os.path.join(OUT_DIR, 'precision_parity.json'), 'w') as f:
            json.dump(summary, f, indent=1)
    assert summary['median_rel_loss'] < 0.02 and summary['max_rel_loss'] < 0.1, summary
    assert summary['median_rel_gnorm'] < 0.05 and summary['max_rel_gnorm'] < 0.2, summary
    assert cos > 0.9 and 0.8 < summary['update_norm_ratio'] < 1.25, summary
