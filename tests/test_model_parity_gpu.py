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
CFG = {'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16'}, 'model': {'enable_baselines': ['winloss']}}
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


def _bf16_grad_errors(cpu, batch, ref_grads, native: bool):
    """Per-group relative gradient error of the mixed-precision trainer against the fp32 oracle, with the
    native kernels on, or off (PyTorch's own bf16 autocast path: the control)."""
    from applestar_amd import ops
    ops.set_native(native)
    try:
        tr = RLTrainer(CFG, device='cuda')
        assert tr.master is not None
        tr.load_model_state_dict(cpu.state_dict())
        info = tr._fwd_bwd(to_device(copy.deepcopy(batch), 'cuda'))
        tr._reduce()
        with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False), torch.no_grad():
            out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
        views = tr.master._master_grad_views()
        got = {}
        for p in tr.master.reducer.params:
            g = views.get(p, p.grad)
            if g is not None:
                got[tr.master.names[p]] = g.float()
        torch.cuda.synchronize()
    finally:
        ops.set_native(True)
    return _group_errors(got, ref_grads), out, info


def _su_logit_spread(cpu, seeds, control_runs: int = 3):
    """Mean selected-units logit error of the bf16 trainer over several batches, native kernels on and off.  The
    torch control is not deterministic run to run (0.028-0.039 over four runs of the same batches on one box,
    r6p), so - as for the gradient groups - its level is the largest of ``control_runs`` runs."""
    from applestar_amd import ops
    res = {}
    for native in [True] + [False] * control_runs:
        ops.set_native(native)
        try:
            tr = RLTrainer(CFG, device='cuda')
            tr.load_model_state_dict(cpu.state_dict())
            errs = []
            for s in seeds:
                batch = rl_batch(2, 4, max_entities=48, seed=s)
                with torch.no_grad():
                    ref = cpu.rl_learner_forward(**copy.deepcopy(batch))['target_logit']['selected_units']
                with torch.autocast('cuda', dtype=torch.bfloat16, cache_enabled=False), torch.no_grad():
                    out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
                errs.append(_masked_rel(out['target_logit']['selected_units'].float(), ref))
        finally:
            ops.set_native(True)
        key = 'native' if native else 'torch'
        res[key] = max(res.get(key, 0.0), sum(errs) / len(errs))
    return res


def test_full_model_bf16_gpu_vs_cpu_fp32(reference):
    """The mixed-precision trainer (bf16 compute weights + autocast) against the same fp32 oracle: all six
    heads' logits and the value within bf16 rounding, the loss within 2 %, and every parameter-group
    gradient (read from the fp32 master gradient) no further from the oracle than PyTorch's own bf16
    autocast path is (native kernels off, same weights and batch): the native kernels add no error of their
    own on top of bf16 compute.  Both error tables go to gpurun_out/bf16_grad_group_errors.json."""
    batch, (cpu, ref_out, ref_info, ref_grads) = reference
    errs, out, info = _bf16_grad_errors(cpu, batch, ref_grads, native=True)
    # the control (torch's own bf16 autocast backward) is not deterministic run to run - its head-gradient errors
    # moved 0.042 -> 0.106 over four runs of the same test on one box, while the native ones were bit-identical
    # (profiles/r4u_bf16_control_spread.txt) - so its noise level is the max over three runs
    runs = [_bf16_grad_errors(cpu, batch, ref_grads, native=False)[0] for _ in range(3)]
    errs_torch = {k: max(r[k] for r in runs) for k in runs[0]}
    logit_errs = {h: _masked_rel(out['target_logit'][h].float(), ref_out['target_logit'][h]) for h in HEADS}
    print('bf16 logit errors vs the fp32 oracle:', logit_errs)
    for h, e in logit_errs.items():
        if h != 'selected_units':
            assert e < 3e-2, (h, e, logit_errs)
    # the selected-units logits run through an autoregressive chain + a 32-wide LSTM: on one B=2 x T=4 batch
    # their bf16 error is 2-6 % for either bf16 path depending on the batch (profiles/r4q_bf16_logit_spread.jsonl:
    # torch's own autocast 2.1-5.6 %, native 1.8-4.9 %, means 3.4 / 3.1 %), so they are judged on the mean over
    # four batches against the torch control's mean instead of one seed's value
    # Over round 5's boxes the four-batch mean was 0.028-0.039 for the torch control and 0.0297-0.0343 for the native
    # path.  The check is an absolute ceiling that sits above the native path's measured range and below the one real
    # regression seen (rounding the core output to bf16 in front of a GLU: 0.0407, r7a) - it does not widen with the
    # control.  The control is reported, not bounded against: it moves box to box as well (its max of three runs was
    # 0.0271 on the round-6 box where the native value was 0.0343 - a 1.25x relative bound failed there - and 0.0372
    # on the next run of the same tree), and the native forward is bit-identical across reruns and under allocator
    # poisoning (tools/diag/poison_probe.py, profiles/r10g_poison_probe_fwd.txt: no read of unwritten memory), so its
    # box-to-box spread is not an uninitialised read in these kernels.
    su = _su_logit_spread(cpu, [3, 0, 1, 2])
    props = torch.cuda.get_device_properties(0)
    print('selected-units logit error, mean of four batches:', su, 'device CUs', props.multi_processor_count,
          getattr(props, 'gcnArchName', ''))
    assert su['native'] <= 0.036, su
    assert _rel(out['value']['winloss'].float(), ref_out['value']['winloss']) < 3e-2
    a, r = float(info['total_loss']), float(ref_info['total_loss'])
    assert abs(a - r) <= 2e-2 * max(1.0, abs(r)), (a, r)
    table = {k: {'native_bf16': errs[k], 'torch_bf16': errs_torch[k]} for k in errs}
    if os.path.isdir(OUT_DIR):
        with open(os.path.join(OUT_DIR, 'bf16_grad_group_errors.json'), 'w') as f:
            json.dump(table, f, indent=1, sort_keys=True)
    # r3b (profiles/r3b_bf16_grad_group_errors.json): 16 of 18 groups within +-15 % of torch's own bf16 error.
    # No absolute floors: the control is the max over three runs, and why the head groups sit at 8-10 % in both
    # paths is pinned down by test_bf16_head_grad_error_is_upstream_amplification below
    bad = {k: v for k, v in table.items() if v['native_bf16'] > 1.5 * v['torch_bf16']}
    assert not bad, bad
    # and in absolute terms: the big groups (transformer, spatial ResNet, LSTM, heads) within 15 %
    assert all(v['native_bf16'] < 0.15 for k, v in table.items() if k.startswith(('core_lstm', 'policy'))), table


def _tensor_leaves(tree, prefix=''):
    if isinstance(tree, dict):
        for k, v in tree.items():
            yield from _tensor_leaves(v, f'{prefix}/{k}')
    elif isinstance(tree, (list, tuple)):
        for i, v in enumerate(tree):
            yield from _tensor_leaves(v, f'{prefix}/{i}')
    elif torch.is_tensor(tree) and tree.is_floating_point() and tree.requires_grad:
        yield prefix, tree


def _pinned_grad_errors(cpu, batch, ref_grads, pins, native: bool):
    """Group gradient errors of the bf16 trainer when every model output's upstream gradient is pinned to the
    fp32 oracle's (the surrogate loss sum_i <out_i, g_i> has exactly the oracle's parameter gradient); also the
    relative error of the upstream gradients the bf16 step computes itself from the real loss."""
    from applestar_amd import ops
    ops.set_native(native)
    try:
        tr = RLTrainer(CFG, device='cuda')
        tr.load_model_state_dict(cpu.state_dict())
        from applestar_amd.runtime.train_engine import amp_context
        with amp_context(tr.device, tr.amp_dtype):
            out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
        leaves = dict(_tensor_leaves(out))
        # the upstream gradients of the real loss, computed in this path's own precision
        info = tr.loss.compute_loss(out)
        names = [k for k in pins if k in leaves]
        own = torch.autograd.grad(info['total_loss'], [leaves[k] for k in names], retain_graph=True, allow_unused=True)
        up_err = {}
        for k, g in zip(names, own):
            ref = pins[k]
            if g is not None and float(ref.norm()) > 0:
                up_err[k] = _rel(g.float(), ref)
        sur = sum((leaves[k].float() * pins[k].to('cuda', torch.float32)).sum() for k in names)
        tr.backward(sur)
        tr._reduce()
        views = tr.master._master_grad_views()
        got = {}
        for p in tr.master.reducer.params:
            g = views.get(p, p.grad)
            if g is not None:
                got[tr.master.names[p]] = g.float()
        torch.cuda.synchronize()
    finally:
        ops.set_native(True)
    return _group_errors(got, ref_grads), up_err


def test_bf16_head_grad_error_not_from_upstream_or_loss(reference):
    """The 8-10 % bf16 gradient error of the small heads (action type / delay / queued), shared by the native
    kernels and PyTorch's own autocast path, does not come from the loss: the upstream gradients the bf16 step
    derives from the real loss are within a few percent of the oracle's, and with every model output's upstream
    gradient PINNED to the oracle's the head groups keep the same error.  With the upstream pinned, the native
    path is within 1.5x of the control in EVERY group, no floor (tables in gpurun_out/bf16_pinned_upstream_errors.json;
    the cause is pinned down by test_bf16_head_grad_error_is_weight_rounding_sensitivity)."""
    batch, (cpu, ref_out, ref_info, ref_grads) = reference
    out = cpu.rl_learner_forward(**copy.deepcopy(batch))
    info = ReinforcementLoss(RLTrainer(CFG).cfg.learner, 'MP0').compute_loss(out)
    leaves = dict(_tensor_leaves(out))
    names = list(leaves)
    gs = torch.autograd.grad(info['total_loss'], [leaves[k] for k in names], allow_unused=True)
    pins = {k: g.detach() for k, g in zip(names, gs) if g is not None}
    assert any('target_logit' in k for k in pins) and any('value' in k for k in pins), list(pins)
    nat, up_nat = _pinned_grad_errors(cpu, batch, ref_grads, pins, native=True)
    # the control's error on these groups moves run to run (0.04-0.10: atomics-order noise through flipped ReLU
    # gates); as in test_full_model_bf16_gpu_vs_cpu_fp32, the bound is against the largest of three control runs
    ctl, up_ctl = _pinned_grad_errors(cpu, batch, ref_grads, pins, native=False)
    for _ in range(2):
        c2, _ = _pinned_grad_errors(cpu, batch, ref_grads, pins, native=False)
        ctl = {k: max(ctl[k], c2.get(k, ctl[k])) for k in ctl}
    table = {k: {'native_bf16_pinned': nat[k], 'torch_bf16_pinned': ctl[k]} for k in nat}
    ups = {k: {'native_bf16': up_nat.get(k), 'torch_bf16': up_ctl.get(k)} for k in pins}
    print('pinned-upstream group errors:', json.dumps(table, indent=1, sort_keys=True))
    print('upstream (d loss / d output) errors of the bf16 paths:', json.dumps(ups, indent=1, sort_keys=True))
    if os.path.isdir(OUT_DIR):
        with open(os.path.join(OUT_DIR, 'bf16_pinned_upstream_errors.json'), 'w') as f:
            json.dump({'pinned_group_errors': table, 'upstream_errors': ups}, f, indent=1, sort_keys=True)
    # r5g: upstream errors 0.1-1.9 % (native) / 0.1-0.9 % (torch); pinned head groups 0.083 / 0.099 / 0.081 native
    # vs 0.083 / 0.097 / 0.080 torch - the same as under the real loss
    for k, v in ups.items():
        if v['native_bf16'] is not None:
            assert v['native_bf16'] < 0.05, (k, v)
    bad = {k: v for k, v in table.items() if v['native_bf16_pinned'] > 1.5 * v['torch_bf16_pinned']}
    assert not bad, bad


def test_bf16_head_grad_error_is_weight_rounding_sensitivity(reference):
    """Root cause of the shared 8-10 % head-gradient error: the gradient's sensitivity to rounding the weights to
    bf16 at all.  The fp32 step (fp32 kernels, accurate to ~1e-5 against the oracle with the oracle's weights) run
    with every weight rounded to bf16 - no bf16 arithmetic anywhere - already moves the head groups' gradients by
    most of that error: a 2^-9 relative weight perturbation flips the ReLU gates (and max-pool / selection
    decisions) whose pre-activations sit within that margin of the boundary, and each flipped gate reroutes a whole
    unit's gradient.  The bf16 paths inherit this from their bf16 compute weights; it is not kernel error."""
    batch, (cpu, ref_out, ref_info, ref_grads) = reference
    fp32_cfg = {**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None}}
    res = {}
    for tag, rnd in (('fp32_exact_weights', False), ('fp32_bf16_rounded_weights', True)):
        tr = RLTrainer(fp32_cfg, device='cuda')
        sd = {k: (v.to(torch.bfloat16).float() if rnd and v.is_floating_point() else v)
              for k, v in cpu.state_dict().items()}
        tr.model.load_state_dict(sd)
        out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
        tr.loss.compute_loss(out)['total_loss'].backward()
        got = {n: p.grad for n, p in tr.model.named_parameters() if p.grad is not None}
        res[tag] = _group_errors(got, ref_grads)
    errs, _, _ = _bf16_grad_errors(cpu, batch, ref_grads, native=True)
    table = {k: {'fp32_exact_weights': res['fp32_exact_weights'][k],
                 'fp32_bf16_rounded_weights': res['fp32_bf16_rounded_weights'][k], 'native_bf16': errs[k]}
             for k in errs}
    print('weight-rounding sensitivity:', json.dumps(table, indent=1, sort_keys=True))
    if os.path.isdir(OUT_DIR):
        with open(os.path.join(OUT_DIR, 'bf16_weight_rounding_sensitivity.json'), 'w') as f:
            json.dump(table, f, indent=1, sort_keys=True)
    for k in ('policy.action_type_head', 'policy.delay_head', 'policy.queued_head'):
        v = table[k]
        assert v['fp32_exact_weights'] < 1e-3, (k, v)
        # rounding the weights alone accounts for at least half of the bf16 path's error
        assert v['fp32_bf16_rounded_weights'] > 0.5 * v['native_bf16'], (k, v)


def _trajectory(cfg, batches, steps, w_init, native=True):
    from applestar_amd import ops
    ops.set_native(native)
    try:
        tr = RLTrainer(cfg, device='cuda')
        tr.load_model_state_dict(w_init)
        rec = []
        for s in range(steps):
            info = tr.step(copy.deepcopy(batches[s % len(batches)]))
            rec.append((float(info['total_loss']), float(info['gradient'])))
        w = {k: v.detach().double().clone() for k, v in tr.model_state_dict().items()}
        torch.cuda.synchronize()
    finally:
        ops.set_native(True)
    return rec, w


def _compare(rec_a, w_a, rec_b, w_b, w0):
    num = da = db = 0.0
    for k, v0 in w0.items():
        if not v0.is_floating_point():
            continue
        x = (w_a[k] - v0.double().cuda()).flatten()
        y = (w_b[k] - v0.double().cuda()).flatten()
        num += float((x * y).sum())
        da += float(x.square().sum())
        db += float(y.square().sum())
    rel_loss = sorted(abs(b[0] - a[0]) / max(abs(a[0]), 1e-2) for a, b in zip(rec_a, rec_b))
    rel_gn = sorted(abs(b[1] - a[1]) / max(a[1], 1e-6) for a, b in zip(rec_a, rec_b))
    return {'update_cosine': num / max((da * db) ** 0.5, 1e-60), 'update_norm_ratio': (db / max(da, 1e-60)) ** 0.5,
            'median_rel_loss': rel_loss[len(rel_loss) // 2], 'max_rel_loss': rel_loss[-1],
            'median_rel_gnorm': rel_gn[len(rel_gn) // 2], 'max_rel_gnorm': rel_gn[-1]}


def test_bf16_training_tracks_fp32():
    """30 learner steps at the reference RL settings (lr 1e-5, Adam betas (0, 0.99) eps 1e-5, pytorch_norm clip
    1.0: distar/agent/default/rl_learner.py) of the fp32 and the bf16 trainer from the same weights over the
    same 6 batches: total loss and gradient norm track step by step and the accumulated update points the same
    way.  Control: an fp32 run on the plain PyTorch kernels (same precision, different kernels / summation
    order) shows how far two fp32 runs drift apart on their own.  Summary -> gpurun_out/precision_parity.json."""
    steps = 30
    cfg32 = {**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None}}
    torch.manual_seed(0)
    w0 = {k: v.detach().clone() for k, v in RLTrainer(cfg32, device='cuda').model_state_dict().items()}
    batches = [to_device(rl_batch(2, 8, max_entities=64, seed=100 + i), 'cuda') for i in range(6)]
    r32, w32 = _trajectory(cfg32, batches, steps, w0)
    r16, w16 = _trajectory(CFG, batches, steps, w0)
    rct, wct = _trajectory(cfg32, batches, steps, w0, native=False)
    summary = {'bf16_vs_fp32': _compare(r32, w32, r16, w16, w0),
               'control_fp32_torch_vs_fp32_native': _compare(r32, w32, rct, wct, w0),
               'steps': [{'step': i, 'loss_fp32': a[0], 'loss_bf16': b[0], 'loss_fp32_torch': c[0],
                          'gnorm_fp32': a[1], 'gnorm_bf16': b[1], 'gnorm_fp32_torch': c[1]}
                         for i, (a, b, c) in enumerate(zip(r32, r16, rct))]}
    if os.path.isdir(OUT_DIR):
        with open(os.path.join(OUT_DIR, 'precision_parity.json'), 'w') as f:
            json.dump(summary, f, indent=1)
    s = summary['bf16_vs_fp32']
    assert s['median_rel_loss'] < 0.01 and s['max_rel_loss'] < 0.05, summary
    assert s['median_rel_gnorm'] < 0.03 and s['max_rel_gnorm'] < 0.15, summary
    assert s['update_cosine'] > 0.95 and 0.9 < s['update_norm_ratio'] < 1.1, summary


def _count_native(monkeypatch, names):
    """Wrap the extension's entry points to count calls (and record the gemm_f32 epilogues used)."""
    from applestar_amd.ops import native as N
    C = N.ensure_loaded()
    calls = {n: [] for n in names}
    for n in names:
        f = getattr(C, n)

        def wrap(*a, _f=f, _n=n):
            # (residual given, epilogue act, rows): gemm_f32(a, b, bias, res, act), gemm_f32_psb(a, planes, N, K,
            # bias, res, act, variant)
            ri, ai = {'gemm_f32': (3, 4), 'gemm_f32_psb': (5, 6)}.get(_n, (None, None))
            calls[_n].append((a[ri] is not None if ri is not None else None, a[ai] if ai is not None else None,
                              int(a[0].shape[0]) if torch.is_tensor(a[0]) else None))
            return _f(*a)
        monkeypatch.setattr(C, n, wrap)
    return calls


def test_fp32_benchmark_composition_matches_cpu(monkeypatch):
    """The benchmarked fp32 composition at a shape that routes through it: B = 2, T = 16
    (34 observations) with entity counts up to 300 (~5k packed entity rows), so the entity transformer's linears
    take the native f32 GEMM (>= 128 output tiles) with the residual GradLink and ReLU-mask (ACT_DRELU) epilogues
    and the varlen attention runs multi-block (> 64 keys) sequences.  Forward logits / value, loss and every
    parameter-group gradient vs the fp32 CPU model, per-group bound 2e-3."""
    batch = rl_batch(2, 16, max_entities=300, seed=11)
    assert int(batch['entity_num'].max()) > 128
    cpu, ref_out, ref_info, ref_grads = _cpu_reference(batch)
    calls = _count_native(monkeypatch, ['gemm_f32', 'gemm_f32_psb', 'varlen_attn_fwd_f32', 'varlen_attn_bwd_f32'])
    tr = RLTrainer({**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None}}, device='cuda')
    tr.model.load_state_dict(cpu.state_dict())
    out = tr.model.rl_learner_forward(**to_device(copy.deepcopy(batch), 'cuda'))
    info = tr.loss.compute_loss(out)
    info['total_loss'].backward()
    torch.cuda.synchronize()
    g = calls['gemm_f32'] + calls['gemm_f32_psb']                  # the split ring or the pre-split-plane kernel
    assert len(g) >= 12, len(g)                                    # transformer linears fwd + dX on the f32 GEMM
    assert any(e[1] == 4 for e in g), 'no ReLU-mask (ACT_DRELU) dX epilogue'
    assert any(e[0] and e[1] == 0 for e in g), 'no residual (GradLink) dX epilogue'
    assert len(calls['varlen_attn_fwd_f32']) == 3 and len(calls['varlen_attn_bwd_f32']) == 3
    for h in HEADS:
        a, b = out['target_logit'][h], ref_out['target_logit'][h]
        assert _masked_rel(a, b) < 1e-4, (h, _masked_rel(a, b))
    assert _rel(out['value']['winloss'], ref_out['value']['winloss']) < 1e-4
    a, r = float(info['total_loss']), float(ref_info['total_loss'])
    assert abs(a - r) <= 1e-4 * max(1.0, abs(r)), (a, r)
    got = {n: p.grad for n, p in tr.model.named_parameters() if p.grad is not None}
    errs = _group_errors(got, ref_grads)
    bad = {k: v for k, v in errs.items() if v > 2e-3}
    assert not bad, bad


def test_fp32_trainer_trajectory_native_vs_torch():
    """Three fp32 trainer steps (derived weight forms refreshed after every update, fused clip + Adam) with the
    native kernels vs the torch fp32 path (native off) from the same weights on the same batches: per-step loss
    and gradient norm agree to 1e-3 and the accumulated update points the same way."""
    from applestar_amd import ops
    batches = [rl_batch(2, 8, max_entities=200, seed=s) for s in (21, 22, 23)]
    res = {}
    w0 = None
    for native in (True, False):
        ops.set_native(native)
        try:
            torch.manual_seed(0)
            tr = RLTrainer({**CFG, 'learner': {**CFG['learner'], 'amp_dtype': None, 'learning_rate': 1e-4}},
                           device='cuda')
            if w0 is None:
                w0 = {k: v.detach().clone() for k, v in tr.model.state_dict().items()}
            tr.model.load_state_dict(w0)
            tr.on_model_changed()
            traj = []
            for b in batches:
                info = tr.step(to_device(copy.deepcopy(b), 'cuda'))
                traj.append((float(info['total_loss']), float(info['gradient'])))
            torch.cuda.synchronize()
            res[native] = (traj, {k: v.detach().clone() for k, v in tr.model.state_dict().items()})
        finally:
            ops.set_native(True)
    (tn, wn), (tt, wt) = res[True], res[False]
    for (ln, gn), (lt, gt) in zip(tn, tt):
        assert abs(ln - lt) <= 1e-3 * max(1.0, abs(lt)), (ln, lt)
        assert abs(gn - gt) <= 1e-3 * max(1.0, abs(gt)), (gn, gt)
    dn = torch.cat([(wn[k] - w0[k]).reshape(-1).double() for k in w0 if w0[k].is_floating_point()])
    dt = torch.cat([(wt[k] - w0[k]).reshape(-1).double() for k in w0 if w0[k].is_floating_point()])
    cos = float((dn * dt).sum() / (dn.norm() * dt.norm()))
    assert cos > 0.999, cos
