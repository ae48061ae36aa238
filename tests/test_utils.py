"""ctools-equivalent utilities: config layering, safe serialization, checkpoints (shape-matched load,
auto-checkpoint), gradient clipping, LR warm-up, learner hooks, log meters."""
import os

import pytest
import torch

from applestar_amd.utils import serialize
from applestar_amd.utils.checkpoint import CheckpointHelper, auto_checkpoint, load_state_dict_matched
from applestar_amd.utils.config import deep_merge_dicts, deep_update, read_config, save_config
from applestar_amd.utils.grad_clip import build_grad_clip
from applestar_amd.utils.lr_scheduler import build_lr_scheduler


def test_config_merge_update_roundtrip(tmp_path):
    base = {'a': {'b': 1, 'c': [1, 2]}, 'd': 'x'}
    m = deep_merge_dicts(base, {'a': {'b': 2, 'new': 3}})
    assert m.a.b == 2 and m.a.c == [1, 2] and m.a.new == 3 and m.d == 'x' and base['a']['b'] == 1
    deep_update(m, {'a': {'c': [3]}})
    assert m.a.c == [3]
    p = tmp_path / 'c.yaml'
    save_config(m, str(p))
    r = read_config(str(p))
    assert r.a.b == 2 and r.a.new == 3


@pytest.mark.parametrize('compress', [False, True])
def test_serialize_roundtrip(compress):
    tree = {'f': torch.randn(3, 5), 'bf': torch.randn(4).bfloat16(), 'i8': torch.tensor([-1, 2], dtype=torch.int8),
            'b': torch.tensor([True, False]), 'scalar': torch.tensor(2.5), 'empty': torch.zeros(0, 7),
            'nested': [{'x': torch.arange(5)}, (1, 'two', None, 3.5)], 'nc': torch.randn(4, 4).t()}
    out = serialize.loads(serialize.dumps(tree, compress=compress))
    for k in ('f', 'bf', 'i8', 'b', 'scalar', 'nc'):
        assert torch.equal(out[k], tree[k]) and out[k].dtype == tree[k].dtype
    assert out['empty'].shape == (0, 7)
    assert torch.equal(out['nested'][0]['x'], torch.arange(5)) and out['nested'][1] == (1, 'two', None, 3.5)
    if not compress:
        header, body = serialize.parse(serialize.dumps(tree))
        assert '__d__' in header and len(body) > 0


def test_checkpoint_matched_load_and_auto_checkpoint(tmp_path):
    a = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    b = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 5))
    helper = CheckpointHelper()
    path = str(tmp_path / 'ck.pth.tar')
    opt = torch.optim.Adam(a.parameters())
    helper.save(path, a, opt, last_iter=7, extra={'map_name': 'KairosJunction'})
    obj = helper.load(path, b, None)
    assert obj['last_iter'] == 7 and obj['map_name'] == 'KairosJunction'
    assert sorted(obj['report']['mismatched']) == ['1.bias', '1.weight']
    assert torch.equal(b[0].weight, a[0].weight)
    rep = load_state_dict_matched(b, {'module.0.weight': a[0].weight, 'extra': torch.zeros(1)}, drop=('1.',))
    assert rep['unexpected'] == ['extra'] and '0.bias' in rep['missing']

    class Runner:
        saved = 0

        def save_checkpoint(self):
            self.saved += 1

        @auto_checkpoint('save_checkpoint')
        def run(self):
            raise RuntimeError('boom')
    r = Runner()
    with pytest.raises(RuntimeError):
        r.run()
    assert r.saved == 1


def test_grad_clip_variants():
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(10)) for _ in range(3)]
    for p in ps:
        p.grad = torch.randn(10) * 5
    ref = [p.grad.clone() for p in ps]
    total = build_grad_clip({'type': 'pytorch_norm', 'threshold': 1.0}).apply(ps)
    qs = [torch.nn.Parameter(torch.zeros(10)) for _ in range(3)]
    for q, g in zip(qs, ref):
        q.grad = g.clone()
    t2 = torch.nn.utils.clip_grad_norm_(qs, 1.0)
    assert abs(float(total) - float(t2)) < 1e-4
    for p, q in zip(ps, qs):
        assert torch.allclose(p.grad, q.grad, atol=1e-6)
    c = build_grad_clip({'type': 'clip_const', 'threshold': 0.5})
    for p in ps:
        p.grad = torch.randn(10) * 5
    c.apply(ps)
    assert max(float(p.grad.abs().max()) for p in ps) <= 0.5
    m = build_grad_clip({'type': 'momentum_norm', 'threshold': 1.0, 'momentum_mode': 'ema'})
    for p in ps:
        p.grad = torch.ones(10)
    m.apply(ps)                      # first step initialises the per-parameter EMA
    for p in ps:
        p.grad = torch.ones(10) * 100
    m.apply(ps)                      # a 100x spike is scaled back to the EMA norm
    assert all(abs(float(p.grad.norm()) - 10 ** 0.5) < 1e-3 for p in ps)


def _reference_momentum_norm_apply(state, parameters, threshold=1.0, norm_type=2.0):
    """A line-level port of the reference's momentum_norm branch (distar/ctools/torch_utils/grad_clip.py:73-106),
    list bookkeeping included: the oracle for the 'reference' mode."""
    parameters = list(parameters)
    if state['flag'] == 0:
        state['norm_mom'] = [None] * len(parameters)
    total = 0.0
    for idx, p in enumerate(parameters):
        if p.grad is not None:
            g = p.grad.data.norm(norm_type)
            m = state['norm_mom'][idx]
            s = 1.0 if m is None else (1.0 if g < threshold * m else threshold * m / (g + 1e-6))
            p.grad.data.mul_(s)
    for idx, p in enumerate(parameters):
        if p.grad is not None:
            g = p.grad.data.norm(norm_type)
            if state['norm_mom'][idx] is None:
                state['norm_mom'].append(float(g))
            else:
                state['norm_mom'][idx] = state['norm_mom'][idx] * 0.99 + float(g) * 0.01
            total += g.item() ** norm_type
    state['flag'] = 1
    return total ** (1.0 / norm_type)


def test_momentum_norm_reference_mode_matches_reference_apply():
    """the reference's momentum_norm never scales a gradient (norm_mom[idx] stays None, the new norms
    are appended past the end) and reports the unclipped global norm.  The default 'reference' mode reproduces
    that over steps with 100x spikes; the 'ema' mode does clip them."""
    torch.manual_seed(0)
    shapes = [(10,), (4, 7), (3, 3, 3)]
    ref_ps = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    ps = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    clip = build_grad_clip({'type': 'momentum_norm', 'threshold': 1.0})
    assert clip.momentum_mode == 'reference'
    ema = build_grad_clip({'type': 'momentum_norm', 'threshold': 1.0, 'momentum_mode': 'ema'})
    ema_ps = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
    state = {'flag': 0, 'norm_mom': None}
    for step in range(6):
        gs = [torch.randn(s) * (100.0 if step % 2 else 1.0) for s in shapes]
        for a, b, c, g in zip(ref_ps, ps, ema_ps, gs):
            a.grad, b.grad, c.grad = g.clone(), g.clone(), g.clone()
        want = _reference_momentum_norm_apply(state, ref_ps)
        got = clip.apply(ps)
        ema.apply(ema_ps)
        assert abs(float(got) - want) <= 1e-5 * want, step
        for a, b in zip(ref_ps, ps):
            assert torch.equal(a.grad, b.grad), step
        if step % 2:
            assert sum(float(c.grad.norm()) for c in ema_ps) < 0.1 * sum(float(b.grad.norm()) for b in ps)
    assert len(state['norm_mom']) == len(shapes) * 7     # the reference's list growth, not reproduced here


def test_momentum_norm_ema_gated_first_step_keeps_ema_uninitialised():
    """a gated-off FIRST step must not mark the EMA initialised (with a host flag, every later scale
    would be thr * 0 = 0 and all updates zero)."""
    ps = [torch.nn.Parameter(torch.zeros(5)) for _ in range(2)]
    clip = build_grad_clip({'type': 'momentum_norm', 'threshold': 1.0, 'momentum_mode': 'ema'})
    for p in ps:
        p.grad = torch.full((5,), float('nan'))
    clip.apply(ps, gate=torch.zeros(()))
    assert float(clip.mom_init) == 0.0
    for p in ps:
        p.grad = torch.ones(5)
    clip.apply(ps, gate=torch.ones(()))
    assert all(torch.equal(p.grad, torch.ones(5)) for p in ps)          # scale 1 on the initialising step
    assert float(clip.mom_init) == 1.0 and torch.allclose(clip.norm_mom, torch.full((2,), 5 ** 0.5))
    sd = clip.state_dict()
    fresh = build_grad_clip({'type': 'momentum_norm', 'threshold': 1.0, 'momentum_mode': 'ema'})
    fresh.load_state_dict(sd)
    for p in ps:
        p.grad = torch.ones(5) * 100
    fresh.apply(ps)
    assert all(abs(float(p.grad.norm()) - 5 ** 0.5) < 1e-3 for p in ps)


def test_lr_warmup_schedule():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = build_lr_scheduler(opt, {'type': 'warmup', 'warm_up_steps': 4, 'multiplier': 1.0})
    lrs = []
    for _ in range(6):
        lrs.append(opt.param_groups[0]['lr'])
        opt.step()
        sch.step()
    assert lrs[0] < lrs[2] < lrs[4] <= 1.0 + 1e-9 and abs(lrs[5] - 1.0) < 1e-9


def test_hooks_priority_and_save_freq(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    from applestar_amd.learner.hooks import build_learner_hooks, LearnerHook, add_learner_hook
    from applestar_amd.learner.sl_learner import SLLearner
    calls = []

    class H(LearnerHook):
        def __call__(self, engine):
            calls.append(self.name)
    hooks = build_learner_hooks({})
    add_learner_hook(hooks, H('late', 50, 'after_iter'))
    add_learner_hook(hooks, H('early', 0, 'after_iter'))
    names = [h.name for h in hooks['after_iter']]
    assert names.index('early') < names.index('late')
    lr = SLLearner({'common': {'experiment_name': 'hk'},
                    'learner': {'use_cuda': False, 'ignore_steps': 0, 'max_iterations': 3, 'log_to_stdout': False,
                                'data': {'fake_data': True, 'batch_size': 1, 'trajectory_length': 2,
                                         'fake_max_entities': 6},
                                'hook': {'save_ckpt_after_iter': {'name': 's', 'type': 'save_ckpt', 'priority': 40,
                                                                  'position': 'after_iter', 'ext_args': {'freq': 2}}}}})
    lr.run()
    ck = sorted(os.listdir(tmp_path / 'experiments' / 'hk' / 'checkpoint'))
    assert ck == ['hk_iteration_2.pth.tar', 'hk_iteration_3.pth.tar']  # every 2 iters + after run


def test_meters():
    from applestar_amd.utils.log import VariableRecord, AverageMeter
    m = AverageMeter(3)
    for v in (1, 2, 3, 4):
        m.update(v)
    assert m.avg == 3.0
    r = VariableRecord(2)
    r.update_var({'a': 1.0, 'b': 2.0})
    r.update_var({'a': 3.0})
    assert r.get_vars_dict()['a'] == 2.0 and 'a' in r.get_vars_text()


def test_stopwatch_and_alphastar_table():
    from applestar_amd.utils.stopwatch import StopWatch
    from applestar_amd.utils.log import AlphaStarVarRecord
    s = StopWatch(enabled=True)
    for _ in range(3):
        with s('outer'):
            with s('inner'):
                pass

    @s.decorate('fn')
    def f():
        return 1
    f()
    assert s.times['outer'].num == 3 and s.times['outer.inner'].num == 3 and s.times['fn'].num == 1
    assert 'outer.inner' in s.str()
    r = AlphaStarVarRecord(4)
    r.update_var({'winloss/action_type': 0.5, 'total_loss': 2.0, 'kl/total': 0.1})
    txt = r.get_vars_text()
    assert 'winloss' in txt and '0.5' in txt and 'total_loss' in txt


def test_take_rows_consumed_skip_link_returns_full_gradient():
    """SkipLink hand-over (ops/native.py): an unconsumed link takes the gradient (no autograd gradient here); a
    link whose ResBlock backward already ran returns the ordinary full-height gradient instead of dropping it."""
    import torch
    from applestar_amd.models.model import _TakeRows
    from applestar_amd.ops.native import SkipLink
    for consumed in (False, True):
        x = torch.randn(5, 3, 2, 2, requires_grad=True)
        link = SkipLink()
        link.consumed = consumed
        _TakeRows.apply(x, 2, link).sum().backward()
        if consumed:
            assert link.g is None and torch.equal(x.grad[:2], torch.ones(2, 3, 2, 2)) and not x.grad[2:].any()
        else:
            assert x.grad is None and link.g.shape == (2, 2, 2, 3)


def test_single_consumer_params_counts_every_autograd_use():
    """Deferred fp32 weight gradients (ops/native.py _Deferred) are allowed only for parameters with ONE consumer in
    the step's autograd graph: a weight also reached through an uncounted path (F.linear, a view) is excluded."""
    import torch
    from applestar_amd.ops.native import single_consumer_params
    a = torch.nn.Parameter(torch.randn(4, 4))
    b = torch.nn.Parameter(torch.randn(4, 4))
    c = torch.nn.Parameter(torch.randn(4))
    x = torch.randn(3, 4)
    y = torch.nn.functional.linear(torch.relu(x @ a.t()), b, c)
    loss = y.sum() + (x @ b.t()).sum()          # b: a second consumer through another op
    ids = {id(p) for p in single_consumer_params(loss)}
    assert id(a) in ids and id(c) in ids and id(b) not in ids
    y2 = (x @ a.t()).sum() + a.t().sum()         # a view of a: two edges into its AccumulateGrad
    assert id(a) not in {id(p) for p in single_consumer_params(y2)}
