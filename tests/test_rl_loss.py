"""RL loss: batched scans vs the step-by-step reference formulas, and the full loss (every logged
term) vs the reference ReinforcementLoss on the same model outputs."""
import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.ops import reference as R
from applestar_amd.rl import rl_utils
from applestar_amd.rl.loss import ReinforcementLoss, HEADS
from applestar_amd.rl.synthetic import rl_batch
from applestar_amd.models.model import Model


def test_vtrace_matches_loop():
    g = torch.Generator().manual_seed(0)
    T, B = 7, 5
    rho = torch.rand(T, B, generator=g)
    r = torch.randn(T, B, generator=g)
    v = torch.randn(T + 1, B, generator=g)
    for gamma in (1.0, 0.997):
        a = rl_utils.vtrace_advantages(rho, rho, r, v, gamma=gamma, lambda_=1.0)
        b = R.vtrace_advantages(rho, rho, r, v, gamma=gamma, lambda_=1.0)
        assert torch.allclose(a, b, atol=1e-5)
    # batched over heads
    rho6 = torch.rand(6, T, B, generator=g)
    a6 = rl_utils.vtrace_advantages(rho6, rho6, r, v)
    for k in range(6):
        assert torch.allclose(a6[k], R.vtrace_advantages(rho6[k], rho6[k], r, v), atol=1e-5)


def test_lambda_and_upgo_returns_match_loop():
    g = torch.Generator().manual_seed(1)
    T, B = 9, 4
    r = torch.randn(T, B, generator=g)
    v = torch.randn(T + 1, B, generator=g)
    assert torch.allclose(rl_utils.lambda_returns(r, v, 1.0, 0.8), R.lambda_returns(r, v, 1.0, 0.8), atol=1e-5)
    assert torch.allclose(rl_utils.upgo_returns(r, v), R.upgo_returns(r, v), atol=1e-5)


@pytest.mark.skipif(not reference_available(), reason='reference tree not available')
def test_full_loss_matches_reference():
    import_reference()
    import distar.agent.default.rl_training.rl_loss as rref
    torch.manual_seed(0)
    cfg = {'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}
    model = Model(cfg, use_value_network=True)
    out = model.rl_learner_forward(**rl_batch(2, 3, max_entities=30, seed=1))
    lcfg = {f'{n}_head_weights': {h: 1.0 for h in HEADS} for n in ('pg', 'upgo', 'entropy', 'kl', 'dapo')}
    lcfg.update({'loss_weights': {'kl': 0.002}, 'kl': {'action_type_kl_steps': 5200}, 'use_dapo': False,
                 'dapo': {'dapo_steps': 2400}})
    mine = ReinforcementLoss(lcfg).compute_loss(dict(out, value=dict(out['value'])))
    ref_loss = rref.ReinforcementLoss(rref.deep_merge_dicts(rref.default_config.learner, lcfg), 'MP0')
    theirs = ref_loss.compute_loss(dict(out, value={k: v.clone() for k, v in out['value'].items()}))
    for k, rv in theirs.items():
        if k in mine:
            assert abs(float(mine[k]) - float(rv)) <= 1e-4 * max(1.0, abs(float(rv))), k
    params = [p for p in model.parameters() if p.requires_grad]
    g1 = torch.autograd.grad(mine['total_loss'], params, allow_unused=True, retain_graph=True)
    g2 = torch.autograd.grad(theirs["total_loss"], params, allow_unused=True)
    for a, b in zip(g1, g2):
        if a is None:
            assert b is None or b.abs().max() == 0
            continue
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)
