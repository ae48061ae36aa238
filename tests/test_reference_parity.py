"""Numerical parity of the whole model against the reference implementation (CPU, fp32).

The reference model is built from /root/reference (read-only), its random-init state_dict is loaded
into our Model with ``strict=True`` (proves the key schema of SURVEY Appendix A), and both run on
the same synthetic observations.  Skipped where the reference tree is not present.
"""
import copy

import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.models.model import Model
from applestar_amd.lib.features import random_obs, random_actions

pytestmark = pytest.mark.skipif(not reference_available(), reason='reference tree not available')


def _pair(cfg, use_value_network=True, seed=0):
    ref = import_reference()
    cfg = dict(cfg, common={'type': 'train'})
    torch.manual_seed(seed)
    rm = ref.Model(cfg, use_value_network=use_value_network).eval()
    mm = Model(cfg, use_value_network=use_value_network).eval()
    missing = mm.load_state_dict(rm.state_dict(), strict=True)
    return rm, mm


def _inputs(B=3, seed=0, value_feature=False, max_entities=40):
    g = torch.Generator().manual_seed(seed)
    obs = random_obs(B, max_entities=max_entities, generator=g, value_feature=value_feature)
    act, su_num = random_actions(B, obs['entity_num'], generator=g)
    hidden = [(torch.randn(B, 384, generator=g), torch.randn(B, 384, generator=g)) for _ in range(3)]
    return obs, act, su_num, hidden


def _close(a, b, atol=2e-4, rtol=2e-4):
    a, b = a.float(), b.float()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), err


def test_state_dict_schema_matches_reference():
    rm, mm = _pair({}, use_value_network=True)
    assert list(rm.state_dict().keys()) == list(mm.state_dict().keys())
    for k, v in rm.state_dict().items():
        assert mm.state_dict()[k].shape == v.shape, k
    cfg = {'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}
    rm, mm = _pair(cfg)
    assert set(rm.state_dict()) == set(mm.state_dict())
    assert len(mm.state_dict()) == 515


def test_teacher_logits_match_reference():
    rm, mm = _pair({}, use_value_network=False)
    obs, act, su_num, hidden = _inputs(B=4)
    with torch.no_grad():
        r = rm.compute_teacher_logit(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                     selected_units_num=su_num.clone(), action_info=copy.deepcopy(act))
        m = mm.compute_teacher_logit(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                     selected_units_num=su_num.clone(), action_info=copy.deepcopy(act))
    for k in ['action_type', 'delay', 'queued', 'target_unit', 'target_location']:
        _close(r['logit'][k], m['logit'][k])
    _close(r['logit']['selected_units'], m['logit']['selected_units'])
    for (rh, rc), (mh, mc) in zip(r['hidden_state'], m['hidden_state']):
        _close(rh, mh)
        _close(rc, mc)


def test_rl_learner_forward_matches_reference():
    cfg = {'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}
    rm, mm = _pair(cfg)
    T, B = 3, 2
    obs, _, _, hidden = _inputs(B=(T + 1) * B, value_feature=True)
    act, su_num = random_actions(T * B, obs['entity_num'][:T * B], generator=torch.Generator().manual_seed(5))
    act = {k: v.view(T, B, *v.shape[1:]) for k, v in act.items()}
    su_num = su_num.view(T, B)
    kw = dict(batch_size=B, unroll_len=T, behaviour_logp=None, teacher_logit=None, mask=None, reward=None, step=None)
    with torch.no_grad():
        r = rm.rl_learner_forward(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                  action_info=copy.deepcopy(act), selected_units_num=su_num.clone(), **kw)
        m = mm.rl_learner_forward(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                  action_info=copy.deepcopy(act), selected_units_num=su_num.clone(), **kw)
    for k in r['target_logit']:
        _close(r['target_logit'][k], m['target_logit'][k])
    _close(r['value']['winloss'], m['value']['winloss'])


@pytest.mark.parametrize('reduce_type', ['attention_pool', 'attention_pool_add_num'])
def test_attention_pool_selected_units_match_reference(reduce_type):
    """entity_reduce_type attention variants: our prefix-softmax (all steps at once) vs the reference's
    per-step masked attention pooling (action_arg_head.py:201-206)."""
    rm, mm = _pair({'model': {'entity_reduce_type': reduce_type}}, use_value_network=False)
    assert 'policy.head.selected_units_head.attention_pool.queries' in mm.state_dict() or \
        any('attention_pool.queries' in k for k in mm.state_dict())
    obs, act, su_num, hidden = _inputs(B=4, seed=3)
    with torch.no_grad():
        r = rm.compute_teacher_logit(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                     selected_units_num=su_num.clone(), action_info=copy.deepcopy(act))
        m = mm.compute_teacher_logit(**copy.deepcopy(obs), hidden_state=copy.deepcopy(hidden),
                                     selected_units_num=su_num.clone(), action_info=copy.deepcopy(act))
    for k in ['selected_units', 'target_unit', 'target_location']:
        _close(r['logit'][k], m['logit'][k], atol=5e-4, rtol=5e-4)
