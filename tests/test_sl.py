"""Supervised loss parity with the reference and an SL trainer smoke step on CPU."""
import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.models.model import Model
from applestar_amd.rl.synthetic import sl_batch
from applestar_amd.sl.loss import SupervisedLoss
from applestar_amd.sl.trainer import SLTrainer


@pytest.mark.skipif(not reference_available(), reason='reference tree not available')
@pytest.mark.parametrize('su_mask', [True, False])
def test_sl_loss_matches_reference(su_mask):
    import_reference()
    import distar.agent.default.sl_training.sl_loss as rsl
    torch.manual_seed(0)
    m = Model({})
    b = sl_batch(2, 3, max_entities=30, seed=4)
    logits, act, _ = m.sl_train(**{k: v for k, v in b.items() if k not in ('new_episodes',)})
    cfg = {'learner': {'su_mask': su_mask}}
    ref = rsl.SupervisedLoss(rsl.deep_merge_dicts(rsl.default_config, cfg)).compute_loss(
        logits, b['action_info'], b['action_mask'], b['selected_units_num'], b['entity_num'], act)
    mine = SupervisedLoss({'su_mask': su_mask}).compute_loss(
        logits, b['action_info'], b['action_mask'], b['selected_units_num'], b['entity_num'], act)
    for k, v in ref.items():
        assert abs(float(mine[k]) - float(v)) <= 1e-4 * max(1.0, abs(float(v))), k


def test_sl_trainer_steps_cpu():
    torch.manual_seed(0)
    tr = SLTrainer({'learner': {'ignore_steps': 1, 'data': {'batch_size': 2}}})
    b = sl_batch(2, 3, max_entities=20, seed=1)
    info0 = tr.step(b)
    info1 = tr.step(b)
    assert torch.isfinite(info1['total_loss'])
    assert 'gradient' in info1 and 'gradient' not in info0
