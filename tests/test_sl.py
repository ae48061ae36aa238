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


def test_replay_dataloader_slots_carry_and_pad():
    """Slots consume consecutive chunks of one trajectory (new_episodes on the first), short tails are
    padded with masked steps, and the batch trains."""
    import torch
    from applestar_amd.learner.replay_dataloader import ReplayDataLoader
    from applestar_amd.lib.features import random_obs, random_actions, actions_mask
    from applestar_amd.utils.config import AttrDict

    def traj(L, seed):
        g = torch.Generator().manual_seed(seed)
        steps = []
        for i in range(L):
            o = random_obs(1, max_entities=12, generator=g)
            a, su = random_actions(1, o['entity_num'], generator=g)
            one = lambda t: t[0]
            s = {'spatial_info': {k: one(v) for k, v in o['spatial_info'].items()},
                 'entity_info': {k: one(v)[:int(o['entity_num'][0])] for k, v in o['entity_info'].items()},
                 'scalar_info': {k: one(v) for k, v in o['scalar_info'].items()},
                 'entity_num': o['entity_num'][0], 'selected_units_num': su[0],
                 'action_info': {k: one(v)[:max(int(su[0]), 1)] if k == 'selected_units' else one(v)
                                 for k, v in a.items()},
                 'action_mask': {'action_type': torch.tensor(True), 'delay': torch.tensor(True),
                                 **{k: one(v).bool() for k, v in actions_mask(a['action_type']).items()}}}
            steps.append(s)
        return steps
    src = iter([traj(5, 0), traj(3, 1), traj(4, 2), traj(6, 3), traj(4, 4)])
    cfg = AttrDict({'learner': {'data': {'batch_size': 2, 'trajectory_length': 4}}})
    dl = ReplayDataLoader(cfg, source=src)
    b1 = next(dl)
    assert b1['traj_lens'] == [4, 3] and b1['new_episodes'] == [True, True]
    assert b1['entity_info']['unit_type'].shape[0] == 8
    assert not bool(b1['action_mask']['action_type'][7])   # padded step of slot 1
    b2 = next(dl)
    assert b2['traj_lens'] == [1, 4] and b2['new_episodes'] == [False, True]
    from applestar_amd.sl.trainer import SLTrainer
    tr = SLTrainer({'learner': {'data': {'batch_size': 2, 'trajectory_length': 4}, 'ignore_steps': 0}}, device='cpu')
    info = tr.step(b1)
    assert torch.isfinite(info['total_loss'])
