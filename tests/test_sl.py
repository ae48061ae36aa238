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
    from applestar_amd.utils.config import AttrDict

    from applestar_amd.rl.synthetic import sl_trajectory as traj
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


def test_replay_dataloader_shared_batch_process_matches_in_process():
    """The shared-batch path (collator process -> shared slab -> views) yields exactly the batches of the
    in-process path for the same trajectories, slot bookkeeping included."""
    import functools
    import torch
    from applestar_amd.learner.replay_dataloader import ReplayDataLoader
    from applestar_amd.rl.synthetic import sl_trajectories
    from applestar_amd.utils.config import AttrDict
    lengths = [5, 3, 4, 6, 4, 7, 2]
    cfg = AttrDict({'learner': {'data': {'batch_size': 2, 'trajectory_length': 4, 'shared_batch': True,
                                         'slab_mb': 16}}})
    shared = ReplayDataLoader(cfg, source_factory=functools.partial(sl_trajectories, lengths, 3))
    plain = ReplayDataLoader(AttrDict({'learner': {'data': {'batch_size': 2, 'trajectory_length': 4}}}),
                             source=sl_trajectories(lengths, 3))
    assert shared._shared is not None and plain._shared is None

    def cmp(a, b, path=''):
        if isinstance(a, dict):
            assert set(a) == set(b), path
            for k in a:
                cmp(a[k], b[k], f'{path}/{k}')
        elif isinstance(a, (list, tuple)):
            assert len(a) == len(b), path
            for x, y in zip(a, b):
                cmp(x, y, path)
        elif torch.is_tensor(a):
            assert a.dtype == b.dtype and torch.equal(a, b), path
        else:
            assert a == b, path
    try:
        for _ in range(4):
            cmp(next(shared), next(plain))
    finally:
        shared.close()


def test_shared_batch_shm_capacity_check():
    """the slabs are checked against /dev/shm's free space up front."""
    from applestar_amd.runtime.shared_batch import check_shm_capacity
    check_shm_capacity(1 << 20)
    with pytest.raises(RuntimeError, match='slab'):
        check_shm_capacity(1 << 62)
