"""Synthetic learner batches with the exact structure the RL/SL learners consume.

Mirrors what ``rl_dataloader.collate_fn`` (``distar/agent/default/rl_training/rl_dataloader.py:45-76,
206-245``) builds from actor trajectories: observations flattened time-major to (T+1)*B with
entities padded to the batch max, actions/logp/teacher logits/masks/rewards as [T,B,...].
Used by ``bench.py``, the smoke test and the GPU tests (no SC2 / no checkpoints on the boxes).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..lib import game_data as gd
from ..lib.features import (random_obs, random_actions, actions_mask, MAX_SELECTED_UNITS_NUM, LOCATION_NUM,
                            MAX_ENTITY_NUM)
from ..ops.reference import sequence_mask


def _tree_to(x, device, non_blocking=False):
    if torch.is_tensor(x):
        return x.to(device, non_blocking=non_blocking)
    if isinstance(x, dict):
        return {k: _tree_to(v, device, non_blocking) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_tree_to(v, device, non_blocking) for v in x)
    return x


def rl_batch(batch_size: int, unroll_len: int, max_entities: int = MAX_ENTITY_NUM, seed: int = 0,
             use_value_feature: bool = True, baselines=('winloss',), hidden_size: int = 384,
             num_layers: int = 3, entity_num: Optional[torch.Tensor] = None) -> Dict:
    g = torch.Generator().manual_seed(seed)
    B, T = batch_size, unroll_len
    n_obs = (T + 1) * B
    obs = random_obs(n_obs, entity_num=entity_num, max_entities=max_entities, generator=g,
                     value_feature=use_value_feature)
    N = obs['entity_info']['unit_type'].shape[1]
    en = obs['entity_num']
    act, su_num = random_actions(T * B, en[:T * B], generator=g)
    am = actions_mask(act['action_type'])
    act = {k: v.view(T, B, *v.shape[1:]) for k, v in act.items()}
    su_num = su_num.view(T, B)
    am = {k: v.view(T, B) for k, v in am.items()}
    en_tb = en[:T * B].view(T, B)
    behaviour_logp = {k: -torch.rand(T, B, generator=g) * 3 for k in
                      ['action_type', 'delay', 'queued', 'target_unit', 'target_location']}
    behaviour_logp['selected_units'] = -torch.rand(T, B, MAX_SELECTED_UNITS_NUM, generator=g) * 3
    teacher = {
        'action_type': torch.randn(T, B, gd.NUM_ACTIONS, generator=g),
        'delay': torch.randn(T, B, 128, generator=g),
        'queued': torch.randn(T, B, 2, generator=g),
        'selected_units': torch.randn(T, B, MAX_SELECTED_UNITS_NUM, N + 1, generator=g),
        'target_unit': torch.randn(T, B, N, generator=g),
        'target_location': torch.randn(T, B, LOCATION_NUM, generator=g),
    }
    # padded teacher logits carry -1e9 exactly like padding_entity_info (rl_dataloader.py:228-236)
    tu_valid = sequence_mask(en_tb.reshape(-1), N).view(T, B, N)
    teacher['target_unit'] = teacher['target_unit'].masked_fill(~tu_valid, -1e9)
    su_valid = sequence_mask(en_tb.reshape(-1) + 1, N + 1).view(T, B, 1, N + 1)
    # the teacher runs the same teacher-forced selected-units head as the student (agent.py:569,
    # model.py:76-162), so its logits carry the same masks: at step i the units already chosen at steps < i,
    # and the end token at step 0.  Random logits there would put a ~1e9 KL on every masked unit.
    labels = act['selected_units'].clamp(max=N)                                         # [T,B,S]
    prev = torch.nn.functional.one_hot(labels, N + 1).bool()                             # [T,B,S,N+1]
    prev_excl = torch.cat([torch.zeros_like(prev[:, :, :1]), (torch.cumsum(prev.int(), 2) > 0)[:, :, :-1]], 2)
    end0 = torch.zeros(T, B, MAX_SELECTED_UNITS_NUM, N + 1, dtype=torch.bool)
    end0[:, :, 0] = torch.nn.functional.one_hot(en_tb.clamp(max=N), N + 1).bool()
    teacher['selected_units'] = teacher['selected_units'].masked_fill(~su_valid | prev_excl | end0, -1e9)
    mask = {
        'actions_mask': am,
        'selected_units_mask': sequence_mask(su_num.reshape(-1), MAX_SELECTED_UNITS_NUM).view(T, B, -1),
        'selected_units_logits_mask': su_valid.view(T, B, N + 1),
        'target_units_logits_mask': tu_valid,
        'cum_action_mask': torch.ones(T, B),
        'build_order_mask': torch.zeros(T, B),
        'built_unit_mask': torch.zeros(T, B),
    }
    winloss = torch.zeros(T, B)
    winloss[-1] = torch.randint(-1, 2, (B,), generator=g).float()
    reward = {'winloss': winloss, 'build_order': torch.randn(T, B, generator=g) * 0.1,
              'built_unit': torch.randn(T, B, generator=g) * 0.1, 'battle': torch.randn(T, B, generator=g) * 0.1,
              'effect': torch.zeros(T, B), 'upgrade': torch.zeros(T, B)}
    hidden = [(torch.randn(n_obs, hidden_size, generator=g) * 0.1, torch.randn(n_obs, hidden_size, generator=g) * 0.1)
              for _ in range(num_layers)]
    batch = dict(obs)
    batch.update({
        'hidden_state': hidden,
        'action_info': act,
        'selected_units_num': su_num,
        'behaviour_logp': behaviour_logp,
        'teacher_logit': teacher,
        'mask': mask,
        'reward': reward,
        'step': torch.randint(0, 8000, (T, B), generator=g).float(),
        'batch_size': B,
        'unroll_len': T,
        'model_last_iter': torch.zeros(B),
    })
    return batch


def sl_batch(batch_size: int, traj_len: int, max_entities: int = MAX_ENTITY_NUM, seed: int = 0,
             hidden_size: int = 384, num_layers: int = 3) -> Dict:
    """Batch-major [B*T] supervised batch (sl_dataloader.py:19-94 layout)."""
    g = torch.Generator().manual_seed(seed)
    B, T = batch_size, traj_len
    obs = random_obs(B * T, max_entities=max_entities, generator=g)
    act, su_num = random_actions(B * T, obs['entity_num'], generator=g)
    am = actions_mask(act['action_type'])
    batch = dict(obs)
    batch.update({
        'action_info': act,
        'selected_units_num': su_num,
        'action_mask': {'action_type': torch.ones(B * T, dtype=torch.bool), 'delay': torch.ones(B * T, dtype=torch.bool),
                        **{k: v.bool() for k, v in am.items()}},
        'traj_lens': [T] * B,
        'hidden_state': [(torch.zeros(B, hidden_size), torch.zeros(B, hidden_size)) for _ in range(num_layers)],
        'new_episodes': [False] * B,
    })
    return batch


to_device = _tree_to


def sl_trajectory(length: int, seed: int = 0, max_entities: int = 12):
    """A decoded-replay-shaped trajectory (list of per-step dicts with the ReplayDecoder's keys, entities and
    selected units trimmed to their counts) of random observations / actions, for SL data-path tests."""
    g = torch.Generator().manual_seed(seed)
    steps = []
    for _ in range(length):
        o = random_obs(1, max_entities=max_entities, generator=g)
        a, su = random_actions(1, o['entity_num'], generator=g)
        n = int(o['entity_num'][0])
        steps.append({
            'spatial_info': {k: v[0] for k, v in o['spatial_info'].items()},
            'entity_info': {k: v[0][:n] for k, v in o['entity_info'].items()},
            'scalar_info': {k: v[0] for k, v in o['scalar_info'].items()},
            'entity_num': o['entity_num'][0], 'selected_units_num': su[0],
            'action_info': {k: v[0][:max(int(su[0]), 1)] if k == 'selected_units' else v[0] for k, v in a.items()},
            'action_mask': {'action_type': torch.tensor(True), 'delay': torch.tensor(True),
                            **{k: v[0].bool() for k, v in actions_mask(a['action_type']).items()}}})
    return steps


def sl_trajectories(lengths, seed: int = 0, max_entities: int = 12):
    """Iterator of :func:`sl_trajectory` (picklable through functools.partial: a collator-process source)."""
    for i, L in enumerate(lengths):
        yield sl_trajectory(L, seed + i, max_entities)
