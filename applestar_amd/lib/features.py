"""Observation / action tensor schema (agent <-> model contract) and synthetic data.

Schema constants follow ``distar/agent/default/lib/features.py:31-82``.  The
synthetic generators produce tensors with exactly the dtypes/shapes the agent emits; they replace the
reference's ``fake_step_data`` / ``fake_model_output`` (``features.py:95-145``) and are what the
benchmarks and GPU tests run on (there is no SC2 binary on the MI355X boxes).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .game_data import (NUM_ACTIONS, NUM_UNIT_TYPES, NUM_UPGRADES, NUM_CUMULATIVE_STAT_ACTIONS,
                        NUM_UNIT_MIX_ABILITIES, NUM_BEGINNING_ORDER_ACTIONS, SELECTED_UNITS_MASK,
                        ACTION_ARG_MASK)

SPATIAL_SIZE = (152, 160)  # (y, x)
MAX_DELAY = 127
BEGINNING_ORDER_LENGTH = 20
MAX_SELECTED_UNITS_NUM = 64
MAX_ENTITY_NUM = 512
EFFECT_LEN = 100
UPGRADE_LENGTH = 20
LOCATION_NUM = SPATIAL_SIZE[0] * SPATIAL_SIZE[1]  # 24320

u8, i8, i16, f16, f32, i64 = torch.uint8, torch.int8, torch.int16, torch.float16, torch.float32, torch.int64

SPATIAL_INFO = [('height_map', u8), ('visibility_map', u8), ('creep', u8), ('player_relative', u8),
                ('alerts', u8), ('pathable', u8), ('buildable', u8), ('effect_PsiStorm', i16),
                ('effect_NukeDot', i16), ('effect_LiberatorDefenderZone', i16), ('effect_BlindingCloud', i16),
                ('effect_CorrosiveBile', i16), ('effect_LurkerSpines', i16)]

# one-hot width of each categorical spatial plane (in encoder channel order)
SPATIAL_ONE_HOT = [('visibility_map', 4), ('creep', 2), ('player_relative', 5), ('alerts', 2),
                   ('pathable', 2), ('buildable', 2)]
EFFECT_KEYS = [k for k, _ in SPATIAL_INFO if k.startswith('effect_')]

SCALAR_INFO = [('home_race', u8, ()), ('away_race', u8, ()), ('upgrades', i16, (NUM_UPGRADES,)),
               ('time', f32, ()), ('unit_counts_bow', u8, (NUM_UNIT_TYPES,)), ('agent_statistics', f32, (10,)),
               ('cumulative_stat', u8, (NUM_CUMULATIVE_STAT_ACTIONS,)),
               ('beginning_order', i16, (BEGINNING_ORDER_LENGTH,)), ('last_queued', i16, ()),
               ('last_delay', i16, ()), ('last_action_type', i16, ()),
               ('bo_location', i16, (BEGINNING_ORDER_LENGTH,)),
               ('unit_order_type', u8, (NUM_UNIT_MIX_ABILITIES,)), ('unit_type_bool', u8, (NUM_UNIT_TYPES,)),
               ('enemy_unit_type_bool', u8, (NUM_UNIT_TYPES,))]

# (name, dtype, encoding, width): encoding 'one_hot' (clamped index), 'binary' (11 bits) or 'scalar'.
# Order == column order of the 997-wide entity embedding input (actor_critic_default_config.yaml).
ENTITY_FIELDS = [
    ('unit_type', i16, 'one_hot', NUM_UNIT_TYPES), ('alliance', u8, 'one_hot', 5),
    ('cargo_space_taken', u8, 'one_hot', 9), ('build_progress', f16, 'scalar', 1),
    ('health_ratio', f16, 'scalar', 1), ('shield_ratio', f16, 'scalar', 1), ('energy_ratio', f16, 'scalar', 1),
    ('display_type', u8, 'one_hot', 5), ('x', u8, 'binary', 11), ('y', u8, 'binary', 11),
    ('cloak', u8, 'one_hot', 5), ('is_blip', u8, 'one_hot', 2), ('is_powered', u8, 'one_hot', 2),
    ('mineral_contents', f16, 'scalar', 1), ('vespene_contents', f16, 'scalar', 1),
    ('cargo_space_max', u8, 'one_hot', 9), ('assigned_harvesters', u8, 'one_hot', 24),
    ('weapon_cooldown', u8, 'one_hot', 32), ('order_length', u8, 'one_hot', 9),
    ('order_id_0', i16, 'one_hot', NUM_ACTIONS), ('order_id_1', i16, 'one_hot', 49),
    ('is_hallucination', u8, 'one_hot', 2), ('buff_id_0', u8, 'one_hot', 50), ('buff_id_1', u8, 'one_hot', 50),
    ('addon_unit_type', u8, 'one_hot', 9), ('is_active', u8, 'one_hot', 2),
    ('order_progress_0', f16, 'scalar', 1), ('order_progress_1', f16, 'scalar', 1),
    ('order_id_2', i16, 'one_hot', 49), ('order_id_3', i16, 'one_hot', 49), ('is_in_cargo', u8, 'one_hot', 2),
    ('attack_upgrade_level', u8, 'one_hot', 4), ('armor_upgrade_level', u8, 'one_hot', 4),
    ('shield_upgrade_level', u8, 'one_hot', 4), ('last_selected_units', i8, 'one_hot', 2),
    ('last_targeted_unit', i8, 'one_hot', 2),
]
ENTITY_INFO = [(n, d) for n, d, _, _ in ENTITY_FIELDS]
ENTITY_EMBED_DIM = sum(w for *_, w in ENTITY_FIELDS)
assert ENTITY_EMBED_DIM == 997

ACTION_HEADS = ['action_type', 'delay', 'queued', 'selected_units', 'target_unit', 'target_location']
ARG_HEADS = ['queued', 'selected_units', 'target_unit', 'target_location']

VALUE_FEATURE_INFO = [('unit_type', i16, (MAX_ENTITY_NUM,)), ('enemy_unit_counts_bow', u8, (NUM_UNIT_TYPES,)),
                      ('enemy_unit_type_bool', u8, (NUM_UNIT_TYPES,)), ('unit_x', u8, (MAX_ENTITY_NUM,)),
                      ('unit_y', u8, (MAX_ENTITY_NUM,)), ('unit_alliance', torch.bool, (MAX_ENTITY_NUM,)),
                      ('total_unit_count', i64, ()), ('enemy_agent_statistics', f32, (10,)),
                      ('enemy_upgrades', u8, (NUM_UPGRADES,)),
                      ('own_units_spatial', torch.bool, (1,) + SPATIAL_SIZE),
                      ('enemy_units_spatial', torch.bool, (1,) + SPATIAL_SIZE),
                      ('beginning_order', i64, (BEGINNING_ORDER_LENGTH,)), ('bo_location', i64, (BEGINNING_ORDER_LENGTH,)),
                      ('cumulative_stat', i64, (NUM_CUMULATIVE_STAT_ACTIONS,))]


def _rand_field(g: torch.Generator, dtype, shape, hi: int):
    if dtype in (f16, f32):
        return torch.rand(shape, generator=g).to(dtype)
    if dtype == torch.bool:
        return torch.rand(shape, generator=g) < 0.5
    return torch.randint(0, max(hi, 1), shape, generator=g).to(dtype)


def random_obs(batch: int, entity_num: Optional[torch.Tensor] = None, max_entities: int = MAX_ENTITY_NUM,
               generator: Optional[torch.Generator] = None, value_feature: bool = False) -> Dict:
    """A batch of random observations in the agent's exact schema.

    ``entity_num`` defaults to U[1, max_entities) per sample (the reference's fake_step_data draws
    U[0, 512); 0 is excluded because the reference divides by entity_num).  Entity tensors are
    padded to ``max(entity_num)`` like the learner collate (rl_dataloader.py:45-76)."""
    g = generator or torch.Generator().manual_seed(0)
    if entity_num is None:
        entity_num = torch.randint(1, max_entities, (batch,), generator=g)
    N = int(entity_num.max())
    H, W = SPATIAL_SIZE
    spatial = {
        'height_map': torch.randint(0, 256, (batch, H, W), generator=g).to(u8),
        'visibility_map': torch.randint(0, 4, (batch, H, W), generator=g).to(u8),
        'creep': torch.randint(0, 2, (batch, H, W), generator=g).to(u8),
        'player_relative': torch.randint(0, 5, (batch, H, W), generator=g).to(u8),
        'alerts': torch.randint(0, 2, (batch, H, W), generator=g).to(u8),
        'pathable': torch.randint(0, 2, (batch, H, W), generator=g).to(u8),
        'buildable': torch.randint(0, 2, (batch, H, W), generator=g).to(u8),
    }
    for k in EFFECT_KEYS:
        eff = torch.randint(0, H * W, (batch, EFFECT_LEN), generator=g)
        eff[:, torch.randint(1, EFFECT_LEN, (1,), generator=g).item():] = 0  # zero padded tail
        spatial[k] = eff.to(i16)
    scalar = {}
    for name, dtype, size in SCALAR_INFO:
        hi = {'home_race': 5, 'away_race': 5, 'last_queued': 2, 'last_delay': 128, 'last_action_type': NUM_ACTIONS,
              'beginning_order': NUM_BEGINNING_ORDER_ACTIONS, 'bo_location': H * W, 'upgrades': 2,
              'unit_counts_bow': 20, 'cumulative_stat': 2, 'unit_order_type': 2, 'unit_type_bool': 2,
              'enemy_unit_type_bool': 2}.get(name, 2)
        if name == 'time':
            scalar[name] = torch.randint(0, 20000, (batch,), generator=g).float()
        else:
            scalar[name] = _rand_field(g, dtype, (batch,) + tuple(size), hi)
    entity = {}
    for name, dtype, enc, width in ENTITY_FIELDS:
        hi = 256 if enc == 'binary' else width
        entity[name] = _rand_field(g, dtype, (batch, N), hi)
    valid = torch.arange(N)[None, :] < entity_num[:, None]
    for k in entity:
        entity[k] = torch.where(valid, entity[k], torch.zeros_like(entity[k]))
    obs = {'spatial_info': spatial, 'scalar_info': scalar, 'entity_info': entity,
           'entity_num': entity_num.long()}
    if value_feature:
        vf = {}
        for name, dtype, size in VALUE_FEATURE_INFO:
            hi = {'unit_type': NUM_UNIT_TYPES, 'unit_x': W, 'unit_y': H, 'total_unit_count': MAX_ENTITY_NUM,
                  'beginning_order': NUM_BEGINNING_ORDER_ACTIONS, 'bo_location': H * W}.get(name, 2)
            vf[name] = _rand_field(g, dtype, (batch,) + tuple(size), hi)
        vf['enemy_agent_statistics'] = vf['enemy_agent_statistics'] * 5
        obs['value_feature'] = vf
    return obs


def random_actions(batch: int, entity_num: torch.Tensor, generator: Optional[torch.Generator] = None,
                   max_su: int = MAX_SELECTED_UNITS_NUM) -> Dict:
    """Random behaviour actions consistent with ``entity_num`` (labels used teacher-forced).

    selected_units labels follow what the actor's sampler emits: distinct units, terminated by the
    end token (== entity_num) unless 64 units were chosen; ``selected_units_num`` counts the end
    token (action_arg_head.py:296-302)."""
    g = generator or torch.Generator().manual_seed(1)
    B = batch
    action_type = torch.randint(0, NUM_ACTIONS, (B,), generator=g)
    su = torch.zeros(B, max_su, dtype=torch.long)
    su_num = torch.zeros(B, dtype=torch.long)
    for b in range(B):
        n = int(entity_num[b])
        if not bool(SELECTED_UNITS_MASK[action_type[b]]):
            continue
        k = int(torch.randint(1, min(n, max_su - 1) + 1, (1,), generator=g))
        perm = torch.randperm(n, generator=g)[:k]
        su[b, :k] = perm
        if k < max_su:
            su[b, k] = n
            su_num[b] = k + 1
        else:
            su_num[b] = max_su
    return {
        'action_type': action_type,
        'delay': torch.randint(0, MAX_DELAY + 1, (B,), generator=g),
        'queued': torch.randint(0, 2, (B,), generator=g),
        'selected_units': su,
        'target_unit': (torch.rand(B, generator=g) * entity_num.float()).long(),
        'target_location': torch.randint(0, LOCATION_NUM, (B,), generator=g),
    }, su_num


def actions_mask(action_type: torch.Tensor) -> Dict[str, torch.Tensor]:
    m = ACTION_ARG_MASK[action_type.long()]
    return {'queued': m[..., 0].long(), 'selected_units': m[..., 1].long(), 'target_unit': m[..., 2].long(),
            'target_location': m[..., 3].long()}
