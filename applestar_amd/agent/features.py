"""Raw SC2 observation -> model tensors, agent action -> SC2 command, replay action -> labels.

Behaviour follows ``distar/agent/default/lib/features.py``:

* ``transform_obs`` (``:463-767``): 7 minimap planes padded to 152x160; effect positions as flat
  ``x + (map_h - y) * 160`` indices (owner-1 LiberatorDefenderZone / LurkerSpines skipped), zero
  padded to 100; units + cargo passengers as 38 raw columns truncated to 512, remapped through the
  reorder tables; scalar features (log1p player stats, upgrade/unit bags, order types); optional
  value features from the opponent's observation (``:690-765``).
* ``get_z`` (``:419-460``), ``reverse_raw_action`` (``:854-952``), ``compute_battle_score``.

MI355X-side design: the per-unit Python loop of the reference (one list per unit, then a
NamedNumpyArray) is replaced by one flat row-builder per unit and *vectorised* numpy column
transforms; the featurizer accepts real protobuf messages or :mod:`applestar_amd.envs.raw` mirrors.
"""
from __future__ import annotations

import random
from collections import defaultdict
from typing import Dict, List, Optional

import numpy as np
import torch

from ..utils.stopwatch import sw
from ..lib.features import (SPATIAL_SIZE, SPATIAL_INFO, ENTITY_INFO, EFFECT_LEN, MAX_ENTITY_NUM,
                            MAX_SELECTED_UNITS_NUM, BEGINNING_ORDER_LENGTH, UPGRADE_LENGTH)
from ..lib.game_data import (ACTIONS, NUM_UNIT_TYPES, NUM_UPGRADES, NUM_UNIT_MIX_ABILITIES,
                             NUM_CUMULATIVE_STAT_ACTIONS, BEGINNING_ORDER_ACTIONS, CUMULATIVE_STAT_ACTIONS,
                             UNIT_TYPES_REORDER_ARRAY, BUFFS_REORDER_ARRAY, UPGRADES_REORDER_ARRAY,
                             ADDON_REORDER_ARRAY, UNIT_ABILITY_REORDER, ABILITY_TO_QUEUE_ACTION, RAW_ABILITY_FUNCS,
                             FUNC_ID_TO_ACTION_TYPE_DICT)

MINIMAP_LAYERS = ['height_map', 'visibility_map', 'creep', 'player_relative', 'alerts', 'pathable', 'buildable']
EFFECT_NAMES = {1: 'PsiStorm', 2: 'GuardianShield', 3: 'TemporalFieldGrowing', 4: 'TemporalField',
                5: 'ThermalLance', 6: 'ScannerSweep', 7: 'NukeDot', 8: 'LiberatorDefenderZoneSetup',
                9: 'LiberatorDefenderZone', 10: 'BlindingCloud', 11: 'CorrosiveBile', 12: 'LurkerSpines'}
SCORE_CATEGORIES = ['none', 'army', 'economy', 'technology', 'upgrade']
BASE_UNIT_TYPES = (59, 18, 86)  # Nexus, CommandCenter, Hatchery
OBSERVER_TYPE = 3

# raw unit columns (features.py FeatureUnit enum order)
RAW_COLS = ['unit_type', 'alliance', 'cargo_space_taken', 'build_progress', 'health_max', 'shield_max',
            'energy_max', 'display_type', 'owner', 'x', 'y', 'cloak', 'is_blip', 'is_powered', 'mineral_contents',
            'vespene_contents', 'cargo_space_max', 'assigned_harvesters', 'weapon_cooldown', 'order_length',
            'order_id_0', 'order_id_1', 'is_hallucination', 'buff_id_0', 'buff_id_1', 'addon_unit_type',
            'is_active', 'order_progress_0', 'order_progress_1', 'order_id_2', 'order_id_3', 'is_in_cargo',
            'attack_upgrade_level', 'armor_upgrade_level', 'shield_upgrade_level', 'health', 'shield', 'energy']
COL = {n: i for i, n in enumerate(RAW_COLS)}

_UNIT_TYPES_NP = UNIT_TYPES_REORDER_ARRAY.numpy()
_BUFFS_NP = BUFFS_REORDER_ARRAY.numpy()
_UPGRADES_NP = UPGRADES_REORDER_ARRAY.numpy()
_ADDON_NP = ADDON_REORDER_ARRAY.numpy()
_ABILITY_NP = UNIT_ABILITY_REORDER.numpy()
_QUEUE_NP = ABILITY_TO_QUEUE_ACTION.numpy()
_BO_INDEX = {a: i for i, a in enumerate(BEGINNING_ORDER_ACTIONS)}
_CUM_INDEX = {a: i for i, a in enumerate(CUMULATIVE_STAT_ACTIONS)}

_TORCH_TO_NP = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int16: np.int16, torch.float16: np.float16,
                torch.float32: np.float32, torch.int64: np.int64}


def compute_battle_score(obs) -> float:
    """killed minerals + 1.5 * killed vespene over all score categories (features.py:354-363)."""
    if obs is None:
        return 0.0
    sd = obs.observation.score.score_details
    km = sum(getattr(sd.killed_minerals, c) for c in SCORE_CATEGORIES)
    kv = sum(getattr(sd.killed_vespene, c) for c in SCORE_CATEGORIES)
    return float(km + 1.5 * kv)


def unpack_layer(plane) -> Optional[np.ndarray]:
    sx, sy = plane.size.x, plane.size.y
    if sx == 0 and sy == 0:
        return None
    if plane.bits_per_pixel == 1:
        data = np.unpackbits(np.frombuffer(plane.data, dtype=np.uint8))[:sx * sy]
    else:
        dt = {8: np.uint8, 16: np.uint16, 32: np.int32}[plane.bits_per_pixel]
        data = np.frombuffer(plane.data, dtype=dt)
    return data.reshape(sy, sx)


def _pad_plane(d: np.ndarray, padding: bool) -> torch.Tensor:
    """A copy of minimap plane d, zero-padded / cropped to SPATIAL_SIZE when ``padding`` (one numpy fill + one
    slice copy: the torch pad of the plain form cost ~30 us a plane)."""
    if not padding:
        return torch.from_numpy(np.array(d, copy=True))
    H, W = SPATIAL_SIZE
    h, w = min(d.shape[0], H), min(d.shape[1], W)
    out = np.zeros((H, W), dtype=d.dtype)
    out[:h, :w] = d[:h, :w]
    return torch.from_numpy(out)


def _unit_row(u, tag_types) -> list:
    orders = u.orders
    no = len(orders)
    buffs = u.buff_ids
    return [u.unit_type, u.alliance, u.cargo_space_taken, u.build_progress, u.health_max, u.shield_max,
            u.energy_max, u.display_type, u.owner, u.pos.x, u.pos.y, u.cloak, u.is_blip, u.is_powered,
            u.mineral_contents, u.vespene_contents, u.cargo_space_max, u.assigned_harvesters, u.weapon_cooldown,
            no, orders[0].ability_id if no > 0 else 0, orders[1].ability_id if no > 1 else 0,
            u.is_hallucination, buffs[0] if len(buffs) > 0 else 0, buffs[1] if len(buffs) > 1 else 0,
            tag_types.get(u.add_on_tag, 0) if u.add_on_tag else 0, u.is_active,
            orders[0].progress if no > 0 else 0, orders[1].progress if no > 1 else 0,
            orders[2].ability_id if no > 2 else 0, orders[3].ability_id if no > 3 else 0, 0,
            u.attack_upgrade_level, u.armor_upgrade_level, u.shield_upgrade_level, u.health, u.shield, u.energy]


def _passenger_row(v, u) -> list:
    row = [0.0] * len(RAW_COLS)
    row[COL['unit_type']] = v.unit_type
    row[COL['alliance']] = u.alliance
    row[COL['health_max']], row[COL['shield_max']], row[COL['energy_max']] = v.health_max, v.shield_max, v.energy_max
    row[COL['owner']] = u.owner
    row[COL['x']], row[COL['y']] = u.pos.x, u.pos.y
    row[COL['is_in_cargo']] = 1
    row[COL['health']], row[COL['shield']], row[COL['energy']] = v.health, v.shield, v.energy
    return row


def _player_stats(player) -> torch.Tensor:
    s = torch.from_numpy(np.array([player.minerals, player.vespene, player.food_used, player.food_cap,
                                   player.food_army, player.food_workers, player.idle_worker_count,
                                   player.army_count, player.warp_gate_count, player.larva_count], dtype=np.float32))
    return torch.log(s + 1)


def _upgrade_bag(upgrade_ids) -> torch.Tensor:
    up = np.zeros(NUM_UPGRADES, dtype=np.uint8)
    ids = list(upgrade_ids)[:UPGRADE_LENGTH]
    if ids:
        up[_UPGRADES_NP[ids]] = 1
    return torch.from_numpy(up)


def _bag(idx: np.ndarray, n: int, count: bool) -> torch.Tensor:
    """uint8 [n]: occurrences of each index (wrapping mod 256 like a uint8 scatter_add) or their presence."""
    if count:
        return torch.from_numpy(np.bincount(idx, minlength=n).astype(np.uint8))
    b = np.zeros(n, dtype=np.uint8)
    b[idx] = 1
    return torch.from_numpy(b)


# per-key column plan of transform_obs: (key, kind, column(s), numpy dtype), resolved once
def _entity_plan():
    plan = []
    tables = {'unit_type': _UNIT_TYPES_NP, 'order_id_0': _ABILITY_NP, 'addon_unit_type': _ADDON_NP}
    for k, dtype in ENTITY_INFO:
        if k.startswith('last_'):
            continue
        npt = _TORCH_TO_NP.get(dtype)
        if k in tables:
            plan.append((k, 'table', (COL[k], tables[k]), npt))
        elif k.startswith('order_id_'):
            plan.append((k, 'table', (COL[k], _QUEUE_NP), npt))
        elif k.startswith('buff_id'):
            plan.append((k, 'table', (COL[k], _BUFFS_NP), npt))
        elif k in ('cargo_space_taken', 'cargo_space_max'):
            plan.append((k, 'clip8', COL[k], npt))
        elif k in ('health_ratio', 'shield_ratio', 'energy_ratio'):
            base = k.split('_')[0]
            plan.append((k, 'ratio', (COL[base], COL[base + '_max']), npt))
        elif k == 'mineral_contents':
            plan.append((k, 'scale', (COL[k], np.float16(1800)), npt))
        elif k == 'vespene_contents':
            plan.append((k, 'scale', (COL[k], np.float16(2500)), npt))
        elif k == 'y':
            plan.append((k, 'flip_y', COL[k], npt))
        else:
            plan.append((k, 'col', COL[k], npt))
    return plan


_ENTITY_PLAN = _entity_plan()


class Features:
    def __init__(self, game_info, raw_ob, cfg: Optional[dict] = None):
        cfg = cfg or {}
        self._map_size = game_info.start_raw.map_size
        self._requested_races = {p.player_id: p.race_requested for p in game_info.player_info
                                 if p.type != OBSERVER_TYPE}
        self._map_name = game_info.map_name
        self._start_location = game_info.start_raw.start_locations[0]
        fcfg = cfg.get('feature', {}) or {}
        self._bo_zergling_num = fcfg.get('bo_zergling_num', 8)
        self._beginning_order_flag = random.random() < fcfg.get('beginning_order_prob', 1.0)
        self._cumulative_stat_flag = random.random() < fcfg.get('cumulative_stat_prob', 1.0)
        self._zero_z_value = fcfg.get('zero_z_value', 1.0)
        self._filter_spine = fcfg.get('filter_spine', True)
        bases = [u for u in raw_ob.observation.raw_data.units if u.unit_type in BASE_UNIT_TYPES]
        assert len(bases) == 1, 'expected exactly one own base at game start (no fog of war / corrupt replay?)'
        b = bases[0]
        self._born_location = int(b.pos.x) + int(self._map_size.y - b.pos.y) * SPATIAL_SIZE[1]
        a = game_info.start_raw.start_locations[0]
        self._away_born_location = int(a.x) + int(self._map_size.y - a.y) * SPATIAL_SIZE[1]

    # ------------------------------------------------------------------ properties
    home_born_location = property(lambda self: self._born_location)
    away_born_location = property(lambda self: self._away_born_location)
    start_location = property(lambda self: self._start_location)
    map_name = property(lambda self: self._map_name)
    map_size = property(lambda self: self._map_size)
    requested_races = property(lambda self: self._requested_races)

    # ------------------------------------------------------------------ Z from a trajectory
    def get_z(self, traj_data: List[dict]):
        zerglings = 0
        bo, bo_loc = [], []
        cum = torch.zeros(NUM_CUMULATIVE_STAT_ACTIONS, dtype=torch.int8)
        W = SPATIAL_SIZE[1]
        ox, oy = self._born_location % W, self._born_location // W
        ax, ay = self._away_born_location % W, self._away_born_location // W
        for step in traj_data:
            at = int(step['action_info']['action_type'])
            if at == 322:
                zerglings += 1
                if zerglings > self._bo_zergling_num:
                    continue
            if at in _BO_INDEX:
                loc = int(step['action_info']['target_location'])
                if self._filter_spine and at == 54:
                    x, y = loc % W, loc // W
                    if (ox - x) ** 2 + (oy - y) ** 2 < (ax - x) ** 2 + (ay - y) ** 2:
                        continue
                bo.append(_BO_INDEX[at])
                bo_loc.append(loc)
            if at in _CUM_INDEX:
                cum[_CUM_INDEX[at]] = 1
        n = len(bo)
        bo = (bo + [0] * BEGINNING_ORDER_LENGTH)[:BEGINNING_ORDER_LENGTH]
        bo_loc = (bo_loc + [0] * BEGINNING_ORDER_LENGTH)[:BEGINNING_ORDER_LENGTH]
        bo = torch.as_tensor(bo, dtype=torch.short) * self._beginning_order_flag
        bo_loc = torch.as_tensor(bo_loc, dtype=torch.short) * self._beginning_order_flag
        if not self._cumulative_stat_flag:
            cum = 0 * cum + self._zero_z_value
        return bo, cum, n, bo_loc

    # ------------------------------------------------------------------ observation
    @sw.decorate('transform_obs')
    def transform_obs(self, obs, padding_spatial: bool = False, opponent_obs=None) -> Dict:
        o = obs.observation
        raw = o.raw_data
        map_y = self._map_size.y
        W = SPATIAL_SIZE[1]
        spatial_info = {}
        for name in MINIMAP_LAYERS:
            spatial_info[name] = _pad_plane(unpack_layer(getattr(o.feature_layer_data.minimap_renders, name)),
                                            padding_spatial)
        effects = defaultdict(list)
        for e in raw.effects:
            name = EFFECT_NAMES.get(e.effect_id)
            if name is None or (name in ('LiberatorDefenderZone', 'LurkerSpines') and e.owner == 1):
                continue
            for p in e.pos:
                effects[name].append(int(p.x) + int(map_y - p.y) * W)
        for k, _ in SPATIAL_INFO:
            if k.startswith('effect_'):
                v = (effects[k[7:]] + [0] * EFFECT_LEN)[:EFFECT_LEN]
                spatial_info[k] = torch.as_tensor(v, dtype=torch.int16)

        # entities (units followed by their cargo passengers), truncated to 512
        tag_types = {u.tag: u.unit_type for u in raw.units} if any(u.add_on_tag for u in raw.units) else {}
        tags, rows = [], []
        for u in raw.units:
            tags.append(u.tag)
            rows.append(_unit_row(u, tag_types))
            for v in u.passengers:
                tags.append(v.tag)
                rows.append(_passenger_row(v, u))
        tags, rows = tags[:MAX_ENTITY_NUM], rows[:MAX_ENTITY_NUM]
        # column-major copy: every column below is one contiguous row of RT
        RT = np.ascontiguousarray(np.asarray(rows, dtype=np.float32).reshape(-1, len(RAW_COLS)).T)
        entity_info = {}
        np_cols = {}
        for k, kind, arg, npt in _ENTITY_PLAN:
            if kind == 'col':
                v = RT[arg]
            elif kind == 'table':
                v = arg[1][RT[arg[0]].astype(np.int64)]
            elif kind == 'flip_y':
                v = map_y - RT[arg]
            elif kind == 'clip8':
                v = np.clip(RT[arg], 0, 8)
            elif kind == 'ratio':
                # reference computes the ratio in fp16
                with np.errstate(over='ignore', divide='ignore', invalid='ignore'):
                    v = RT[arg[0]].astype(np.float16) / (RT[arg[1]].astype(np.float16) + np.float16(1e-6))
            else:   # scale
                v = RT[arg[0]].astype(np.float16) / arg[1]
            v = v.astype(npt)
            np_cols[k] = v
            entity_info[k] = torch.from_numpy(v)

        scalar_info = {'time': torch.tensor(o.game_loop, dtype=torch.float),
                       'agent_statistics': _player_stats(o.player_common)}
        pid = o.player_common.player_id
        scalar_info['home_race'] = torch.tensor(self._requested_races[pid], dtype=torch.uint8)
        for p, race in self._requested_races.items():
            if p != pid:
                scalar_info['away_race'] = torch.tensor(race, dtype=torch.uint8)
        scalar_info['upgrades'] = _upgrade_bag(raw.player.upgrade_ids)
        alliance = np_cols['alliance']
        own = alliance == 1
        own_types = np_cols['unit_type'][own].astype(np.int64)
        scalar_info['unit_counts_bow'] = _bag(own_types, NUM_UNIT_TYPES, True)
        scalar_info['unit_type_bool'] = (scalar_info['unit_counts_bow'] > 0).to(torch.uint8)
        scalar_info['unit_order_type'] = _bag(np_cols['order_id_0'][own].astype(np.int64), NUM_UNIT_MIX_ABILITIES,
                                              False)
        scalar_info['enemy_unit_type_bool'] = _bag(np_cols['unit_type'][alliance == 4].astype(np.int64),
                                                   NUM_UNIT_TYPES, False)

        game_info = {'map_name': self._map_name, 'action_result': [e.result for e in obs.action_errors],
                     'game_loop': o.game_loop, 'tags': tags, 'battle_score': compute_battle_score(obs),
                     'opponent_battle_score': 0.0}
        ret = {'spatial_info': spatial_info, 'scalar_info': scalar_info,
               'entity_num': torch.tensor(len(tags), dtype=torch.long), 'entity_info': entity_info,
               'game_info': game_info}
        if opponent_obs:
            ret['value_feature'] = self._value_feature(opponent_obs, np_cols, own, own_types, spatial_info,
                                                       padding_spatial)
            game_info['opponent_battle_score'] = compute_battle_score(opponent_obs)
        return ret

    def _value_feature(self, opponent_obs, np_cols, own, own_types, spatial_info, padding_spatial):
        oo = opponent_obs.observation
        enemy = [u for u in oo.raw_data.units if u.alliance == 1]
        e_type = _UNIT_TYPES_NP[np.asarray([u.unit_type for u in enemy], dtype=np.int64)].astype(np.int16)
        bow = _bag(e_type.astype(np.int64), NUM_UNIT_TYPES, True)
        ne = len(enemy)
        ex = np.asarray([u.pos.x for u in enemy], dtype=np.float32).astype(np.uint8)
        ey = (self._map_size.y - np.asarray([u.pos.y for u in enemy], dtype=np.float32)).astype(np.uint8)
        own_x, own_y = np_cols['x'][own], np_cols['y'][own]
        total = ne + len(own_types)
        n = min(total, MAX_ENTITY_NUM)

        def fit(first, second, dtype):
            out = np.zeros(MAX_ENTITY_NUM, dtype=dtype)
            out[:min(len(first), n)] = first[:n]
            if n > len(first):
                out[len(first):n] = second[:n - len(first)]
            return torch.from_numpy(out)
        alliance = np.zeros(MAX_ENTITY_NUM, dtype=np.bool_)
        alliance[:min(ne, n)] = True
        d = _pad_plane(unpack_layer(oo.feature_layer_data.minimap_renders.player_relative), padding_spatial)
        return {'unit_type': fit(e_type, own_types.astype(np.int16), np.int16), 'enemy_unit_counts_bow': bow,
                'enemy_unit_type_bool': (bow > 0).to(torch.uint8),
                'unit_x': fit(ex, own_x, np_cols['x'].dtype), 'unit_y': fit(ey, own_y, np_cols['y'].dtype),
                'unit_alliance': torch.from_numpy(alliance), 'total_unit_count': torch.tensor(total, dtype=torch.long),
                'enemy_agent_statistics': _player_stats(oo.player_common),
                'enemy_upgrades': _upgrade_bag(oo.raw_data.player.upgrade_ids),
                'own_units_spatial': (spatial_info['player_relative'] == 1).unsqueeze(0),
                'enemy_units_spatial': (d == 1).unsqueeze(0)}

    # ------------------------------------------------------------------ replay action -> labels
    @sw.decorate('reverse_raw_action')
    def reverse_raw_action(self, action, raw_tags: List[int]):
        """Replay ``ActionRaw`` -> (labels, mask, selected_units_num, last_su_tags, last_tu_tag, invalid)."""
        ret = {'action_type': None, 'delay': torch.tensor(0, dtype=torch.long), 'queued': None,
               'selected_units': None, 'target_unit': None, 'target_location': None}
        last_su_tags, last_tu_tag, invalid = None, None, False
        units, tags = [], []
        tag_index = {t: i for i, t in enumerate(raw_tags)}

        raw_act = getattr(action, 'action_raw', action)
        uc = _field(raw_act, 'unit_command')
        if uc is not None:
            ret['queued'] = torch.tensor(int(bool(uc.queue_command)), dtype=torch.long)
            for t in uc.unit_tags:
                if t in tag_index:
                    units.append(tag_index[t])
                    tags.append(t)
            tgt_unit = _field(uc, 'target_unit_tag')
            tgt_pos = _field(uc, 'target_world_space_pos')
            if tgt_unit:
                if tgt_unit in tag_index:
                    ret['target_unit'] = torch.tensor(tag_index[tgt_unit], dtype=torch.long)
                    last_tu_tag = tgt_unit
                else:
                    invalid = True
                ret['action_type'] = action_type_from_ability(uc.ability_id, 'unit')
            elif tgt_pos is not None:
                x = min(int(tgt_pos.x), self._map_size.x - 1)
                y = min(self._map_size.y - int(tgt_pos.y), self._map_size.y - 1)
                ret['target_location'] = torch.tensor(y * SPATIAL_SIZE[1] + x, dtype=torch.long)
                ret['action_type'] = action_type_from_ability(uc.ability_id, 'pt')
            else:
                ret['action_type'] = action_type_from_ability(uc.ability_id, 'quick')
        ta = _field(raw_act, 'toggle_autocast')
        if ta is not None:
            ret['action_type'] = action_type_from_ability(ta.ability_id, 'autocast')
            for t in ta.unit_tags:
                if t in tag_index:
                    units.append(tag_index[t])
                    tags.append(t)
        if ret['action_type'] is not None:
            ret['action_type'] = torch.tensor(ret['action_type'], dtype=torch.long)
        else:
            invalid = True
        if units and not invalid:
            last_su_tags = tags
            units.append(len(raw_tags))  # end flag
            ret['selected_units'] = torch.tensor(units, dtype=torch.long)
            su_num = torch.tensor(len(units), dtype=torch.long)
        else:
            invalid = True
            su_num = torch.tensor(0, dtype=torch.long)
        defaults = {'action_type': 0, 'delay': 0, 'queued': 0, 'target_unit': 0, 'target_location': 0}
        mask = {}
        for k, v in ret.items():
            mask[k] = torch.tensor(v is not None, dtype=torch.bool)
            if v is None:
                ret[k] = torch.tensor([0], dtype=torch.long) if k == 'selected_units' else \
                    torch.tensor(defaults[k], dtype=torch.long)
        ret['selected_units'] = ret['selected_units'][:MAX_SELECTED_UNITS_NUM]
        su_num.clamp_(max=MAX_SELECTED_UNITS_NUM)
        return ret, mask, su_num, last_su_tags, last_tu_tag, invalid


def _field(msg, name):
    """``msg.name`` if set (protobuf HasField semantics for messages; truthiness for mirrors)."""
    if hasattr(msg, 'HasField'):
        try:
            return getattr(msg, name) if msg.HasField(name) else None
        except ValueError:
            return getattr(msg, name, None) or None
    return getattr(msg, name, None)


_CANCEL_SLOT = {313, 1039, 305, 307, 309, 1832, 1834, 3672}
_UNLOAD_UNIT = {410, 415, 397, 1440, 2373, 1409, 914, 3670}
_FRIVOLOUS = {6, 7}
_CMD_TYPE = {'quick': 'raw_cmd', 'pt': 'raw_cmd_pt', 'unit': 'raw_cmd_unit', 'autocast': 'raw_autocast'}


def action_type_from_ability(ability_id: int, kind: str) -> Optional[int]:
    """Map a raw ability id + command kind (quick / pt / unit / autocast) to an action type index, as the reference's
    ``transfer_action_type`` (``features.py:862-880``): frivolous abilities drop, unloads become unload-all and slot
    cancels cancel-quick, a specific ability becomes its general one, then the raw function of that command type.
    None where the reference prints an invalid ability (no such function, or one outside the action table)."""
    if ability_id in _FRIVOLOUS:
        return None
    if ability_id in _UNLOAD_UNIT:
        ability_id = 3664
    elif ability_id in _CANCEL_SLOT:
        ability_id = 3671
    fns = RAW_ABILITY_FUNCS.get(ability_id)
    if not fns:
        return None
    gen = next(iter(fns.values()))[1]
    if gen:
        ability_id = gen
    f = RAW_ABILITY_FUNCS.get(ability_id, {}).get(_CMD_TYPE[kind])
    return FUNC_ID_TO_ACTION_TYPE_DICT.get(f[0]) if f is not None else None


@sw.decorate('transform_action')
def transform_action(action: dict, map_size=None):
    """Agent action dict -> (list of RawUnitCommand, skip_steps) (env.py:457-480)."""
    from ..envs.raw import RawUnitCommand, Point
    at = FUNC_ID_TO_ACTION_TYPE_DICT[action['func_id']]
    a = ACTIONS[at]
    skip = int(action.get('skip_steps', 0))
    if at == 0 or not a['general_ability_id']:
        return [], skip
    cmd = RawUnitCommand(ability_id=a['general_ability_id'], unit_tags=list(action.get('unit_tags', [])),
                         queue_command=bool(action.get('queued', 0)) and a['queued'])
    if a['target_unit']:
        cmd.target_unit_tag = action['target_unit_tag']
    elif a['target_location']:
        x, y = action['location']
        cmd.target_world_space_pos = Point(float(x), float(y))
    return [cmd], skip
