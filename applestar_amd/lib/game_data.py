"""StarCraft II game-fact tables and the tables derived from them.

The raw lists live in ``data/game_data.json`` (extracted by ``tools/extract_game_data.py`` from
``distar/agent/default/lib/actions.py:5-333``, ``distar/pysc2/lib/static_data.py:123-331`` and
``distar/agent/default/lib/stat.py:533-631``).  The derived tables below follow the definitions in
``distar/agent/default/lib/actions.py:339-425`` so released checkpoints see identical indices:

* ``UNIT_TYPES_REORDER_ARRAY`` etc. map raw game ids -> dense index (-1 = unknown)
* ``QUEUE_ACTIONS`` (49), ``BEGINNING_ORDER_ACTIONS`` (174), ``CUMULATIVE_STAT_ACTIONS`` (167)
* ``SELECTED_UNITS_MASK`` [327] bool, ``ACTION_RACE_MASK`` {race: [327] bool}
"""
from __future__ import annotations

import gzip
import json
import os
from collections import defaultdict
from functools import lru_cache

import numpy as np
import torch

_DATA_DIR = os.path.join(os.path.dirname(__file__), 'data')

with open(os.path.join(_DATA_DIR, 'game_data.json')) as _f:
    _RAW = json.load(_f)

ACTIONS = _RAW['actions']
UNIT_TYPES = _RAW['unit_types']
BUFFS = _RAW['buffs']
UPGRADES = _RAW['upgrades']
ADDON = _RAW['addon']
UNIT_SPECIFIC_ABILITIES = _RAW['unit_specific_abilities']
UNIT_GENERAL_ABILITIES = _RAW['unit_general_abilities']
UNIT_MIX_ABILITIES = _RAW['unit_mix_abilities']

NUM_ACTIONS = len(ACTIONS)                  # 327
NUM_UNIT_TYPES = len(UNIT_TYPES)            # 260
NUM_BUFFS = len(BUFFS)                      # 50
NUM_UPGRADES = len(UPGRADES)                # 90
NUM_ADDON = len(ADDON)                      # 9
NUM_UNIT_MIX_ABILITIES = len(UNIT_MIX_ABILITIES)  # 269


def _reorder_array(ids):
    arr = torch.full((max(ids) + 1,), -1, dtype=torch.long)
    arr[torch.tensor(ids, dtype=torch.long)] = torch.arange(len(ids), dtype=torch.long)
    return arr


UNIT_TYPES_REORDER_ARRAY = _reorder_array(UNIT_TYPES)
BUFFS_REORDER_ARRAY = _reorder_array(BUFFS)
UPGRADES_REORDER_ARRAY = _reorder_array(UPGRADES)
ADDON_REORDER_ARRAY = _reorder_array(ADDON)
UNIT_TYPES_REORDER = {u: i for i, u in enumerate(UNIT_TYPES)}
UPGRADES_REORDER = {u: i for i, u in enumerate(UPGRADES)}
BUFFS_REORDER = {u: i for i, u in enumerate(BUFFS)}

# ability id -> general ability id (identity where no general ability exists)
ABILITY_TO_GABILITY = {
    a: (a if g == 0 else g) for a, g in zip(UNIT_SPECIFIC_ABILITIES, UNIT_GENERAL_ABILITIES)
}

UNIT_ABILITY_REORDER = torch.full((max(UNIT_MIX_ABILITIES) + 1,), -1, dtype=torch.long)
_mix_index = {a: i for i, a in enumerate(UNIT_MIX_ABILITIES)}
for _a, _g in ABILITY_TO_GABILITY.items():
    UNIT_ABILITY_REORDER[_a] = _mix_index[_g]
UNIT_ABILITY_REORDER[0] = 0

FUNC_ID_TO_ACTION_TYPE_DICT = {a['func_id']: i for i, a in enumerate(ACTIONS)}

# raw ability id -> {command type: (func id, general ability id)} from the pysc2 raw function table
# (distar/pysc2/lib/actions.py:1183-1763 RAW_ABILITY_IDS; every ability has at most one function per command type
# and one general id, so the table is order-free): replay decoding (agent/features.py action_type_from_ability)
RAW_ABILITY_FUNCS = {}
for _fid, _name, _ftype, _ab, _gen in _RAW['raw_functions']:
    RAW_ABILITY_FUNCS.setdefault(_ab, {})[_ftype] = (_fid, _gen)

# queue actions: every Train_* / Research* action, indexed from 1 (0 = no-op)
QUEUE_ACTIONS = [i for i, a in enumerate(ACTIONS) if 'Train_' in a['name'] or 'Research' in a['name']]
# later entries sharing a general ability overwrite earlier ones (reference dict-insertion order)
GABILITY_TO_QUEUE_ACTION = {}
_queue_index = {a: q for q, a in enumerate(QUEUE_ACTIONS, start=1)}
for _i, _a in enumerate(ACTIONS):
    GABILITY_TO_QUEUE_ACTION[_a['general_ability_id']] = _queue_index.get(_i, 0)

ABILITY_TO_QUEUE_ACTION = torch.full((max(ABILITY_TO_GABILITY) + 1,), -1, dtype=torch.long)
ABILITY_TO_QUEUE_ACTION[0] = 0
for _a, _g in ABILITY_TO_GABILITY.items():
    ABILITY_TO_QUEUE_ACTION[_a] = GABILITY_TO_QUEUE_ACTION.get(_g, 0)

EXCLUDE_ACTIONS = ['Build_Pylon_pt', 'Train_Overlord_quick', 'Build_SupplyDepot_pt', 'Train_Drone_quick',
                   'Train_SCV_quick', 'Train_Probe_quick', 'Build_CreepTumor_pt', '']
CUM_EXCLUDE_ACTIONS = ['Build_SpineCrawler_pt', 'Build_SporeCrawler_pt', 'Build_PhotonCannon_pt',
                       'Build_ShieldBattery_pt', 'Build_Bunker_pt', 'Morph_Overseer_quick', 'Build_MissileTurret_pt']

BEGINNING_ORDER_ACTIONS = [0] + [
    i for i, a in enumerate(ACTIONS) if a['goal'] in ('unit', 'build', 'research') and a['name'] not in EXCLUDE_ACTIONS]
CUMULATIVE_STAT_ACTIONS = [0] + [
    i for i, a in enumerate(ACTIONS) if a['goal'] in ('unit', 'build', 'research')
    and a['name'] not in EXCLUDE_ACTIONS and a['name'] not in CUM_EXCLUDE_ACTIONS]

NUM_QUEUE_ACTIONS = len(QUEUE_ACTIONS)                          # 109 table entries
MODEL_NUM_QUEUE_ACTIONS = 49  # one-hot width the model uses for order_id_1..3 (ids are clamped), config yaml
NUM_BEGINNING_ORDER_ACTIONS = len(BEGINNING_ORDER_ACTIONS)      # 174
NUM_CUMULATIVE_STAT_ACTIONS = len(CUMULATIVE_STAT_ACTIONS)      # 167

SELECTED_UNITS_MASK = torch.tensor([bool(a['selected_units']) for a in ACTIONS], dtype=torch.bool)
TARGET_UNIT_MASK = torch.tensor([bool(a['target_unit']) for a in ACTIONS], dtype=torch.bool)
TARGET_LOCATION_MASK = torch.tensor([bool(a['target_location']) for a in ACTIONS], dtype=torch.bool)
QUEUED_MASK = torch.tensor([bool(a['queued']) for a in ACTIONS], dtype=torch.bool)

# per action: which argument heads are meaningful (used to build 'actions_mask' in trajectories)
ACTION_ARG_MASK = torch.stack([QUEUED_MASK, SELECTED_UNITS_MASK, TARGET_UNIT_MASK, TARGET_LOCATION_MASK], dim=1)

UNIT_BUILD_ACTIONS = [a['func_id'] for a in ACTIONS if a['goal'] == 'build']
UNIT_TRAIN_ACTIONS = [a['func_id'] for a in ACTIONS if a['goal'] == 'unit']
GENERAL_ABILITY_IDS = [a['general_ability_id'] for a in ACTIONS]
UNIT_ABILITY_TO_ACTION = {i: GENERAL_ABILITY_IDS.index(a) for i, a in enumerate(UNIT_MIX_ABILITIES)
                          if a in GENERAL_ABILITY_IDS}

UNIT_TO_CUM = defaultdict(lambda: -1)
UPGRADE_TO_CUM = defaultdict(lambda: -1)
_cum_index = {a: i for i, a in enumerate(CUMULATIVE_STAT_ACTIONS)}
for _i, _a in enumerate(ACTIONS):
    if 'game_id' in _a and _i in _cum_index:
        if _a['goal'] in ('unit', 'build'):
            UNIT_TO_CUM[_a['game_id']] = _cum_index[_i]
        elif _a['goal'] == 'research':
            UPGRADE_TO_CUM[_a['game_id']] = _cum_index[_i]

ACTION_RACE_MASK = {r: torch.tensor(m, dtype=torch.bool) for r, m in _RAW['action_race_mask'].items()}
RACE_NAMES = ['random', 'zerg', 'terran', 'protoss']  # frac_id order used by the league (player.py:12)


@lru_cache(maxsize=None)
def z_library() -> dict:
    """All bundled Z (strategy statistic) files keyed by their reference file name."""
    with gzip.open(os.path.join(_DATA_DIR, 'z_library.json.gz'), 'rt') as f:
        return json.load(f)


def load_z(name_or_path: str) -> dict:
    """Load a Z file: a bundled name (``3map.json``) or a path on disk."""
    if os.path.exists(name_or_path):
        with open(name_or_path) as f:
            return json.load(f)
    lib = z_library()
    base = os.path.basename(name_or_path)
    if base not in lib:
        raise FileNotFoundError(f'unknown Z file {name_or_path}; bundled: {sorted(lib)}')
    return lib[base]


def action_arg_masks(action_type: int) -> dict:
    a = ACTIONS[int(action_type)]
    return {k: int(bool(a[k])) for k in ('queued', 'selected_units', 'target_unit', 'target_location')}


def as_numpy(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy()
