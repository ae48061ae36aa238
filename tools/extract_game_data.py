"""One-off extractor: reads game-fact tables (action table, unit/buff/upgrade/addon id lists,
ability id lists, per-race action masks) out of the reference tree by *parsing* its Python
sources with ``ast`` (nothing from the reference is imported or executed) and writes them to
``applestar_amd/lib/data/game_data.json``.

These tables are facts about StarCraft II 4.10 that released checkpoints depend on
(reorder arrays index into one-hot tables), so they must be bit-identical to the reference.

Sources:
  distar/agent/default/lib/actions.py:5-333       ACTIONS
  distar/pysc2/lib/static_data.py:123-201,318-331 UNIT_TYPES, BUFFS, UPGRADES, ADDON, *_ABILITIES
  distar/agent/default/lib/stat.py:533-631        ACTION_RACE_MASK
  distar/agent/default/lib/stat.py:73-330         unit_dict, cum_dict, action_result_dict (league stats)
  distar/pysc2/lib/units.py, upgrades.py          unit / upgrade enum names (ids -> names for logs)
  distar/envs/map_info.py:8-258                   MAPS (bnet name, path, cropped / full size)
  distar/pysc2/run_configs/lib.py:36-…            SC2 VERSIONS (game version -> build, data hash)
  distar/pysc2/lib/actions.py:1183-1757           _RAW_FUNCTIONS (func id, name, command type, ability id,
                                                  general ability id): replay decoding (reverse_raw_action)
"""
import ast
import json
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
OUT = os.path.join(os.path.dirname(__file__), '..', 'applestar_amd', 'lib', 'data', 'game_data.json')


def _assignments(path):
    tree = ast.parse(open(path).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            out[node.targets[0].id] = node.value
    return out


def _literal(node):
    return ast.literal_eval(node)


def _torch_tensor_arg(node):
    # torch.tensor([...]) -> python list
    assert isinstance(node, ast.Call)
    return ast.literal_eval(node.args[0])


def _enum_classes(path):
    tree = ast.parse(open(path).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.ClassDef):
            out[node.name] = {t.targets[0].id: ast.literal_eval(t.value) for t in node.body
                              if isinstance(t, ast.Assign) and isinstance(t.targets[0], ast.Name)}
    return out


def _raw_functions(path):
    """[[func_id, name, function_type, ability_id, general_id], ...] of the ``_RAW_FUNCTIONS`` list, in list order."""
    tree = ast.parse(open(path).read())
    for node in tree.body:
        if isinstance(node, ast.Assign) and getattr(node.targets[0], 'id', None) == '_RAW_FUNCTIONS':
            out = []
            for call in node.value.elts:
                kind = call.func.attr
                args = call.args
                fid, name, ftype = ast.literal_eval(args[0]), ast.literal_eval(args[1]), args[2].id
                if kind == 'raw_ability':
                    ab = ast.literal_eval(args[3])
                    gen = ast.literal_eval(args[4]) if len(args) > 4 else 0
                    for kw in call.keywords:
                        if kw.arg == 'general_id':
                            gen = ast.literal_eval(kw.value)
                else:                                       # raw_ui_func: no ability
                    ab, gen = 0, 0
                out.append([fid, name, ftype, ab, gen])
            return out
    raise ValueError('_RAW_FUNCTIONS not found')


def _versions(path):
    tree = ast.parse(open(path).read())
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, 'id', None) == 'Version' and len(node.args) == 4:
            out.append([ast.literal_eval(a) for a in node.args])
    return out


def main():
    acts = _assignments(os.path.join(REF, 'distar/agent/default/lib/actions.py'))
    static = _assignments(os.path.join(REF, 'distar/pysc2/lib/static_data.py'))
    stat = _assignments(os.path.join(REF, 'distar/agent/default/lib/stat.py'))
    actions = _literal(acts['ACTIONS'])
    race_mask_node = stat['ACTION_RACE_MASK']
    race_mask = {}
    for k, v in zip(race_mask_node.keys, race_mask_node.values):
        race_mask[ast.literal_eval(k)] = [bool(x) for x in _torch_tensor_arg(v)]
    data = {
        'actions': actions,
        'unit_types': _literal(static['UNIT_TYPES']),
        'buffs': _literal(static['BUFFS']),
        'upgrades': _literal(static['UPGRADES']),
        'addon': _literal(static['ADDON']),
        'unit_specific_abilities': _literal(static['UNIT_SPECIFIC_ABILITIES']),
        'unit_general_abilities': _literal(static['UNIT_GENERAL_ABILITIES']),
        'unit_mix_abilities': _literal(static['UNIT_MIX_ABILITIES']),
        'action_race_mask': race_mask,
        'unit_dict': {race: {str(k): v for k, v in d.items()} for race, d in _literal(stat['unit_dict']).items()},
        'cum_dict': _literal(stat['cum_dict']),
        'action_result_dict': _literal(stat['action_result_dict']),
        'unit_enums': _enum_classes(os.path.join(REF, 'distar/pysc2/lib/units.py')),
        'upgrade_enums': _enum_classes(os.path.join(REF, 'distar/pysc2/lib/upgrades.py'))['Upgrades'],
        'sc2_versions': _versions(os.path.join(REF, 'distar/pysc2/run_configs/lib.py')),
        'raw_functions': _raw_functions(os.path.join(REF, 'distar/pysc2/lib/actions.py')),
        'maps': {k: list(v) for k, v in _literal(_assignments(os.path.join(REF, 'distar/envs/map_info.py'))['MAPS']).items()},
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, 'w') as f:
        json.dump(data, f, separators=(',', ':'))
    print({k: len(v) for k, v in data.items()})


if __name__ == '__main__':
    main()
