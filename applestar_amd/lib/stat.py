"""Per-game unit counts and action success statistics reported to the league (``lib/stat.py:6-72``).

The lookup tables (``unit_dict`` func_id -> unit name per race, ``cum_dict``, ``action_result_dict``)
are game facts extracted into ``data/game_data.json`` by ``tools/extract_game_data.py``.
"""
from __future__ import annotations

from collections import defaultdict

from .game_data import ACTIONS, _RAW

UNIT_DICT = {race: {int(k): v for k, v in d.items()} for race, d in _RAW['unit_dict'].items()}
CUM_DICT = _RAW['cum_dict']
ACTION_RESULT_DICT = _RAW['action_result_dict']
ENTITY_DICT = {v: k for race in ('Neutral', 'Protoss', 'Terran', 'Zerg') for k, v in _RAW['unit_enums'][race].items()}
UPGRADE_NAMES = {v: k for k, v in _RAW['upgrade_enums'].items()}


class Stat:
    def __init__(self, race: str):
        self._race = race
        self._unit_num = defaultdict(int)
        self._unit_num['max_unit_num'] = 0
        for name in UNIT_DICT.get(race, {}).values():
            self._unit_num[name] = 0
        self._action_success_count = defaultdict(int)

    def update(self, last_action_type: int, action_result: int, observation, game_step: int) -> None:
        if action_result < 1:
            return
        if action_result == 1:
            self._count_unit(int(last_action_type))
        if observation is not None:
            ei, n = observation['entity_info'], int(observation['entity_num'])
            if int((ei['alliance'][:n] == 1).sum()) > 10:
                name = ACTIONS[int(last_action_type)]['name']
                self._action_success_count[f'rate/{name}/{ACTION_RESULT_DICT[action_result]}'] += 1
                self._action_success_count[f'rate/{name}/count'] += 1

    def _count_unit(self, action_type: int) -> None:
        name = UNIT_DICT.get(self._race, {}).get(ACTIONS[action_type]['func_id'])
        if not name:
            return
        self._unit_num[name] += 1
        self._unit_num['max_unit_num'] = max(self._unit_num[name], self._unit_num['max_unit_num'])

    def get_stat_data(self) -> dict:
        data = {}
        mx = self._unit_num['max_unit_num']
        for k, v in self._unit_num.items():
            if k != 'max_unit_num':
                data['units/' + k] = v / mx if mx else 0.0
        for k, v in self._action_success_count.items():
            action = k.split('rate/')[1].split('/')[0]
            data[k] = v if k.endswith('/count') else v / (self._action_success_count[f'rate/{action}/count'] + 1e-6)
        return data

    @property
    def unit_num(self):
        return self._unit_num
