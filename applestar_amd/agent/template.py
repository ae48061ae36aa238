"""Minimal agent plugin contract (``distar/agent/template/agent.py``).

An agent pipeline is any class with these attributes/methods; the actor selects it by name through
:func:`applestar_amd.agent.registry.import_agent`.  ``step`` returns a list of SC2 action dicts
``{func_id, skip_steps, queued, unit_tags, target_unit_tag, location}``.
"""
from __future__ import annotations


class Agent:
    HAS_MODEL = False
    HAS_TEACHER_MODEL = False
    HAS_SUCCESSIVE_MODEL = False

    def __init__(self, cfg=None, env_id: int = 0, **kwargs):
        self.cfg = cfg
        self.env_id = env_id
        self.player_id = None

    def reset(self, map_name, race, game_info, obs):
        self.map_name, self.race = map_name, race

    def step(self, obs):
        return [{'func_id': 0, 'skip_steps': 1, 'queued': 0, 'unit_tags': [], 'target_unit_tag': 0,
                 'location': (0, 0)}]
