"""Agent pipelines by name (``distar/agent/import_helper.py:3-14``): ``default`` is the AlphaStar
agent, ``template`` the minimal no-op agent, ``<name>`` resolves ``applestar_amd.agent.<name>`` and
``pkg.module:Class`` any importable class.  ``register_agent`` adds pipelines at runtime."""
from __future__ import annotations

import importlib
from typing import Dict

_REGISTRY: Dict[str, str] = {'default': 'applestar_amd.agent.agent:Agent',
                             'template': 'applestar_amd.agent.template:Agent'}


def register_agent(name: str, target) -> None:
    _REGISTRY[name] = target


def import_agent(name: str = 'default', attr: str = 'Agent'):
    target = _REGISTRY.get(name, name)
    if not isinstance(target, str):
        return target
    if ':' in target:
        mod, cls = target.split(':', 1)
    elif '.' in target:
        mod, cls = target, attr
    else:
        mod, cls = f'applestar_amd.agent.{target}', attr
    return getattr(importlib.import_module(mod), cls)
