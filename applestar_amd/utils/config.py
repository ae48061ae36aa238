"""Layered YAML configuration.

Behavioural parity with the reference's ``read_config`` / ``deep_merge_dicts`` / ``deep_update``
(``distar/ctools/utils/config_helper.py:10-112``): component defaults are merged under a user file,
which is merged under CLI overrides; merging may introduce new keys.  Attribute access on nested
dicts mirrors EasyDict so configs read as ``cfg.learner.data.batch_size``.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Mapping

import yaml

__all__ = ['AttrDict', 'read_config', 'save_config', 'deep_merge_dicts', 'deep_update', 'to_plain']


class AttrDict(dict):
    """dict with attribute access; nested dicts are converted on construction and assignment."""

    def __init__(self, d: Mapping | None = None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, AttrDict):
            return v
        if isinstance(v, Mapping):
            return AttrDict(v)
        if isinstance(v, list):
            return [AttrDict._wrap(x) for x in v]
        return v

    def __setitem__(self, k, v):
        super().__setitem__(k, self._wrap(v))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def __deepcopy__(self, memo):
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = default
        return self[k]

    def update(self, other=(), **kw):
        for k, v in dict(other, **kw).items():
            self[k] = v


def to_plain(d: Any) -> Any:
    if isinstance(d, Mapping):
        return {k: to_plain(v) for k, v in d.items()}
    if isinstance(d, (list, tuple)):
        return [to_plain(x) for x in d]
    return d


def read_config(path: str) -> AttrDict:
    with open(path, 'r') as f:
        return AttrDict(yaml.safe_load(f) or {})


def save_config(cfg: Mapping, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, 'w') as f:
        yaml.safe_dump(to_plain(cfg), f, sort_keys=False)


def deep_update(base: dict, new: Mapping, new_keys_allowed: bool = True) -> dict:
    """In-place recursive update of ``base`` with ``new``."""
    for k, v in new.items():
        if k in base and isinstance(base[k], Mapping) and isinstance(v, Mapping):
            deep_update(base[k], v, new_keys_allowed)
        else:
            if k not in base and not new_keys_allowed:
                raise KeyError(f'unknown config key: {k}')
            base[k] = copy.deepcopy(v)
    return base


def deep_merge_dicts(base: Mapping, new: Mapping | None) -> AttrDict:
    """Return a new AttrDict = ``base`` recursively overridden by ``new``."""
    merged = AttrDict(copy.deepcopy(to_plain(base)))
    if new:
        deep_update(merged, to_plain(new))
    return AttrDict(merged)
