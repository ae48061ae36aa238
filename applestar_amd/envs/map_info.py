"""Map table (``distar/envs/map_info.py:8-278``): formatted name -> (battle.net name, map path,
cropped playable size (x, y), full size, localized names)."""
from __future__ import annotations

from ..lib.game_data import _RAW

MAPS = {k: tuple(v) for k, v in _RAW['maps'].items()}


def get_map_size(map_name: str, cropped: bool = True):
    return tuple(MAPS[map_name][2 if cropped else 3])


def get_localized_map_name(map_name: str, cleared: bool = True) -> str:
    return MAPS[map_name][5 if cleared else 4]


def _inverse(indices):
    out = {}
    for k, v in MAPS.items():
        for i in indices:
            if i < len(v):
                out[v[i]] = k
    return out


LOCALIZED_BNET_NAME_TO_NAME_LUT = _inverse([0, 4, 5, 6])
