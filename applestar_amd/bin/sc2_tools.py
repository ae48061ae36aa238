"""SC2 utility commands (the upstream pysc2 ``bin`` tools: map_list.py, valid_actions.py,
replay_info.py, benchmark_observe.py, mem_leak_check.py, check_apm.py, replay_actions.py).

``python -m applestar_amd.bin.sc2_tools <command> [...]``

* ``map_list``                      - the map table (name, path, cropped / full size)
* ``valid_actions [--race zerg]``   - the 327-entry action table with argument heads (race filtered)
* ``replay_info REPLAY``            - game version, map, players, results, length (needs SC2)
* ``benchmark_observe``             - env steps / s and observe latency percentiles (``--fake`` env or SC2)
* ``mem_leak_check``                - RSS of this process (+ SC2 children) over episodes
* ``check_apm REPLAY...``           - actions-per-minute of each player in replays (needs SC2)

Every command returns a JSON-serialisable dict (printed as one JSON document), so they are scriptable.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional

from ..lib import game_data as gd


def map_list() -> Dict:
    from ..envs.map_info import MAPS, get_map_size
    return {name: {'path': v[1], 'cropped_size': list(get_map_size(name, True)),
                   'full_size': list(get_map_size(name, False))} for name, v in sorted(MAPS.items())}


def valid_actions(race: Optional[str] = None) -> Dict:
    mask = None
    if race:
        mask = gd.ACTION_RACE_MASK[race.lower()]
    out = []
    for i, a in enumerate(gd.ACTIONS):
        if mask is not None and not bool(mask[i]):
            continue
        out.append({'action_type': i, 'name': a['name'], 'func_id': a['func_id'], 'queued': bool(a['queued']),
                    'selected_units': bool(a['selected_units']), 'target_unit': bool(a['target_unit']),
                    'target_location': bool(a['target_location'])})
    return {'race': race, 'count': len(out), 'actions': out}


def _controller():
    from ..envs.sc2.launcher import SC2Process
    from ..envs.sc2.controller import RemoteController
    proc = SC2Process()
    return proc, RemoteController(proc.host, proc.port)


def replay_info(path: str) -> Dict:
    with open(path, 'rb') as f:
        data = f.read()
    proc, ctrl = _controller()
    try:
        info = ctrl.replay_info(data)
    finally:
        ctrl.quit()
        proc.close()
    players = [{'player_id': p.player_info.player_id, 'race': int(p.player_info.race_actual),
                'result': int(p.player_result.result), 'apm': p.player_apm, 'mmr': p.player_mmr}
               for p in info.player_info]
    return {'map_name': info.map_name, 'game_version': info.game_version, 'data_build': info.data_build,
            'game_duration_loops': info.game_duration_loops,
            'game_duration_seconds': info.game_duration_seconds, 'players': players}


def _percentiles(xs: List[float]) -> Dict:
    xs = sorted(xs)
    if not xs:
        return {}
    pick = lambda q: xs[min(len(xs) - 1, int(q * len(xs)))]  # noqa: E731
    return {'p50_ms': 1e3 * pick(0.5), 'p90_ms': 1e3 * pick(0.9), 'p99_ms': 1e3 * pick(0.99),
            'mean_ms': 1e3 * sum(xs) / len(xs)}


def _make_env(fake: bool, map_name: str, steps_per_episode: int):
    cfg = {'env': {'player_ids': ['agent1', 'bot7'], 'map_name': map_name, 'fake': fake,
                   'game_steps_per_episode': steps_per_episode}}
    from ..envs import make_env
    return make_env(cfg)


def benchmark_observe(fake: bool = True, steps: int = 500, map_name: str = 'KairosJunction',
                      steps_per_episode: int = 2000) -> Dict:
    env = _make_env(fake, map_name, steps_per_episode)
    lat = []
    n = 0
    t0 = time.perf_counter()
    try:
        env.reset()
        while n < steps:
            t = time.perf_counter()
            _, _, done = env.step({0: []})
            lat.append(time.perf_counter() - t)
            n += 1
            if done:
                env.reset()
    finally:
        env.close()
    wall = time.perf_counter() - t0
    return {'env': 'fake' if fake else 'sc2', 'steps': n, 'steps_per_s': n / wall, **_percentiles(lat)}


def _rss_mb(pid: int) -> float:
    try:
        with open(f'/proc/{pid}/status') as f:
            for line in f:
                if line.startswith('VmRSS:'):
                    return int(line.split()[1]) / 1024.0
    except OSError:
        pass
    return 0.0


def _tree_rss_mb(pid: int) -> float:
    total = _rss_mb(pid)
    try:
        for child in open(f'/proc/{pid}/task/{pid}/children').read().split():
            total += _tree_rss_mb(int(child))
    except OSError:
        pass
    return total


def mem_leak_check(fake: bool = True, episodes: int = 5, steps_per_episode: int = 500,
                   map_name: str = 'KairosJunction') -> Dict:
    env = _make_env(fake, map_name, steps_per_episode)
    samples = []
    try:
        for _ in range(episodes):
            env.reset()
            done = False
            while not done:
                _, _, done = env.step({0: []})
            samples.append(_tree_rss_mb(os.getpid()))
    finally:
        env.close()
    growth = samples[-1] - samples[0] if len(samples) > 1 else 0.0
    return {'env': 'fake' if fake else 'sc2', 'rss_mb': samples, 'growth_mb': growth,
            'growth_per_episode_mb': growth / max(1, len(samples) - 1)}


def check_apm(paths: List[str]) -> Dict:
    out = {}
    proc, ctrl = _controller()
    try:
        for p in paths:
            with open(p, 'rb') as f:
                info = ctrl.replay_info(f.read())
            out[p] = {int(pl.player_info.player_id): pl.player_apm for pl in info.player_info}
    finally:
        ctrl.quit()
        proc.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog='applestar_amd.bin.sc2_tools')
    sub = ap.add_subparsers(dest='cmd', required=True)
    sub.add_parser('map_list')
    va = sub.add_parser('valid_actions')
    va.add_argument('--race', default=None)
    ri = sub.add_parser('replay_info')
    ri.add_argument('replay')
    for name in ('benchmark_observe', 'mem_leak_check'):
        p = sub.add_parser(name)
        p.add_argument('--fake', action='store_true')
        p.add_argument('--map', default='KairosJunction')
        p.add_argument('--steps', type=int, default=500)
        p.add_argument('--episodes', type=int, default=5)
    ca = sub.add_parser('check_apm')
    ca.add_argument('replays', nargs='+')
    a = ap.parse_args(argv)
    if a.cmd == 'map_list':
        res = map_list()
    elif a.cmd == 'valid_actions':
        res = valid_actions(a.race)
    elif a.cmd == 'replay_info':
        res = replay_info(a.replay)
    elif a.cmd == 'benchmark_observe':
        res = benchmark_observe(a.fake, a.steps, a.map)
    elif a.cmd == 'mem_leak_check':
        res = mem_leak_check(a.fake, a.episodes, a.steps, a.map)
    else:
        res = check_apm(a.replays)
    print(json.dumps(res, indent=1, default=str))
    return res


if __name__ == '__main__':
    main()
