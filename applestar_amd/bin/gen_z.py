"""Build a Z (strategy statistics) library from winning players' replays (``distar/bin/gen_z.py``).

Output JSON: ``z[map][race][born_location] = [[beginning_order(20), cumulative_stat_indices,
bo_location(20), last_action_loop], ...]`` — the format the agent samples from (``agent.py:206-317``).
Only the winner of each replay contributes, and only if its build order has >= 10 entries.
Decoding uses the fast action-only pass of :class:`ReplayDecoder` (needs SC2).

    python -m applestar_amd.bin.gen_z --data /replays --name my_z --num_workers 4
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
from collections import defaultdict
from typing import List, Optional, Tuple

from ..agent.features import Features
from ..agent.replay_decoder import RACE_DICT, _pb  # noqa: F401


def z_entry(feature: Features, action_steps: List[dict], last_loop: int) -> Tuple[list, list, list, int, int]:
    """(beginning_order, cumulative_stat indices, bo_location, bo_len, loop) from decoded actions."""
    bo, cum, bo_len, bo_loc = feature.get_z(action_steps)
    return bo.tolist(), cum.nonzero().flatten().tolist(), bo_loc.tolist(), bo_len, int(last_loop)


def add_entry(lib: dict, map_name: str, race: str, born: int, entry: list) -> None:
    lib.setdefault(map_name, {}).setdefault(race, {}).setdefault(str(born), []).append(entry)


def _worker(cfg_dict, jobs, out):
    from ..utils.config import AttrDict
    from ..agent.replay_decoder import ReplayDecoder
    from ..envs.map_info import get_map_size
    dec = ReplayDecoder(AttrDict(cfg_dict))
    while True:
        path = jobs.get()
        if path is None:
            break
        try:
            if dec._ctl is None:
                dec._start()
            info = dec.replay_info(path)
            for p in range(2):
                if info['result'][p] != 'W' or info['player_type'][p] == 2:
                    continue
                dec._map_size = get_map_size(info['map_name'])
                actions = dec._collect_actions(os.path.abspath(path), p + 1, info['game_steps'])
                if not actions:
                    continue
                ctl = dec._ctl
                ctl.start_replay(_pb().RequestStartReplay(replay_path=os.path.abspath(path),
                                                          options=dec._interface(dec._map_size),
                                                          observed_player_id=p + 1))
                feature = Features(ctl.game_info(), ctl.observe(), cfg_dict)
                steps = [{'action_info': feature.reverse_raw_action(a, [])[0]} for a in dec._filter.run(actions)]
                bo, cum, bo_loc, bo_len, loop = z_entry(feature, steps, actions[-1].game_loop)
                if bo_len >= 10:
                    out.put((info['map_name'], info['race'][p], feature.home_born_location, [bo, cum, bo_loc, loop]))
        except Exception as e:  # noqa: BLE001
            print(f'[gen_z] {path}: {e}')
    dec.close()
    out.put(None)


def main(argv=None):
    ap = argparse.ArgumentParser(description='gen_z')
    ap.add_argument('--data', required=True, help='replay directory or a file with replay paths')
    ap.add_argument('--name', required=True, help='output Z file name (without .json)')
    ap.add_argument('--out_dir', default=os.path.join(os.path.dirname(__file__), '..', 'lib', 'data'))
    ap.add_argument('--num_workers', type=int, default=1)
    ap.add_argument('--parse_race', default='Z')
    args = ap.parse_args(argv)
    from ..learner.replay_dataloader import replay_paths
    cfg = {'learner': {'data': {'parse_race': list(args.parse_race), 'filter_action': True}}, 'feature': {}}
    ctx = mp.get_context('spawn')
    jobs, out = ctx.Queue(), ctx.Queue()
    for p in replay_paths(args.data):
        jobs.put(p)
    procs = []
    for _ in range(args.num_workers):
        jobs.put(None)
        pr = ctx.Process(target=_worker, args=(cfg, jobs, out), daemon=True)
        pr.start()
        procs.append(pr)
    lib: dict = {}
    done = n = 0
    path = os.path.join(args.out_dir, f'{args.name}.json')
    while done < args.num_workers:
        item = out.get()
        if item is None:
            done += 1
            continue
        add_entry(lib, *item)
        n += 1
        if n % 10 == 0:
            json.dump(lib, open(path, 'w'))
    json.dump(lib, open(path, 'w'))
    print(f'{n} Z entries written to {os.path.abspath(path)}')


if __name__ == '__main__':
    main()
