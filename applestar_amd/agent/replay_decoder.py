"""Replay -> supervised trajectories (``distar/agent/default/replay_decoder.py:216-435``).

Two passes over a replay with an SC2 client (requires the SC2 binary + ``s2clientprotocol``):
1. fast pass at 1x1 minimap resolution stepping 50 loops at a time, collecting the observed player's
   raw actions (camera moves dropped), optionally de-spammed by :class:`FilterActions`;
2. full-resolution pass that observes right before each action: ``transform_obs`` +
   ``reverse_raw_action`` -> one step dict per action with ``delay`` = loops until the next action
   (clamped to ``MAX_DELAY - 1``) and the last-action / last-selection scalars the agent also feeds.
The Z (build order, cumulative stat, build-order locations) is computed from the filtered actions
and broadcast to every step (``:337-347``).  The SC2 version is taken from the replay itself
(``RequestReplayInfo.base_build``) — the reference parses the MPQ header with ``mpyq``; here the
client is (re)started only when the build changes, or every 10 replays (``:383-390``).
"""
from __future__ import annotations

import os
import random
import time
import traceback
from typing import List, Optional

import torch

from ..envs.map_info import LOCALIZED_BNET_NAME_TO_NAME_LUT, get_map_size
from ..lib.features import MAX_DELAY
from ..lib.game_data import NUM_UNIT_TYPES, ACTIONS
from .features import Features

RACE_DICT = {1: 'terran', 2: 'zerg', 3: 'protoss', 4: 'random'}
RESULT_DICT = {1: 'W', 2: 'L', 3: 'D', 4: 'U'}
# neutral resource / rock unit types whose tags change between passes (matched by position)
_RESOURCE_TYPES = {665, 666, 341, 1961, 483, 884, 885, 796, 797, 146, 147, 608, 880, 344, 881, 342}
_TARGET_NAMES = ('Train_', 'Research_', 'Morph_')


def _pb():
    from s2clientprotocol import sc2api_pb2
    return sc2api_pb2


def resource_tags(obs) -> dict:
    return {u.tag: (u.pos.x, u.pos.y) for u in obs.observation.raw_data.units if u.unit_type in _RESOURCE_TYPES}


def fix_missed_target(obs, action, saved: dict):
    """Re-target a command whose resource target tag no longer exists (same position, new tag)."""
    ar = action.action_raw
    if ar.HasField('unit_command') and ar.unit_command.HasField('target_unit_tag'):
        t = ar.unit_command.target_unit_tag
        live = {u.tag for u in obs.observation.raw_data.units}
        if t not in live and t in saved:
            for u in obs.observation.raw_data.units:
                if (u.pos.x, u.pos.y) == saved[t]:
                    ar.unit_command.target_unit_tag = u.tag
                    break
    return action


class FilterActions:
    """Optional de-spam of production commands: a train / research / morph command repeated for the
    same units within ``max_loop`` game loops is kept once (the reference checks unit-count deltas
    between observations; this keeps the same intent with the command stream alone)."""

    def __init__(self, enabled: bool = False, max_loop: int = 4):
        self.enabled = enabled
        self.max_loop = max_loop
        self._target = {a['general_ability_id'] for a in ACTIONS
                        if a['general_ability_id'] and a['name'].startswith(_TARGET_NAMES)}

    @staticmethod
    def _key(a):
        ar = a.action_raw
        uc = ar.unit_command if ar.HasField('unit_command') else ar.toggle_autocast
        return uc.ability_id, tuple(sorted(uc.unit_tags))

    def run(self, actions: List) -> List:
        if not self.enabled:
            return list(actions)
        out, last = [], {}
        for a in actions:
            k = self._key(a)
            if k[0] in self._target and k in last and a.game_loop - last[k] <= self.max_loop:
                continue
            last[k] = a.game_loop
            out.append(a)
        return out


class ReplayDecoder:
    def __init__(self, cfg):
        from ..envs.sc2.launcher import SC2Process  # noqa: F401 (fail early without SC2 support code)
        d = cfg.learner.data
        self._cfg = cfg
        self._parse_race = [r.upper() for r in d.get('parse_race', ['Z'])]
        self._filter = FilterActions(bool(d.get('filter_action', False)))
        self._min_len = int(cfg.get('minimum_action_length', 128))
        self._proc = None
        self._ctl = None
        self._build = None
        self._count = 0

    # ---------------------------------------------------------------- SC2 process
    def _start(self, version: Optional[str] = None):
        from ..envs.sc2.launcher import SC2Process
        from ..envs.sc2.controller import RemoteController
        self._close()
        for i in range(10):
            try:
                self._proc = SC2Process(version)
                self._ctl = RemoteController(self._proc.host, self._proc.port)
                return True
            except Exception as e:  # noqa: BLE001
                print(f'[replay] SC2 start failed ({i}): {e}')
                self._close()
        return False

    def _close(self):
        if self._ctl is not None:
            self._ctl.quit()
        if self._proc is not None:
            self._proc.close()
        self._ctl = self._proc = None

    def _version_for(self, base_build: int) -> Optional[str]:
        from ..envs.sc2.launcher import VERSIONS
        for v in VERSIONS.values():
            if v.build_version == base_build:
                return v.game_version
        return None

    # ---------------------------------------------------------------- decode
    def _interface(self, minimap):
        sc_pb = _pb()
        opt = sc_pb.InterfaceOptions(raw=True, score=False, raw_crop_to_playable_area=True)
        opt.feature_layer.width = 1
        opt.feature_layer.crop_to_playable_area = True
        opt.feature_layer.resolution.x = opt.feature_layer.resolution.y = 1
        opt.feature_layer.minimap_resolution.x, opt.feature_layer.minimap_resolution.y = minimap
        return opt

    def _collect_actions(self, path: str, player: int, loops: int):
        sc_pb = _pb()
        self._ctl.start_replay(sc_pb.RequestStartReplay(replay_path=path, options=self._interface((1, 1)),
                                                        observed_player_id=player))
        cur, actions = 0, []
        while cur < loops:
            nxt = min(loops, cur + 50)
            self._ctl.step(nxt - cur)
            cur = nxt
            ob = self._ctl.observe()
            actions += [a for a in ob.actions if a.HasField('action_raw') and not a.action_raw.HasField('camera_move')]
            if len(ob.player_result):
                break
        return actions

    def _decode(self, path: str, player: int, info: dict) -> List[dict]:
        sc_pb = _pb()
        actions = self._collect_actions(path, player, info['game_steps'])
        if not actions:
            return []
        filtered = self._filter.run(actions)
        self._ctl.start_replay(sc_pb.RequestStartReplay(replay_path=path, options=self._interface(self._map_size),
                                                        observed_player_id=player, disable_fog=False))
        raw = self._ctl.observe()
        saved = resource_tags(raw)
        feature = Features(self._ctl.game_info(), raw, self._cfg)
        last_su, last_tu = None, None
        last_delay = last_at = last_q = torch.tensor(0, dtype=torch.long)
        enemy_bool = torch.zeros(NUM_UNIT_TYPES, dtype=torch.uint8)
        self._ctl.step(max(actions[0].game_loop - 2, 0))
        traj = []
        for i, a in enumerate(actions):
            delay = random.randint(0, MAX_DELAY) if i == len(actions) - 1 else actions[i + 1].game_loop - a.game_loop
            raw = self._ctl.observe()
            if len(raw.player_result):
                break
            if delay > 0:
                self._ctl.step(delay)
            a = fix_missed_target(raw, a, saved)
            step = feature.transform_obs(raw)
            tags = step['game_info']['tags']
            index = {t: k for k, t in enumerate(tags)}
            n = int(step['entity_num'])
            lsu = torch.zeros(n, dtype=torch.int8)
            ltu = torch.zeros(n, dtype=torch.int8)
            for t in last_su or ():
                if t in index:
                    lsu[index[t]] = 1
            if last_tu is not None and last_tu in index:
                ltu[index[last_tu]] = 1
            step['entity_info']['last_selected_units'] = lsu
            step['entity_info']['last_targeted_unit'] = ltu
            si = step['scalar_info']
            si['last_delay'], si['last_action_type'], si['last_queued'] = last_delay, last_at, last_q
            si['enemy_unit_type_bool'] = (enemy_bool | si['enemy_unit_type_bool']).to(torch.uint8)
            act, mask, su_num, last_su, last_tu, invalid = feature.reverse_raw_action(a, tags)
            if invalid:
                continue
            act['delay'] = torch.tensor(delay, dtype=torch.long).clamp_(max=MAX_DELAY - 1)
            last_at, last_delay, last_q = act['action_type'], act['delay'], act['queued']
            enemy_bool = si['enemy_unit_type_bool']
            step.pop('game_info')
            step.update({'action_info': act, 'action_mask': mask, 'selected_units_num': su_num})
            traj.append(step)
        z_steps = [{'action_info': feature.reverse_raw_action(a, [])[0]} for a in filtered]
        bo, cum, _, bo_loc = feature.get_z(z_steps)
        for s in traj:
            s['scalar_info']['beginning_order'] = bo
            s['scalar_info']['cumulative_stat'] = cum
            s['scalar_info']['bo_location'] = bo_loc
        return traj

    def replay_info(self, path: str) -> dict:
        r = self._ctl.replay_info(open(path, 'rb').read())
        return {'race': [RACE_DICT[p.player_info.race_actual] for p in r.player_info],
                'result': [RESULT_DICT[p.player_result.result] for p in r.player_info],
                'player_type': [p.player_info.type for p in r.player_info],
                'mmr': [p.player_mmr for p in r.player_info],
                'map_name': LOCALIZED_BNET_NAME_TO_NAME_LUT.get(r.map_name, r.map_name),
                'game_steps': r.game_duration_loops, 'base_build': r.base_build}

    def run(self, path: str, player_index: int) -> Optional[List[dict]]:
        path = path.strip()
        try:
            if self._ctl is None and not self._start():
                return None
            info = self.replay_info(path)
            version = self._version_for(info['base_build'])
            if info['base_build'] != self._build or self._count >= 10:
                if not self._start(version):
                    return None
                self._build, self._count = info['base_build'], 0
            if info['player_type'][player_index] == 2:  # computer
                return None
            if info['race'][player_index][0].upper() not in self._parse_race:
                return None
            self._map_size = get_map_size(info['map_name'])
            self._count += 1
            t0 = time.time()
            data = self._decode(os.path.abspath(path), player_index + 1, info)
            if len(data) < self._min_len:
                return None
            print(f'[replay] {path}: {len(data)} actions in {time.time() - t0:.1f}s')
            return data
        except Exception as e:  # noqa: BLE001 - a bad replay must not kill the worker
            print(f'[replay] decode failed for {path}: {e}\n{traceback.format_exc()}')
            self._close()
            self._build = None
            return None

    def close(self):
        self._close()
