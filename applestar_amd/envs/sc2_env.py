"""Real StarCraft II environment (``distar/envs/env.py:96-503``) on top of the in-house launcher and
websocket RPC client (``envs/sc2``).  Requires the SC2 binary (``$SC2PATH``) and the
``s2clientprotocol`` message classes; everything else is self-contained.

Contract identical to :class:`~applestar_amd.envs.fake_env.FakeSC2Env`:
``reset() -> (obs, game_info, map_name)``, ``step(actions) -> (obs, reward, done)`` with
``obs[idx] = {'raw_obs', 'opponent_obs', 'action_result'}``.  Behaviour kept from the reference:
raw interface with the feature minimap at the map's playable size (``:150-177``), launch retried
x10 (``:179-209``), create/join with reserved ports (``:211-274``), SC2 restarted every 10 episodes
(``:309-311``), per-agent ``skip_steps`` scheduling plus a random 0-3 loop latency in non-realtime
mode (``:333-375``), outcome from ``player_result`` (``:377-455``), replay saved on episode end.
"""
from __future__ import annotations

import os
import random
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List

from .map_info import MAPS, get_map_size
from .sc2.launcher import SC2Process, pick_ports, map_path, DEFAULT_VERSION

RANDOM_MAPS = ['KairosJunction', 'KingsCove', 'NewRepugnancy']
MAX_STEP_COUNT = 524000
BOT_DIFFICULTY = {i: i + 1 for i in range(11)}  # bot0..bot10 -> VeryEasy..CheatInsane (sc2api Difficulty)
RESULTS = {1: 1, 2: -1, 3: 0, 4: 0}            # Victory, Defeat, Tie, Undecided


def _pb():
    from s2clientprotocol import sc2api_pb2, common_pb2, raw_pb2
    return sc2api_pb2, common_pb2, raw_pb2


def find_sc2_binary():
    from .sc2.launcher import find_sc2_binary as f
    return f(DEFAULT_VERSION)


class SC2Env:
    def __init__(self, cfg):
        env = cfg['env'] if 'env' in cfg else cfg
        self._cfg = env
        self._whole_cfg = cfg
        self._player_ids = list(env.get('player_ids', ['agent1', 'bot7']))
        self._races = list(env.get('races', ['zerg', 'zerg']))
        self._human = any('human' in p for p in self._player_ids)
        self._agent_slots = [i for i, p in enumerate(self._player_ids) if 'bot' not in p]
        self._num_agents = len(self._agent_slots)
        name = env.get('map_name', 'KairosJunction')
        self._ori_map_name, self._born_location = (name.split('_') + [None])[:2] if '_' in name else (name, None)
        self._realtime = bool(env.get('realtime', False))
        self._save_replay_episodes = int(env.get('save_replay_episodes', 0))
        self._replay_dir = env.get('replay_dir', '.')
        seed = env.get('random_seed', None)
        self._seed = None if seed in (None, 'none') else int(seed)
        self._episode_length = int(env.get('game_steps_per_episode', 100000))
        self._version = env.get('version', DEFAULT_VERSION)
        self._update_both_obs = bool(env.get('update_both_obs', False)) and not self._human
        self._delay_weights = env.get('random_delay_weights', [0, 0.7, 0.2, 0.1])
        self._map_size_res = env.get('map_size_resolutions', [True, True])
        self._minimap_res = env.get('minimap_resolutions', [[160, 152], [160, 152]])
        self._procs: List[SC2Process] = []
        self._controllers = None
        self._ports: List[int] = []
        self._episode_count = 0
        self._pool = ThreadPoolExecutor(max_workers=max(2, self._num_agents))
        self._done = True

    # ---------------------------------------------------------------- setup
    def _interface(self, i: int):
        sc_pb, _, _ = _pb()
        mx, my = get_map_size(self._map_name)
        opt = sc_pb.InterfaceOptions(raw=True, show_cloaked=False, show_burrowed_shadows=False,
                                     show_placeholders=False, raw_affects_selection=self._human,
                                     raw_crop_to_playable_area=True, score=True)
        opt.feature_layer.width = 24
        opt.feature_layer.resolution.x = 1
        opt.feature_layer.resolution.y = 1
        if self._map_size_res[i]:
            opt.feature_layer.minimap_resolution.x, opt.feature_layer.minimap_resolution.y = mx, my
        else:
            opt.feature_layer.minimap_resolution.x, opt.feature_layer.minimap_resolution.y = self._minimap_res[i]
        opt.feature_layer.crop_to_playable_area = True
        return opt

    def _launch(self):
        from .sc2.controller import RemoteController
        last = None
        for attempt in range(10):
            try:
                self._ports = pick_ports(self._num_agents * 2) if self._num_agents > 1 else []
                self._procs = [SC2Process(self._version, full_screen=(self._human and i == 1))
                               for i in range(self._num_agents)]
                self._controllers = [RemoteController(p.host, p.port) for p in self._procs]
                return
            except Exception as e:  # noqa: BLE001 - retried like the reference
                last = e
                self.close()
                time.sleep(2)
        raise RuntimeError(f'SC2 launch failed 10 times: {last}')

    def _create_join(self):
        sc_pb, common_pb, _ = _pb()
        create = sc_pb.RequestCreateGame(disable_fog=False, realtime=self._realtime)
        path = MAPS[self._map_name][1]
        if self._born_location is not None:
            path = path.replace('.SC2Map', f'_{self._born_location}.SC2Map')
        create.local_map.map_path = map_path(path)
        if self._seed is not None:
            create.random_seed = self._seed
        for i, pid in enumerate(self._player_ids):
            if 'bot' in pid:
                lvl = int(pid.split('bot')[1])
                create.player_setup.add(type=sc_pb.Computer, race=common_pb.Race.Value(self._races[i].capitalize()),
                                        difficulty=BOT_DIFFICULTY[lvl])
            else:
                create.player_setup.add(type=sc_pb.Participant)
        host = self._controllers[1] if self._num_agents > 1 else self._controllers[0]
        host.create_game(create)
        joins = []
        for k, slot in enumerate(self._agent_slots):
            join = sc_pb.RequestJoinGame(options=self._interface(k))
            join.race = common_pb.Race.Value(self._races[slot].capitalize())
            join.player_name = self._player_ids[slot][:32]
            if self._ports:
                join.shared_port = 0
                join.server_ports.game_port, join.server_ports.base_port = self._ports[0], self._ports[1]
                for j in range(self._num_agents - 1):
                    join.client_ports.add(game_port=self._ports[2 * j + 2], base_port=self._ports[2 * j + 3])
            joins.append(join)
        list(self._pool.map(lambda cj: cj[0].join_game(cj[1]), zip(self._controllers, joins)))
        self._game_info = list(self._pool.map(lambda c: c.game_info(), self._controllers))

    # ---------------------------------------------------------------- API
    def reset(self, players=None):
        if players is not None:
            self._player_ids = list(players)
        self._map_name = random.choice(RANDOM_MAPS) if self._ori_map_name == 'random' else self._ori_map_name
        if self._controllers is None or (self._episode_count + 1) % 10 == 0:  # restart to bound SC2 memory
            self.close()
            self._launch()
        elif self._episode_count:
            list(self._pool.map(lambda c: c.leave(), self._controllers))
        self._create_join()
        self._episode_count += 1
        self._episode_steps = 0
        self._next_obs_step = [0] * self._num_agents
        if self._human:
            self._next_obs_step[1] = 9999999
        self._action_result = [[0] for _ in range(self._num_agents)]
        self._obs = [None] * self._num_agents
        self._done = False
        obs, _, _ = self._observe(0)
        return obs, {i: g for i, g in enumerate(self._game_info)}, self._map_name

    def step(self, actions: Dict[int, list]):
        if self._done:
            return self.reset()
        sc_pb, _, _ = _pb()
        max_skip = 0
        reqs = {}
        for slot in range(self._num_agents):
            if slot not in actions:
                continue
            cmds, skip = self.transform_action(actions[slot])
            reqs[slot] = cmds
            self._next_obs_step[slot] = self._episode_steps + skip
            max_skip = max(max_skip, skip)
        if not self._realtime and max_skip < 4 and not self._controllers[0].status_ended:
            rs = random.choices(range(len(self._delay_weights)), weights=self._delay_weights)[0]
            if rs:
                list(self._pool.map(lambda c: c.step(rs), self._controllers))
                self._episode_steps += rs
        for slot, cmds in reqs.items():
            if cmds and not self._controllers[0].status_ended:
                res = self._controllers[slot].actions(sc_pb.RequestAction(actions=cmds))
                if res is not None and len(res.result):
                    self._action_result[slot] = list(res.result)
        target = max(min(self._next_obs_step), self._episode_steps)
        if not self._controllers[0].status_ended and target > self._episode_steps:
            list(self._pool.map(lambda c: c.step(target - self._episode_steps), self._controllers))
        return self._observe(target)

    def _observe(self, target: int):
        due = [i for i in range(self._num_agents) if self._next_obs_step[i] <= target]
        if self._human:
            due = [0]
        idx = list(range(self._num_agents)) if self._update_both_obs else due
        obs = list(self._pool.map(lambda i: self._controllers[i].observe(target_game_loop=target), idx))
        for i, o in zip(idx, obs):
            self._obs[i] = o
        loop = self._obs[idx[0]].observation.game_loop if idx else self._episode_steps
        outcome = [0] * self._num_agents
        done = any(o is not None and len(o.player_result) for o in self._obs)
        if done:
            for i, o in enumerate(self._obs):
                if o is None:
                    continue
                me = o.observation.player_common.player_id
                for r in o.player_result:
                    if r.player_id == me:
                        outcome[i] = RESULTS.get(r.result, 0)
                    elif self._num_agents == 2:
                        outcome[1 - i] = RESULTS.get(r.result, 0)
        self._episode_steps = loop
        if loop >= min(self._episode_length, MAX_STEP_COUNT):
            done = True
        if done:
            self._done = True
            due = list(range(self._num_agents))
            if self._save_replay_episodes and self._episode_count % self._save_replay_episodes == 0:
                self.save_replay(self._replay_dir, f'{self._map_name}_{"_vs_".join(self._player_ids)}_{outcome}')
        ret = {}
        for i in due:
            ret[i] = {'raw_obs': self._obs[i], 'opponent_obs': self._obs[1 - i] if self._num_agents == 2 else None,
                      'action_result': self._action_result[i]}
        return ret, outcome, done

    def transform_action(self, actions: List[dict]):
        """Agent action dicts -> ``sc_pb.Action`` list + min skip_steps (``env.py:457-480``)."""
        sc_pb, _, raw_pb = _pb()
        from ..agent.features import transform_action as to_cmd
        out, skip = [], MAX_STEP_COUNT
        for a in actions:
            cmds, s = to_cmd(a)
            skip = min(skip, s)
            for c in cmds:
                act = sc_pb.Action()
                uc = act.action_raw.unit_command
                uc.ability_id = c.ability_id
                uc.unit_tags.extend(c.unit_tags)
                uc.queue_command = c.queue_command
                if c.target_unit_tag:
                    uc.target_unit_tag = c.target_unit_tag
                elif c.target_world_space_pos is not None:
                    uc.target_world_space_pos.x = c.target_world_space_pos.x
                    uc.target_world_space_pos.y = c.target_world_space_pos.y
                out.append(act)
        return out, (0 if skip == MAX_STEP_COUNT else skip)

    def save_replay(self, replay_dir: str, prefix: str = None) -> str:
        os.makedirs(replay_dir, exist_ok=True)
        data = self._controllers[0].save_replay()
        path = os.path.join(os.path.abspath(replay_dir),
                            f'{prefix or self._map_name}_{time.strftime("%Y-%m-%d-%H-%M-%S")}.SC2Replay')
        with open(path, 'wb') as f:
            f.write(data)
        return path

    @property
    def game_info(self):
        return {i: g for i, g in enumerate(self._game_info)}

    @property
    def map_name(self):
        return self._map_name

    def close(self):
        if self._controllers:
            for c in self._controllers:
                c.quit()
        self._controllers = None
        for p in self._procs:
            p.close()
        self._procs = []
        self._ports = []
        self._done = True
