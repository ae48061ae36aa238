"""FakeSC2Env: a 2-player SC2 stand-in that emits raw observations in the API schema.

There is no SC2 binary on the MI355X boxes, so every actor / inference / end-to-end test runs on
this env (SURVEY §7.1 ``FakeSC2Env``).  It keeps the exact contract of ``distar/envs/env.py``
(``reset() -> (obs, game_info, map_name)``, ``step(actions) -> (obs, reward, done)``,
``obs[idx] = {'raw_obs', 'opponent_obs', 'action_result'}``, per-agent ``skip_steps`` scheduling,
the random 0-3 loop latency weights ``[0, .7, .2, .1]`` in non-realtime mode, episode length cut),
and produces a plausible, slowly growing unit population so featurization, varlen batching and the
model see realistic entity counts (tens early, hundreds later, capped at 512 after cargo).

Game dynamics are synthetic: actions are accepted (``action_result`` Success with a small error
rate), units appear/die at random, and by default the outcome is decided by accumulated "army value" with
noise - no action influences it.

Learnable mode (``env.fake_learnable: true``) makes the actions matter, so a training run can show that the
whole pipeline learns (agent -> inference server -> data plane -> HBM ring -> learner -> model push -> actor):
a fixed quarter of the 327 action types is "rewarded" (:data:`REWARDED_ACTION_TYPES`); an episode lasts
``fake_episode_agent_steps`` agent steps; player i's rate r_i is the fraction of its steps whose action type is
rewarded (a bot plays ``fake_bot_rate``, the rate of a uniform policy); player 1 wins with probability
clip(0.5 + r_1 - r_2, 0, 1).  A uniform policy wins half its games against the bot, a policy that learned the
set wins all of them.  ``fake_stats_path``: every finished episode appends one JSON line (time, episode, each
agent slot's rate and result) - the actor-side learning curve.
"""
from __future__ import annotations

import json
import os
import random
import time
from typing import Dict, List, Optional

import numpy as np

from . import raw as R
from .map_info import get_map_size
from ..agent.features import transform_action, MINIMAP_LAYERS
from ..lib.game_data import UNIT_TYPES, UNIT_SPECIFIC_ABILITIES, ABILITY_TO_QUEUE_ACTION, BUFFS, ACTIONS
from ..lib.game_data import FUNC_ID_TO_ACTION_TYPE_DICT

RANDOM_MAPS = ['KairosJunction', 'KingsCove', 'NewRepugnancy']  # env.py:64
POSSIBLE_RESULTS = {R.RESULT_VICTORY: 1, R.RESULT_DEFEAT: -1, R.RESULT_TIE: 0, R.RESULT_UNDECIDED: 0}
BASES = {'zerg': 86, 'terran': 18, 'protoss': 59}
WORKERS = {'zerg': 104, 'terran': 45, 'protoss': 84}
_QUEUE_ABILITIES = [a for a in range(len(ABILITY_TO_QUEUE_ACTION)) if int(ABILITY_TO_QUEUE_ACTION[a]) > 0]
_ORDER_ABILITIES = [a for a in UNIT_SPECIFIC_ABILITIES if a]
_UNIT_POOL = [u for u in UNIT_TYPES if u not in (86, 18, 59)]
_BUFF_POOL = [b for b in BUFFS if b]
# learnable mode: the rewarded action types (a fixed quarter of the 327, no_op excluded)
REWARDED_ACTION_TYPES = frozenset(a for a in range(len(ACTIONS)) if a % 4 == 1)


class _PlayerState:
    def __init__(self, player_id: int, race: str, base_xy, rng: np.random.Generator, tag_base: int):
        self.player_id = player_id
        self.race = race
        self.rng = rng
        self.tag = tag_base
        self.units: List[R.Unit] = []
        self.army_value = 0.0
        self.upgrades: List[int] = []
        self.killed = 0.0
        self.base = self._mk(BASES[race], base_xy, build=1.0)
        for _ in range(12):
            self._mk(WORKERS[race], self._near(base_xy, 6))

    def _near(self, xy, r):
        return (float(xy[0] + self.rng.uniform(-r, r)), float(xy[1] + self.rng.uniform(-r, r)))

    def _mk(self, unit_type, xy, build=1.0):
        self.tag += 1
        hp = float(self.rng.integers(20, 1500))
        emax = float(self.rng.choice([0, 200]))
        u = R.Unit(tag=self.tag, unit_type=int(unit_type), alliance=1, owner=self.player_id,
                   pos=R.Point(*xy), build_progress=build, health=hp * float(self.rng.uniform(0.2, 1.0)),
                   health_max=hp, energy_max=emax, energy=float(self.rng.uniform(0, emax)),
                   is_powered=bool(self.rng.integers(0, 2)), weapon_cooldown=float(self.rng.integers(0, 20)),
                   assigned_harvesters=int(self.rng.integers(0, 16)), is_active=bool(self.rng.integers(0, 2)),
                   attack_upgrade_level=int(self.rng.integers(0, 4)), display_type=1)
        if self.rng.random() < 0.3:
            k = int(self.rng.integers(1, 5))
            u.orders = [R.UnitOrder(ability_id=int(self.rng.choice(_ORDER_ABILITIES)),
                                    progress=float(self.rng.random()))]
            u.orders += [R.UnitOrder(ability_id=int(self.rng.choice(_QUEUE_ABILITIES)),
                                     progress=float(self.rng.random())) for _ in range(k - 1)]
        if self.rng.random() < 0.1:
            u.buff_ids = [int(self.rng.choice(_BUFF_POOL))]
        if self.rng.random() < 0.02:
            u.passengers = [R.PassengerUnit(tag=self.tag + 10_000_000 + i, unit_type=int(self.rng.choice(_UNIT_POOL)),
                                            health=40.0, health_max=40.0) for i in range(int(self.rng.integers(1, 4)))]
            u.cargo_space_taken = len(u.passengers)
            u.cargo_space_max = 8
        self.units.append(u)
        return u

    def tick(self, loops: int, map_xy):
        # grow / shrink the population at a rate proportional to elapsed game loops
        n_new = self.rng.poisson(0.02 * loops)
        for _ in range(int(n_new)):
            if len(self.units) > 420:
                break
            ut = int(self.rng.choice(_UNIT_POOL))
            self._mk(ut, (float(self.rng.uniform(1, map_xy[0] - 1)), float(self.rng.uniform(1, map_xy[1] - 1))),
                     build=float(self.rng.choice([1.0, self.rng.random()])))
            self.army_value += 1.0
        n_dead = self.rng.poisson(0.008 * loops)
        for _ in range(int(n_dead)):
            if len(self.units) > 14:
                self.units.pop(int(self.rng.integers(1, len(self.units))))
                self.army_value -= 0.5
        for u in self.units:
            if u.orders and self.rng.random() < 0.2:
                u.orders = u.orders[1:]
        if self.rng.random() < 0.002 * loops and len(self.upgrades) < 20:
            self.upgrades.append(int(self.rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12])))


class FakeSC2Env:
    """Drop-in replacement for ``SC2Env`` with synthetic dynamics (no SC2 binary)."""

    def __init__(self, cfg):
        env = cfg['env'] if 'env' in cfg else cfg
        self._cfg = env
        self._player_ids = list(env.get('player_ids', ['agent1', 'bot7']))
        self._races = list(env.get('races', ['zerg', 'zerg']))
        self._ori_map_name = env.get('map_name', 'KairosJunction').split('_')[0]
        self._map_name = self._ori_map_name
        self._episode_length = int(env.get('game_steps_per_episode', 100000))
        self._realtime = bool(env.get('realtime', False))
        self._random_delay_weights = env.get('random_delay_weights', [0, 0.7, 0.2, 0.1])
        self._error_rate = float(env.get('fake_action_error_rate', 0.05))
        seed = env.get('random_seed', None)
        self._seed = None if seed in (None, 'none') else int(seed)
        self._agent_slots = [i for i, p in enumerate(self._player_ids) if 'bot' not in p]
        self._num_agents = len(self._agent_slots)
        self._learnable = bool(env.get('fake_learnable', False))
        self._ep_agent_steps = int(env.get('fake_episode_agent_steps', 32))
        self._bot_rate = float(env.get('fake_bot_rate', len(REWARDED_ACTION_TYPES) / len(ACTIONS)))
        self._stats_path = env.get('fake_stats_path', None)
        self._episode_count = 0
        self._rng = np.random.default_rng(self._seed)
        self._done = True

    # ---------------------------------------------------------------- helpers
    def _planes(self):
        mx, my = self._map_xy
        rng = self._rng
        h = rng.integers(0, 256, (my, mx), dtype=np.uint8)
        self._static = {'height_map': h,
                        'pathable': (rng.random((my, mx)) < 0.7).astype(np.uint8),
                        'buildable': (rng.random((my, mx)) < 0.4).astype(np.uint8)}

    def _minimap(self, me: _PlayerState, opp: _PlayerState) -> R.MinimapRenders:
        mx, my = self._map_xy
        rng = self._rng
        pr = np.zeros((my, mx), dtype=np.uint8)
        for u in me.units:
            pr[min(int(my - u.pos.y), my - 1) if u.pos.y > 0 else my - 1, min(int(u.pos.x), mx - 1)] = 1
        for u in opp.units[::3]:
            pr[min(int(my - u.pos.y), my - 1) if u.pos.y > 0 else my - 1, min(int(u.pos.x), mx - 1)] = 4

        def img(a):
            return R.ImageData(bits_per_pixel=8, size=R.Size2D(mx, my), data=np.ascontiguousarray(a).tobytes())
        return R.MinimapRenders(height_map=img(self._static['height_map']),
                                visibility_map=img(rng.integers(0, 3, (my, mx), dtype=np.uint8)),
                                creep=img((rng.random((my, mx)) < 0.1).astype(np.uint8)),
                                player_relative=img(pr),
                                alerts=img(np.zeros((my, mx), np.uint8)),
                                pathable=img(self._static['pathable']),
                                buildable=img(self._static['buildable']))

    def _observation(self, i: int, results=None) -> R.ResponseObservation:
        me, opp = self._players[i], self._players[1 - i]
        units = [u for u in me.units]
        # a visible subset of the enemy (alliance 4) and neutral resources (alliance 3)
        vis = opp.units[3::3]  # the enemy base (index 0) stays hidden
        units += [R.Unit(**{**u.__dict__, 'alliance': 4, 'orders': [], 'passengers': [], 'cargo_space_taken': 0,
                            'cargo_space_max': 0, 'assigned_harvesters': 0}) for u in vis]
        units += self._neutral
        effects = []
        if self._rng.random() < 0.1:
            effects.append(R.Effect(effect_id=int(self._rng.integers(1, 13)), owner=2,
                                    pos=[R.Point(float(self._rng.uniform(0, self._map_xy[0])),
                                                 float(self._rng.uniform(1, self._map_xy[1])))]))
        pc = R.PlayerCommon(player_id=me.player_id, minerals=int(self._rng.integers(0, 2000)),
                            vespene=int(self._rng.integers(0, 1000)), food_used=min(200, len(me.units)),
                            food_cap=200, food_workers=12, army_count=max(0, len(me.units) - 13),
                            larva_count=int(self._rng.integers(0, 10)))
        sd = R.ScoreDetails(killed_minerals=R.CategoryScoreDetails(army=me.killed),
                            killed_vespene=R.CategoryScoreDetails(army=me.killed * 0.3))
        ob = R.Observation(game_loop=self._game_loop, player_common=pc,
                           raw_data=R.ObservationRaw(player=R.PlayerRaw(list(me.upgrades)), units=units,
                                                     effects=effects),
                           feature_layer_data=R.FeatureLayerData(self._minimap(me, opp)),
                           score=R.Score(sd))
        resp = R.ResponseObservation(observation=ob)
        if results is not None:
            resp.player_result = results
        return resp

    # ---------------------------------------------------------------- API
    def reset(self, players=None):
        if players is not None:
            self._player_ids = list(players)
        self._episode_count += 1
        if self._ori_map_name == 'random':
            self._map_name = random.choice(RANDOM_MAPS)
        self._map_xy = get_map_size(self._map_name)
        mx, my = self._map_xy
        locs = [(mx * 0.2, my * 0.8), (mx * 0.8, my * 0.2)]
        self._players = [_PlayerState(i + 1, self._races[i], locs[i], self._rng, (i + 1) * 1_000_000)
                         for i in range(2)]
        self._neutral = []
        for k in range(16):
            x, y = self._rng.uniform(2, mx - 2), self._rng.uniform(2, my - 2)
            self._neutral.append(R.Unit(tag=5_000_000 + k, unit_type=341 if k % 4 else 342, alliance=3, owner=16,
                                        pos=R.Point(float(x), float(y)), mineral_contents=1800 if k % 4 else 0,
                                        vespene_contents=0 if k % 4 else 2250, display_type=2))
        self._planes()
        self._game_loop = 0
        self._next_obs_step = [0] * self._num_agents
        self._action_result = [[0] for _ in range(self._num_agents)]
        self._steps = [0] * self._num_agents            # learnable mode: agent steps / rewarded steps per slot
        self._rewarded = [0] * self._num_agents
        self._done = False
        self._game_info = []
        for slot in range(self._num_agents):
            i = self._agent_slots[slot]
            gi = R.GameInfo(map_name=self._map_name,
                            player_info=[R.PlayerInfo(player_id=p + 1, race_requested=R.RACE[self._races[p]],
                                                      type=R.PLAYER_TYPE_COMPUTER if 'bot' in self._player_ids[p]
                                                      else R.PLAYER_TYPE_PARTICIPANT) for p in range(2)],
                            start_raw=R.StartRaw(map_size=R.Size2D(mx, my),
                                                 start_locations=[R.Point(*locs[1 - i])]))
            self._game_info.append(gi)
        obs, _, _ = self._observe()
        return obs, {idx: g for idx, g in enumerate(self._game_info)}, self._map_name

    def step(self, actions: Dict[int, list]):
        if self._done:
            return self.reset()
        max_skip = 0
        for slot in range(self._num_agents):
            if slot in actions:
                cmds, skip = [], 0
                for a in actions[slot]:
                    c, s = transform_action(a)
                    cmds += c
                    skip = max(skip, s) if skip else s
                if actions[slot]:
                    self._steps[slot] += 1
                    at = FUNC_ID_TO_ACTION_TYPE_DICT.get(actions[slot][0].get('func_id'), 0)
                    self._rewarded[slot] += int(at in REWARDED_ACTION_TYPES)
                self._next_obs_step[slot] = self._game_loop + max(1, skip)
                max_skip = max(max_skip, skip)
                ok = self._rng.random() > self._error_rate
                self._action_result[slot] = [1 if ok else int(self._rng.integers(2, 214))]
        random_step = 0
        if not self._realtime and max_skip < 4:
            random_step = random.choices(range(len(self._random_delay_weights)), weights=self._random_delay_weights)[0]
        target = max(min(self._next_obs_step), self._game_loop + random_step)
        elapsed = target - self._game_loop
        for p in self._players:
            p.tick(elapsed, self._map_xy)
        self._players[0].killed += self._rng.random() * elapsed
        self._players[1].killed += self._rng.random() * elapsed
        self._game_loop = target
        return self._observe()

    def _rates(self):
        """Learnable mode: each player's rewarded-action rate (bots: ``fake_bot_rate``)."""
        rates = [self._bot_rate, self._bot_rate]
        for slot, i in enumerate(self._agent_slots):
            rates[i] = self._rewarded[slot] / max(self._steps[slot], 1)
        return rates

    def _log_episode(self, rates, res):
        if not self._stats_path:
            return
        line = json.dumps({'t': time.time(), 'pid': os.getpid(), 'episode': self._episode_count,
                           'agent_steps': list(self._steps),
                           'rate': [round(rates[i], 4) for i in self._agent_slots],
                           'win': [int(res[i] == R.RESULT_VICTORY) for i in self._agent_slots]}) + '\n'
        fd = os.open(self._stats_path, os.O_WRONLY | os.O_APPEND | os.O_CREAT, 0o644)
        try:
            os.write(fd, line.encode())      # one O_APPEND write per line: whole lines from many env processes
        finally:
            os.close(fd)

    def _observe(self):
        done = self._game_loop >= self._episode_length or \
            (self._learnable and max(self._steps) >= self._ep_agent_steps)
        reward = [0] * self._num_agents
        results = None
        if done and self._learnable:
            rates = self._rates()
            p1_wins = self._rng.random() < min(1.0, max(0.0, 0.5 + rates[0] - rates[1]))
        elif done:
            a, b = self._players[0].army_value, self._players[1].army_value
            p1_wins = (a + self._rng.normal(0, 5)) >= b
        if done:
            res = [R.RESULT_VICTORY, R.RESULT_DEFEAT] if p1_wins else [R.RESULT_DEFEAT, R.RESULT_VICTORY]
            results = [R.PlayerResult(player_id=1, result=res[0]), R.PlayerResult(player_id=2, result=res[1])]
            for slot in range(self._num_agents):
                reward[slot] = POSSIBLE_RESULTS[res[self._agent_slots[slot]]]
            if self._learnable:
                self._log_episode(rates, res)
            self._done = True
        agent_slots = [s for s in range(self._num_agents) if done or self._next_obs_step[s] <= self._game_loop]
        full = {s: self._observation(self._agent_slots[s], results) for s in range(self._num_agents)}
        ret = {}
        for s in agent_slots:
            opp_obs = self._observation(1 - self._agent_slots[s], results) if self._num_agents == 1 else \
                full.get(1 - s)
            ret[s] = {'raw_obs': full[s], 'opponent_obs': opp_obs, 'action_result': self._action_result[s]}
        return ret, reward, done

    @property
    def game_info(self):
        return {i: g for i, g in enumerate(self._game_info)}

    @property
    def map_name(self):
        return self._map_name

    def save_replay(self, replay_dir, prefix=None):
        return None

    def close(self):
        self._done = True
