"""The default StarCraft II agent: per-game state, Z selection, featurization, model call,
action decoding, teacher forward, trajectory assembly and pseudo-rewards.

Behaviour follows ``distar/agent/default/agent.py`` (``Agent :92``): per-game LSTM state and last
action bookkeeping (``:162-205``), Z selection by map / race / born location with ``z_type`` and
``fake_reward_prob`` gating (``:206-317``), ``_pre_process`` (``:319-370``), ``_post_process``
(``:413-459``: indices -> ``{func_id, skip_steps, queued, unit_tags, target_unit_tag, location}`` with
the y flip ``map_h - y``), ``collect_data`` (``:541-673``: teacher forward, step data, trajectory of
``traj_len`` steps + bootstrap obs), pseudo-rewards (``:685-779``: build-order Levenshtein with
location, time-decayed cumulative Hamming, battle score delta).

MI355X design differences:
* the model call goes through an :class:`InferenceClient` when the actor batches inference on the
  GPU (one server per GPU batching every env; :mod:`applestar_amd.actor.inference`) instead of the
  reference's shared-memory slots polled with ``sleep(0.01)``;
* observation tensors stay on the host; the server moves one collated batch per call.
"""
from __future__ import annotations

import copy
import random
from collections import deque, defaultdict
from functools import partial
from typing import Dict, List, Optional

import torch

from ..lib.features import SPATIAL_SIZE, BEGINNING_ORDER_LENGTH, MAX_SELECTED_UNITS_NUM
from ..lib.game_data import (ACTIONS, NUM_UNIT_TYPES, NUM_CUMULATIVE_STAT_ACTIONS, BEGINNING_ORDER_ACTIONS,
                             CUMULATIVE_STAT_ACTIONS, QUEUE_ACTIONS, UNIT_ABILITY_TO_ACTION, UNIT_TO_CUM,
                             UPGRADE_TO_CUM, ACTION_RACE_MASK, load_z)
from ..lib.metrics import levenshtein_distance, hamming_distance, l2_distance
from ..lib.stat import Stat, CUM_DICT
from ..utils.config import AttrDict, deep_merge_dicts
from .features import Features, compute_battle_score, BASE_UNIT_TYPES
from .collate import collate_obs, decollate_output

RACE_DICT = {1: 'terran', 2: 'zerg', 3: 'protoss', 4: 'random'}
_BO_INDEX = {a: i for i, a in enumerate(BEGINNING_ORDER_ACTIONS)}
_CUM_INDEX = {a: i for i, a in enumerate(CUMULATIVE_STAT_ACTIONS)}

DEFAULT_AGENT_CONFIG = {
    'common': {'type': 'play'},
    'agent': {'z_path': '7map_filter_spine.json', 'show_Z': False, 'zero_z_exceed_loop': True,
              'extra_units': False, 'bo_zergling_num': 8, 'fake_reward_prob': 1.0, 'clip_bo': True,
              'cum_type': 'action'},
    'feature': {'zero_z_value': 1.0},
    'actor': {'job_type': 'eval_test', 'gpu_batch_inference': False, 'use_cuda': False, 'traj_len': 64},
    'env': {'realtime': False},
    'learner': {'use_value_feature': False, 'use_dapo': False, 'only_cum_action_kl': False,
                'bo_norm': 20, 'cum_norm': 30, 'battle_norm': 30},
}


class Agent:
    HAS_MODEL = True
    HAS_TEACHER_MODEL = True
    HAS_SUCCESSIVE_MODEL = False

    def __init__(self, cfg=None, env_id: int = 0, model=None, teacher_model=None, inference_client=None,
                 teacher_client=None):
        self._whole_cfg = deep_merge_dicts(DEFAULT_AGENT_CONFIG, cfg or {})
        c = self._whole_cfg
        self._job_type = c.actor.job_type
        self._z_path = c.agent.z_path
        self._bo_norm = c.learner.get('bo_norm', 20)
        self._cum_norm = c.learner.get('cum_norm', 30)
        self._battle_norm = c.learner.get('battle_norm', 30)
        self._only_cum_action_kl = c.learner.get('only_cum_action_kl', False)
        self._use_value_feature = c.learner.get('use_value_feature', False)
        self._use_dapo = c.learner.get('use_dapo', False)
        self._zero_z_value = c.feature.get('zero_z_value', 1.0)
        self._zero_z_exceed_loop = c.agent.get('zero_z_exceed_loop', False)
        self._extra_units = c.agent.get('extra_units', False)
        self._bo_zergling_num = c.agent.get('bo_zergling_num', 8)
        self._fake_reward_prob = c.agent.get('fake_reward_prob', 1.0)
        self._clip_bo = c.agent.get('clip_bo', True)
        self._cum_type = c.agent.get('cum_type', 'action')
        self._use_cuda = bool(c.actor.get('use_cuda', False)) and torch.cuda.is_available()
        self._env_id = env_id
        self._player_id = None
        self._client = inference_client
        self._teacher_client = teacher_client
        # 'policy+teacher' client: the server returns the teacher's logits for the sampled action with the policy
        # reply (one round trip per agent step); collect_data then uses the cached half
        self._merged = inference_client is not None and getattr(inference_client, 'kind', '') == 'policy+teacher'
        self._teacher_out = None
        self.z_idx = None
        if model is None and inference_client is None:
            from ..models.model import Model
            model = Model(c)
        self.model = model
        if self.model is not None:
            self.model.eval()
            if self._use_cuda:
                self.model.cuda()
        self.teacher_model = teacher_model
        if 'train' in self._job_type and teacher_model is None and teacher_client is None and not self._merged:
            from ..models.model import Model
            self.teacher_model = Model(c).eval()
        self.successive_model = None
        self._num_layers = 3
        self._hidden_size = 384
        self._reset_z_defaults()

    # ------------------------------------------------------------------ per-game state
    def _reset_z_defaults(self):
        self._target_z_loop = 99999999
        self._target_building_order = torch.zeros(0, dtype=torch.long)
        self._target_bo_location = torch.zeros(0, dtype=torch.long)
        self._target_cumulative_stat = torch.zeros(NUM_CUMULATIVE_STAT_ACTIONS, dtype=torch.float)
        self.use_cum_reward = False
        self.use_bo_reward = False
        self._exceed_flag = True
        self._old_bo_reward = torch.tensor(0.)
        self._old_cum_reward = torch.tensor(0.)
        self._total_bo_reward = torch.zeros(())
        self._total_cum_reward = torch.zeros(())

    def _zero_state(self):
        return [(torch.zeros(self._hidden_size), torch.zeros(self._hidden_size)) for _ in range(self._num_layers)]

    def reset(self, map_name: str, race: str, game_info, obs) -> None:
        self._stat_api = Stat(race)
        self._race = race
        if self.model is not None:
            self.model.race_mask = ACTION_RACE_MASK[race] if self._whole_cfg.common.type == 'play' else None
        self._map_name = map_name
        self._hidden_state = self._zero_state()
        self._last_action_type = torch.tensor(0, dtype=torch.long)
        self._last_delay = torch.tensor(0, dtype=torch.long)
        self._last_queued = torch.tensor(0, dtype=torch.long)
        self._last_selected_unit_tags = None
        self._last_target_unit_tag = None
        self._last_location = None
        self._enemy_unit_type_bool = torch.zeros(NUM_UNIT_TYPES, dtype=torch.uint8)
        self._observation = None
        self._output = None
        self._iter_count = 0
        self._success_iter_count = 0
        self._model_last_iter = 0
        self._game_step = 0
        self._behaviour_building_order: List[int] = []
        self._behaviour_bo_location: List[int] = []
        self._bo_zergling_count = 0
        self._behaviour_cumulative_stat = [0] * NUM_CUMULATIVE_STAT_ACTIONS
        self._reset_z_defaults()
        self._feature = Features(game_info, obs['raw_obs'], self._whole_cfg)
        if 'train' in self._job_type:
            self._hidden_state_backup = self._zero_state()
            self._teacher_hidden_state = self._zero_state()
            self._successive_hidden_state = self._zero_state()
            self._data_buffer = deque(maxlen=self._whole_cfg.actor.traj_len)
            self._push_count = 0
        self._select_z(obs)

    def _select_z(self, obs) -> None:
        raw_ob = obs['raw_obs']
        bases = [u for u in raw_ob.observation.raw_data.units if u.unit_type in BASE_UNIT_TYPES]
        assert len(bases) == 1, 'expected exactly one own base at game start'
        self._born_location = [bases[0].pos.x, bases[0].pos.y]
        bx = int(bases[0].pos.x)
        by = int(self._feature.map_size.y - bases[0].pos.y)
        born_str = str(bx + by * SPATIAL_SIZE[1])
        try:
            z_data = load_z(self._z_path)
        except FileNotFoundError:
            return
        pid = raw_ob.observation.player_common.player_id
        race = RACE_DICT[self._feature.requested_races[pid]]
        by_map = z_data.get(self._map_name, {}).get(race)
        if not by_map:
            return
        if born_str not in by_map:
            # unknown start position (e.g. the fake env): use the closest recorded born location
            W = SPATIAL_SIZE[1]
            born_str = min(by_map, key=lambda k: (int(k) % W - bx) ** 2 + (int(k) // W - by) ** 2)
        z_type = None
        if self.z_idx is not None:
            entry = self.z_idx.get(self._map_name, {}).get(race, {}).get(born_str)
            if not entry:
                return
            idx, z_type = random.choice(entry)
            z = by_map[born_str][idx]
        else:
            z = random.choice(by_map[born_str])
        if len(z) == 5:
            bo, cum, bo_loc, self._target_z_loop, z_type = z
        else:
            bo, cum, bo_loc, self._target_z_loop = z
        self.use_cum_reward = self.use_bo_reward = True
        if z_type is not None:
            if z_type in (2, 3):
                self.use_cum_reward = False
            if z_type in (1, 3):
                self.use_bo_reward = False
        if random.random() > self._fake_reward_prob:
            self.use_cum_reward = False
        if random.random() > self._fake_reward_prob:
            self.use_bo_reward = False
        self._bo_norm = len(bo)
        self._cum_norm = len(cum)
        self._target_building_order = torch.tensor(bo, dtype=torch.long)
        self._target_bo_location = torch.tensor(bo_loc, dtype=torch.long)
        self._target_cumulative_stat = torch.zeros(NUM_CUMULATIVE_STAT_ACTIONS, dtype=torch.float)
        self._target_cumulative_stat[torch.tensor(cum, dtype=torch.long)] = 1.0
        if self._whole_cfg.agent.get('show_Z', False):
            print(self._z_text(born_str))
        if not self._whole_cfg.env.realtime:
            self._old_bo_reward = torch.tensor(0.) if self._clip_bo else -levenshtein_distance(
                torch.as_tensor(self._behaviour_building_order, dtype=torch.long),
                self._target_building_order) / self._bo_norm
            self._old_cum_reward = -hamming_distance(
                torch.as_tensor(self._behaviour_cumulative_stat, dtype=torch.float),
                self._target_cumulative_stat) / self._cum_norm

    def _z_text(self, born_str: str) -> str:
        W = SPATIAL_SIZE[1]
        s = f'Map: {self._map_name} Race: {self._race}, Born location: {born_str}, loop: {self._target_z_loop}\n'
        s += 'Building order:\n'
        for a, loc in zip(self._target_building_order.tolist(), self._target_bo_location.tolist()):
            if a:
                s += f'  {ACTIONS[BEGINNING_ORDER_ACTIONS[a]]["name"]}, ({loc % W}, {loc // W})\n'
        s += 'Cumulative stat:\n'
        for i in torch.nonzero(self._target_cumulative_stat).flatten().tolist():
            s += f'  {ACTIONS[CUMULATIVE_STAT_ACTIONS[i]]["name"]}\n'
        return s

    # ------------------------------------------------------------------ step
    def _pre_process(self, obs) -> Dict:
        agent_obs = self._feature.transform_obs(obs['raw_obs'], padding_spatial=True,
                                                opponent_obs=obs.get('opponent_obs') if self._use_value_feature
                                                else None)
        self._game_info = agent_obs.pop('game_info')
        self._game_step = self._game_info['game_loop']
        if self._zero_z_exceed_loop and self._game_step > self._target_z_loop:
            self._exceed_flag = False
            self._target_z_loop = 99999999
        n = int(agent_obs['entity_num'])
        tags = self._game_info['tags']
        index = {t: i for i, t in enumerate(tags)}
        last_su = torch.zeros(n, dtype=torch.int8)
        last_tu = torch.zeros(n, dtype=torch.int8)
        for t in self._last_selected_unit_tags or ():
            if t in index:
                last_su[index[t]] = 1
        if self._last_target_unit_tag is not None and self._last_target_unit_tag in index:
            last_tu[index[self._last_target_unit_tag]] = 1
        ei, si = agent_obs['entity_info'], agent_obs['scalar_info']
        ei['last_selected_units'] = last_su
        ei['last_targeted_unit'] = last_tu
        agent_obs['hidden_state'] = self._hidden_state
        si['last_delay'] = self._last_delay
        si['last_action_type'] = self._last_action_type
        si['last_queued'] = self._last_queued
        si['enemy_unit_type_bool'] = (self._enemy_unit_type_bool | si['enemy_unit_type_bool']).to(torch.uint8)
        use_bo = self.use_bo_reward and self._exceed_flag
        si['beginning_order'] = self._pad_bo(self._target_building_order) * use_bo
        si['bo_location'] = self._pad_bo(self._target_bo_location) * use_bo
        if self.use_cum_reward and self._exceed_flag:
            si['cumulative_stat'] = self._target_cumulative_stat
        else:
            si['cumulative_stat'] = self._target_cumulative_stat * 0 + self._zero_z_value
        self._observation = agent_obs
        return agent_obs

    @staticmethod
    def _pad_bo(t: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(BEGINNING_ORDER_LENGTH, dtype=torch.long)
        n = min(len(t), BEGINNING_ORDER_LENGTH)
        out[:n] = t[:n]
        return out

    def _model_input(self, agent_obs: Dict) -> Dict:
        keys = ('spatial_info', 'entity_info', 'scalar_info', 'entity_num', 'hidden_state')
        return {k: agent_obs[k] for k in keys}

    def step(self, observation) -> List[dict]:
        if 'eval' in self._job_type and self._iter_count > 0 and not self._whole_cfg.env.realtime:
            self._update_fake_reward(self._last_action_type, self._last_location, observation)
        agent_obs = self._pre_process(observation)
        self._stat_api.update(int(self._last_action_type), observation['action_result'][0], self._observation,
                              self._game_step)
        if self._client is not None:
            req = self._model_input(agent_obs)
            if self._merged:
                req['teacher_hidden_state'] = self._teacher_hidden_state
            out = self._client.infer(req)
            self._teacher_out = out.pop('teacher', None)
            self._model_last_iter = int(out.pop('model_last_iter', self._model_last_iter))
        else:
            batch = collate_obs([self._model_input(agent_obs)])
            if self._use_cuda:
                batch = _to(batch, 'cuda')
            out = decollate_output(self.model.compute_logp_action(**batch), 0)
        action = self._post_process(out)
        self._iter_count += 1
        return action

    def _post_process(self, output: Dict) -> List[dict]:
        self._hidden_state = output['hidden_state']
        ai = output['action_info']
        self._last_queued = ai['queued']
        self._last_action_type = ai['action_type']
        self._last_delay = ai['delay']
        self._last_location = ai['target_location']
        self._output = output
        at = int(ai['action_type'])
        act = ACTIONS[at]
        tags = self._game_info['tags']
        info = {'func_id': act['func_id'], 'skip_steps': int(ai['delay']), 'queued': int(ai['queued'])}
        su_num = int(output['selected_units_num'])
        info['unit_tags'] = [tags[i] for i in ai['selected_units'][:max(su_num - 1, 0)].tolist() if i < len(tags)]
        if self._extra_units and output.get('extra_units') is not None:
            for i in torch.nonzero(output['extra_units']).flatten().tolist():
                if i < len(tags):
                    info['unit_tags'].append(tags[i])
        self._last_selected_unit_tags = info['unit_tags'] if act['selected_units'] else None
        tu = int(ai['target_unit'])
        info['target_unit_tag'] = tags[tu] if tu < len(tags) else 0
        self._last_target_unit_tag = info['target_unit_tag'] if act['target_unit'] else None
        loc = int(ai['target_location'])
        x, y = loc % SPATIAL_SIZE[1], loc // SPATIAL_SIZE[1]
        info['location'] = (x, max(self._feature.map_size.y - y, 0))
        if 'test' in self._job_type and self._whole_cfg.actor.get('print_action', False):
            print(f'{self.player_id} step {self._game_step}: {act["name"]} delay {int(ai["delay"])} '
                  f'su {len(info["unit_tags"])} loc {(x, y)}')
        return [info]

    # ------------------------------------------------------------------ stats
    def get_unit_num_info(self):
        return {'unit_num': self._stat_api.unit_num}

    def get_behavior_z(self) -> Dict:
        pad = BEGINNING_ORDER_LENGTH
        bo = (self._behaviour_building_order + [0] * pad)[:pad]
        loc = (self._behaviour_bo_location + [0] * pad)[:pad]
        return {'beginning_order': torch.as_tensor(bo, dtype=torch.long),
                'bo_location': torch.as_tensor(loc, dtype=torch.long),
                'cumulative_stat': torch.as_tensor(self._behaviour_cumulative_stat, dtype=torch.bool).long()}

    def get_stat_data(self) -> Dict:
        data = self._stat_api.get_stat_data()
        bb = torch.as_tensor(self._behaviour_building_order, dtype=torch.int)
        tb = torch.as_tensor(self._target_building_order, dtype=torch.int)
        bo_dist = levenshtein_distance(bb, tb).item()
        bo_dist_loc = levenshtein_distance(bb, tb, torch.as_tensor(self._behaviour_bo_location, dtype=torch.int),
                                           torch.as_tensor(self._target_bo_location, dtype=torch.int),
                                           partial(l2_distance, spatial_x=SPATIAL_SIZE[1])).item()
        stat = {'race_id': self._race, 'step': self._game_step, 'dist/bo': bo_dist,
                'dist/bo_location': bo_dist_loc - bo_dist,
                'dist/cum': hamming_distance(torch.as_tensor(self._behaviour_cumulative_stat, dtype=torch.bool),
                                             self._target_cumulative_stat.bool()).item(),
                'bo_reward': self._total_bo_reward.item(), 'cum_reward': self._total_cum_reward.item(),
                'bo_len': len(self._behaviour_building_order)}
        z0 = z1 = 0
        if not self.use_bo_reward:
            stat.update({'dist/bo': None, 'bo_reward': None, 'bo_len': None, 'dist/bo_location': None})
            z0 = 1
        if not self.use_cum_reward:
            stat.update({'dist/cum': None, 'cum_reward': None})
            z1 = 1
        stat['z_type'] = 2 * z1 + z0
        data.update(stat)
        for i, b in enumerate(self._behaviour_cumulative_stat):
            if self._race not in CUM_DICT[i]['race']:
                continue
            name = CUM_DICT[i]['name']
            key = ('cum_in/' if self._target_cumulative_stat[i] > 1e-3 else 'cum_out/') + name
            data[key] = 1 if b >= 1 else 0
        return data

    # ------------------------------------------------------------------ training data
    def collect_data(self, next_obs, reward, done: bool, idx: int = 0) -> Optional[List[dict]]:
        if next_obs is not None and 'Success' in str(next_obs.get('action_result')):
            self._success_iter_count += 1
        behaviour_z = self.get_behavior_z()
        bo_reward, cum_reward, battle_reward = self._update_fake_reward(self._last_action_type, self._last_location,
                                                                        next_obs)
        agent_obs = self._observation
        teacher_in = {'spatial_info': agent_obs['spatial_info'], 'entity_info': agent_obs['entity_info'],
                      'scalar_info': agent_obs['scalar_info'], 'entity_num': agent_obs['entity_num'],
                      'hidden_state': self._teacher_hidden_state,
                      'selected_units_num': self._output['selected_units_num'],
                      'action_info': self._output['action_info']}
        if self._teacher_out is not None:        # computed with the policy step (merged request)
            t_out, self._teacher_out = self._teacher_out, None
        elif self._teacher_client is not None:
            t_out = self._teacher_client.infer(teacher_in)
        else:
            batch = collate_obs([teacher_in])
            if self._use_cuda:
                batch = _to(batch, 'cuda')
            t_out = decollate_output(self.teacher_model.compute_teacher_logit(**batch), 0)
        self._teacher_hidden_state = t_out['hidden_state']
        if self._use_dapo and self.successive_model is not None:
            s_in = dict(teacher_in, hidden_state=self._successive_hidden_state)
            s_out = decollate_output(self.successive_model.compute_teacher_logit(**collate_obs([s_in])), 0)
            self._successive_hidden_state = s_out['hidden_state']

        ai = {k: v.clone() for k, v in self._output['action_info'].items()}
        act = ACTIONS[int(ai['action_type'])]
        mask = {'actions_mask': {k: torch.tensor(int(act[k]), dtype=torch.long)
                                 for k in ('queued', 'selected_units', 'target_unit', 'target_location')},
                'cum_action_mask': torch.tensor(0.0 if self._only_cum_action_kl else 1.0),
                'build_order_mask': torch.tensor(1.0 if self.use_bo_reward else 0.0),
                'built_unit_mask': torch.tensor(1.0 if self.use_cum_reward else 0.0)}
        if self.use_cum_reward:
            mask['cum_action_mask'] = torch.tensor(1.0)
        step_data = {
            'map_name': self._map_name, 'spatial_info': agent_obs['spatial_info'],
            'model_last_iter': torch.tensor(float(self._model_last_iter)),
            'entity_info': agent_obs['entity_info'], 'scalar_info': agent_obs['scalar_info'],
            'entity_num': agent_obs['entity_num'], 'selected_units_num': self._output['selected_units_num'],
            'hidden_state': self._hidden_state_backup, 'action_info': ai,
            'behaviour_logp': self._output['action_logp'], 'teacher_logit': t_out['logit'],
            'reward': {'winloss': torch.tensor(float(reward)), 'build_order': bo_reward, 'built_unit': cum_reward,
                       'battle': battle_reward},
            'step': torch.tensor(float(self._game_step)), 'mask': mask}
        if self._use_value_feature:
            step_data['value_feature'] = dict(agent_obs['value_feature'], **behaviour_z)
        if self._use_dapo and self.successive_model is not None:
            step_data['successive_logit'] = s_out['logit']
        self._hidden_state_backup = self._hidden_state
        self._data_buffer.append(step_data)
        self._push_count += 1
        if self._push_count < self._whole_cfg.actor.traj_len and not done:
            return None
        if not done:
            self._pre_process(next_obs)
        last_obs = self._observation
        last = {'map_name': self._map_name, 'spatial_info': last_obs['spatial_info'],
                'entity_info': last_obs['entity_info'], 'scalar_info': last_obs['scalar_info'],
                'entity_num': last_obs['entity_num'], 'hidden_state': self._hidden_state}
        if self._use_value_feature:
            last['value_feature'] = dict(last_obs['value_feature'], **self.get_behavior_z())
        traj = list(self._data_buffer) + [copy.copy(last)]
        self._push_count = 0
        return traj

    # ------------------------------------------------------------------ pseudo rewards
    @staticmethod
    def _time_factor(game_step: int) -> float:
        return 1.0 if game_step < 10000 else 0.5 if game_step < 20000 else 0.25 if game_step < 30000 else 0.0

    def _update_fake_reward(self, action_type, location, next_obs):
        bo_reward = torch.zeros(())
        cum_reward = torch.zeros(())
        if next_obs is None:
            return bo_reward, cum_reward, torch.zeros(())
        battle = (compute_battle_score(next_obs['raw_obs']) - self._game_info['battle_score']
                  - (compute_battle_score(next_obs.get('opponent_obs')) - self._game_info['opponent_battle_score']))
        battle_reward = torch.tensor(battle, dtype=torch.float) / self._battle_norm
        if not self._exceed_flag:
            return bo_reward, cum_reward, battle_reward
        at = int(action_type)
        ok = next_obs['action_result'][0] == 1
        if at in _BO_INDEX and ok:
            skip_bo = False
            if at == 322:
                self._bo_zergling_count += 1
                skip_bo = self._bo_zergling_count > self._bo_zergling_num
            idx = _BO_INDEX[at]
            if idx == 39 and 39 not in self._target_building_order.tolist():
                skip_bo = True
            if skip_bo:
                return bo_reward, cum_reward, battle_reward
            if len(self._behaviour_building_order) < len(self._target_building_order):
                self._behaviour_building_order.append(idx)
                self._behaviour_bo_location.append(int(location) if ACTIONS[at]['target_location'] else 0)
                if self.use_bo_reward:
                    n = len(self._behaviour_building_order)
                    tz = self._target_building_order[:n] if self._clip_bo else self._target_building_order
                    tl = self._target_bo_location[:n] if self._clip_bo else self._target_bo_location
                    new = -levenshtein_distance(torch.as_tensor(self._behaviour_building_order, dtype=torch.int),
                                                tz.int(), torch.as_tensor(self._behaviour_bo_location, dtype=torch.int),
                                                tl.int(), partial(l2_distance, spatial_x=SPATIAL_SIZE[1])) / self._bo_norm
                    bo_reward = new - self._old_bo_reward
                    self._old_bo_reward = new
        cum_flag = False
        if self._cum_type == 'observation':
            cum_flag = True
            ro = next_obs['raw_obs'].observation
            for u in ro.raw_data.units:
                if u.alliance == 1 and u.unit_type in BASE_UNIT_TYPES and \
                        [u.pos.x, u.pos.y] == self._born_location:
                    continue
                if u.alliance == 1 and u.build_progress == 1 and UNIT_TO_CUM[u.unit_type] != -1:
                    self._behaviour_cumulative_stat[UNIT_TO_CUM[u.unit_type]] = 1
            for u in ro.raw_data.player.upgrade_ids:
                if UPGRADE_TO_CUM[u] != -1:
                    self._behaviour_cumulative_stat[UPGRADE_TO_CUM[u]] = 1
        elif self._cum_type == 'action':
            name = ACTIONS[at]['name']
            if name in ('Cancel_quick', 'Cancel_Last_quick'):
                ai = self._output['action_info']
                u = int(ai['selected_units'][0])
                ei = self._observation['entity_info']
                order_len = int(ei['order_length'][u])
                if order_len == 0:
                    cancelled = 0
                elif order_len == 1:
                    cancelled = UNIT_ABILITY_TO_ACTION.get(int(ei['order_id_0'][u]), 0)
                else:
                    cancelled = QUEUE_ACTIONS[int(ei[f'order_id_{min(order_len, 4) - 1}'][u]) - 1]
                if cancelled in _CUM_INDEX:
                    cum_flag = True
                    ci = _CUM_INDEX[cancelled]
                    self._behaviour_cumulative_stat[ci] = max(0, self._behaviour_cumulative_stat[ci] - 1)
            if at in _CUM_INDEX:
                cum_flag = True
                self._behaviour_cumulative_stat[_CUM_INDEX[at]] += 1
        else:
            raise NotImplementedError(self._cum_type)
        if self.use_cum_reward and cum_flag and (self._cum_type == 'observation' or ok):
            new = -hamming_distance(torch.as_tensor(self._behaviour_cumulative_stat, dtype=torch.bool),
                                    self._target_cumulative_stat.bool()) / self._cum_norm
            cum_reward = (new - self._old_cum_reward) * self._time_factor(self._game_step)
            self._old_cum_reward = new
        self._total_bo_reward += bo_reward
        self._total_cum_reward += cum_reward
        return bo_reward, cum_reward, battle_reward

    # ------------------------------------------------------------------ properties
    @property
    def player_id(self):
        return self._player_id

    @player_id.setter
    def player_id(self, v):
        self._player_id = v

    @property
    def env_id(self):
        return self._env_id

    @env_id.setter
    def env_id(self, v):
        self._env_id = v

    @property
    def race(self):
        return self._race

    @property
    def iter_count(self):
        return self._iter_count

    @property
    def model_last_iter(self):
        return self._model_last_iter

    @model_last_iter.setter
    def model_last_iter(self, v):
        self._model_last_iter = int(v)


def _to(tree, device):
    if isinstance(tree, torch.Tensor):
        return tree.to(device, non_blocking=True)
    if isinstance(tree, dict):
        return {k: _to(v, device) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return type(tree)(_to(v, device) for v in tree)
    return tree
