"""League manager: job dispatch, result ingestion, snapshot/reset of active players, resume.

Capabilities of ``distar/ctools/worker/league/league.py:30-875``:

* active players from config (player type from the id prefix) + initial historical players;
* ``actor_ask_for_job``: choose an active player by ``chosen_weight``; vs-bot jobs (``bot_probs``),
  training jobs from the player's branch policy (sp / pfsp / eval / vs_main ...), or ladder jobs
  among historical players; a map sampled by ``map_id_weights``;
* ``actor_send_result``: queued, applied by a worker thread: payoffs (both sides), ELO, per-race stats;
* ``learner_send_train_info``: adds trained frames, snapshots the player into a historical player
  when trained enough, and resets it (new checkpoint) when its policy says so;
* resume: periodic JSON snapshot of all players / payoffs / ELO (the reference pickles with dill).
"""
from __future__ import annotations

import itertools
import json
import os
import re
import queue
import random
import shutil
import threading
import time
from typing import Dict, Optional

from ..utils.config import AttrDict, deep_merge_dicts
from ..utils.log import TextLogger
from .players import (ActivePlayer, HistoricalPlayer, MainPlayer, active_player_type, player_from_dict)
from .stats import ELORating, TrueSkillRating

DEFAULT_LEAGUE_CONFIG = AttrDict({
    'common': {'experiment_name': 'rl_train'},
    'learner': {'use_dapo': False},
    'league': {
        'resume_path': '', 'use_historical_players': True, 'fake_model': True, 'vs_bot': False,
        'pfsp_train_bot': False, 'bot_probs': [0, 0, 0, 1.0, 0, 0, 0, 0, 0, 0, 0],
        'save_initial_snapshot': False, 'map_names': ['KairosJunction'], 'map_id_weights': [1],
        'stat_decay': 0.995, 'stat_warm_up_size': 1000, 'payoff_min_win_rate_games': 100, 'print_freq': 100,
        'save_resume_freq': 3600, 'ladder_bots': ['bot7', 'bot10'],
        'active_players': {'checkpoint_path': ['default'], 'player_id': ['MP0'], 'pipeline': ['default'],
                           'frac_id': [1], 'z_prob': [0.0], 'teacher_id': ['teacher_model'],
                           'teacher_path': ['default'], 'z_path': ['3map.json'], 'one_phase_step': ['4e8'],
                           'chosen_weight': [1]},
        'historical_players': {'player_id': ['sl'], 'checkpoint_path': ['default'], 'pipeline': ['default'],
                               'frac_id': [1], 'z_prob': [0.0], 'z_path': ['3map.json']},
        'branch_probs': {
            'MainPlayer': {'sp': 0.5, 'pfsp': 0.5, 'eval': 0.0},
            'ExploiterPlayer': {'pfsp': 0.95, 'eval': 0.05},
            'ExpertExploiterPlayer': {'pfsp': 0.95, 'eval': 0.05},
            'MainExploiterPlayer': {'vs_main': 0.5, 'pfsp': 0.45, 'eval': 0.05},
            'AdaptiveEvolutionaryExploiterPlayer': {'vs_main': 0.45, 'pfsp': 0.45, 'eval': 0.1},
            'ExpertPlayer': {'pfsp': 0.95, 'eval': 0.05},
        },
    },
})


class League:
    def __init__(self, cfg: Optional[dict] = None, root: str = '.', start_threads: bool = True):
        self.whole_cfg = deep_merge_dicts(DEFAULT_LEAGUE_CONFIG, cfg or {})
        self.cfg = self.whole_cfg.league
        exp = self.whole_cfg.common.experiment_name
        self.root = os.path.abspath(os.path.join(root, 'experiments', exp))
        # admin routes may only read checkpoints / write backups under these directories (default: the directory
        # the league runs in, which holds experiments/); extend with ``league.checkpoint_roots``
        self.allowed_roots = [os.path.realpath(os.path.abspath(root))] + \
            [os.path.realpath(os.path.abspath(r)) for r in (self.cfg.get('checkpoint_roots') or [])]
        self.model_dir = os.path.join(self.root, 'league_models')
        self.resume_dir = os.path.join(self.root, 'league_resume')
        os.makedirs(self.model_dir, exist_ok=True)
        os.makedirs(self.resume_dir, exist_ok=True)
        self.logger = TextLogger(os.path.join(self.root, 'log'), 'league', to_stdout=False)
        from ..utils.log import ScalarLogger
        self.scalar_logger = ScalarLogger(os.path.join(self.root, 'league_scalars')) \
            if self.cfg.get('scalar_log', True) else None
        self.lock = threading.RLock()
        from ..runtime.health import HeartbeatRegistry
        self.health = HeartbeatRegistry(float(self.cfg.get('heartbeat_timeout', 120.0)))
        self.elo = ELORating()
        self.trueskill = TrueSkillRating()
        self.active_players: Dict[str, ActivePlayer] = {}
        self.historical_players: Dict[str, HistoricalPlayer] = {}
        self.learner_info = {}
        self._results: 'queue.Queue[dict]' = queue.Queue()
        self._stop = threading.Event()
        self._init_players()
        self._threads = []
        if start_threads:
            for fn in (self._result_loop, self._resume_loop):
                t = threading.Thread(target=fn, daemon=True)
                t.start()
                self._threads.append(t)

    # ------------------------------------------------------------------ setup
    @property
    def all_players(self):
        return {**self.historical_players, **self.active_players}

    def _player_kw(self):
        return dict(decay=self.cfg.stat_decay, warm_up_size=self.cfg.stat_warm_up_size,
                    min_win_rate_games=self.cfg.payoff_min_win_rate_games)

    def _init_players(self):
        if self.cfg.resume_path and os.path.isfile(self.cfg.resume_path):
            self.load_resume(self.cfg.resume_path)
            return
        ap = self.cfg.active_players
        for ckpt, pid, pipe, frac, zp, zprob, tid, tpath, ops, cw in zip(
                ap.checkpoint_path, ap.player_id, ap.pipeline, ap.frac_id, ap.z_path, ap.z_prob, ap.teacher_id,
                ap.teacher_path, ap.one_phase_step, ap.chosen_weight):
            self.add_active_player(ckpt, pid, pipe, frac, zp, zprob, tid, tpath, ops, cw)
        if self.cfg.use_historical_players:
            hp = self.cfg.historical_players
            ids = hp.get('player_id') or [f'HP{i}' for i in range(len(hp.checkpoint_path))]
            for pid, ckpt, pipe, frac, zp, zprob in zip(ids, hp.checkpoint_path, hp.pipeline, hp.frac_id, hp.z_path,
                                                        hp.z_prob):
                self.historical_players[pid] = HistoricalPlayer(ckpt, pid, pipe, frac, zp, zprob, **self._player_kw())
        self.logger.info(f'league active={list(self.active_players)} historical={list(self.historical_players)}')

    def add_active_player(self, ckpt_path, player_id, pipeline, frac_id, z_path, z_prob, teacher_id, teacher_path,
                          one_phase_step, chosen_weight=1.0) -> bool:
        cls = active_player_type(player_id)
        if cls is None:
            return False
        dst = os.path.join(self.model_dir, f'{player_id}_ckpt.pth.tar')
        p = cls(dst, player_id, pipeline, frac_id, z_path, z_prob, teacher_id, teacher_path,
                chosen_weight=chosen_weight, one_phase_step=one_phase_step, **self._player_kw())
        if os.path.exists(str(ckpt_path)):
            shutil.copyfile(ckpt_path, dst)
        elif not self.cfg.get('fake_model', True):
            raise FileNotFoundError(ckpt_path)
        with self.lock:
            self.active_players[player_id] = p
        if isinstance(p, MainPlayer) and self.cfg.save_initial_snapshot:
            self.save_snapshot(p)
        return True

    # ------------------------------------------------------------------ learner side
    def register_learner(self, info: Dict) -> Dict:
        pid = info['player_id']
        if pid not in self.active_players:
            raise KeyError(f'{pid} not an active player ({list(self.active_players)})')
        self.health.beat('learner', f"{pid}/rank{info.get('rank', 0)}", info)
        self.learner_info.setdefault(pid, []).append({k: info.get(k) for k in ('ip', 'port', 'rank', 'world_size')})
        return {'ckpt_path': self.active_players[pid].checkpoint_path}

    def save_snapshot(self, player: ActivePlayer) -> str:
        hp = player.snapshot()
        hp.checkpoint_path = os.path.join(self.model_dir, hp.player_id + '_' + os.path.basename(player.checkpoint_path))
        if os.path.exists(player.checkpoint_path):
            shutil.copyfile(player.checkpoint_path, hp.checkpoint_path)
        with self.lock:
            self.historical_players[hp.player_id] = hp
        self.logger.info(f'snapshot {player.player_id} -> {hp.player_id}')
        return hp.player_id

    def learner_send_train_info(self, info: Dict) -> Dict:
        pid = info['player_id']
        p = self.active_players[pid]
        with self.lock:
            p.total_agent_step += int(info['train_steps'])
            if info.get('checkpoint_path'):
                p.checkpoint_path = info['checkpoint_path']
        hist = self.historical_players if self.cfg.pfsp_train_bot else {
            k: v for k, v in self.historical_players.items() if v.pipeline != 'bot'}
        reset = p.reset_flag
        new_hp = None
        if p.is_trained_enough(hist, self.active_players, pfsp_train_bot=self.cfg.pfsp_train_bot):
            new_hp = self.save_snapshot(p)
            reset |= p.is_reset()
        if reset:
            p.reset_flag = False
            with self.lock:
                p.reset_stats()
                src = p.reset_checkpoint(self.active_players, self.historical_players, new_hp)
                p.checkpoint_path = os.path.join(self.model_dir, f'{pid}_ckpt.pth.tar')
                if src and os.path.exists(src) and os.path.abspath(src) != os.path.abspath(p.checkpoint_path):
                    shutil.copyfile(src, p.checkpoint_path)
            self.logger.info(f'reset {pid} from {src}')
            return {'reset_checkpoint_path': p.checkpoint_path}
        return {'reset_checkpoint_path': 'none'}

    # ------------------------------------------------------------------ actor side
    def choose_active_player(self) -> ActivePlayer:
        ids = list(self.active_players)
        w = [self.active_players[i].chosen_weight for i in ids]
        return self.active_players[random.choices(ids, weights=w, k=1)[0]]

    def actor_ask_for_job(self, info: Dict) -> Dict:
        job_type = info.get('job_type', 'train')
        if info.get('actor_id'):
            self.health.beat('actor', info['actor_id'])
        with self.lock:
            if job_type == 'ladder':
                branch, job = self._ladder_job()
            else:
                p = self.choose_active_player()
                branch, job = self._vs_bot_job(p) if self.cfg.vs_bot else self._train_job(p)
        job['branch'] = branch
        job['env_info']['map_name'] = random.choices(self.cfg.map_names, weights=self.cfg.map_id_weights, k=1)[0]
        return job

    def _vs_bot_job(self, p: ActivePlayer):
        lvl = random.choices(range(len(self.cfg.bot_probs)), weights=self.cfg.bot_probs, k=1)[0]
        job = {'player_ids': [p.player_id], 'side_ids': [0], 'checkpoint_paths': [p.checkpoint_path],
               'successive_ids': [p.player_id if isinstance(p, MainPlayer) else 'none'],
               'pipelines': [p.pipeline], 'z_path': [p.z_path], 'z_prob': [p.z_prob],
               'teacher_player_ids': [p.teacher_id], 'teacher_checkpoint_paths': [p.teacher_checkpoint_path],
               'send_data_players': [p.player_id], 'update_players': [p.player_id],
               'frac_ids': [p.frac_id, self.cfg.get('frac_id', 1)], 'bot_id': f'bot{lvl}',
               'env_info': {'player_ids': [p.player_id, f'bot{lvl}'], 'side_id': [0, 1]}}
        return 'train_bot', job

    def _train_job(self, p: ActivePlayer):
        branch, home, away = p.get_branch_opponent(self.historical_players, self.active_players,
                                                   self.cfg.branch_probs, self.cfg.pfsp_train_bot)
        players = list(itertools.chain.from_iterable(zip(away, home)))
        active_ids = sorted({q.player_id for q in players if isinstance(q, ActivePlayer)})
        job = {'player_ids': [q.player_id for q in players], 'side_ids': list(range(len(players))),
               'pipelines': [q.pipeline for q in players], 'checkpoint_paths': [q.checkpoint_path for q in players],
               'successive_ids': [q.player_id if isinstance(q, MainPlayer) else 'none' for q in players],
               'z_path': [q.z_path for q in players], 'z_prob': [q.z_prob for q in players],
               'teacher_player_ids': [q.teacher_id for q in players],
               'teacher_checkpoint_paths': [q.teacher_checkpoint_path for q in players],
               'send_data_players': active_ids, 'update_players': active_ids,
               'frac_ids': [q.frac_id for q in players],
               'env_info': {'player_ids': [q.player_id for q in players], 'side_id': [0, 1]}}
        if branch == 'vs_main':
            for i, q in enumerate(players):
                if isinstance(q, MainPlayer):
                    job['teacher_player_ids'][i] = job['teacher_checkpoint_paths'][i] = 'none'
            job['send_data_players'] = sorted({q.player_id for q in players if isinstance(q, ActivePlayer)
                                               and not isinstance(q, MainPlayer)})
        elif 'eval' in branch:
            job['teacher_player_ids'] = ['none'] * len(players)
            job['teacher_checkpoint_paths'] = ['none'] * len(players)
            job['send_data_players'] = []
        return branch, job

    def _ladder_job(self):
        """Pair historical players (and ladder bots) favouring pairs with few games (league.py:486-533)."""
        entrants = list(self.historical_players) + list(self.cfg.ladder_bots or [])
        pairs = [(a, b) for a in entrants for b in entrants if a != b and not (a.startswith('bot') and b.startswith('bot'))]
        if not pairs:
            raise RuntimeError('ladder needs at least two entrants')
        few = [pr for pr in pairs if self.elo.games[pr[0]][pr[1]] < 100]
        a, b = random.choice(few or pairs)
        ids, paths, pipes, zps, zpr, fr = [], [], [], [], [], []
        for pid in (a, b):
            if pid in self.historical_players:
                q = self.historical_players[pid]
                ids.append(q.player_id); paths.append(q.checkpoint_path); pipes.append(q.pipeline)
                zps.append(q.z_path); zpr.append(q.z_prob); fr.append(q.frac_id)
            else:
                ids.append(pid); paths.append('none'); pipes.append('bot'); zps.append('none'); zpr.append(0.0)
                fr.append(1)
        job = {'player_ids': ids, 'side_ids': [0, 1], 'pipelines': pipes, 'checkpoint_paths': paths,
               'successive_ids': ['none', 'none'], 'z_path': zps, 'z_prob': zpr,
               'teacher_player_ids': ['none', 'none'], 'teacher_checkpoint_paths': ['none', 'none'],
               'send_data_players': [], 'update_players': [], 'frac_ids': fr,
               'env_info': {'player_ids': ids, 'side_id': [0, 1]}}
        return 'ladder', job

    def actor_send_result(self, info: Dict) -> bool:
        self._results.put(info)
        return True

    def apply_result(self, info: Dict) -> None:
        info = dict(info)
        steps = info.pop('game_steps', 0)
        iters = info.pop('game_iters', 0)
        dur = info.pop('game_duration', 0.0)
        with self.lock:
            for side, r in info.items():
                pid, opp = r['player_id'], r['opponent_id']
                p = self.all_players.get(pid)
                if p is None:
                    continue
                if pid != opp:
                    p.payoff.update(opp, {'winrate': (1 + r['winloss']) / 2, 'game_steps': steps,
                                          'game_iters': iters, 'game_duration': dur})
                p.total_game_count += 1
                if isinstance(p, ActivePlayer):
                    race = r.get('race_id', 'unknown')
                    p.dist_stat.update(race, {k: v for k, v in r.items() if k.startswith('dist')})
                    p.cum_stat.update(race, {k: v for k, v in r.items() if k.startswith('cum')})
                    p.unit_num_stat.update(race, {k: v for k, v in r.items() if k.startswith('units/')})
                    self._log_player(p, opp)
            first = info.get('0') or next(iter(info.values()))
            self.elo.update(first['player_id'], first['opponent_id'], int(first['winloss']))
            self.trueskill.update(first['player_id'], first['opponent_id'], int(first['winloss']))
            if self.elo.game_count % max(int(self.cfg.print_freq), 1) == 0:
                self.logger.info('ELO\n' + self.elo.text())

    def _log_player(self, p, opp: str) -> None:
        """Per-player scalars (league.py:351-375): win rate / game length per opponent, Z distances,
        cumulative-stat in/out rates, unit counts; step = games played by the player."""
        if self.scalar_logger is None:
            return
        step = p.total_game_count
        for k, v in p.payoff.stat_info_dict().get(opp, {}).items():
            self.scalar_logger.add_scalar(f'{p.player_id}/{opp}/{k}', v, step)
        for stat in (p.dist_stat, p.cum_stat, p.unit_num_stat):
            for race, vals in stat.stat_info_dict().items():
                for k, v in vals.items():
                    self.scalar_logger.add_scalar(f'{p.player_id}/{race}/{k}', v, step)

    def _result_loop(self):
        while not self._stop.is_set():
            try:
                info = self._results.get(timeout=0.1)
            except queue.Empty:
                continue
            try:
                self.apply_result(info)
            except Exception as e:  # a malformed result must not kill the league
                self.logger.error(f'bad result {info}: {e!r}')

    def drain_results(self, timeout: float = 5.0):
        t = time.time()
        while not self._results.empty() and time.time() - t < timeout:
            time.sleep(0.01)

    # ------------------------------------------------------------------ resume
    def state_dict(self) -> Dict:
        with self.lock:
            return {'active': {k: v.to_dict() for k, v in self.active_players.items()},
                    'historical': {k: v.to_dict() for k, v in self.historical_players.items()},
                    'elo': self.elo.to_dict(), 'trueskill': self.trueskill.to_dict()}

    def save_resume(self, path: Optional[str] = None) -> str:
        path = path or os.path.join(self.resume_dir, f'league.resume.{int(time.time())}.json')
        tmp = path + '.tmp'
        with open(tmp, 'w') as f:
            json.dump(self.state_dict(), f)
        os.replace(tmp, path)
        return path

    def load_resume(self, path: str) -> None:
        with open(path) as f:
            d = json.load(f)
        with self.lock:
            self.active_players = {k: player_from_dict(v) for k, v in d['active'].items()}
            self.historical_players = {k: player_from_dict(v) for k, v in d['historical'].items()}
            self.elo = ELORating.from_dict(d['elo'])
            if 'trueskill' in d:
                self.trueskill = TrueSkillRating.from_dict(d['trueskill'])

    # ------------------------------------------------------------------ admin (league_api.py:56-305)
    def correspondent_player_ids(self, player_id):
        """'all' / 'active' / 'hist' / a list / one id -> the matching player ids (league.py:847-862)."""
        if player_id == 'all':
            return list(self.all_players)
        if player_id == 'active':
            return list(self.active_players)
        if player_id == 'hist':
            return list(self.historical_players)
        if isinstance(player_id, (list, tuple)):
            return [p for p in player_id if p in self.all_players]
        return [player_id] if player_id in self.all_players else []

    def show_stat(self, stat_type: str, historical: bool = False) -> Dict:
        """One statistic of every active (or historical) player, as a dict; also written to the league log."""
        players = self.historical_players if historical else self.active_players
        out = {}
        with self.lock:
            for pid, p in players.items():
                st = getattr(p, stat_type, None)
                if st is None:
                    continue
                out[pid] = st.stat_info_dict()
                self.logger.info('=' * 20 + pid + '=' * 20 + f'\n{stat_type}: {json.dumps(out[pid], default=str)}')
        return out

    def save_elo_ratings(self, zero_min: bool = False) -> str:
        path = os.path.join(self.root, 'elo_ratings' + ('_zero' if zero_min else '') + '.json')
        with open(path, 'w') as f:
            json.dump(self.elo.ratings(start_from_zero=zero_min), f, indent=1)
        return path

    def update_elo(self, info: Dict) -> bool:
        """{player_id: elo} (absolute ratings; the stored value is relative to init_elo)."""
        with self.lock:
            for pid, v in (info or {}).items():
                self.elo.elos[pid] = float(v) - self.elo.init_elo
        return True

    def save_trueskill_ratings(self) -> str:
        path = os.path.join(self.root, 'trueskill_ratings.json')
        with open(path, 'w') as f:
            json.dump(self.trueskill.ratings(), f, indent=1)
        return path

    def update_trueskill(self, info: Dict) -> bool:
        """{player_id: {'mu': .., 'sigma': ..}}."""
        with self.lock:
            for pid, v in (info or {}).items():
                self.trueskill.set(pid, v.get('mu'), v.get('sigma'))
        return True

    _SAFE_ID = re.compile(r'^[A-Za-z0-9_]+$')

    def _allowed_path(self, path: str) -> bool:
        """True when ``path`` resolves (symlinks too) inside one of the league's allowed roots."""
        real = os.path.realpath(os.path.abspath(path))
        return any(real == r or real.startswith(r + os.sep) for r in self.allowed_roots)

    def add_hist_player(self, info: Dict) -> bool:
        """Copy a checkpoint into the league and add it as a historical player (league.py:558-588).  The player id
        must match ``[A-Za-z0-9_]+`` (it names a file under league_models/) and the checkpoint must lie under an
        allowed root."""
        ckpt = info.get('checkpoint_path', 'none')
        if ckpt == 'none' or not os.path.isfile(ckpt) or not self._allowed_path(ckpt):
            return False
        pid = info.get('player_id') or 'none'
        if pid != 'none' and not self._SAFE_ID.match(str(pid)):
            return False
        if pid == 'none':
            self._added = getattr(self, '_added', 0) + 1
            pid = f'HP_ADD{self._added}'
        dst = os.path.join(self.model_dir, pid + '_' + os.path.basename(ckpt))
        shutil.copyfile(ckpt, dst)
        hp = HistoricalPlayer(dst, pid, info.get('pipeline', 'default'), info.get('frac_id', 1),
                              info.get('z_path', '3map.json'), info.get('z_prob', 0.0), **self._player_kw())
        with self.lock:
            self.historical_players[pid] = hp
        self.logger.info(f'added historical player {pid}')
        return True

    def remove_hist_player(self, info: Dict) -> bool:
        """Drop historical players and every payoff record against them (league.py:739-758)."""
        ids = [p for p in self.correspondent_player_ids(info['player_id']) if p in self.historical_players]
        with self.lock:
            for pid in ids:
                self.historical_players.pop(pid, None)
                for p in self.all_players.values():
                    for k in ('payoff', 'teammate_payoff', 'opponent_payoff'):
                        getattr(p, k).record.pop(pid, None)
                self.logger.info(f'removed historical player {pid}')
        return bool(ids)

    _UPDATABLE = ('checkpoint_path', 'pipeline', 'frac_id', 'z_path', 'teacher_id', 'teacher_checkpoint_path',
                  'chosen_weight', 'total_agent_step', 'decay', 'warm_up_size', 'total_game_count', 'parent_id',
                  'one_phase_step', 'last_enough_step', 'snapshot_times', 'strong_win_rate', 'snapshot_flag',
                  'reset_flag', 'z_prob')

    def update_player(self, info: Dict) -> bool:
        """Set attributes of one player (league.py:617-635)."""
        p = self.all_players.get(info.get('player_id'))
        if p is None:
            return False
        with self.lock:
            for k in self._UPDATABLE:
                if k in info and hasattr(p, k):
                    v = info[k]
                    if k == 'one_phase_step':
                        v = int(float(v))
                    setattr(p, k, v)
        return True

    def display_player(self, info: Dict) -> Dict:
        out = {}
        for pid in self.correspondent_player_ids(info['player_id']):
            p = self.all_players[pid]
            d = {'repr': repr(p)}
            for st in info.get('stat_types', []):
                if hasattr(p, st):
                    d[st] = getattr(p, st).stat_info_dict()
            out[pid] = d
            self.logger.info(f'{pid}: {json.dumps(d, default=str)}')
        return out

    def reset_player_stat(self, info: Dict) -> bool:
        ids = self.correspondent_player_ids(info['player_id'])
        with self.lock:
            for pid in ids:
                self.all_players[pid].reset_stats(info.get('stat_types'))
        return bool(ids)

    def _refresh(self, players: Dict) -> None:
        """Rebuild player objects from their persisted state with the current league settings (new code or
        config takes effect without a restart; league.py:637-705)."""
        with self.lock:
            for pid, old in list(players.items()):
                d = old.to_dict()
                d['min_win_rate_games'] = self.cfg.payoff_min_win_rate_games
                players[pid] = player_from_dict(d)
                self.logger.info(f'refreshed player {pid}')

    def refresh_active_player(self) -> bool:
        self._refresh(self.active_players)
        return True

    def refresh_hist_player(self) -> bool:
        self._refresh(self.historical_players)
        return True

    def backup_models(self, info: Optional[Dict] = None) -> str:
        """Copy the checkpoints of the selected players (default all) into ``league_models_backup/<time>``."""
        info = info or {}
        dst = info.get('backup_dir') or os.path.join(self.root, 'league_models_backup',
                                                     time.strftime('%Y-%m-%d-%H-%M-%S'))
        if not self._allowed_path(dst):
            raise ValueError(f'backup_dir {dst!r} is outside the league roots')
        os.makedirs(dst, exist_ok=True)
        n = 0
        for pid in self.correspondent_player_ids(info.get('player_id', 'all')):
            src = self.all_players[pid].checkpoint_path
            if src and os.path.isfile(src):
                shutil.copyfile(src, os.path.join(dst, os.path.basename(src)))
                n += 1
        self.logger.info(f'backed up {n} checkpoints to {dst}')
        return dst

    def _resume_loop(self):
        freq = float(self.cfg.save_resume_freq)
        last = time.time()
        while not self._stop.wait(1.0):
            if time.time() - last >= freq:
                try:
                    self.save_resume()
                except Exception as e:
                    self.logger.error(f'save_resume failed: {e!r}')
                last = time.time()

    def close(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2)
