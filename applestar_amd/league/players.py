"""League players and their matchmaking policies.

Player types are decoded from the id prefix like the reference (``league.py:793-825``,
``player.py:253-760``):

====  ==============================  =======================================================
MP    MainPlayer                      sp (self-play, falls back to a PFSP-chosen snapshot of
                                      the opponent when its win rate < 0.3) / pfsp (squared) / eval
EP    ExploiterPlayer (league expl.)  pfsp (normal) / eval; reset with prob 0.25 on snapshot
EE    ExpertExploiterPlayer           like EP, rotates themed Z files; reset to latest MP snapshot
ME    MainExploiterPlayer             vs_main while beating it > 0.2 else pfsp vs MP snapshots
EX    ExpertPlayer                    pfsp (variance) over non-expert history / eval
AE    AdaptiveEvolutionaryExploiter   vs a random MP / pfsp; evolutionary reset pool
====  ==============================  =======================================================

``is_trained_enough`` gates snapshots: ``one_phase_step`` frames, or (after half a phase) beating
every relevant opponent at ``strong_win_rate`` over ``warm_up_size`` games.
"""
from __future__ import annotations

import os
import random
from typing import Dict, List, Optional, Tuple

from .stats import Payoff, RaceStat, pfsp

FRAC_ID = {0: ['zerg', 'terran', 'protoss'], 1: ['zerg'], 2: ['terran'], 3: ['protoss']}


class Player:
    kind = 'base'
    persist = ['checkpoint_path', 'player_id', 'pipeline', 'frac_id', 'z_path', 'z_prob', 'teacher_id',
               'teacher_checkpoint_path', 'total_agent_step', 'decay', 'warm_up_size', 'min_win_rate_games',
               'total_game_count']

    def __init__(self, checkpoint_path: str, player_id: str, pipeline: str = 'default', frac_id: int = 1,
                 z_path='3map.json', z_prob: float = 0.0, teacher_id: str = 'none',
                 teacher_checkpoint_path: str = 'none', total_agent_step: int = 0, decay: float = 0.995,
                 warm_up_size: int = 1000, min_win_rate_games: int = 200, total_game_count: int = 0, **_):
        self.checkpoint_path = checkpoint_path
        self.player_id = player_id
        self.pipeline = pipeline
        self.frac_id = frac_id
        self.z_path = z_path
        self.z_prob = z_prob
        self.teacher_id = teacher_id
        self.teacher_checkpoint_path = teacher_checkpoint_path
        self.total_agent_step = int(total_agent_step)
        self.decay = decay
        self.warm_up_size = warm_up_size
        self.min_win_rate_games = min_win_rate_games
        self.total_game_count = total_game_count
        self.payoff = Payoff(decay, warm_up_size, min_win_rate_games)
        # team-game payoffs of the reference's Player (kept and persisted; 1v1 results only feed ``payoff``)
        self.teammate_payoff = Payoff(decay, warm_up_size, min_win_rate_games)
        self.opponent_payoff = Payoff(decay, warm_up_size, min_win_rate_games)

    def get_race(self) -> str:
        return random.choice(FRAC_ID[self.frac_id])

    STAT_TYPES = ('payoff', 'teammate_payoff', 'opponent_payoff')

    def reset_stats(self, stat_types=None):
        for k in (Player.STAT_TYPES if stat_types is None else stat_types):
            if k in Player.STAT_TYPES:
                setattr(self, k, Payoff(self.decay, self.warm_up_size, self.min_win_rate_games))

    def to_dict(self) -> Dict:
        d = {k: getattr(self, k) for k in self.persist}
        d['kind'] = self.kind
        for k in self.STAT_TYPES:
            d[k] = getattr(self, k).to_dict()
        return d

    def __repr__(self):
        return f'{type(self).__name__}({self.player_id}, step={self.total_agent_step})'


class HistoricalPlayer(Player):
    kind = 'historical'
    persist = Player.persist + ['parent_id']

    def __init__(self, *a, parent_id: str = 'none', **kw):
        kw.setdefault('teacher_id', 'none')
        kw.setdefault('teacher_checkpoint_path', 'none')
        super().__init__(*a, **kw)
        self.parent_id = parent_id


def _hist_ids(historical: Dict[str, HistoricalPlayer], include_bots: bool, pred=None) -> List[str]:
    out = []
    for pid, p in historical.items():
        if not include_bots and p.pipeline == 'bot':
            continue
        if pred is not None and not pred(p):
            continue
        out.append(pid)
    return out


class ActivePlayer(Player):
    kind = 'active'
    persist = Player.persist + ['one_phase_step', 'chosen_weight', 'last_enough_step', 'snapshot_times',
                                'strong_win_rate', 'successive_model_path', 'last_successive_step']

    def __init__(self, *a, chosen_weight: float = 1.0, one_phase_step: float = 2e8, last_enough_step: int = 0,
                 snapshot_times: int = 0, strong_win_rate: float = 0.7, successive_model_path: Optional[str] = None,
                 last_successive_step: int = 0, **kw):
        super().__init__(*a, **kw)
        self.chosen_weight = chosen_weight
        self.one_phase_step = int(float(one_phase_step))
        self.last_enough_step = last_enough_step
        self.snapshot_times = snapshot_times
        self.strong_win_rate = strong_win_rate
        self.successive_model_path = successive_model_path or self.checkpoint_path
        self.last_successive_step = last_successive_step
        self.snapshot_flag = False
        self.reset_flag = False
        self.dist_stat = RaceStat(self.decay, self.warm_up_size)
        self.cum_stat = RaceStat(self.decay, self.warm_up_size)
        self.unit_num_stat = RaceStat(self.decay, self.warm_up_size)

    # ---------------------------------------------------------------- matchmaking
    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False) -> Tuple[str, list, list]:
        raise NotImplementedError

    def _pick_branch(self, branch_probs) -> str:
        probs = branch_probs[type(self).__name__]
        return random.choices(list(probs.keys()), weights=list(probs.values()), k=1)[0]

    def _pfsp_pick(self, keys: List[str], historical, weighting: str, default: float = 0.5):
        if not keys:
            raise RuntimeError(f'{self.player_id}: no historical opponent available for pfsp')
        w = [self.payoff.pfsp_winrate_info_dict.get(k, default) for k in keys]
        return historical[random.choices(keys, weights=list(pfsp(w, weighting)), k=1)[0]]

    # ---------------------------------------------------------------- snapshot / reset
    def _beats(self, opponent_ids: List[str], margin: float = 0.0) -> bool:
        for pid in opponent_ids:
            e = self.payoff.record.get(pid)
            if e is None or not (e['winrate'].val > self.strong_win_rate + margin and
                                 e['winrate'].count >= self.warm_up_size):
                return False
        return True

    def _phase_gate(self, half_phase: bool = True) -> Optional[bool]:
        """Common prefix of is_trained_enough: True/False when decided, None to continue."""
        if self.snapshot_flag:
            self.snapshot_flag = False
            self.last_enough_step = self.total_agent_step
            return True
        passed = self.total_agent_step - self.last_enough_step
        if half_phase and passed < self.one_phase_step / 2:
            return False
        if passed >= self.one_phase_step:
            self.last_enough_step = self.total_agent_step
            return True
        return None

    def is_trained_enough(self, historical, active, pfsp_train_bot=False) -> bool:
        raise NotImplementedError

    def is_save_successive_model(self) -> bool:
        if self.total_agent_step - self.last_successive_step > self.one_phase_step / 2:
            self.last_successive_step = self.total_agent_step
            return True
        return False

    def is_reset(self) -> bool:
        return False

    def reset_checkpoint(self, active, historical, new_player_id) -> str:
        return self.teacher_checkpoint_path

    def snapshot(self) -> HistoricalPlayer:
        self.snapshot_times += 1
        hid = self.player_id + f'H{self.snapshot_times}'
        root, ext = os.path.splitext(self.checkpoint_path)
        return HistoricalPlayer(checkpoint_path=f'{root}_{self.total_agent_step}{ext or ".pth"}', player_id=hid,
                                pipeline=self.pipeline, frac_id=self.frac_id, z_path=self.z_path, z_prob=self.z_prob,
                                total_agent_step=self.total_agent_step, decay=self.decay,
                                warm_up_size=self.warm_up_size, min_win_rate_games=self.min_win_rate_games,
                                parent_id=self.player_id)

    STAT_TYPES = Player.STAT_TYPES + ('dist_stat', 'cum_stat', 'unit_num_stat')

    def reset_stats(self, stat_types=None):
        types = stat_types or self.STAT_TYPES
        super().reset_stats([k for k in types if k in Player.STAT_TYPES])
        for k in ('dist_stat', 'cum_stat', 'unit_num_stat'):
            if k in types:
                setattr(self, k, RaceStat(self.decay, self.warm_up_size))

    def to_dict(self):
        d = super().to_dict()
        d.update(dist_stat=self.dist_stat.to_dict(), cum_stat=self.cum_stat.to_dict(),
                 unit_num_stat=self.unit_num_stat.to_dict())
        return d


class MainPlayer(ActivePlayer):
    kind = 'MP'

    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False):
        branch = self._pick_branch(branch_probs)
        if branch == 'sp':
            opp = random.choice([p for p in active.values() if isinstance(p, MainPlayer)])
            if opp is not self and self.payoff.pfsp_winrate_info_dict.get(opp.player_id, 0.5) < 0.3:
                keys = _hist_ids(historical, True, lambda p: p.parent_id == opp.player_id)
                if not keys:
                    keys = _hist_ids(historical, False)
                opp = self._pfsp_pick(keys, historical, 'variance')
            return branch, [self], [opp]
        if branch == 'pfsp':
            return branch, [self], [self._pfsp_pick(_hist_ids(historical, pfsp_train_bot), historical, 'squared')]
        if branch == 'eval':
            return branch, [self], [historical[random.choice(list(historical))]]
        raise NotImplementedError(branch)

    def is_trained_enough(self, historical, active, pfsp_train_bot=False):
        g = self._phase_gate()
        if g is not None:
            return g
        hist = _hist_ids(historical, pfsp_train_bot)
        if self._beats(hist, margin=0.1):
            return True
        if self._beats(hist + [p for p in active if p != self.player_id]):
            self.last_enough_step = self.total_agent_step
            return True
        return False


class ExploiterPlayer(ActivePlayer):
    kind = 'EP'
    reset_prob = 0.25

    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False):
        branch = self._pick_branch(branch_probs)
        if branch == 'pfsp':
            return branch, [self], [self._pfsp_pick(_hist_ids(historical, pfsp_train_bot), historical, 'normal')]
        if branch == 'eval':
            return branch, [self], [historical[random.choice(list(historical))]]
        raise NotImplementedError(branch)

    def is_trained_enough(self, historical, active, pfsp_train_bot=False):
        g = self._phase_gate()
        if g is not None:
            return g
        if self._beats(_hist_ids(historical, pfsp_train_bot)):
            self.last_enough_step = self.total_agent_step
            return True
        return False

    def is_reset(self):
        if self.reset_flag:
            self.reset_flag = False
            return True
        return random.random() < self.reset_prob


class ExpertExploiterPlayer(ExploiterPlayer):
    kind = 'EE'

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.z_paths = list(self.z_path) if isinstance(self.z_path, (list, tuple)) else [self.z_path]
        self.z_path = random.choice(self.z_paths)

    def is_reset(self):
        self.z_path = random.choice(self.z_paths)
        return True

    def snapshot(self):
        hp = super().snapshot()
        hp.player_id = hp.player_id + '_' + os.path.basename(str(self.z_path)).split('.')[0]
        return hp

    def reset_checkpoint(self, active, historical, new_player_id):
        mains = sorted([p for p in historical if 'MP' in p and 'H' in p], key=lambda x: int(x.split('H')[-1].split('_')[0]))
        return historical[mains[-1]].checkpoint_path if mains else self.teacher_checkpoint_path

    def to_dict(self):
        d = super().to_dict()
        d['z_path'] = self.z_paths
        return d


class MainExploiterPlayer(ActivePlayer):
    kind = 'ME'

    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False):
        main = active.get(f'MP{self.player_id[-1]}') or next(p for p in active.values() if isinstance(p, MainPlayer))
        branch = self._pick_branch(branch_probs)
        if branch == 'vs_main':
            if self.payoff.pfsp_winrate_info_dict.get(main.player_id, 0.5) > 0.2:
                return branch, [self], [main]
            branch = 'pfsp'
        elif branch == 'eval':
            return 'vs_main_eval', [self], [main]
        if branch == 'pfsp':
            keys = _hist_ids(historical, True, lambda p: p.parent_id == main.player_id)
            if not keys:  # the main agent has no snapshot yet: train against it directly
                return 'vs_main', [self], [main]
            return branch, [self], [self._pfsp_pick(keys, historical, 'variance')]
        raise NotImplementedError(branch)

    def is_trained_enough(self, historical, active, pfsp_train_bot=False):
        g = self._phase_gate(half_phase=False)
        if g is not None:
            return g
        if self._beats([p for p in active if 'MP' in p]):
            self.last_enough_step = self.total_agent_step
            return True
        return False

    def is_reset(self):
        return True


class ExpertPlayer(ActivePlayer):
    kind = 'EX'

    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False):
        branch = self._pick_branch(branch_probs)
        if branch == 'pfsp':
            keys = [k for k in historical if 'EX' not in k]
            return branch, [self], [self._pfsp_pick(keys, historical, 'variance', default=0.1)]
        if branch == 'eval':
            return branch, [self], [historical[random.choice(list(historical))]]
        raise NotImplementedError(branch)

    def is_trained_enough(self, historical, active, pfsp_train_bot=False):
        g = self._phase_gate(half_phase=False)
        return bool(g)


class AdaptiveEvolutionaryExploiterPlayer(MainExploiterPlayer):
    kind = 'AE'
    persist = ActivePlayer.persist + ['init_players']

    def __init__(self, *a, init_players=None, **kw):
        super().__init__(*a, **kw)
        self.init_players = list(init_players or [])
        self.reset_prob = 0.25

    def get_branch_opponent(self, historical, active, branch_probs, pfsp_train_bot=False):
        mains = [p for p in active.values() if 'MP' in p.player_id]
        main = random.choice(mains)
        branch = self._pick_branch(branch_probs)
        if branch == 'vs_main':
            if self.payoff.pfsp_winrate_info_dict.get(main.player_id, 0.5) > 0.2:
                return branch, [self], [main]
            branch = 'pfsp'
        elif branch == 'eval':
            return 'vs_main_eval', [self], [main]
        keys = _hist_ids(historical, True, lambda p: p.parent_id == main.player_id)
        if not keys:
            return 'vs_main', [self], [main]
        return 'pfsp', [self], [self._pfsp_pick(keys, historical, 'variance')]

    def reset_checkpoint(self, active, historical, new_player_id):
        """Evolutionary reset: restart from the teacher with prob 0.25, else from the pool member whose
        win rate against a main player is in [0.2, 0.5] (closest to a fair fight)."""
        mains = [p for p in active if 'MP' in p]
        main = random.choice(mains)
        if random.random() < self.reset_prob:
            self.init_players.append(new_player_id)
            return self.teacher_checkpoint_path
        best_id, best_wr, best_idx = None, 0.0, None
        wr = self.payoff.win_rate(main, respect_min_games=False)
        if 0.2 <= wr <= 0.5:
            best_id, best_wr, best_idx = new_player_id, wr, -1
        for i, pid in enumerate(self.init_players):
            w = 1 - active[main].payoff.win_rate(pid, respect_min_games=False)
            if 0.2 <= w <= 0.5 and w > best_wr:
                best_id, best_wr, best_idx = pid, w, i
        if best_idx is not None and best_idx != -1:
            del self.init_players[best_idx]
            if new_player_id is not None:
                self.init_players.append(new_player_id)
        if best_id is None or best_id not in historical:
            return self.teacher_checkpoint_path
        return historical[best_id].checkpoint_path


PLAYER_TYPES = {'MP': MainPlayer, 'EP': ExploiterPlayer, 'EE': ExpertExploiterPlayer, 'ME': MainExploiterPlayer,
                'EX': ExpertPlayer, 'AE': AdaptiveEvolutionaryExploiterPlayer}


def active_player_type(player_id: str):
    for prefix, cls in PLAYER_TYPES.items():
        if prefix in player_id:
            return cls
    return None


def player_from_dict(d: Dict) -> Player:
    d = dict(d)
    kind = d.pop('kind')
    payoffs = {k: d.pop(k, None) for k in Player.STAT_TYPES}
    stats = {k: d.pop(k, None) for k in ('dist_stat', 'cum_stat', 'unit_num_stat')}
    if kind == 'historical':
        p = HistoricalPlayer(**d)
    else:
        p = PLAYER_TYPES[kind](**d)
        for k, v in stats.items():
            if v is not None:
                setattr(p, k, RaceStat.from_dict(v))
    for k, v in payoffs.items():
        if v is not None:
            setattr(p, k, Payoff.from_dict(v))
    return p
