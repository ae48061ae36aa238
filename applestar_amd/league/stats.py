"""League statistics: payoff tables, PFSP weighting, ELO, per-race distance/cumulative stats.

Behaviour follows ``distar/ctools/worker/league/{payoff,algorithms,dist_stat,cum_stat}.py`` and
``ctools/worker/ladder/{elo,trueskill_algo}.py``:

* ``Payoff``: per-opponent moving averages (window = warm-up size) of win rate, game steps / iters /
  duration; PFSP sees 0.5 until ``min_win_rate_games`` games were played.
* ``pfsp``: squared (1-x)^2, variance x(1-x), normal min(0.5, 1-x); uniform if all win rates ~0.
* ``ELORating``: K=44 pairwise updates.
All state is plain Python data so the league can be checkpointed as JSON (no pickling).
"""
from __future__ import annotations

import math
from collections import defaultdict, deque
from typing import Optional, Dict, Iterable, List

import numpy as np


class MovingAverage:
    __slots__ = ('length', 'history', 'count')

    def __init__(self, length: int = 1000):
        self.length = length
        self.history = deque(maxlen=length)
        self.count = 0

    def update(self, v: float):
        self.history.append(float(v))
        self.count += 1

    @property
    def val(self) -> float:
        return sum(self.history) / len(self.history) if self.history else 0.0

    def to_dict(self):
        return {'length': self.length, 'history': list(self.history), 'count': self.count}

    @classmethod
    def from_dict(cls, d):
        m = cls(d['length'])
        m.history.extend(d['history'])
        m.count = d['count']
        return m


class Payoff:
    keys = ('winrate', 'game_steps', 'game_iters', 'game_duration')

    def __init__(self, decay: float = 0.999, warm_up_size: int = 1000, min_win_rate_games: int = 1000):
        self.decay = decay
        self.warm_up_size = warm_up_size
        self.min_win_rate_games = min_win_rate_games
        self.record: Dict[str, Dict[str, MovingAverage]] = {}

    def _entry(self, opponent_id: str):
        if opponent_id not in self.record:
            self.record[opponent_id] = {k: MovingAverage(self.warm_up_size) for k in self.keys}
        return self.record[opponent_id]

    def update(self, opponent_id: str, info: Dict[str, float]) -> None:
        e = self._entry(opponent_id)
        for k in self.keys:
            e[k].update(info[k])

    def win_rate(self, opponent_id: str, respect_min_games: bool = True) -> float:
        e = self.record.get(opponent_id)
        if e is None or (respect_min_games and e['winrate'].count < self.min_win_rate_games):
            return 0.5
        return e['winrate'].val

    def games(self, opponent_id: str) -> int:
        e = self.record.get(opponent_id)
        return 0 if e is None else e['winrate'].count

    @property
    def pfsp_winrate_info_dict(self) -> Dict[str, float]:
        return {p: self.win_rate(p) for p in self.record}

    def stat_info_dict(self) -> Dict[str, Dict[str, float]]:
        return {p: {k: m.val for k, m in e.items()} for p, e in self.record.items()}

    def table(self) -> str:
        rows = [['opponent', *self.keys, 'games']]
        for p, e in sorted(self.record.items()):
            rows.append([p] + [f'{e[k].val:.3f}' for k in self.keys] + [str(e['winrate'].count)])
        w = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
        return '\n'.join(' | '.join(c.ljust(w[i]) for i, c in enumerate(r)) for r in rows)

    def to_dict(self):
        return {'decay': self.decay, 'warm_up_size': self.warm_up_size, 'min_win_rate_games': self.min_win_rate_games,
                'record': {p: {k: m.to_dict() for k, m in e.items()} for p, e in self.record.items()}}

    @classmethod
    def from_dict(cls, d):
        p = cls(d['decay'], d['warm_up_size'], d['min_win_rate_games'])
        p.record = {o: {k: MovingAverage.from_dict(m) for k, m in e.items()} for o, e in d['record'].items()}
        return p


_PFSP = {
    'squared': lambda x: (1 - x) ** 2,
    'variance': lambda x: x * (1 - x),
    'normal': lambda x: np.minimum(0.5, 1 - x),
}


def pfsp(win_rates: Iterable[float], weighting: str = 'variance') -> np.ndarray:
    """Prioritised fictitious self-play selection probabilities (algorithms.py:58-85)."""
    x = np.asarray(list(win_rates), dtype=np.float64)
    if x.size == 0:
        raise ValueError('pfsp needs at least one opponent')
    if weighting not in _PFSP:
        raise KeyError(f'invalid pfsp weighting {weighting}')
    if x.sum() < 1e-8:
        return np.full_like(x, 1.0 / len(x))
    f = _PFSP[weighting](x)
    s = f.sum()
    if s < 1e-12:
        return np.full_like(x, 1.0 / len(x))
    return f / s


class ELORating:
    WIN, DRAW, LOSS = 1, 0, -1

    def __init__(self, K: float = 44, init_elo: float = 1000):
        self.K = K
        self.init_elo = init_elo
        self.elos: Dict[str, float] = defaultdict(float)
        self.games: Dict[str, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
        self.wins: Dict[str, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
        self.game_count = 0

    def expected(self, p1: str, p2: str) -> float:
        return 1.0 / (1.0 + 10 ** ((self.elos[p2] - self.elos[p1]) / 400.0))

    def update(self, p1: str, p2: str, result: int) -> None:
        e1 = self.expected(p1, p2)
        s = 1.0 if result == self.WIN else (0.0 if result == self.LOSS else 0.5)
        if result == self.WIN:
            self.wins[p1][p2] += 1
        elif result == self.LOSS:
            self.wins[p2][p1] += 1
        self.games[p1][p2] += 1
        self.games[p2][p1] += 1
        self.elos[p1] += self.K * (s - e1)
        self.elos[p2] -= self.K * (s - e1)
        self.game_count += 1

    def ratings(self, start_from_zero: bool = True) -> Dict[str, float]:
        r = {k: v + self.init_elo for k, v in self.elos.items()}
        if start_from_zero and r:
            lo = min(r.values())
            r = {k: v - lo for k, v in r.items()}
        return dict(sorted(r.items(), key=lambda kv: kv[1]))

    def text(self) -> str:
        return '\n'.join(f'{k:24s} {v:8.1f}' for k, v in self.ratings().items())

    def to_dict(self):
        return {'K': self.K, 'init_elo': self.init_elo, 'elos': dict(self.elos),
                'games': {k: dict(v) for k, v in self.games.items()},
                'wins': {k: dict(v) for k, v in self.wins.items()}, 'game_count': self.game_count}

    @classmethod
    def from_dict(cls, d):
        e = cls(d['K'], d['init_elo'])
        e.elos.update(d['elos'])
        for k, v in d['games'].items():
            e.games[k].update(v)
        for k, v in d['wins'].items():
            e.wins[k].update(v)
        e.game_count = d['game_count']
        return e


def trueskill_win_probability(mu1: float, sigma1: float, mu2: float, sigma2: float, beta: float = 25 / 6) -> float:
    """P(player1 beats player2) under TrueSkill (trueskill_algo.py:8)."""
    delta = mu1 - mu2
    denom = math.sqrt(2 * beta * beta + sigma1 * sigma1 + sigma2 * sigma2)
    return 0.5 * (1 + math.erf(delta / (denom * math.sqrt(2))))


def _norm_pdf(x: float) -> float:
    return math.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)


def _norm_cdf(x: float) -> float:
    return 0.5 * (1 + math.erf(x / math.sqrt(2)))


def _norm_ppf(p: float) -> float:
    lo, hi = -10.0, 10.0
    for _ in range(100):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if _norm_cdf(mid) < p else (lo, mid)
    return 0.5 * (lo + hi)


class TrueSkillRating:
    """1v1 TrueSkill (Herbrich et al. 2006) for the league's players: Gaussian skill N(mu, sigma^2), dynamics
    noise tau, performance noise beta, draw margin from ``draw_probability``.  The reference's league API exposes
    show / save / update_trueskill routes (``league_api.py:230-247``) whose league methods it never defines;
    this is the working version (win probability: :func:`trueskill_win_probability`)."""

    def __init__(self, mu: float = 25.0, sigma: float = 25 / 3, beta: float = 25 / 6, tau: float = 25 / 300,
                 draw_probability: float = 0.1):
        self.mu0, self.sigma0, self.beta, self.tau, self.draw_probability = mu, sigma, beta, tau, draw_probability
        self.eps = _norm_ppf((draw_probability + 1) / 2) * math.sqrt(2) * beta
        self.mu: Dict[str, float] = {}
        self.sigma: Dict[str, float] = {}
        self.game_count = 0

    def get(self, pid: str):
        return self.mu.get(pid, self.mu0), self.sigma.get(pid, self.sigma0)

    def update(self, p1: str, p2: str, result: int) -> None:
        """result: 1 = p1 won, -1 = p2 won, 0 = draw."""
        if result < 0:
            p1, p2 = p2, p1
        (m1, s1), (m2, s2) = self.get(p1), self.get(p2)
        s1, s2 = math.sqrt(s1 * s1 + self.tau ** 2), math.sqrt(s2 * s2 + self.tau ** 2)
        c = math.sqrt(2 * self.beta ** 2 + s1 * s1 + s2 * s2)
        t, e = (m1 - m2) / c, self.eps / c
        if result == 0:
            den = max(_norm_cdf(e - t) - _norm_cdf(-e - t), 1e-12)
            v = (_norm_pdf(-e - t) - _norm_pdf(e - t)) / den
            w = v * v + ((e - t) * _norm_pdf(e - t) + (e + t) * _norm_pdf(e + t)) / den
        else:
            den = max(_norm_cdf(t - e), 1e-12)
            v = _norm_pdf(t - e) / den
            w = v * (v + t - e)
        self.mu[p1] = m1 + s1 * s1 / c * v
        self.mu[p2] = m2 - s2 * s2 / c * v
        self.sigma[p1] = s1 * math.sqrt(max(1 - s1 * s1 / (c * c) * w, 1e-6))
        self.sigma[p2] = s2 * math.sqrt(max(1 - s2 * s2 / (c * c) * w, 1e-6))
        self.game_count += 1

    def set(self, pid: str, mu: Optional[float] = None, sigma: Optional[float] = None) -> None:
        if mu is not None:
            self.mu[pid] = float(mu)
        if sigma is not None:
            self.sigma[pid] = float(sigma)

    def win_probability(self, p1: str, p2: str) -> float:
        (m1, s1), (m2, s2) = self.get(p1), self.get(p2)
        return trueskill_win_probability(m1, s1, m2, s2, self.beta)

    def ratings(self) -> Dict[str, Dict[str, float]]:
        """Sorted by the conservative skill mu - 3 sigma."""
        ids = sorted(set(self.mu) | set(self.sigma), key=lambda k: self.get(k)[0] - 3 * self.get(k)[1])
        return {k: {'mu': self.get(k)[0], 'sigma': self.get(k)[1], 'skill': self.get(k)[0] - 3 * self.get(k)[1]}
                for k in ids}

    def text(self) -> str:
        return '\n'.join(f'{k:24s} mu {v["mu"]:7.2f} sigma {v["sigma"]:6.2f} skill {v["skill"]:7.2f}'
                         for k, v in self.ratings().items())

    def to_dict(self):
        return {'mu0': self.mu0, 'sigma0': self.sigma0, 'beta': self.beta, 'tau': self.tau,
                'draw_probability': self.draw_probability, 'mu': self.mu, 'sigma': self.sigma,
                'game_count': self.game_count}

    @classmethod
    def from_dict(cls, d):
        t = cls(d['mu0'], d['sigma0'], d['beta'], d['tau'], d['draw_probability'])
        t.mu, t.sigma, t.game_count = dict(d['mu']), dict(d['sigma']), d['game_count']
        return t


class RaceStat:
    """Per-race exponential moving averages of arbitrary scalar game statistics (DistStat / CumStat /
    UnitNumStat: Z-distance rewards, cumulative-stat in/out rates, unit counts)."""

    def __init__(self, decay: float = 0.99, warm_up_size: int = 100):
        self.decay = decay
        self.warm_up_size = warm_up_size
        self.values: Dict[str, Dict[str, float]] = {}
        self.game_count: Dict[str, int] = defaultdict(int)

    def update(self, race: str, info: Dict[str, float]) -> None:
        race = str(race)
        v = self.values.setdefault(race, {})
        n = self.game_count[race]
        for k, x in info.items():
            if not isinstance(x, (int, float)):
                continue
            if k not in v or n < self.warm_up_size:
                # running mean while warming up, EMA afterwards
                v[k] = x if k not in v else v[k] + (x - v[k]) / (n + 1)
            else:
                v[k] = self.decay * v[k] + (1 - self.decay) * x
        self.game_count[race] = n + 1

    def stat_info_dict(self):
        return {r: dict(v) for r, v in self.values.items()}

    def to_dict(self):
        return {'decay': self.decay, 'warm_up_size': self.warm_up_size, 'values': self.values,
                'game_count': dict(self.game_count)}

    @classmethod
    def from_dict(cls, d):
        s = cls(d['decay'], d['warm_up_size'])
        s.values = d['values']
        s.game_count.update(d['game_count'])
        return s
