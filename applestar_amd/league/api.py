"""HTTP control plane of the league (routes of ``distar/ctools/worker/league/league_api.py``) and the
matching client with retries (``Retry(total=20, backoff_factor=1)`` in the reference comm helpers).

The control plane is low-rate JSON (jobs, results, train info); the high-rate data plane
(trajectories, model weights) goes through :mod:`applestar_amd.comm`.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional

from .league import League


def create_league_app(league: League):
    from flask import Flask, jsonify, request

    app = Flask('applestar_league')

    def ok(info: Any = None):
        return jsonify({'code': 0, 'info': info})

    def bad(msg: str):
        return jsonify({'code': 1, 'info': msg})

    @app.route('/league/register_learner', methods=['POST'])
    def register_learner():
        try:
            return ok(league.register_learner(request.json))
        except KeyError as e:
            return bad(str(e))

    @app.route('/league/learner_send_train_info', methods=['POST'])
    def learner_send_train_info():
        return ok(league.learner_send_train_info(request.json))

    @app.route('/league/actor_ask_for_job', methods=['POST'])
    def actor_ask_for_job():
        return ok(league.actor_ask_for_job(request.json or {}))

    @app.route('/league/actor_send_result', methods=['POST'])
    def actor_send_result():
        return ok(league.actor_send_result(request.json))

    @app.route('/league/heartbeat', methods=['POST'])
    def heartbeat():
        d = request.json or {}
        league.health.beat(d.get('role', 'unknown'), str(d.get('id')), d.get('info'))
        return ok(True)

    @app.route('/league/health', methods=['GET'])
    def health():
        return ok({'members': league.health.status(), 'dead': league.health.dead()})

    @app.route('/league/update_config', methods=['GET'])
    def reload_config():
        """Hot reload: re-read ``experiments/<exp>/user_config.yaml`` and merge its league section."""
        from ..utils.config import read_config, deep_update
        path = os.path.join(league.root, 'user_config.yaml')
        if not os.path.exists(path):
            return bad(f'{path} not found')
        new = read_config(path)
        with league.lock:
            deep_update(league.cfg, new.get('league', {}))
        return ok(True)

    @app.route('/league/save_resume', methods=['GET', 'POST'])
    def save_resume():
        return ok(league.save_resume())

    @app.route('/league/load_resume', methods=['POST'])
    def load_resume():
        d = request.json or {}
        path = d.get('resume_path') or d.get('path')
        if not path or not os.path.exists(path):
            return bad(f'resume file {path} not found')
        league.load_resume(path)
        return ok(True)

    @app.route('/league/show_elo', methods=['GET'])
    def show_elo():
        return ok(league.elo.ratings())

    @app.route('/league/show_payoff', methods=['GET'])
    def show_payoff():
        pid = request.args.get('player_id')
        players = league.all_players
        if pid:
            return ok({pid: players[pid].payoff.stat_info_dict()}) if pid in players else bad(f'unknown {pid}')
        return ok({k: p.payoff.stat_info_dict() for k, p in players.items()})

    @app.route('/league/display_players', methods=['GET'])
    def display_players():
        return ok({'active': {k: repr(v) for k, v in league.active_players.items()},
                   'historical': {k: repr(v) for k, v in league.historical_players.items()}})

    @app.route('/league/add_active_player', methods=['POST'])
    def add_active_player():
        d = request.json
        done = league.add_active_player(d['checkpoint_path'], d['player_id'], d.get('pipeline', 'default'),
                                        d.get('frac_id', 1), d.get('z_path', '3map.json'), d.get('z_prob', 0.0),
                                        d.get('teacher_id', 'none'), d.get('teacher_path', 'none'),
                                        d.get('one_phase_step', 2e8), d.get('chosen_weight', 1.0))
        return ok(done)

    @app.route('/league/update_config', methods=['POST'])
    def update_config():
        from ..utils.config import deep_update
        with league.lock:
            deep_update(league.cfg, request.json or {})
        return ok(True)

    @app.route('/league/reset_player_stat', methods=['POST'])
    def reset_player_stat():
        d = request.json or {}
        return ok(True) if league.reset_player_stat(d) else bad(f"unknown player {d.get('player_id')}")

    # ---- statistics views (league_api.py:56-138): active and historical players
    def stat_route(stat, hist):
        def view():
            return ok(league.show_stat(stat, historical=hist))
        view.__name__ = f'show_{"hist_" if hist else ""}{stat}'
        return view

    for stat, name in (('dist_stat', 'dist_stat'), ('cum_stat', 'cum_stat'), ('unit_num_stat', 'unit_num_stat'),
                       ('opponent_payoff', 'opponent_payoff'), ('teammate_payoff', 'teammate_payoff'),
                       ('payoff', 'payoff')):
        if name != 'payoff':
            app.add_url_rule(f'/league/show_{name}', view_func=stat_route(stat, False), methods=['GET'])
        app.add_url_rule(f'/league/show_hist_{name}', view_func=stat_route(stat, True), methods=['GET'])

    # ---- ratings (league_api.py:205-247)
    @app.route('/league/save_elo', methods=['GET'])
    def save_elo():
        return ok(league.save_elo_ratings(zero_min=False))

    @app.route('/league/save_zero_elo', methods=['GET'])
    def save_zero_elo():
        return ok(league.save_elo_ratings(zero_min=True))

    @app.route('/league/update_elo', methods=['POST'])
    def update_elo():
        return ok(league.update_elo(request.json or {}))

    @app.route('/league/show_trueskill', methods=['GET'])
    def show_trueskill():
        return ok(league.trueskill.ratings())

    @app.route('/league/save_trueskill', methods=['GET'])
    def save_trueskill():
        return ok(league.save_trueskill_ratings())

    @app.route('/league/update_trueskill', methods=['POST'])
    def update_trueskill():
        return ok(league.update_trueskill(request.json or {}))

    # ---- player management (league_api.py:188-199,257-313)
    @app.route('/league/add_hist_player', methods=['POST'])
    def add_hist_player():
        return ok(True) if league.add_hist_player(request.json or {}) else bad('checkpoint not found')

    @app.route('/league/remove_hist_player', methods=['POST'])
    def remove_hist_player():
        return ok(True) if league.remove_hist_player(request.json or {}) else bad('no such historical player')

    @app.route('/league/update_player', methods=['POST'])
    def update_player():
        d = request.json or {}
        return ok(True) if league.update_player(d) else bad(f"unknown player {d.get('player_id')}")

    @app.route('/league/display_player', methods=['POST'])
    def display_player():
        return ok(league.display_player(request.json or {}))

    @app.route('/league/refresh_active_player', methods=['GET'])
    def refresh_active_player():
        return ok(league.refresh_active_player())

    @app.route('/league/refresh_hist_player', methods=['GET'])
    def refresh_hist_player():
        return ok(league.refresh_hist_player())

    @app.route('/league/refresh_all_player', methods=['GET'])
    def refresh_all_player():
        return ok(league.refresh_active_player() and league.refresh_hist_player())

    @app.route('/league/backup_models', methods=['POST'])
    def backup_models():
        try:
            return ok(league.backup_models(request.json or {}))
        except ValueError as e:
            return bad(str(e))

    @app.route('/league/show_config', methods=['GET'])
    def show_config():
        return ok(json.loads(json.dumps(league.cfg, default=str)))

    return app


class HttpClient:
    """Minimal JSON client with exponential back-off retries."""

    def __init__(self, ip: str, port: int, retries: int = 20, backoff: float = 1.0, timeout: float = 30.0):
        self.base = f'http://{ip}:{port}'
        self.retries = retries
        self.backoff = backoff
        self.timeout = timeout

    def post(self, route: str, data: Optional[Dict] = None) -> Any:
        import requests
        err = None
        for i in range(self.retries + 1):
            try:
                r = requests.post(self.base + route, json=data or {}, timeout=self.timeout)
                r.raise_for_status()
                body = r.json()
                if body.get('code', 0) != 0:
                    raise RuntimeError(body.get('info'))
                return body.get('info')
            except (requests.ConnectionError, requests.Timeout) as e:
                err = e
                time.sleep(min(self.backoff * (2 ** i), 30.0))
        raise ConnectionError(f'{route}: {err}')

    def get(self, route: str, params: Optional[Dict] = None) -> Any:
        import requests
        r = requests.get(self.base + route, params=params, timeout=self.timeout)
        r.raise_for_status()
        return r.json().get('info')


def serve(league: League, host: str = '0.0.0.0', port: int = 23335, threaded: bool = True):
    app = create_league_app(league)
    app.run(host=host, port=port, threaded=threaded, use_reloader=False)
