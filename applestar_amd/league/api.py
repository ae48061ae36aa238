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
        league.load_resume(request.json['resume_path'])
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
        pid = request.json['player_id']
        league.all_players[pid].reset_stats()
        return ok(True)

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
