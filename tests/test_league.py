"""League: PFSP, payoff, ELO, job dispatch per player type, snapshot/reset, JSON resume, HTTP API."""
import os
import random

import numpy as np
import pytest

from applestar_amd.league.league import League
from applestar_amd.league.players import MainPlayer, MainExploiterPlayer, ExploiterPlayer, HistoricalPlayer
from applestar_amd.league.stats import pfsp, Payoff, ELORating, trueskill_win_probability


def test_pfsp_weightings():
    w = np.array([0.1, 0.5, 0.9])
    assert np.allclose(pfsp(w, 'squared'), (1 - w) ** 2 / ((1 - w) ** 2).sum())
    assert np.allclose(pfsp(w, 'variance'), w * (1 - w) / (w * (1 - w)).sum())
    nm = np.minimum(0.5, 1 - w)
    assert np.allclose(pfsp(w, 'normal'), nm / nm.sum())
    assert np.allclose(pfsp(np.zeros(4)), 0.25)


def test_payoff_min_games_and_elo():
    p = Payoff(warm_up_size=10, min_win_rate_games=3)
    for r in (1, 1):
        p.update('x', {'winrate': r, 'game_steps': 1, 'game_iters': 1, 'game_duration': 1})
    assert p.win_rate('x') == 0.5
    p.update('x', {'winrate': 0, 'game_steps': 1, 'game_iters': 1, 'game_duration': 1})
    assert abs(p.win_rate('x') - 2 / 3) < 1e-9
    e = ELORating()
    e.update('a', 'b', 1)
    assert e.elos['a'] > 0 > e.elos['b'] and abs(e.elos['a'] - 22) < 1e-9
    assert abs(trueskill_win_probability(25, 8, 25, 8) - 0.5) < 1e-9


def _cfg(tmp, players=('MP0', 'ME0', 'EP0')):
    n = len(players)
    return {'league': {'active_players': {'checkpoint_path': ['none'] * n, 'player_id': list(players),
                                          'pipeline': ['default'] * n, 'frac_id': [1] * n, 'z_prob': [0.0] * n,
                                          'teacher_id': ['t'] * n, 'teacher_path': ['none'] * n,
                                          'z_path': ['3map.json'] * n, 'one_phase_step': [1000] * n,
                                          'chosen_weight': [1] * n},
                       'historical_players': {'player_id': ['sl'], 'checkpoint_path': ['none'], 'pipeline': ['default'],
                                              'frac_id': [1], 'z_prob': [0.0], 'z_path': ['3map.json']},
                       'stat_warm_up_size': 5, 'payoff_min_win_rate_games': 2, 'save_resume_freq': 1e9}}


def test_jobs_snapshot_reset_resume(tmp_path):
    random.seed(0)
    lg = League(_cfg(tmp_path), root=str(tmp_path), start_threads=False)
    assert isinstance(lg.active_players['MP0'], MainPlayer)
    assert isinstance(lg.active_players['ME0'], MainExploiterPlayer)
    assert isinstance(lg.active_players['EP0'], ExploiterPlayer)
    branches = set()
    for _ in range(60):
        job = lg.actor_ask_for_job({'job_type': 'train'})
        assert len(job['player_ids']) == 2 and job['env_info']['map_name'] == 'KairosJunction'
        branches.add(job['branch'])
        lg.apply_result({'0': {'player_id': job['player_ids'][0], 'opponent_id': job['player_ids'][1], 'winloss': 1,
                               'race_id': 'zerg'},
                         '1': {'player_id': job['player_ids'][1], 'opponent_id': job['player_ids'][0], 'winloss': -1,
                               'race_id': 'zerg'},
                         'game_steps': 100, 'game_iters': 10, 'game_duration': 1.0})
    assert branches & {'sp', 'pfsp'} and branches & {'vs_main', 'vs_main_eval', 'pfsp'}
    assert lg.elo.game_count == 60
    # trained enough by steps -> snapshot becomes a historical player with the parent id
    out = lg.learner_send_train_info({'player_id': 'MP0', 'train_steps': 1000, 'checkpoint_path': ''})
    snaps = [h for h in lg.historical_players.values() if h.parent_id == 'MP0']
    assert len(snaps) == 1 and snaps[0].player_id == 'MP0H1'
    assert out['reset_checkpoint_path'] == 'none'            # main players never reset
    out = lg.learner_send_train_info({'player_id': 'ME0', 'train_steps': 1000, 'checkpoint_path': ''})
    assert out['reset_checkpoint_path'] != 'none'            # main exploiters always reset after a snapshot
    # ladder job among historical players / bots
    assert lg.actor_ask_for_job({'job_type': 'ladder'})['branch'] == 'ladder'
    # resume round trip
    path = lg.save_resume(os.path.join(tmp_path, 'r.json'))
    lg2 = League(dict(_cfg(tmp_path), league=dict(_cfg(tmp_path)['league'], resume_path=path)), root=str(tmp_path),
                 start_threads=False)
    assert set(lg2.historical_players) == set(lg.historical_players)
    assert lg2.active_players['MP0'].payoff.stat_info_dict() == lg.active_players['MP0'].payoff.stat_info_dict()
    assert lg2.elo.game_count == 60


def test_http_api(tmp_path):
    flask = pytest.importorskip('flask')
    from applestar_amd.league.api import create_league_app
    lg = League(_cfg(tmp_path, players=('MP0',)), root=str(tmp_path), start_threads=True)
    c = create_league_app(lg).test_client()
    r = c.post('/league/register_learner', json={'player_id': 'MP0', 'ip': '127.0.0.1', 'port': 1, 'rank': 0,
                                                 'world_size': 1}).json
    assert r['code'] == 0 and r['info']['ckpt_path'].endswith('MP0_ckpt.pth.tar')
    job = c.post('/league/actor_ask_for_job', json={'job_type': 'train'}).json['info']
    res = {'0': {'player_id': job['player_ids'][0], 'opponent_id': job['player_ids'][1], 'winloss': 0},
           'game_steps': 1, 'game_iters': 1, 'game_duration': 1}
    assert c.post('/league/actor_send_result', json=res).json['code'] == 0
    lg.drain_results()
    assert c.get('/league/show_elo').json['code'] == 0
    lg.close()


def test_http_admin_routes(tmp_path):
    """The league admin surface of league_api.py:56-313: statistics views (active + historical), ELO /
    TrueSkill show-save-update, historical player add / remove, player update / display / stat reset,
    refresh, model backup, config view, resume load - each answers code 0 and has its effect."""
    pytest.importorskip('flask')
    from applestar_amd.league.api import create_league_app
    lg = League(_cfg(tmp_path, players=('MP0',)), root=str(tmp_path), start_threads=True)
    c = create_league_app(lg).test_client()
    for i in range(6):
        job = c.post('/league/actor_ask_for_job', json={'job_type': 'train'}).json['info']
        res = {'0': {'player_id': job['player_ids'][0], 'opponent_id': job['player_ids'][1], 'winloss': 1 - i % 3,
                     'race_id': 'zerg', 'dist/bo': 3.0},
               'game_steps': 10, 'game_iters': 5, 'game_duration': 1.0}
        c.post('/league/actor_send_result', json=res)
    lg.drain_results()
    for route in ('show_dist_stat', 'show_cum_stat', 'show_unit_num_stat', 'show_opponent_payoff',
                  'show_teammate_payoff', 'show_hist_payoff', 'show_hist_dist_stat', 'show_hist_cum_stat',
                  'show_hist_unit_num_stat', 'show_hist_opponent_payoff', 'show_hist_teammate_payoff', 'show_payoff',
                  'show_elo', 'show_trueskill', 'show_config', 'refresh_active_player', 'refresh_hist_player',
                  'refresh_all_player'):
        assert c.get(f'/league/{route}').json['code'] == 0, route
    assert 'zerg' in c.get('/league/show_dist_stat').json['info']['MP0']
    ts = c.get('/league/show_trueskill').json['info']
    assert len(ts) >= 2 and all(v['sigma'] < 25 / 3 for v in ts.values())
    assert c.post('/league/update_trueskill', json={'MP0': {'mu': 30.0}}).json['code'] == 0
    assert lg.trueskill.get('MP0')[0] == 30.0
    assert c.post('/league/update_elo', json={'MP0': 1500}).json['code'] == 0
    assert abs(lg.elo.ratings(start_from_zero=False)['MP0'] - 1500) < 1e-6
    for route in ('save_elo', 'save_zero_elo', 'save_trueskill'):
        path = c.get(f'/league/{route}').json['info']
        assert os.path.exists(path), route
    ckpt = tmp_path / 'extra.pth'
    ckpt.write_bytes(b'weights')
    assert c.post('/league/add_hist_player', json={'player_id': 'HPX', 'checkpoint_path': str(ckpt)}).json['code'] == 0
    assert 'HPX' in lg.historical_players
    assert c.post('/league/add_hist_player', json={'checkpoint_path': '/nonexistent'}).json['code'] == 1
    # no path traversal through the player id, no checkpoint / backup outside the league roots
    assert c.post('/league/add_hist_player', json={'player_id': '../../evil', 'checkpoint_path': str(ckpt)}).json['code'] == 1
    assert c.post('/league/add_hist_player', json={'player_id': 'HPY', 'checkpoint_path': '/etc/hostname'}).json['code'] == 1
    assert c.post('/league/backup_models', json={'backup_dir': '/tmp/../etc/x'}).json['code'] == 1
    assert c.post('/league/update_player', json={'player_id': 'MP0', 'chosen_weight': 3.0,
                                                 'one_phase_step': '1e6'}).json['code'] == 0
    assert lg.active_players['MP0'].chosen_weight == 3.0 and lg.active_players['MP0'].one_phase_step == 1000000
    shown = c.post('/league/display_player', json={'player_id': 'active', 'stat_types': ['payoff']}).json['info']
    assert 'MP0' in shown and 'payoff' in shown['MP0']
    assert c.post('/league/reset_player_stat', json={'player_id': 'MP0', 'stat_types': ['dist_stat']}).json['code'] == 0
    assert lg.active_players['MP0'].dist_stat.stat_info_dict() == {}
    assert sum(len(p.payoff.record) for p in lg.all_players.values()) > 0     # payoffs kept
    lg.active_players['MP0'].checkpoint_path = str(ckpt)
    bdir = c.post('/league/backup_models', json={'player_id': 'all'}).json['info']
    assert os.path.exists(os.path.join(bdir, 'extra.pth'))
    assert c.post('/league/remove_hist_player', json={'player_id': 'HPX'}).json['code'] == 0
    assert 'HPX' not in lg.historical_players
    path = c.get('/league/save_resume').json['info']
    assert c.post('/league/load_resume', json={'path': path}).json['code'] == 0
    assert lg.trueskill.get('MP0')[0] == 30.0                                   # TrueSkill persisted in the resume
    lg.close()
