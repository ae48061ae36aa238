"""Full RL pipeline on CPU: league HTTP + coordinator + actor (train job, spawned env workers with
batched inference) -> trajectories over the data plane -> RL learner iterations -> model broadcast
back to the actor -> results reach the league."""
import socket
import threading
import time

import pytest
import torch


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_rl_pipeline_end_to_end(tmp_path, monkeypatch):
    pytest.importorskip('flask')
    monkeypatch.chdir(tmp_path)
    from werkzeug.serving import make_server
    from applestar_amd.comm.adapter import Coordinator, serve_coordinator
    from applestar_amd.league.league import League
    from applestar_amd.league.api import create_league_app
    from applestar_amd.actor.actor import Actor
    from applestar_amd.learner.rl_learner import RLLearner

    coord = serve_coordinator(Coordinator(), '127.0.0.1', 0)
    cport = coord.server_address[1]
    league = League({'league': {'active_players': {'checkpoint_path': ['none'], 'player_id': ['MP0'],
                                                   'pipeline': ['default'], 'frac_id': [1], 'z_prob': [0.0],
                                                   'teacher_id': ['none'], 'teacher_path': ['none'],
                                                   'z_path': ['3map.json'], 'one_phase_step': [1e9],
                                                   'chosen_weight': [1]},
                                'vs_bot': True, 'bot_probs': [0, 0, 0, 0, 0, 0, 0, 1.0, 0, 0, 0]}},
                    root=str(tmp_path))
    lport = _free_port()
    srv = make_server('127.0.0.1', lport, create_league_app(league), threaded=True)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    comm = {'coordinator_ip': '127.0.0.1', 'coordinator_port': cport, 'league_ip': '127.0.0.1',
            'league_port': lport, 'learner_send_model_freq': 1, 'learner_send_train_info_freq': 2,
            'actor_ask_for_job_interval': 240, 'actor_model_update_interval': 1}
    T = 3
    learner_holder = {}

    def run_learner():
        lrn = RLLearner({'common': {'experiment_name': 'e2e'},
                         'learner': {'use_cuda': False, 'player_id': 'MP0', 'use_value_feature': False,
                                     'data': {'batch_size': 2, 'trajectory_length': T, 'buffer_size': 2},
                                     'hook': {'log_show': {'name': 'log_show', 'type': 'log_show', 'priority': 20,
                                                           'position': 'after_iter', 'ext_args': {'freq': 1}}},
                                     'log_to_stdout': False},
                         'communication': comm})
        learner_holder['l'] = lrn
        lrn.run(max_iterations=3)
    t = threading.Thread(target=run_learner, daemon=True)
    t.start()
    actor = Actor({'common': {'experiment_name': 'e2e'},
                   'actor': {'job_type': 'train', 'env_num': 2, 'gpu_batch_inference': True, 'traj_len': T,
                             'episode_num': 1},
                   'env': {'game_steps_per_episode': 700, 'fake': True},
                   'communication': comm})
    results = actor.run(max_jobs=1)
    t.join(timeout=300)
    lrn = learner_holder.get('l')
    assert lrn is not None and lrn.last_iter.val == 3
    assert results and all(r['0']['player_id'] == 'MP0' for r in results)
    league.drain_results()
    assert sum(league.active_players['MP0'].payoff.games(o) for o in
               league.active_players['MP0'].payoff.record) == len(results)
    from applestar_amd.comm.adapter import Adapter
    st = Adapter('127.0.0.1', cport).stats()
    assert 'MP0model' in st['broadcast'] and st['pull'].get('MP0traj', 0) >= 2
    actor.close()
    lrn.close()
    srv.shutdown()
    coord.shutdown()


def test_rl_dataloader_ring_mode_cpu():
    """Ring-mode replay buffer (device collate path, run on the host here): batches come from the
    trajectory ring, each trajectory is reused max_reuse times then dropped."""
    import torch
    from applestar_amd.comm.adapter import Coordinator, serve_coordinator, Adapter
    from applestar_amd.learner.dataloader import RLDataLoader
    from test_agent import _run_episode
    _, trajs, _, _ = _run_episode('train_test', traj_len=3, until_full=6)
    full = [t for t in trajs if len(t) == 4][:4]
    srv = serve_coordinator(Coordinator(), '127.0.0.1', 0)
    port = srv.server_address[1]
    prod = Adapter('127.0.0.1', port)
    for t in full:
        prod.push(t, 'MP0traj')
    dl = RLDataLoader(Adapter('127.0.0.1', port), 'MP0', batch_size=2, buffer_size=4, device='cpu',
                      device_collate=True, max_reuse=2)
    seen = []
    for _ in range(4):
        b = next(dl)
        assert b['entity_info']['x'].shape[0] == 4 * 2 and b['action_info']['action_type'].shape == (3, 2)
        seen.append(b)
    assert len(dl._ring) == 0  # 4 trajectories x 2 uses = 4 batches of 2
    dl.close()
    prod.close()
    srv.shutdown()


def test_learner_admin_routes(tmp_path, monkeypatch):
    """/rl_learner/{update_config, reset_value, reset_comm_setting} (rl_learner.py:263-287): requests are
    applied between iterations - the learning rate changes, and the comm link and dataloader are rebuilt."""
    pytest.importorskip('flask')
    monkeypatch.chdir(tmp_path)
    from applestar_amd.learner.rl_learner import RLLearner, create_learner_app
    lrn = RLLearner({'common': {'experiment_name': 'adm'},
                     'learner': {'use_cuda': False, 'player_id': 'MP0', 'use_value_feature': False,
                                 'data': {'batch_size': 1, 'trajectory_length': 2, 'synthetic': True},
                                 'log_to_stdout': False}})
    c = create_learner_app(lrn).test_client()
    old_comm, old_loader = lrn.comm, lrn.dataloader
    assert c.post('/rl_learner/update_config', json={'learner': {'learning_rate': 3e-4}}).json['code'] == 0
    assert c.get('/rl_learner/reset_comm_setting').json['code'] == 0
    assert c.post('/rl_learner/reset_value', json={}).json['code'] == 0
    lrn.run(max_iterations=1)
    assert lrn.trainer.optimizer.param_groups[0]['lr'] == 3e-4
    assert lrn.comm is not old_comm and lrn.dataloader is not old_loader
    assert c.get('/rl_learner/status').json['info']['iter'] == 1
    lrn.close()


def test_rl_train_two_learner_ranks_identical_replicas(tmp_path):
    """rl_train itself (coordinator, league, the learner role under torch.distributed.run with
    two gloo ranks, an actor with fake-env workers and the batched inference server) runs 2 learner iterations;
    both ranks' weights are then identical (tools/rl_train_dp_rehearsal.py; on a GPU box the same script runs both
    ranks on the one GPU)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(root, 'tools', 'rl_train_dp_rehearsal.py'), '--iters', '2',
                          '--out', str(tmp_path / 'dp2'), '--timeout', '500'], capture_output=True, text=True,
                         timeout=560)
    assert res.returncode == 0, (res.stdout[-2000:], res.stderr[-3000:])
    rec = json.loads(res.stdout.strip().splitlines()[-1])
    assert rec['replicas_identical'] and rec['iterations'] == [2, 2], rec
