"""RL training launcher (``distar/bin/rl_train.py``).

No ``--type``: start coordinator, league, learner and actor on this host (separate processes).
``--type {coordinator,league,learner,actor}`` starts one role (multi-host / multi-GPU layouts).
Learner data parallelism: launch the learner role under ``torch.distributed.run`` (one process per
GPU, RCCL over xGMI) or pass ``--init_method tcp://host:port --rank r --world_size n``.
``--task bot`` trains against built-in bots (no value feature); ``--task selfplay`` uses the league.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import shutil
import threading
import time

from ..utils.config import read_config, save_config

HERE = os.path.dirname(os.path.abspath(__file__))


def _default_model(path: str) -> str:
    return os.path.join(HERE, 'sl_model.pth') if path == 'default' else path


def coordinator_run(cfg, args):
    from ..comm.adapter import Coordinator, serve_coordinator
    srv = serve_coordinator(Coordinator(), cfg.communication.coordinator_ip, int(cfg.communication.coordinator_port))
    print(f'coordinator on {srv.server_address}', flush=True)
    while True:
        time.sleep(3600)


def league_run(cfg, args):
    from ..league.league import League
    from ..league.api import serve
    exp_dir = os.path.join(os.getcwd(), 'experiments', cfg.common.experiment_name)
    os.makedirs(os.path.join(exp_dir, 'config'), exist_ok=True)
    save_config(cfg, os.path.join(exp_dir, 'rl_user_config.yaml'))
    stamp = time.strftime('%Y-%m-%d-%H-%M-%S')
    save_config(cfg, os.path.join(exp_dir, 'config', f'rl_user_config_{stamp}.yaml'))
    ap = cfg.league.active_players
    ap.checkpoint_path = [_default_model(p) for p in ap.checkpoint_path]
    ap.teacher_path = [_default_model(p) for p in ap.teacher_path]
    hp = cfg.league.historical_players
    hp.checkpoint_path = [_default_model(p) for p in hp.checkpoint_path]
    league = League(cfg)
    serve(league, cfg.communication.get('league_ip', cfg.communication.coordinator_ip),
          int(cfg.communication.league_port))


def learner_run(cfg, args):
    from ..learner.rl_learner import RLLearner, create_learner_app
    cfg.learner.player_id = args.player_id
    if args.init_method:
        os.environ.setdefault('MASTER_ADDR', args.init_method.split('//')[-1].split(':')[0])
        os.environ.setdefault('MASTER_PORT', args.init_method.rsplit(':', 1)[-1])
        os.environ['RANK'], os.environ['WORLD_SIZE'] = str(args.rank), str(args.world_size)
        cfg.learner.use_distributed = True
    d = os.path.join(os.getcwd(), 'experiments', cfg.common.experiment_name, args.player_id)
    os.makedirs(d, exist_ok=True)
    save_config(cfg, os.path.join(d, 'rl_user_config.yaml'))
    learner = RLLearner(cfg)
    if learner.rank == 0 and args.admin_port:
        app = create_learner_app(learner)
        threading.Thread(target=lambda: app.run(host='0.0.0.0', port=args.admin_port, use_reloader=False),
                         daemon=True).start()
    learner.run()


def actor_run(cfg, args):
    from ..actor.actor import Actor
    cfg.actor.gpu_batch_inference = str(args.gpu_batch_inference).lower() in ('1', 'true', 'yes')
    if cfg.actor.job_type == 'train':
        cfg.env.replay_dir = os.path.join(os.path.abspath(cfg.env.replay_dir), cfg.common.experiment_name)
    Actor(cfg).run()


ROLES = {'coordinator': coordinator_run, 'league': league_run, 'learner': learner_run, 'actor': actor_run}


def main(argv=None):
    ap = argparse.ArgumentParser(description='rl_train')
    ap.add_argument('--config', default=os.path.join(HERE, 'rl_user_config.yaml'))
    ap.add_argument('--type', default=None, choices=[None] + list(ROLES))
    ap.add_argument('--task', default='bot', choices=['bot', 'selfplay'])
    ap.add_argument('--player_id', default='MP0')
    ap.add_argument('--gpu_batch_inference', default='true')
    ap.add_argument('--init_method', default=None)
    ap.add_argument('--rank', type=int, default=0)
    ap.add_argument('--world_size', type=int, default=1)
    ap.add_argument('--admin_port', type=int, default=0)
    ap.add_argument('--fake-env', action='store_true')
    args = ap.parse_args(argv)
    cfg = read_config(args.config)
    cfg.common.type = 'rl'
    cfg.actor.traj_len = cfg.learner.data.trajectory_length
    if args.task == 'bot':
        cfg.league.vs_bot = True
        cfg.learner.use_value_feature = False
    else:
        cfg.league.vs_bot = False
    if args.fake_env:
        cfg.env.fake = True
    if args.type is not None:
        return ROLES[args.type](cfg, args)
    ctx = mp.get_context('spawn')
    procs = []
    for role in ('coordinator', 'league', 'learner'):
        p = ctx.Process(target=ROLES[role], args=(cfg, args), daemon=True)
        p.start()
        procs.append(p)
        time.sleep(3)
    try:
        actor_run(cfg, args)
    finally:
        for p in procs:
            p.terminate()


if __name__ == '__main__':
    main()
