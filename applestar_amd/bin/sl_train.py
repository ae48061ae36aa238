"""SL training launcher (``distar/bin/sl_train.py``): ``--type learner`` (default) trains from
replays (``--data`` directory / list file) or synthetic batches (``--fake_data``); ``--type
coordinator`` / ``replay_actor`` run the remote replay-decoding data plane.  Single-node runs force
the LR warm-up like the reference (``sl_train.py:39``).  Data parallel: launch under
``torch.distributed.run`` (one process per GPU) or pass ``--init_method/--rank/--world_size``."""
from __future__ import annotations

import argparse
import os
import time

from ..utils.config import read_config

HERE = os.path.dirname(os.path.abspath(__file__))


def main(argv=None):
    ap = argparse.ArgumentParser(description='sl_train')
    ap.add_argument('--config', default=os.path.join(HERE, 'sl_user_config.yaml'))
    ap.add_argument('--type', default='learner', choices=['learner', 'coordinator', 'replay_actor'])
    ap.add_argument('--data', default=None)
    ap.add_argument('--remote', action='store_true')
    ap.add_argument('--fake_data', action='store_true')
    ap.add_argument('--init_method', default=None)
    ap.add_argument('--rank', type=int, default=0)
    ap.add_argument('--world_size', type=int, default=1)
    ap.add_argument('--max_iterations', type=int, default=None)
    args = ap.parse_args(argv)
    cfg = read_config(args.config)
    cfg.common.type = 'sl'
    if args.data:
        cfg.learner.data.train_data_file = args.data
    if args.fake_data:
        cfg.learner.data.fake_data = True
    if args.remote:
        cfg.learner.data.remote = True
    if args.type == 'coordinator':
        from ..comm.adapter import Coordinator, serve_coordinator
        serve_coordinator(Coordinator(), cfg.communication.coordinator_ip, int(cfg.communication.coordinator_port))
        while True:
            time.sleep(3600)
    if args.type == 'replay_actor':
        from ..learner.replay_dataloader import ReplayActor
        return ReplayActor(cfg).run()
    if args.init_method:
        os.environ.setdefault('MASTER_ADDR', args.init_method.split('//')[-1].split(':')[0])
        os.environ.setdefault('MASTER_PORT', args.init_method.rsplit(':', 1)[-1])
        os.environ['RANK'], os.environ['WORLD_SIZE'] = str(args.rank), str(args.world_size)
        cfg.learner.use_distributed = True
    if not cfg.learner.get('use_distributed') and int(os.environ.get('WORLD_SIZE', '1')) == 1:
        cfg.learner.use_warmup = True
    from ..learner.sl_learner import SLLearner
    learner = SLLearner(cfg)
    learner.run(max_iterations=args.max_iterations)
    return learner


if __name__ == '__main__':
    main()
