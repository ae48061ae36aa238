"""Play a match: agent vs bot, agent vs agent, or human vs agent (``distar/bin/play.py:45-199``).

    python -m applestar_amd.bin.play --game_type agent_vs_bot --model1 rl_model --race zerg
    python -m applestar_amd.bin.play --game_type agent_vs_agent --model1 rl_model --model2 sl_model
    python -m applestar_amd.bin.play --game_type human_vs_agent --model1 rl_model

Models: ``<name>.pth`` next to this file, an absolute path, or ``default`` (= ``rl_model.pth``);
a missing file falls back to random weights (warned).  Runs on the MI355X (bf16 inference) unless
``--cpu``; ``--fake-env`` plays against :class:`FakeSC2Env` when no SC2 install is present.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

from ..utils.config import read_config, deep_merge_dicts

HERE = os.path.dirname(os.path.abspath(__file__))


def resolve_model(name: str) -> str:
    if name in ('default', ''):
        name = 'rl_model'
    if os.path.isabs(name) or os.path.exists(name):
        return name
    path = os.path.join(HERE, name if name.endswith(('.pth', '.tar')) else name + '.pth')
    return path


def build_config(args) -> dict:
    cfg = read_config(args.config or os.path.join(HERE, 'user_config.yaml'))
    cfg = deep_merge_dicts(cfg, {'common': {'type': 'play'},
                                 'actor': {'job_type': 'eval_test', 'episode_num': 1}})
    cfg.actor.use_cuda = bool(torch.cuda.is_available() and not args.cpu)
    cfg.actor.model_paths = {'model1': resolve_model(args.model1), 'model2': resolve_model(args.model2)}
    for k, p in cfg.actor.model_paths.items():
        if not os.path.exists(p):
            print(f'[play] {k}: {p} not found, using random weights', file=sys.stderr)
            cfg.actor.fake_model = True
    cfg.env.races = [args.race, args.race2 or args.race]
    bot = f'bot{args.bot_level}'
    if args.game_type == 'agent_vs_agent':
        cfg.env.player_ids = ['model1', 'model2']
        cfg.actor.player_ids = ['model1', 'model2']
    elif args.game_type == 'agent_vs_bot':
        cfg.env.player_ids = ['model1', bot]
        cfg.actor.player_ids = ['model1']
    elif args.game_type == 'human_vs_agent':
        cfg.env.player_ids = ['human', 'model1']
        cfg.actor.player_ids = ['model1']
        cfg.env.realtime = True
    else:
        raise ValueError(args.game_type)
    if args.fake_env:
        cfg.env.fake = True
    if args.map:
        cfg.env.map_name = args.map
    return cfg


def main(argv=None):
    ap = argparse.ArgumentParser(description='play')
    ap.add_argument('--config', default=None)
    ap.add_argument('--model1', default='rl_model')
    ap.add_argument('--model2', default='rl_model')
    ap.add_argument('--cpu', action='store_true')
    ap.add_argument('--game_type', default='agent_vs_bot',
                    choices=['agent_vs_agent', 'agent_vs_bot', 'human_vs_agent'])
    ap.add_argument('--race', default='zerg', choices=['zerg', 'terran', 'protoss'])
    ap.add_argument('--race2', default=None, choices=[None, 'zerg', 'terran', 'protoss'])
    ap.add_argument('--bot_level', type=int, default=10)
    ap.add_argument('--map', default=None)
    ap.add_argument('--fake-env', action='store_true')
    args = ap.parse_args(argv)
    cfg = build_config(args)
    if cfg.env.get('fake') is None:
        from ..envs import sc2_available
        if not sc2_available():
            print('[play] SC2 not found (set SC2PATH); using FakeSC2Env', file=sys.stderr)
            cfg.env.fake = True
    if cfg.actor.use_cuda:
        torch.set_default_device(None)
    from ..actor.actor import Actor
    results = Actor(cfg).run()
    for r in results:
        print({k: v for k, v in r.items() if k in ('game_steps', 'game_iters')},
              {str(s): r[s]['winloss'] for s in r if isinstance(r[s], dict)})
    return results


if __name__ == '__main__':
    main()
