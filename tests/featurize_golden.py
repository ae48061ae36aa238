"""Golden digests of the featurizer (agent/features.py transform_obs + value features) over a FakeSC2Env
episode: ``python tests/featurize_golden.py --write`` records them in tests/data/featurize_golden.json; the
test (tests/test_agent.py::test_transform_obs_matches_golden_digests) re-runs the same episode and demands
byte-identical tensors, so the featurizer can be re-implemented for speed without changing one value."""
import hashlib
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'featurize_golden.json')


def _digest(tree, prefix=''):
    out = {}
    if isinstance(tree, dict):
        for k in sorted(tree):
            out.update(_digest(tree[k], f'{prefix}/{k}'))
    elif isinstance(tree, (list, tuple)):
        out[prefix] = hashlib.sha1(repr(list(tree)).encode()).hexdigest()[:16]
    elif isinstance(tree, torch.Tensor):
        t = tree.contiguous().reshape(-1)
        h = hashlib.sha1(t.view(torch.uint8).numpy().tobytes() if t.numel() else b'')
        out[prefix] = f'{t.dtype}|{tuple(tree.shape)}|{h.hexdigest()[:16]}'
    else:
        out[prefix] = repr(tree)
    return out


def episode_digests(steps=24, seed=3):
    from applestar_amd.agent.features import Features
    from applestar_amd.envs.fake_env import FakeSC2Env
    random.seed(seed)
    env = FakeSC2Env({'env': {'player_ids': ['agent1', 'agent2'], 'races': ['zerg', 'terran'],
                              'game_steps_per_episode': 100000, 'random_seed': seed}})
    obs, gi, _ = env.reset()
    feats = {i: Features(gi[i], obs[i]['raw_obs']) for i in obs}
    rng = np.random.default_rng(seed)
    digests = []
    for _ in range(steps):
        for i in sorted(obs):
            o = feats[i].transform_obs(obs[i]['raw_obs'], padding_spatial=True, opponent_obs=obs[i]['opponent_obs'])
            digests.append(_digest(o))
        acts = {}
        for i in obs:
            tags = [u.tag for u in obs[i]['raw_obs'].observation.raw_data.units]
            acts[i] = [{'func_id': 0, 'skip_steps': int(rng.integers(1, 4)), 'queued': 0,
                        'unit_tags': tags[:2], 'target_unit_tag': 0, 'location': (10, 10)}]
        obs, _, done = env.step(acts)
        if done:
            break
    return digests


if __name__ == '__main__':
    if '--write' in sys.argv:
        os.makedirs(os.path.dirname(GOLDEN), exist_ok=True)
        with open(GOLDEN, 'w') as f:
            json.dump(episode_digests(), f, indent=0, sort_keys=True)
        print('wrote', GOLDEN)
