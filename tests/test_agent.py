"""Agent layer: featurization of raw observations, Z selection, action decoding, trajectory assembly,
pseudo-reward metrics (parity vs the reference metric code), learner collate."""
import importlib.util
import random
from functools import partial

import pytest
import torch

from applestar_amd.agent.agent import Agent
from applestar_amd.agent.collate import collate_trajectories, collate_obs
from applestar_amd.agent.features import Features, action_type_from_ability, transform_action
from applestar_amd.envs.fake_env import FakeSC2Env
from applestar_amd.envs import raw as R
from applestar_amd.lib.features import SPATIAL_INFO, ENTITY_INFO, SCALAR_INFO, MAX_ENTITY_NUM
from applestar_amd.lib.game_data import ACTIONS
from applestar_amd.lib.metrics import levenshtein_distance, hamming_distance, l2_distance

REF_METRIC = '/root/reference/distar/ctools/torch_utils/metric.py'


def _env(player_ids=('agent1', 'agent2'), steps=1200, seed=0):
    return FakeSC2Env({'env': {'player_ids': list(player_ids), 'races': ['zerg', 'zerg'],
                               'game_steps_per_episode': steps, 'random_seed': seed}})


def test_transform_obs_schema():
    env = _env()
    obs, gi, _ = env.reset()
    f = Features(gi[0], obs[0]['raw_obs'])
    o = f.transform_obs(obs[0]['raw_obs'], padding_spatial=True, opponent_obs=obs[0]['opponent_obs'])
    for k, dt in SPATIAL_INFO:
        assert o['spatial_info'][k].dtype == dt
        assert o['spatial_info'][k].shape == ((100,) if k.startswith('effect') else (152, 160))
    n = int(o['entity_num'])
    for k, dt in ENTITY_INFO:
        if not k.startswith('last_'):
            assert o['entity_info'][k].dtype == dt and o['entity_info'][k].shape == (n,), k
    assert (o['entity_info']['unit_type'] >= 0).all() and (o['entity_info']['order_id_0'] >= 0).all()
    assert (o['entity_info']['order_id_1'] >= 0).all()
    for k, dt, size in SCALAR_INFO:
        if k in o['scalar_info']:
            assert o['scalar_info'][k].shape == size, k
    assert o['value_feature']['unit_type'].shape == (MAX_ENTITY_NUM,)
    # y is flipped to screen coordinates; passengers carry is_in_cargo
    u0 = obs[0]['raw_obs'].observation.raw_data.units[0]
    assert int(o['entity_info']['y'][0]) == int(f.map_size.y - u0.pos.y)


def test_effects_and_minimap_padding():
    env = _env()
    obs, gi, _ = env.reset()
    ro = obs[0]['raw_obs']
    ro.observation.raw_data.effects = [R.Effect(effect_id=1, pos=[R.Point(10.5, 20.2)], owner=2),
                                       R.Effect(effect_id=12, pos=[R.Point(3, 3)], owner=1)]
    f = Features(gi[0], ro)
    o = f.transform_obs(ro, padding_spatial=True)
    assert int(o['spatial_info']['effect_PsiStorm'][0]) == 10 + int(f.map_size.y - 20.2) * 160
    assert int(o['spatial_info']['effect_LurkerSpines'].abs().sum()) == 0  # own lurker spines are skipped
    my, mx = f.map_size.y, f.map_size.x
    assert int(o['spatial_info']['pathable'][my:].sum()) == 0 and int(o['spatial_info']['pathable'][:, mx:].sum()) == 0


def test_transform_and_reverse_action_roundtrip():
    env = _env()
    obs, gi, _ = env.reset()
    f = Features(gi[0], obs[0]['raw_obs'])
    tags = [u.tag for u in obs[0]['raw_obs'].observation.raw_data.units]
    for at in (3, 5, 15, 40, 100, 200, 300):
        a = ACTIONS[at]
        if not a['general_ability_id']:
            continue
        act = {'func_id': a['func_id'], 'skip_steps': 3, 'queued': 1, 'unit_tags': tags[:3],
               'target_unit_tag': tags[4], 'location': (17, 33)}
        cmds, skip = transform_action(act)
        assert skip == 3 and cmds[0].ability_id == a['general_ability_id']
        if a['name'].endswith('_autocast'):
            continue
        class _Raw:  # ActionRaw mirror
            unit_command = cmds[0]
            toggle_autocast = None
        labels, mask, su_num, *_ = f.reverse_raw_action(_Raw, tags)
        assert int(labels['action_type']) == at, (at, a['name'])
        assert labels['selected_units'].tolist() == [0, 1, 2, len(tags)] and int(su_num) == 4
        if a['target_location']:
            assert int(labels['target_location']) == (f.map_size.y - 33) * 160 + 17
        if a['target_unit']:
            assert int(labels['target_unit']) == 4


@pytest.mark.skipif(not importlib.util.find_spec('torch'), reason='torch')
def test_metrics_match_reference():
    spec = importlib.util.spec_from_file_location('refmetric', REF_METRIC)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rng = random.Random(0)
    for _ in range(200):
        a = torch.tensor([rng.randint(0, 4) for _ in range(rng.randint(0, 7))], dtype=torch.long)
        b = torch.tensor([rng.randint(0, 4) for _ in range(rng.randint(0, 7))], dtype=torch.long)
        assert float(levenshtein_distance(a, b)) == float(m.levenshtein_distance(a, b))
        if len(a) and len(b):
            la = torch.randint(0, 24320, (len(a),))
            lb = torch.randint(0, 24320, (len(b),))
            r = m.levenshtein_distance(a, b, la, lb, partial(m.l2_distance, spatial_x=160))
            assert abs(float(levenshtein_distance(a, b, la, lb, partial(l2_distance, spatial_x=160))) - float(r)) < 1e-5
    x = torch.randint(0, 2, (5, 30)).bool()
    y = torch.randint(0, 2, (5, 30)).bool()
    assert torch.equal(hamming_distance(x, y), m.hamming_distance(x, y))


def _run_episode(job_type, steps=900, traj_len=3, value_feature=False, until_full=None):
    """Play one fake-env episode with two agents; train jobs collect trajectories.  ``until_full``: stop once
    that many full (traj_len + 1 step) trajectories exist - the trajectory tests need a handful, not the
    whole 900-step episode (~10 min of CPU forwards)."""
    torch.manual_seed(0)
    random.seed(0)
    cfg = {'actor': {'job_type': job_type, 'traj_len': traj_len}, 'common': {'type': 'rl'},
           'agent': {'z_path': '3map.json'}, 'learner': {'use_value_feature': value_feature}}
    env = _env(steps=steps)
    a0 = Agent(cfg)
    a1 = Agent(cfg, model=a0.model, teacher_model=a0.teacher_model)
    agents = [a0, a1]
    obs, gi, m = env.reset()
    for i, a in enumerate(agents):
        a.reset(m, 'zerg', gi[i], obs[i])
    trajs, done, acts_seen = [], False, []
    while not done:
        acts = {i: agents[i].step(o) for i, o in obs.items()}
        acts_seen += [a[0] for a in acts.values()]
        nobs, rew, done = env.step(acts)
        if 'train' in job_type:
            for i in nobs:
                t = agents[i].collect_data(nobs[i], rew[i], done, i)
                if t:
                    trajs.append(t)
        obs = nobs
        if until_full is not None and sum(len(t) == traj_len + 1 for t in trajs) >= until_full:
            break
    return agents, trajs, acts_seen, rew


def test_agent_eval_episode_actions_valid():
    agents, _, acts, rew = _run_episode('eval_test')
    assert sorted(rew) == [-1, 1]
    for a in acts:
        assert set(a) == {'func_id', 'skip_steps', 'queued', 'unit_tags', 'target_unit_tag', 'location'}
        assert 0 <= a['skip_steps'] <= 127
    st = agents[0].get_stat_data()
    assert 'z_type' in st and 'dist/bo' in st


def test_agent_train_trajectories_collate_and_learn():
    from applestar_amd.rl.trainer import RLTrainer
    _, trajs, _, _ = _run_episode('train_test', traj_len=3, value_feature=True, until_full=6)
    full = [t for t in trajs if len(t) == 4]
    assert len(full) >= 2
    step = full[0][0]
    assert step['teacher_logit']['action_type'].shape == (327,)
    assert step['teacher_logit']['selected_units'].shape[-1] == int(step['entity_num']) + 1
    assert set(step['reward']) == {'winloss', 'build_order', 'built_unit', 'battle'}
    b = collate_trajectories(full[:2])
    N = b['entity_info']['unit_type'].shape[1]
    assert b['entity_info']['unit_type'].shape[0] == 4 * 2
    assert b['teacher_logit']['selected_units'].shape == (3, 2, 64, N + 1)
    assert b['mask']['target_units_logits_mask'].shape == (3, 2, N)
    tr = RLTrainer({'learner': {'use_value_feature': True}}, device='cpu')
    info = tr.step(b)
    assert all(torch.isfinite(torch.as_tensor(v)).all() for v in info.values() if torch.is_tensor(v) or
               isinstance(v, float))


def test_agent_registry_and_template_plugin():
    from applestar_amd.agent.registry import import_agent, register_agent
    from applestar_amd.agent.template import Agent as T
    from applestar_amd.actor.actor import run_episodes, _job_from_config, DEFAULT_ACTOR_CONFIG
    from applestar_amd.utils.config import deep_merge_dicts
    assert import_agent('default') is Agent and import_agent('template') is T
    register_agent('noop', T)
    cfg = deep_merge_dicts(DEFAULT_ACTOR_CONFIG, {'actor': {'agents': {'model1': 'noop'}},
                                                  'env': {'game_steps_per_episode': 200, 'fake': True}})
    res = run_episodes(cfg, _job_from_config(cfg))
    assert len(res) == 1 and res[0]['0']['player_id'] == 'model1'


def test_trajectory_ring_matches_host_collate():
    """The HBM ring's on-device batch assembly reproduces collate_trajectories exactly (host path)."""
    from applestar_amd.runtime.traj_ring import TrajectoryRing
    from applestar_amd.utils import serialize
    _, trajs, _, _ = _run_episode('train_test', traj_len=3, value_feature=True, until_full=6)
    full = [t for t in trajs if len(t) == 4][:3]
    ref = collate_trajectories(full)
    ring = TrajectoryRing(64 << 20, device='cpu')
    ids = [ring.put(serialize.dumps(t)) for t in full]
    got = ring.batch(ids)

    def cmp(a, b, path=''):
        if isinstance(a, dict):
            for k in a:
                if k in ('batch_size', 'unroll_len'):
                    assert a[k] == b[k]
                    continue
                assert k in b, path + '/' + str(k)
                cmp(a[k], b[k], path + '/' + str(k))
        elif isinstance(a, (list, tuple)):
            for x, y in zip(a, b):
                cmp(x, y, path)
        elif torch.is_tensor(a):
            assert a.shape == b.shape, (path, a.shape, b.shape)
            assert torch.equal(a.to(b.dtype), b), path
    cmp(ref, got)
    # eviction when the ring wraps
    frames = [serialize.dumps(t) for t in full]
    small = TrajectoryRing(max(len(f) for f in frames) * 2 + 4096, device='cpu')
    tids = [small.put(f) for f in frames]
    assert tids[-1] in small.ids() and tids[0] not in small.ids() and 1 <= len(small) <= 2


def test_transform_obs_matches_golden_digests():
    """The featurizer reproduces, byte for byte, the digests recorded from the plain per-column implementation
    (tests/featurize_golden.py) over a FakeSC2Env episode: its speed work changes no value."""
    import json
    import tests.featurize_golden as fg
    with open(fg.GOLDEN) as f:
        golden = json.load(f)
    got = fg.episode_digests()
    assert len(got) == len(golden)
    for i, (g, r) in enumerate(zip(got, golden)):
        diff = {k for k in set(g) | set(r) if g.get(k) != r.get(k)}
        assert not diff, (i, sorted(diff)[:8])


def test_dense_segments_varlen_equals_masked_attention():
    """The static (graph-captured) entity path runs attention as varlen over 2B segments - each row's real
    tokens, then its padding tokens (models/transformer.py dense_segments): on every real row it equals the
    dense masked attention; empty segments (no entities / no padding) are fine."""
    from applestar_amd.models.transformer import dense_segments
    from applestar_amd.ops import reference as ref
    torch.manual_seed(0)
    B, N, H, D = 4, 16, 2, 8
    lens = torch.tensor([5, 0, 16, 9])
    qkv = torch.randn(B, N, 3 * H * D, dtype=torch.float64)
    cu = dense_segments(lens, N)
    assert cu.tolist() == [0, 5, 16, 16, 32, 48, 48, 57, 64]
    a = ref.varlen_attention(qkv.reshape(B * N, -1), cu, N, H, D).view(B, N, -1)
    q, k, v = qkv.view(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    mask = torch.arange(N)[None, :] < lens[:, None]
    b = ref.masked_attention(q, k, v, mask).permute(0, 2, 1, 3).reshape(B, N, H * D)
    for i in range(B):
        n = int(lens[i])
        assert torch.allclose(a[i, :n], b[i, :n], atol=1e-12), i
    assert torch.isfinite(a).all()
