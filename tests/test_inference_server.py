"""Actor inference server (actor/inference.py) on the CPU: the merged 'policy+teacher' request returns exactly
the policy reply plus the teacher reply of the two-request path, and a multi-process synthetic-client run over
routed pipes (native frame collation, two-stage launch/finish pipeline) answers every request with the same
result as a direct in-process call."""
import multiprocessing as mp

import torch

from applestar_amd.actor.inference import InferenceClient, InferenceServer
from applestar_amd.lib.features import random_obs
from applestar_amd.models.model import Model


def _requests(n, seed, entity=(12, 90, 40, 7)):
    g = torch.Generator().manual_seed(seed)
    obs = random_obs(n, entity_num=torch.tensor(entity[:n]), generator=g)
    reqs = []
    for i in range(n):
        k = int(obs['entity_num'][i])
        r = {key: ({kk: (vv[i, :k] if key == 'entity_info' else vv[i]) for kk, vv in v.items()}
                   if isinstance(v, dict) else v[i]) for key, v in obs.items()}
        r['hidden_state'] = [(torch.randn(384, generator=g) * 0.1, torch.randn(384, generator=g) * 0.1)
                             for _ in range(3)]
        r['noise'] = {key: torch.rand((), generator=g) for key in ('action_type', 'delay', 'queued', 'target_unit',
                                                                   'target_location')}
        r['noise']['selected_units'] = torch.rand(64, generator=g)
        reqs.append(r)
    return reqs


def _close(a, b, path=''):
    if isinstance(a, dict):
        assert set(a) == set(b), path
        for k in a:
            _close(a[k], b[k], f'{path}/{k}')
    elif isinstance(a, (list, tuple)):
        for x, y in zip(a, b):
            _close(x, y, path)
    elif torch.is_tensor(a):
        assert a.shape == b.shape, path
        assert torch.allclose(a.float(), b.float(), atol=1e-4, rtol=1e-4), path
    else:
        assert a == b, path


def test_policy_teacher_merged_matches_two_requests():
    torch.manual_seed(0)
    pol, tea = Model().eval(), Model().eval()
    srv = InferenceServer('cpu')
    srv.set_model('p', pol)
    srv.set_model('t', tea, teacher=True)
    reqs = _requests(3, 1)
    teacher_hs = [[(torch.randn(384) * 0.1, torch.randn(384) * 0.1) for _ in range(3)] for _ in reqs]
    merged = srv._forward('p', 'policy+teacher', [dict(r, teacher_hidden_state=h) for r, h in zip(reqs, teacher_hs)],
                          teacher_id='t')
    pol_out = srv._forward('p', 'policy', reqs)
    t_reqs = []
    for r, h, o in zip(reqs, teacher_hs, pol_out):
        t = {k: r[k] for k in ('spatial_info', 'entity_info', 'scalar_info', 'entity_num')}
        t.update(hidden_state=h, selected_units_num=o['selected_units_num'], action_info=o['action_info'])
        t_reqs.append(t)
    tea_out = srv._forward('t', 'teacher', t_reqs)
    for m, p, t in zip(merged, pol_out, tea_out):
        m = dict(m)
        mt = m.pop('teacher')
        _close(m, p)
        _close(mt['logit'], t['logit'])
        _close(mt['hidden_state'], t['hidden_state'])


def _client(conn, reqs, q):
    torch.set_num_threads(1)
    cl = InferenceClient(conn, 'p', 'policy')
    from applestar_amd.utils import serialize
    q.put(serialize.dumps([cl.infer(r) for r in reqs]))     # bytes: the child may exit before the get


def test_routed_pipes_serve_every_request():
    torch.manual_seed(0)
    model = Model().eval()
    srv = InferenceServer('cpu', max_wait_ms=5.0)
    srv.set_model('p', model)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs, all_reqs = [], []
    for w in range(3):
        parent, child = ctx.Pipe()
        srv.add_connection(parent, route=('p', 'policy', None))
        reqs = _requests(2, 10 + w, entity=(5 + w, 30 + 7 * w))
        all_reqs.append(reqs)
        p = ctx.Process(target=_client, args=(child, reqs, q), daemon=True)
        p.start()
        procs.append(p)
    got = []
    import time
    t_end = time.time() + 240
    while len(got) < 3 and time.time() < t_end:
        srv.serve_once(timeout=0.05)
        while not q.empty():
            from applestar_amd.utils import serialize
            got.append(serialize.loads(q.get()))
    srv.drain()
    for p in procs:
        p.join(timeout=30)
    assert len(got) == 3 and srv.stats['requests'] == 6
    ref = {}
    for reqs in all_reqs:
        for r in reqs:
            ref[int(r['entity_num'])] = srv._forward('p', 'policy', [r])[0]
    for outs in got:
        for o in outs:
            exp = dict(ref[int(o['entity_num'])])
            exp.pop('logit')                                   # served replies drop the policy logits
            _close(o, exp)
