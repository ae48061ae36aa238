"""Whole-model checks on the MI355X: the native/bf16 learner path agrees with the fp32 CPU oracle,
and a full RL learner iteration (with native kernels) runs and updates weights."""
import copy
import math

import pytest
import torch

from applestar_amd.models.model import Model
from applestar_amd.rl.synthetic import rl_batch, to_device
from applestar_amd.rl.trainer import RLTrainer

pytestmark = pytest.mark.gpu
CFG = {'learner': {'use_value_feature': True, 'amp_dtype': 'bfloat16'}, 'model': {'enable_baselines': ['winloss']}}


def test_rl_forward_gpu_bf16_matches_cpu_fp32():
    torch.manual_seed(0)
    cpu = Model(CFG, use_value_network=True).eval()
    gpu = copy.deepcopy(cpu).cuda().eval()
    batch = rl_batch(2, 3, max_entities=48, seed=3)
    with torch.no_grad():
        ref = cpu.rl_learner_forward(**copy.deepcopy(batch))
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = gpu.rl_learner_forward(**to_device(batch, 'cuda'))
    for k in ['action_type', 'delay', 'queued', 'target_location']:
        a, b = out['target_logit'][k].float().cpu(), ref['target_logit'][k].float()
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() < 0.05 * max(1.0, scale), k
    v_a, v_b = out['value']['winloss'].float().cpu(), ref['value']['winloss']
    assert (v_a - v_b).abs().max().item() < 0.05


def test_trainer_step_updates_weights():
    torch.manual_seed(0)
    tr = RLTrainer(CFG, device='cuda')
    before = {k: v.detach().clone() for k, v in tr.model.named_parameters()}
    info = tr.step(to_device(rl_batch(2, 4, max_entities=64, seed=1), 'cuda'))
    torch.cuda.synchronize()
    assert torch.isfinite(info['total_loss']).item()
    changed = sum(int(not torch.equal(before[k], v)) for k, v in tr.model.named_parameters())
    assert changed > 100


def test_trajectory_ring_on_gpu_matches_host_collate():
    """HBM ring + native segment_copy kernel vs the host collate of the same trajectories."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_agent import _run_episode
    from applestar_amd.agent.collate import collate_trajectories
    from applestar_amd.runtime.traj_ring import TrajectoryRing
    from applestar_amd.utils import serialize
    _, trajs, _, _ = _run_episode('train_test', traj_len=3, value_feature=True, until_full=6)
    full = [t for t in trajs if len(t) == 4][:3]
    ref = collate_trajectories(full)
    ring = TrajectoryRing(256 << 20, device='cuda')
    got = ring.batch([ring.put(serialize.dumps(t)) for t in full])
    torch.cuda.synchronize()

    def cmp(a, b, path=''):
        if isinstance(a, dict):
            for k in a:
                if k not in ('batch_size', 'unroll_len'):
                    cmp(a[k], b[k], f'{path}/{k}')
        elif isinstance(a, (list, tuple)):
            for x, y in zip(a, b):
                cmp(x, y, path)
        elif torch.is_tensor(a):
            assert a.shape == b.shape, path
            assert torch.equal(a.to(b.dtype), b.cpu()), path
    cmp(ref, got)


def test_direct_master_grad_matches_bucket_path():
    """Single-rank autograd.grad + native multi-tensor copy into the fp32 master grad == the bucket path
    (AccumulateGrad into bf16 bucket views, then bucket -> master copy)."""
    torch.manual_seed(0)
    tr = RLTrainer(CFG, device='cuda')
    batch = to_device(rl_batch(2, 4, max_entities=64, seed=3), 'cuda')

    def loss():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = tr.model.rl_learner_forward(**dict(batch))
        return tr.loss.compute_loss(out)['total_loss']

    tr.reducer.zero_grad()
    tr.master.backward(loss())
    tr.master.synchronize()
    direct = tr.master.master.grad.clone()
    fp32_direct = [p.grad.detach().float().clone() for p in tr.master.fp32_params]
    tr.reducer.zero_grad()
    loss().backward()                      # AccumulateGrad into the bucket views
    tr.master._direct = False
    tr.master.synchronize()
    ref = tr.master.master.grad
    scale = ref.abs().max().item()
    assert (direct - ref).abs().max().item() <= 2e-2 * scale
    for a, p in zip(fp32_direct, tr.master.fp32_params):
        assert (a - p.grad.float()).abs().max().item() <= 2e-2 * max(1.0, p.grad.abs().max().item())


def test_entity_total_hint_packing_matches_nonzero():
    """The prefetcher's host-side packed-entity count (nonzero_static, no device sync) gives the same
    learner forward as the synchronising nonzero path."""
    from applestar_amd.runtime.prefetch import DevicePrefetcher, entity_total_hint, pin_tree
    torch.manual_seed(0)
    m = Model(CFG, use_value_network=True).cuda().eval()
    host = pin_tree(rl_batch(2, 3, max_entities=48, seed=5))
    hint = entity_total_hint(host)
    assert hint is not None and hint > 0
    staged = next(DevicePrefetcher(iter([host]), torch.device('cuda')))
    assert staged['entity_total'] == hint
    with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
        a = m.rl_learner_forward(**staged)
        staged.pop('entity_total')
        b = m.rl_learner_forward(**staged)
    for k in a['target_logit']:
        assert torch.equal(a['target_logit'][k], b['target_logit'][k]), k


def test_graphed_section_matches_eager():
    """HIP-graph replay of a value baseline (forward + backward) == the eager module."""
    from applestar_amd.models.model import ValueBaseline
    from applestar_amd.runtime.graphs import GraphedSection
    torch.manual_seed(0)
    m = ValueBaseline(1440, atan=True).cuda().train()
    gs = GraphedSection(m, enabled=True)
    for step in range(3):
        x = torch.randn(390, 1440, device='cuda', requires_grad=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = gs(x)
        gx, *gp = torch.autograd.grad(y.sum(), [x] + list(m.parameters()))
        x2 = x.detach().clone().requires_grad_()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y2 = m(x2)
        gx2, *gp2 = torch.autograd.grad(y2.sum(), [x2] + list(m.parameters()))
        assert torch.allclose(y.float(), y2.float(), atol=1e-3, rtol=1e-3), step
        assert torch.allclose(gx.float(), gx2.float(), atol=1e-3, rtol=1e-3)
        for a, b in zip(gp, gp2):
            assert torch.allclose(a.float(), b.float(), atol=1e-2, rtol=1e-2)
        with torch.no_grad():                       # in-place weight update must be seen by the replay
            for p in m.parameters():
                p.add_(0.01)
    assert gs.replays == 3 and len(gs._graphs) == 1


def test_graphed_policy_matches_eager():
    """HIP-graph replay of the actor step (shape-static dense entity path) agrees with the eager packed
    path on logits, and its replays see new inputs."""
    from applestar_amd.lib.features import random_obs
    from applestar_amd.runtime.graphs import GraphedPolicy
    from applestar_amd.models import encoders
    torch.manual_seed(0)
    m = Model({'agent': {'extra_units': True}}).cuda().eval().to(memory_format=torch.channels_last)
    gp = GraphedPolicy(m, 'compute_logp_action')
    for seed in range(3):
        g = torch.Generator().manual_seed(seed)
        obs = random_obs(2, entity_num=torch.tensor([37 + seed, 300]), generator=g)
        obs['hidden_state'] = [(torch.zeros(2, 384), torch.zeros(2, 384)) for _ in range(3)]
        obs = to_device(obs, 'cuda')
        out_g = gp(**obs)
        lg = {k: v.float().clone() for k, v in out_g['logit'].items()}
        with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
            out_e = m.compute_logp_action(**obs)
        for k in ('action_type',):
            a, b = lg[k], out_e['logit'][k].float()
            assert (a - b).abs().max().item() < 0.05 * max(1.0, b.abs().max().item()), (seed, k)
    assert gp.captures == 1 and not encoders.STATIC_SHAPES


def test_inference_server_graphed_matches_eager():
    """The actor inference server's HIP-graph path (entities padded to 512, batch bucket 4 for 3
    requests) returns the same per-row results as its eager path."""
    from applestar_amd.actor.inference import InferenceServer
    from applestar_amd.lib.features import random_obs

    def split(tree, i):
        if torch.is_tensor(tree):
            return tree[i]
        if isinstance(tree, dict):
            return {k: split(v, i) for k, v in tree.items()}
        return tree

    torch.manual_seed(0)
    m = Model({'agent': {'extra_units': True}}).eval()
    g = torch.Generator().manual_seed(4)
    obs = random_obs(3, entity_num=torch.tensor([12, 200, 77]), generator=g)
    reqs = []
    for i in range(3):
        r = split(obs, i)
        r['hidden_state'] = [(torch.zeros(384), torch.zeros(384)) for _ in range(3)]
        reqs.append(r)
    outs = {}
    for graphs in (False, True):
        srv = InferenceServer('cuda', use_graphs=graphs)
        srv.set_model('p', m)
        outs[graphs] = srv._forward('p', 'policy', reqs)
    for a, b in zip(outs[True], outs[False]):
        la, lb = a['logit']['action_type'].float(), b['logit']['action_type'].float()
        assert (la - lb).abs().max().item() < 0.05 * max(1.0, lb.abs().max().item())
        assert a['entity_num'] == b['entity_num']


def test_inference_server_graphed_sees_hot_weight_load():
    """After ``load_state_dict`` (weights copied in place, graphs kept) the graphed server samples with
    the NEW weights: the fused heads' embedding tables and the selected-units query fold must be
    recomputed inside the replay, not read from a cache captured with the old weights."""
    from applestar_amd.actor.inference import InferenceServer
    from applestar_amd.lib.features import random_obs

    torch.manual_seed(0)
    m_old = Model({'agent': {'extra_units': True}}).eval()
    m_new = Model({'agent': {'extra_units': True}}).eval()
    g = torch.Generator().manual_seed(9)
    obs = random_obs(2, entity_num=torch.tensor([40, 150]), generator=g)
    reqs = []
    for i in range(2):
        r = {k: (v[i] if torch.is_tensor(v) else {kk: vv[i] for kk, vv in v.items()} if isinstance(v, dict) else v)
             for k, v in obs.items()}
        r['hidden_state'] = [(torch.zeros(384), torch.zeros(384)) for _ in range(3)]
        gu = torch.Generator().manual_seed(100 + i)          # fixed sampling noise: same actions both times
        r['noise'] = {k: torch.rand((), generator=gu) for k in ('action_type', 'delay', 'queued', 'target_unit',
                                                                'target_location')}
        r['noise']['selected_units'] = torch.rand(64, generator=gu)
        reqs.append(r)
    srv = InferenceServer('cuda', use_graphs=True)
    srv.set_model('p', copy.deepcopy(m_old))
    srv._forward('p', 'policy', reqs)                               # capture with the old weights
    srv.load_state_dict('p', {k: v.cuda() for k, v in m_new.state_dict().items()})
    got = srv._forward('p', 'policy', reqs)
    ref_srv = InferenceServer('cuda', use_graphs=True)
    ref_srv.set_model('p', copy.deepcopy(m_new))
    ref = ref_srv._forward('p', 'policy', reqs)
    for a, b in zip(got, ref):
        for k in ('action_type', 'delay', 'queued', 'target_unit'):
            assert torch.equal(a['action_info'][k], b['action_info'][k]), k
            la, lb = a['logit'][k].float(), b['logit'][k].float()
            assert (la - lb).abs().max().item() < 1e-3 * max(1.0, lb.abs().max().item()), k


def test_inference_server_policy_teacher_graphed_matches_eager():
    """The training actor's merged request ('policy+teacher': policy sample + the teacher's logits for it, one
    HIP graph per (batch bucket, entity bucket)) agrees with the eager merged path; the routed-frame path
    (native collate_frames into one pinned buffer) gives the same replies as in-process inputs."""
    from applestar_amd.actor.inference import InferenceServer
    from applestar_amd.utils import serialize
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_inference_server import _requests
    torch.manual_seed(0)
    pol, tea = Model().eval(), Model().eval()
    reqs = _requests(3, 5, entity=(12, 200, 77))
    for r in reqs:
        r['teacher_hidden_state'] = [(torch.randn(384) * 0.1, torch.randn(384) * 0.1) for _ in range(3)]
    outs = {}
    for graphs in (False, True):
        srv = InferenceServer('cuda', use_graphs=graphs)
        srv.set_model('p', copy.deepcopy(pol))
        srv.set_model('t', copy.deepcopy(tea), teacher=True)
        outs[graphs] = srv._forward('p', 'policy+teacher', reqs, teacher_id='t')
        if graphs:
            L = srv._launch(('p', 'policy+teacher', 't'), frames=[serialize.dumps(r) for r in reqs], keep_logits=True)
            outs['frames'] = srv._results(L)
            assert {k[2] for k in srv._graphed} == {256}          # entity bucket of max(12, 200, 77)
    for a, b, c in zip(outs[True], outs[False], outs['frames']):
        # the teacher's action-type logits do not depend on the sampled action: graphed == eager up to bf16
        ta, tb = a['teacher']['logit']['action_type'].float(), b['teacher']['logit']['action_type'].float()
        assert (ta - tb).abs().max().item() < 0.05 * max(1.0, tb.abs().max().item())
        for k in ('action_type', 'delay', 'queued', 'target_unit', 'target_location'):   # same graph, same bits
            assert torch.equal(a['action_info'][k], c['action_info'][k]), k
            assert torch.equal(a['teacher']['logit'][k], c['teacher']['logit'][k]), k


@pytest.mark.parametrize('amp', ['bfloat16', None])
def test_graphed_train_step_matches_eager(amp):
    """Whole-step HIP graphs (runtime/step_graph.py: fwd+loss+bwd+clip+Adam in one graph on one rank, fixed
    padded entity packing, the fused clip + Adam reading its bias corrections from a device buffer, derived
    weight forms refreshed inside the graph) train like the eager step: same losses and weights over 5 steps on
    two alternating batches (first sight eager, second capture + replay, then replay)."""
    from applestar_amd.runtime.prefetch import entity_total_hint
    lc = {'use_value_feature': True, 'amp_dtype': amp}
    torch.manual_seed(0)
    eager = RLTrainer({'learner': lc, 'model': CFG['model']}, device='cuda')
    torch.manual_seed(0)
    graphed = RLTrainer({'learner': dict(lc, graph_step=True), 'model': CFG['model']}, device='cuda')
    assert eager.graph is None and graphed.graph is not None and graphed.fused_opt is not None

    def flat(tr):
        if tr.master is not None:
            return tr.master.master.detach().clone()
        return torch.cat([p.detach().reshape(-1) for p in tr.params])
    m0 = flat(graphed)
    assert torch.equal(m0, flat(eager))
    hosts = [rl_batch(2, 4, max_entities=64, seed=s) for s in (11, 12)]
    batches = []
    for h in hosts:
        b = to_device(h, 'cuda')
        b['entity_total'] = entity_total_hint(h)
        batches.append(b)
    for i in range(5):
        b = batches[i % 2]
        ie = eager.step(dict(b))
        ig = graphed.step(dict(b))
        for k in ('total_loss', 'gradient'):
            a, r = float(ig[k]), float(ie[k])
            if not abs(a - r) <= 2e-2 * max(1.0, abs(r)):
                graphed.graph.replay_fwd_bwd_only()
                torch.cuda.synchronize()
                from applestar_amd.ops import native
                lstm_err = int(native.ensure_loaded().lstm_split_error(0).item())
                raise AssertionError((i, k, a, r, 'non-finite after a fwd/bwd replay:', graphed.nonfinite_grads()[:8],
                                      'lstm split timeout flag', lstm_err))
    torch.cuda.synchronize()
    assert graphed.graph.captures == 2 and graphed.graph.replays == 3 and graphed.graph.eager_steps == 2
    eager.optimizer.state_dict(), graphed.optimizer.state_dict()   # lazy per-parameter step counters written
    st_e = eager.optimizer.state[eager.opt_params[0]]['step']
    st_g = graphed.optimizer.state[graphed.opt_params[0]]['step']
    assert float(st_e) == float(st_g) == 5.0
    de, dg = flat(eager) - m0, flat(graphed) - m0
    assert de.abs().max().item() > 0 and dg.abs().max().item() > 0
    cos = float((de * dg).sum() / (de.norm() * dg.norm()))
    assert cos > (0.9 if amp else 0.99), cos   # same updates up to rounding on near-zero gradients (Adam ~ sign)


def test_stacked_lstm_pipelined_matches_layer_by_layer():
    """The wavefront schedule (time chunks x one stream per layer) computes exactly the layer-by-layer
    recurrence: outputs, final states and all gradients agree (fp32 weights, 65 steps, 5 chunks)."""
    import applestar_amd.models.lstm as L
    torch.manual_seed(21)
    m = L.StackedLNLSTM(96, 384, 3).cuda()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) * (0.05 if p.dim() > 1 else 0.1) + (1.0 if p.dim() == 1 else 0.0))
    x = torch.randn(65, 6, 96, device='cuda', requires_grad=True)
    state = [(torch.randn(6, 384, device='cuda') * 0.3, torch.randn(6, 384, device='cuda') * 0.3) for _ in range(3)]
    res = {}
    old = L.PIPELINE_CHUNKS
    try:
        for chunks in (1, 5):
            L.PIPELINE_CHUNKS = chunks
            m.zero_grad()
            x.grad = None
            out, st = m(x, state)
            (out.square().mean() + sum(h.sum() * 0.1 + c.sum() * 0.05 for h, c in st)).backward()
            torch.cuda.synchronize()
            res[chunks] = (out.detach().clone(), [t.detach().clone() for hc in st for t in hc], x.grad.clone(),
                           [p.grad.clone() for p in m.parameters()])
    finally:
        L.PIPELINE_CHUNKS = old
    a, b = res[1], res[5]
    assert (a[0] - b[0]).abs().max().item() < 1e-5
    assert all((u - v).abs().max().item() < 1e-5 for u, v in zip(a[1], b[1]))
    assert (a[2] - b[2]).abs().max().item() < 1e-5
    for u, v in zip(a[3], b[3]):
        assert (u - v).abs().max().item() < 1e-4 * max(1.0, u.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_data_parallel_two_ranks_finite_and_identical(tmp_path, precision):
    """Two ranks (gloo, sharing the one GPU) run the learner step of each precision - fp32: GradientReducer
    buckets + derived weight forms + fused clip/Adam; bf16: master weights - on different data: every step's
    gradient norm is finite and bit-identical on both ranks (the reduced gradient), the loss stays finite, and
    the updated weights are bit-identical (same replica after every step)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, APPLESTAR_DIST_BACKEND='gloo')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(29631 + (precision == 'bf16')), os.path.join(root, 'tools', 'loss_probe.py'),
           '--steps', '3', '--batch', '2', '--unroll', '8', '--precision', precision]
    res = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert res.returncode == 0, res.stderr[-3000:]
    # the two ranks share the launcher's stdout: a line may hold two records back to back
    recs, dec = [], json.JSONDecoder()
    for line in res.stdout.splitlines():
        i = line.find('{')
        while i >= 0:
            obj, end = dec.raw_decode(line, i)
            recs.append(obj)
            i = line.find('{', end)
    assert len(recs) == 6, res.stdout[-2000:]
    for r in recs:
        assert math.isfinite(r['loss']) and math.isfinite(r['grad_norm']), r
        assert 'nonfinite_grads' not in r, r
    for s in range(3):
        a, b = [r for r in recs if r['step'] == s]
        assert a['grad_norm'] == b['grad_norm'] and a['weight_hash'] == b['weight_hash'], (a, b)
        assert a['loss'] != b['loss']          # different data per rank: the equality above is the reduction


@pytest.mark.parametrize('only_value', [False, True])
@pytest.mark.parametrize('bo_pg_weight', [0.5, 0.0])
def test_fused_rl_loss_matches_torch_loss(only_value, bo_pg_weight):
    """rl_loss.hip (the loss after the per-head statistics, with closed-form gradients) vs the torch
    ReinforcementLoss path: total loss, every info entry, and the gradients w.r.t. all head logits and the
    baseline values; two baseline fields (winloss + build_order with its mask)."""
    from applestar_amd.rl import loss as L
    dev = torch.device('cuda')
    T, B = 16, 3
    batch = to_device(rl_batch(B, T, max_entities=40, seed=3), dev)
    g = torch.Generator(device=dev).manual_seed(7)

    def make_inputs():
        logits = {}
        for h, t in batch['teacher_logit'].items():
            x = t + 0.5 * torch.randn(t.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(hash(h) % 1000))
            logits[h] = torch.where(t > -1e8, x, torch.full_like(x, -1e9)).requires_grad_()
        values = {'winloss': (0.3 * torch.randn(T + 1, B, device=dev, generator=torch.Generator(device=dev).manual_seed(1))).requires_grad_(),
                  'build_order': (0.3 * torch.randn(T + 1, B, device=dev, generator=torch.Generator(device=dev).manual_seed(2))).requires_grad_()}
        mask = dict(batch['mask'])
        mask['build_order_mask'] = (torch.rand(T, B, device=dev, generator=g) < 0.7).float()
        return {'target_logit': logits, 'value': values, 'action_log_prob': batch['behaviour_logp'],
                'teacher_logit': batch['teacher_logit'], 'mask': mask, 'action': batch['action_info'],
                'reward': batch['reward'], 'step': batch['step']}

    # pg weight 0 (the reference config's non-winloss fields): pg/<field> is still logged by both paths
    cfg = {'loss_weights': {'pg': {'build_order': bo_pg_weight}, 'baseline': {'build_order': 2.0}}}
    results = []
    inp = make_inputs()
    for fused in (True, False):
        L.FUSED_LOSS = fused
        try:
            loss = L.ReinforcementLoss(cfg)
            loss.only_update_value = only_value
            x = {k: v for k, v in inp.items()}
            info = loss.compute_loss(x)
            leaves = list(inp['target_logit'].values()) + list(inp['value'].values())
            grads = torch.autograd.grad(info['total_loss'], leaves, allow_unused=True)
            results.append((info, grads))
        finally:
            L.FUSED_LOSS = True
    (fi, fg), (ti, tg) = results
    assert set(fi) == set(ti)
    for k in ti:
        a, r = float(fi[k]), float(ti[k])
        assert abs(a - r) <= 1e-4 + 1e-4 * abs(r), (k, a, r)
    for a, r in zip(fg, tg):
        if r is None:
            assert a is None or float(a.abs().max()) == 0.0
            continue
        a = torch.zeros_like(r) if a is None else a
        assert float((a - r).abs().max()) <= 1e-5 + 1e-4 * float(r.abs().max())


def test_replay_dataloader_shared_batch_gpu():
    """SL shared batch on the GPU: collator process -> hipHostRegister'ed shared slab -> one async H2D per
    batch on a side stream; the device batches equal the in-process host collation of the same data."""
    import functools
    from applestar_amd.learner.replay_dataloader import ReplayDataLoader
    from applestar_amd.rl.synthetic import sl_trajectories
    from applestar_amd.utils.config import AttrDict
    lengths = [9, 3, 4, 6, 4, 7, 2, 8, 5]
    cfg = AttrDict({'learner': {'data': {'batch_size': 3, 'trajectory_length': 4, 'slab_mb': 32}}})
    shared = ReplayDataLoader(cfg, device='cuda', source_factory=functools.partial(sl_trajectories, lengths, 5))
    plain = ReplayDataLoader(cfg, source=sl_trajectories(lengths, 5))
    assert shared._shared is not None and len(shared._shared._registered) == 3   # pinned slabs

    def cmp(a, b, path=''):
        if isinstance(a, dict):
            for k in b:
                cmp(a[k], b[k], f'{path}/{k}')
        elif isinstance(a, (list, tuple)):
            for x, y in zip(a, b):
                cmp(x, y, path)
        elif torch.is_tensor(a):
            assert a.is_cuda and torch.equal(a.cpu(), b), path
        else:
            assert a == b, path
    try:
        for _ in range(4):          # the 9 trajectories make exactly 4 batches of 3 slots x 4 steps
            cmp(next(shared), next(plain))
    finally:
        shared.close()
