"""The RL learner step under data parallelism, multi-process on CPU (gloo), world 2 and 4.

Covers the paths the 8-GPU RCCL run takes (``distar/ctools/utils/dist_helper.py:321-344,421-431``), with
the same launch structure at every world size (parallel/dp.py): one ``autograd.grad`` + one multi-tensor
copy into the flat buckets, then one all-reduce per bucket.

* construction broadcasts rank 0's weights, so differently seeded ranks start identical;
* value pre-training (``value_pretrain_iters``): the policy parameters get no gradient on any rank (their
  buckets are zeroed, the update leaves them bit-identical) while the critic moves, identically everywhere;
* a normal step: every rank ends with the same weights, which differ from the start;
* league reset (rl_learner.py LearnerHook: rank 0's checkpoint path broadcast, every rank reloads and resets
  its optimizer): ranks whose weights had drifted apart are identical again, also after the next step;
* the packed log-scalar reduce (``pdist.allreduce_scalars``: ONE collective for the logged scalars)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _fingerprint(tr):
    sd = tr.model_state_dict()
    return {k: float(v.double().sum()) + 1e-3 * float(v.double().abs().sum()) for k, v in sd.items()
            if v.is_floating_point()}


def _worker(rank, world, port, ckpt_dir, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch
    pdist.init(backend='gloo')
    torch.manual_seed(rank)                       # different init per rank: the constructor's broadcast fixes it
    cfg = {'learner': {'use_value_feature': True, 'value_pretrain_iters': 1, 'learning_rate': 1e-3, 'bucket_mb': 4},
           'model': {'enable_baselines': ['winloss']}}
    tr = RLTrainer(cfg, device='cpu')
    out = {'rank': rank, 'buckets': tr.reducer.num_buckets}
    out['init'] = _fingerprint(tr)
    batch = lambda s: rl_batch(1, 2, max_entities=16, seed=100 * s + rank)  # noqa: E731  (per-rank data)

    # 1) value pre-training step: only the critic moves
    before = {k: v.clone() for k, v in tr.model_state_dict().items()}
    info = tr.step(batch(1))
    after = {k: v.clone() for k, v in tr.model_state_dict().items()}
    policy_keys = [k for k in before if k.startswith('policy.') and before[k].is_floating_point()]
    value_keys = [k for k in before if k.startswith('value_networks.') and before[k].is_floating_point()]
    out['policy_unchanged'] = all(torch.equal(before[k], after[k]) for k in policy_keys)
    out['value_moved'] = any(not torch.equal(before[k], after[k]) for k in value_keys)
    out['pretrain'] = _fingerprint(tr)
    out['loss_finite'] = bool(torch.isfinite(info['total_loss']))

    # 2) a normal step
    tr.step(batch(2))
    after2 = tr.model_state_dict()
    out['policy_moved'] = any(not torch.equal(after[k], after2[k]) for k in policy_keys)
    out['step2'] = _fingerprint(tr)

    # 3) league reset: rank 0 saves, everyone drifts apart, rank 0's path is broadcast, everyone reloads
    path = os.path.join(ckpt_dir, 'reset.pth')
    if rank == 0:
        torch.save(tr.state_dict()['model'], path)
    pdist.barrier()
    with torch.no_grad():
        for p in tr.model.parameters():
            p.add_(0.01 * (rank + 1))
    out['drifted'] = _fingerprint(tr)
    got = pdist.broadcast_object(path if rank == 0 else None)
    tr.load_model_state_dict(torch.load(got, weights_only=True))
    tr.reset_optimizer()
    out['reset'] = _fingerprint(tr)
    tr.step(batch(3))
    out['after_reset_step'] = _fingerprint(tr)

    # 4) packed scalar reduce
    sc = pdist.allreduce_scalars({'rank': torch.tensor(float(rank)), 'one': torch.tensor(1.0),
                                  'loss': info['total_loss'].detach()})
    out['scalars'] = sc
    q.put(out)
    pdist.finalize()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world', [2, 4])
def test_rl_trainer_data_parallel(world, tmp_path):
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=500) for _ in range(world)], key=lambda r: r['rank'])
    for p in procs:
        p.join(timeout=60)
    r0 = res[0]
    assert r0['buckets'] > 1
    for r in res:
        assert r['loss_finite'] and r['policy_unchanged'] and r['value_moved'] and r['policy_moved'], r['rank']
        for stage in ('init', 'pretrain', 'step2', 'reset', 'after_reset_step'):
            assert r[stage] == r0[stage], (r['rank'], stage)       # bit-identical across ranks
        assert abs(r['scalars']['rank'] - (world - 1) / 2) < 1e-6 and abs(r['scalars']['one'] - 1.0) < 1e-6
        assert r['scalars'] == r0['scalars']
    assert r0['step2'] != r0['init']
    assert res[1]['drifted'] != r0['drifted']           # the reset really had something to undo
    assert r0['reset'] == {k: v for k, v in r0['step2'].items()}


def test_phased_backward_equals_single_phase(monkeypatch):
    """The two-phase backward (parallel/dp.py backward_phased: loss -> downstream parameters + encoder outputs,
    then encoder outputs -> encoder parameters) writes the same bucket gradients as one autograd.grad."""
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch
    torch.set_num_threads(2)
    grads = {}
    for mode in ('0', '1'):
        monkeypatch.setenv('APPLESTAR_PHASED_BACKWARD', mode)
        torch.manual_seed(0)
        tr = RLTrainer({'learner': {'use_value_feature': True, 'bucket_mb': 4},
                        'model': {'enable_baselines': ['winloss']}}, device='cpu')
        assert tr.reducer.phase_params[0] and tr.reducer.phase_params[1]
        out = tr.model.rl_learner_forward(**rl_batch(1, 2, max_entities=16, seed=3))
        tr.backward(tr.loss.compute_loss(out)['total_loss'])
        grads[mode] = {n: p.grad.clone() for n, p in tr.model.named_parameters() if p.requires_grad}
    assert grads['0'].keys() == grads['1'].keys()
    bad = [n for n in grads['0'] if not torch.allclose(grads['0'][n], grads['1'][n], rtol=1e-5, atol=1e-7)]
    assert not bad, bad[:5]
    assert any(n.startswith('encoder.') and grads['1'][n].abs().sum() > 0 for n in grads['1'])


def _wire_worker(rank, world, port, comm, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch
    pdist.init(backend='gloo')
    torch.manual_seed(0)
    tr = RLTrainer({'learner': {'use_value_feature': True, 'bucket_mb': 4, 'comm_dtype': comm},
                    'model': {'enable_baselines': ['winloss']}}, device='cpu')
    batch = rl_batch(1, 2, max_entities=16, seed=10 + rank)
    # this rank's own gradient, one plain autograd.grad over the uncut graph (the reference for the average)
    params = [p for p in tr.model.parameters() if p.requires_grad]
    assert tr.model.phase_cut
    tr.model.phase_cut = False
    loss = tr.loss.compute_loss(tr.model.rl_learner_forward(**rl_batch(1, 2, max_entities=16, seed=10 + rank)))
    tr.model.phase_cut = True
    local = torch.autograd.grad(loss['total_loss'], params, allow_unused=True)
    local = torch.cat([(g if g is not None else torch.zeros_like(p)).reshape(-1) for g, p in zip(local, params)])
    allg = [torch.zeros_like(local) for _ in range(world)]
    torch.distributed.all_gather(allg, local)
    ref = torch.stack(allg).mean(0)
    # the trainer's phased backward (multi-rank default) + bucket all-reduce
    out = tr.model.rl_learner_forward(**batch)
    tr.backward(tr.loss.compute_loss(out)['total_loss'])
    tr._reduce()
    got = torch.cat([p.grad.reshape(-1) for p in params])
    q.put({'rank': rank, 'err': float((got - ref).abs().max()), 'scale': float(ref.abs().max()),
           'sum': float(got.double().sum())})
    pdist.finalize()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('comm', [None, 'bfloat16'])
def test_phased_allreduce_world2_matches_average(comm):
    """World 2 (gloo): the phased backward with its early all-reduce of the downstream buckets gives every rank
    the average of the ranks' own gradients - exactly on the fp32 wire, within bf16 rounding on the bf16 wire -
    and identical reduced gradients on both ranks."""
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_wire_worker, args=(r, 2, port, comm, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=500) for _ in range(2)], key=lambda r: r['rank'])
    for p in procs:
        p.join(timeout=60)
    tol = 1e-5 if comm is None else 2 ** -7
    for r in res:
        assert r['err'] <= tol * r['scale'], r
    assert res[0]['sum'] == res[1]['sum']
