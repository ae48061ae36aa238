"""Two-phase backward on the GPU (parallel/dp.py backward_phased; the multi-rank default, forced here on one rank):
the model cuts its graph at the encoders' outputs (detached leaves, SkipLinks carried over), phase 1 runs the
heads / LSTM / critics (with the deferred head weight gradients) and would issue their buckets' all-reduce, phase 2
runs the encoders.  Every parameter's gradient equals the one-phase backward's - fp32 (native split-MFMA kernels,
GradientReducer) and bf16 (master weights, MasterWeights)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_phased_backward_matches_single_phase_gpu(precision, monkeypatch):
    from applestar_amd.ops import native
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.rl.synthetic import rl_batch, to_device
    native.ensure_loaded()
    batch = rl_batch(2, 6, max_entities=96, seed=4)
    grads = {}
    for mode in ('0', '0b', '1'):
        monkeypatch.setenv('APPLESTAR_PHASED_BACKWARD', mode[0])
        torch.manual_seed(0)
        tr = RLTrainer({'learner': {'use_value_feature': True,
                                    'amp_dtype': 'bfloat16' if precision == 'bf16' else None},
                        'model': {'enable_baselines': ['winloss']}}, device='cuda')
        assert tr.model.phase_cut == (mode == '1')
        b = to_device(copy.deepcopy(batch), 'cuda')
        from applestar_amd.runtime.train_engine import amp_context
        with amp_context(tr.device, tr.amp_dtype):
            out = tr.model.rl_learner_forward(**b)
        info = tr.loss.compute_loss(out)
        tr.backward(info['total_loss'])
        torch.cuda.synchronize()
        if tr.master is not None:
            g = {'master': tr.master.master.grad.clone()}
            g.update({tr.master.names[p]: p.grad.clone() for p in tr.master.fp32_params})
        else:
            g = {n: p.grad.clone() for n, p in tr.model.named_parameters() if p.requires_grad}
        grads[mode] = g
    # a few kernels reduce with float atomics (run-to-run noise): the one-phase path run twice sets each
    # parameter's noise floor; the phased result must sit within 4x that floor (or the fixed tolerance)
    # A near-cancelling gradient (the last location conv's bias: the softmax gradient sums to ~0 over a row's 24,320
    # locations) has a scale far below the rest; it is judged against the largest gradient of the model (1e-6).
    bad = {}
    tol = 1e-5 if precision == 'fp32' else 2e-2
    top = max(float(a.abs().max()) for a in grads['0'].values())
    for k, a in grads['0'].items():
        scale = max(float(a.abs().max()), 1e-30)
        noise = float((a - grads['0b'][k]).abs().max())
        err = float((a - grads['1'][k]).abs().max())
        if err > max(tol * scale, 4 * noise, 1e-6 * top):
            bad[k] = (err / scale, noise / scale, scale / top)
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:8]
