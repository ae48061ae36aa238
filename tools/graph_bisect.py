"""Which part of the RL learner step breaks HIP-graph capture?  One stage per process (a crash in capture
ends the process); run the stages in order and stop at the first failure.

    python tools/graph_bisect.py <stage>
stages: fwd_nograd | fwd | fwd_loss | fwd_bwd_nomaster | fwd_bwd | update | encoder | heads | lstm | loss_only
"""
from __future__ import annotations

import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    stage = sys.argv[1]
    if stage.startswith('trainer'):
        return trainer_sequence(stage)
    from applestar_amd.models import encoders, model as model_mod
    from applestar_amd.models.encoders import entity_pad_for
    from applestar_amd.rl.synthetic import rl_batch, to_device
    from applestar_amd.rl.trainer import RLTrainer, _amp
    from applestar_amd.runtime.prefetch import entity_total_hint
    encoders.SCALAR_SIDE_STREAM = model_mod.SIDE_STREAMS_ENABLED = os.environ.get('SIDE', '0') == '1'
    torch.manual_seed(0)
    tr = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': os.environ.get('GS', '1') == '1'},
                    'model': {'enable_baselines': ['winloss']}}, device='cuda')
    h = rl_batch(2, 4, max_entities=64, seed=11)
    b = to_device(h, 'cuda')
    b['entity_pad'] = entity_pad_for(entity_total_hint(h), b['entity_info']['unit_type'].shape[1])
    dev = torch.device('cuda')

    def run():
        if stage == 'fwd_nograd':
            with torch.no_grad(), _amp(dev, 'bfloat16'):
                return tr.model.rl_learner_forward(**b)['target_logit']['action_type']
        if stage == 'fwd':
            with _amp(dev, 'bfloat16'):
                return tr.model.rl_learner_forward(**b)['target_logit']['action_type']
        if stage == 'fwd_loss':
            with _amp(dev, 'bfloat16'):
                out = tr.model.rl_learner_forward(**b)
            return tr.loss.compute_loss(out)['total_loss']
        if stage == 'fwd_bwd_nomaster':
            with _amp(dev, 'bfloat16'):
                out = tr.model.rl_learner_forward(**b)
            loss = tr.loss.compute_loss(out)['total_loss']
            return torch.autograd.grad(loss, tr.reducer.params, allow_unused=True)[0]
        if stage == 'fwd_bwd':
            return tr._fwd_bwd(b)['total_loss']
        if stage == 'update':
            return tr._update()
        raise SystemExit(f'unknown stage {stage}')

    if os.environ.get('SIDE_WARM', '0') == '1':   # eager warm-up WITH side streams, capture without
        encoders.SCALAR_SIDE_STREAM = model_mod.SIDE_STREAMS_ENABLED = True
    for _ in range(2):           # warm-up (eager)
        run()
    torch.cuda.synchronize()
    if os.environ.get('SIDE_WARM', '0') == '1':
        encoders.SCALAR_SIDE_STREAM = model_mod.SIDE_STREAMS_ENABLED = os.environ.get('SIDE', '0') == '1'
    g = torch.cuda.CUDAGraph()
    t0 = time.time()
    print(f'[{stage}] capturing', flush=True)
    pool = torch.cuda.graph_pool_handle() if os.environ.get('POOL', '0') == '1' else None
    with torch.cuda.graph(g, pool=pool):
        out = run()
    print(f'[{stage}] captured in {time.time() - t0:.1f}s; replaying', flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f'[{stage}] OK {float(out.float().sum()) if torch.is_tensor(out) else out}', flush=True)


def trainer_sequence(stage):
    """The graphed RLTrainer over b0 b1 b0 b1 b0 (eager, eager, capture+replay, capture+replay, replay);
    'trainer_pair' interleaves an eager trainer (side streams on) like the GPU test."""
    from applestar_amd.rl.synthetic import rl_batch, to_device
    from applestar_amd.rl.trainer import RLTrainer
    from applestar_amd.runtime.prefetch import entity_total_hint
    cfg = {'learner': {'use_value_feature': True, 'graph_step': True}, 'model': {'enable_baselines': ['winloss']}}
    torch.manual_seed(0)
    other = None
    if stage == 'trainer_pair':
        other = RLTrainer({'learner': {'use_value_feature': True, 'graph_step': False},
                           'model': {'enable_baselines': ['winloss']}}, device='cuda')
    tr = RLTrainer(cfg, device='cuda')
    bs = []
    for seed in (11, 12):
        h = rl_batch(2, 4, max_entities=64, seed=seed)
        b = to_device(h, 'cuda')
        b['entity_total'] = entity_total_hint(h)
        bs.append(b)
    for i in range(5):
        if other is not None:
            other.step(dict(bs[i % 2]))
        print(f'[{stage}] step {i} (captures {tr.graph.captures})', flush=True)
        info = tr.step(dict(bs[i % 2]))
        torch.cuda.synchronize()
        print(f'[{stage}] step {i} loss {float(info["total_loss"]):.6g} grad {float(info["gradient"]):.6g}', flush=True)
    print(f'[{stage}] OK captures {tr.graph.captures} replays {tr.graph.replays}', flush=True)


if __name__ == '__main__':
    main()
