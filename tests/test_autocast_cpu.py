"""The learner forward/backward under bf16 autocast (exercised on CPU autocast so dtype plumbing
bugs are caught without a GPU)."""
import torch

from applestar_amd.models.model import Model
from applestar_amd.rl.loss import ReinforcementLoss
from applestar_amd.rl.synthetic import rl_batch


def test_rl_step_under_bf16_autocast_cpu():
    torch.manual_seed(0)
    cfg = {'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}
    m = Model(cfg, use_value_network=True)
    b = rl_batch(2, 3, max_entities=24, seed=2)
    with torch.autocast('cpu', dtype=torch.bfloat16):
        out = m.rl_learner_forward(**b)
    info = ReinforcementLoss({}).compute_loss(out)
    info['total_loss'].backward()
    assert torch.isfinite(info['total_loss'])
    n_grad = sum(int(p.grad is not None) for p in m.parameters() if p.requires_grad)
    assert n_grad > 300
