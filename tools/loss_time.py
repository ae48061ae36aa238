import os, sys, time, torch
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
from applestar_amd.rl.trainer import RLTrainer, _amp
from applestar_amd.rl.synthetic import rl_batch, to_device
from applestar_amd.runtime.prefetch import entity_total_hint
dev = torch.device('cuda', 0)
tr = RLTrainer({'learner': {'use_value_feature': True}, 'model': {'enable_baselines': ['winloss']}}, device=dev)
h = rl_batch(6, 64, seed=0); b = to_device(h, dev); b['entity_total'] = entity_total_hint(h)
with _amp(dev, 'bfloat16'):
    out = tr.model.rl_learner_forward(**b)
leaves = []
def detach_tree(x):
    if torch.is_tensor(x):
        if x.requires_grad:
            y = x.detach().requires_grad_(); leaves.append(y); return y
        return x
    if isinstance(x, dict): return {k: detach_tree(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)): return type(x)(detach_tree(v) for v in x)
    return x
o2 = detach_tree(out)
for i in range(8):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    info = tr.loss.compute_loss(o2)
    t1 = time.perf_counter()
    g = torch.autograd.grad(info['total_loss'], leaves, allow_unused=True)
    t2 = time.perf_counter(); torch.cuda.synchronize(); t3 = time.perf_counter()
    if i >= 3: print(f'loss fwd host {1e3*(t1-t0):.2f} ms, bwd host {1e3*(t2-t1):.2f} ms, total wall {1e3*(t3-t0):.2f} ms, leaves {len(leaves)}')
