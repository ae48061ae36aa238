"""Does the system learn?  Two small, fast learning runs with curves (VERDICT r4 "missing" item 1).

The reference publishes learning outcomes - SL / RL win-rate curves (``docs/guidance_to_small_scale_training.md:
136-140,255-259``) and per-head SL accuracy metrics (``distar/agent/default/sl_training/sl_loss.py:100-136``) - that
need SC2 and days of compute.  These two runs pin the same property on one GPU in seconds, through the production
trainers (native kernels, fused losses, fused clip + Adam):

* :func:`sl_overfit_curve` - the SL trainer memorises one fixed synthetic batch (random observations, random labels
  for all six heads): per-head accuracy / IoU rise and the location L2 falls.  A trainer that does not move the
  weights along the loss gradient cannot memorise random labels.
* :func:`rl_bandit_curve` - an on-policy contextual bandit through the RL learner: every iteration samples the
  action types of a fixed batch of observations from the CURRENT policy (its own teacher-forced forward), rewards
  the ``winloss`` field +1/T at the steps whose action type lies in a fixed half of the 327 types (even ids) and
  -1/T elsewhere (returns inside the atan-squashed winloss value's range), and trains one RL step (V-trace PG + UPGO + TD(lambda) + entropy + KL against the sampling-time
  logits).  The policy's probability mass on the rewarded half must rise from ~0.5, and the winloss value must
  track the return (its TD(lambda) loss falls).

Both return a list of per-step metric dicts (``tools/learn_curves.py`` writes them to ``profiles/``;
``tests/test_learning_gpu.py`` asserts thresholds; the torch fp32 path runs beside the native one as control).
"""
from __future__ import annotations

import time
from typing import Dict, List

import torch

from ..lib.features import actions_mask
from ..rl.synthetic import rl_batch, sl_batch, to_device

SL_HEAD_METRICS = ('action_type_acc', 'delay_distance_L1', 'selected_units_iou', 'target_unit_acc',
                   'target_location_distance_L2', 'total_loss')


def _native_switch(native: bool):
    from .. import ops
    prev = ops.native_enabled()
    ops.set_native(native)
    return prev


@torch.no_grad()
def _sl_eval(tr, b) -> Dict:
    """Teacher-forced argmax accuracy of every head on the batch (the selected-units head per labelled step:
    the reference's SL metrics leave its IoU at 0 in teacher-forced mode, sl_loss.py test_iou off)."""
    m = tr.model
    was = m.training
    m.eval()
    B = len(b['traj_lens'])
    H = m.core_lstm.hidden_size
    z = torch.zeros(B, H, device=tr.device)
    hs = [(z, z) for _ in range(m.core_lstm.num_layers)]
    kw = {k: v for k, v in b.items() if k not in ('hidden_state', 'new_episodes')}
    logits, _, _ = m.sl_train(**kw, hidden_state=hs)
    act, am = b['action_info'], b['action_mask']
    out = {}
    for k in ('action_type', 'delay', 'queued', 'target_unit', 'target_location'):
        hit = (logits[k].argmax(-1) == act[k].long()).float()
        msk = am[k].float()
        out['eval_' + k + '_acc'] = float((hit * msk).sum() / msk.sum().clamp(min=1))
    su = logits['selected_units']                                        # [B*T, S, N+1]
    lab = act['selected_units'][:, :su.shape[1]].long()
    n = b['selected_units_num'].long()
    S = su.shape[1]
    valid = (torch.arange(S, device=su.device)[None, :] < n[:, None]) & am['selected_units'].bool()[:, None]
    # the SL loss's su_mask (sl/loss.py): at step s the OTHER labelled units are forbidden, so rank the label
    # against the unlabelled units only
    lab_v = torch.where(valid, lab, torch.full_like(lab, su.shape[-1]))
    other = torch.nn.functional.one_hot(lab_v, su.shape[-1] + 1)[..., :-1].bool().any(1)      # [B*T, N+1]
    forbid = other[:, None, :].expand(-1, S, -1).clone()
    forbid.scatter_(2, lab.clamp(max=su.shape[-1] - 1)[..., None], False)
    hit = (su.masked_fill(forbid, float('-inf')).argmax(-1) == lab).float()
    out['eval_selected_units_step_acc'] = float((hit * valid).sum() / valid.float().sum().clamp(min=1))
    m.train(was)
    return out


def sl_overfit_curve(device, steps: int = 300, native: bool = True, batch: int = 2, traj: int = 8,
                     max_entities: int = 32, lr: float = 1e-3, seed: int = 0, every: int = 1,
                     eval_every: int = 25) -> List[Dict]:
    """Train the SL trainer on ONE fixed batch for ``steps`` iterations; per-step loss metrics plus a teacher-
    forced argmax evaluation of every head every ``eval_every`` steps and at the end."""
    from ..sl.trainer import SLTrainer
    prev = _native_switch(native)
    try:
        torch.manual_seed(seed)
        tr = SLTrainer({'learner': {'ignore_steps': 0, 'learning_rate': lr, 'weight_decay': 0.0,
                                    'data': {'batch_size': batch, 'trajectory_length': traj}}}, device=device)
        b = to_device(sl_batch(batch, traj, max_entities=max_entities, seed=seed), device)
        b['new_episodes'] = [True] * batch            # same start state every step: a fixed input -> label map
        curve = []
        t0 = time.perf_counter()
        for it in range(steps):
            ev = _sl_eval(tr, b) if (it % eval_every == 0) else {}
            info = tr.step(dict(b))
            if it % every == 0 or it == steps - 1 or ev:
                curve.append({'step': it, **{k: float(info[k].detach()) for k in SL_HEAD_METRICS if k in info},
                              **ev, 'wall_s': round(time.perf_counter() - t0, 3)})
        curve.append({'step': steps, **_sl_eval(tr, b), 'wall_s': round(time.perf_counter() - t0, 3)})
        return curve
    finally:
        _native_switch(prev)


REWARDED_PARITY = 0     # action types with an even id are rewarded


def _rewarded_mask(n_types: int, device) -> torch.Tensor:
    return (torch.arange(n_types, device=device) % 2) == REWARDED_PARITY


def _logp_of(logits: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    return torch.log_softmax(logits.float(), -1).gather(-1, a.long().unsqueeze(-1)).squeeze(-1)


def rl_bandit_curve(device, iters: int = 150, native: bool = True, batch: int = 2, unroll: int = 8,
                    max_entities: int = 32, lr: float = 3e-4, seed: int = 0) -> List[Dict]:
    """On-policy action-type bandit through the RL learner (see the module docstring); per-iteration metrics:
    ``p_rewarded`` (policy mass on the rewarded half, before the update), ``frac_rewarded`` (sampled),
    ``return_mean``, ``value_mean`` (winloss value at t = 0), ``td_loss``, ``pg_loss``."""
    from ..rl.trainer import RLTrainer
    prev = _native_switch(native)
    try:
        torch.manual_seed(seed)
        tr = RLTrainer({'learner': {'use_value_feature': True, 'learning_rate': lr}}, device=device)
        base = to_device(rl_batch(batch, unroll, max_entities=max_entities, seed=seed), device)
        T, B = unroll, batch
        g = torch.Generator(device=device).manual_seed(seed + 1)
        curve = []
        t0 = time.perf_counter()
        for it in range(iters):
            b = dict(base)
            b['action_info'] = dict(base['action_info'])
            b['mask'] = dict(base['mask'])
            with torch.no_grad():
                out = tr.model.rl_learner_forward(**b)
                lt = out['target_logit']['action_type'].float()                     # [T, B, 327]
                rew_mask = _rewarded_mask(lt.shape[-1], lt.device)
                probs = torch.softmax(lt, -1)
                p_rew = probs[..., rew_mask].sum(-1)
                a = torch.multinomial(probs.reshape(-1, lt.shape[-1]), 1, generator=g).view(T, B)
                b['action_info']['action_type'] = a
                b['mask']['actions_mask'] = {k: v.to(device) for k, v in actions_mask(a.cpu()).items()}
                # the other heads' logits depend on the sampled action type (autoregressive embedding): a second
                # teacher-forced pass gives the behaviour log-probs of every head and the KL target
                out = tr.model.rl_learner_forward(**b)
                lg = {k: v.float() for k, v in out['target_logit'].items()}
                act = b['action_info']
                blp = {k: _logp_of(lg[k], act[k]) for k in ('action_type', 'delay', 'queued', 'target_unit',
                                                             'target_location')}
                su = lg['selected_units']                                           # [T, B, 64, N+1]
                labels = act['selected_units'][..., :su.shape[2]].clamp(max=su.shape[-1] - 1)
                blp['selected_units'] = _logp_of(su, labels)
                reward = dict(base['reward'])
                # +-1/T per step: returns stay inside the winloss value's (-1, 1) range (atan-squashed baseline)
                r = (rew_mask[a].float() * 2.0 - 1.0) / T
                r[-1] = 0.0          # a nonzero last winloss reward would read as "game over" (no bootstrap)
                reward['winloss'] = r
                ret = torch.flip(torch.cumsum(torch.flip(r, [0]), 0), [0])        # undiscounted (gamma 1) return
                v0 = out['value']['winloss'][0].float().mean()
            b['behaviour_logp'] = blp
            b['teacher_logit'] = lg
            b['reward'] = reward
            info = tr.step(b)
            curve.append({'iter': it, 'p_rewarded': float(p_rew.mean()),
                          'frac_rewarded': float(rew_mask[a][:-1].float().mean()),
                          'return_mean': float(ret[0].mean()), 'value_mean': float(v0),
                          'td_loss': float(info['winloss/td']), 'pg_loss': float(info['winloss/total']),
                          'entropy': float(info['entropy/total']), 'kl': float(info['kl/total']),
                          'total_loss': float(info['total_loss']), 'wall_s': round(time.perf_counter() - t0, 3)})
        return curve
    finally:
        _native_switch(prev)
