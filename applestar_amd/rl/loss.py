"""IMPALA-style AlphaStar RL loss: V-trace policy gradient per baseline, UPGO, TD(lambda) critic,
entropy, teacher KL (+ extra action-type KL), optional DAPO.

Semantics follow ``distar/agent/default/rl_training/rl_loss.py:33-178`` and ``as_rl_utils.py:1-127``.
Differences by design (not in the math):

* every head's logp(action), entropy and teacher KL come from ONE fused per-row kernel
  (``ops.head_stats``, csrc/kernels/loss.hip) with a one-pass backward, instead of log-softmax / exp /
  gather / product / sum chains over the [T, B, C] logits of both the learner and the teacher;
* the six heads' V-trace (and UPGO) scans run as one batched reverse scan;
* nothing calls ``.item()`` — the info dict holds 0-d device tensors that the logger fetches with a
  single device->host copy (the reference syncs ~40 times per iteration).
"""
from __future__ import annotations

import math
import os
from typing import Dict

import torch
import torch.nn.functional as F

from .. import ops
from ..utils.config import AttrDict, deep_merge_dicts
from . import rl_utils

HEADS = ['action_type', 'delay', 'queued', 'selected_units', 'target_unit', 'target_location']
FUSED_LOSS = os.environ.get('APPLESTAR_FUSED_LOSS', '1') == '1'

DEFAULT_RL_LOSS_CONFIG = AttrDict({
    'loss_weights': {
        'baseline': {'winloss': 10.0, 'build_order': 0.0, 'built_unit': 0.0, 'effect': 0.0, 'upgrade': 0.0, 'battle': 0.0},
        'pg': {'winloss': 1.0, 'build_order': 0.0, 'built_unit': 0.0, 'effect': 0.0, 'upgrade': 0.0, 'battle': 0.0},
        'upgo': {'winloss': 1.0},
        'kl': 0.02, 'action_type_kl': 0.1, 'entropy': 0.0001, 'dapo': 0.0,
    },
    'pg_head_weights': {h: 1.0 for h in HEADS} | {'selected_units': 0.01},
    'upgo_head_weights': {h: 1.0 for h in HEADS} | {'selected_units': 0.01},
    'entropy_head_weights': {h: 1.0 for h in HEADS} | {'selected_units': 0.01},
    'kl_head_weights': {h: 1.0 for h in HEADS} | {'selected_units': 0.01},
    'dapo_head_weights': {h: 1.0 for h in HEADS},
    'kl': {'action_type_kl_steps': 2400},
    'dapo': {'dapo_steps': 2400},
    'use_dapo': False,
    'gammas': {'baseline': {'winloss': 1.0, 'build_order': 1.0, 'built_unit': 1.0, 'effect': 1.0, 'upgrade': 1.0,
                            'battle': 0.997},
               'pg': {'winloss': 1.0, 'build_order': 1.0, 'built_unit': 1.0, 'effect': 1.0, 'upgrade': 1.0,
                      'battle': 0.997}},
})


class ReinforcementLoss:
    def __init__(self, learner_cfg: dict | None = None, player_id: str = 'MP0'):
        self.cfg = deep_merge_dicts(DEFAULT_RL_LOSS_CONFIG, learner_cfg or {})
        self.only_update_value = False
        self.use_dapo = bool(self.cfg.use_dapo) and 'MP' in player_id
        self._refresh()

    def _refresh(self):
        c = self.cfg
        self.w = c.loss_weights
        self.gammas = c.gammas
        self.action_type_kl_steps = c.kl.action_type_kl_steps
        self.dapo_steps = c.dapo.dapo_steps
        # device copies of the weights / gammas are derived from the config: drop them with it
        self.__dict__.pop('_sc_cache', None)
        self.__dict__.pop('_hw_cache', None)

    def reset(self, learner_cfg):
        self.cfg = deep_merge_dicts(self.cfg, learner_cfg)
        self.only_update_value = False
        self._refresh()

    def _head_weights(self, kind: str, device) -> torch.Tensor:
        """Per-head pg / upgo weights as a cached device tensor (building it per call is an H2D copy
        from pageable memory, i.e. a host sync in the middle of the step)."""
        cache = self.__dict__.setdefault('_hw_cache', {})
        key = (kind, str(device))
        if key not in cache:
            w = self.cfg.pg_head_weights if kind == 'pg' else self.cfg.upgo_head_weights
            cache[key] = torch.tensor([w.get(h, 1.0) for h in HEADS], device=device)
        return cache[key]

    # ------------------------------------------------------------------ fused GPU tail (rl_loss.hip)
    _PG_MASKED_FIELDS = ('build_order', 'built_unit', 'effect')

    def _fused_ok(self, inputs: Dict) -> bool:
        if not FUSED_LOSS:
            return False
        v0 = next(iter(inputs['value'].values()))
        if not v0.is_cuda or (self.use_dapo and 'successive_logit' in inputs):
            return False
        n = ops._native(v0)
        if n is None or not n.has('rl_loss'):
            return False
        T, B = inputs['reward']['winloss'].shape if 'winloss' in inputs['reward'] else (0, 0)
        return 0 < T * B <= 2048 and 1 <= len(inputs['value']) <= 6

    def _scalars(self, fields, device) -> torch.Tensor:
        cache = self.__dict__.setdefault('_sc_cache', {})
        key = (tuple(fields), str(device))
        if key not in cache:
            c = self.cfg
            vals = []
            for f in fields:
                vals += [self.w.pg.get(f, 0.0), self.w.baseline.get(f, 0.0), float(self.gammas.pg.get(f, 1.0)),
                         float(self.gammas.baseline.get(f, 1.0))]
            for table in (c.pg_head_weights, c.upgo_head_weights, c.entropy_head_weights, c.kl_head_weights):
                vals += [table.get(h, 1.0) for h in HEADS]
            vals += [self.w.upgo.winloss, self.w.entropy, self.w.kl, self.w.action_type_kl]
            cache[key] = torch.tensor(vals, dtype=torch.float32, device=device)
        return cache[key]

    def _compute_loss_fused(self, inputs: Dict) -> Dict[str, torch.Tensor]:
        """Same loss and info as the torch path below: the per-head statistics and their [T, B] reductions
        here, everything after them (scans, means, gradients) in one native kernel (ops.native.rl_loss_tail)."""
        logits = inputs['target_logit']
        values = inputs['value']
        behaviour_logp = inputs['action_log_prob']
        teacher_logits = inputs['teacher_logit']
        masks = inputs['mask']
        actions = inputs['action']
        rewards = inputs['reward']
        am = masks['actions_mask']
        su_mask = masks['selected_units_mask'].float()
        fields = list(values.keys())
        V = torch.stack([values[k].float() for k in fields], 0)                     # [F, T+1, B]
        not_done = (rewards['winloss'][-1] == 0).to(V.dtype)
        V = torch.cat([V[:, :-1], V[:, -1:] * not_done], 1)
        alps, blps, ents, kls = [], [], [], []
        for h in HEADS:
            alp, ent, kl = ops.head_stats(logits[h], teacher_logits.get(h), actions[h])
            blp = behaviour_logp[h].float()
            if h == 'selected_units':
                n_valid = masks['selected_units_logits_mask'].float().sum(-1)
                alp = (alp * su_mask).sum(-1)
                blp = (blp * su_mask).sum(-1)
                ent = (ent / (1e-9 + torch.log(n_valid + 1).unsqueeze(-1)) * su_mask).sum(-1) / (su_mask.sum(-1) + 1e-9)
                kl = (kl * su_mask).sum(-1)
            elif h == 'target_unit':
                ent = ent / (1e-9 + torch.log(masks['target_units_logits_mask'].float().sum(-1) + 1))
            else:
                ent = ent / math.log(logits[h].shape[-1])
            alps.append(alp)
            blps.append(blp)
            ents.append(ent)
            kls.append(kl)
        ones = torch.ones_like(alps[0])
        hm = torch.stack([ones, ones] + [am[h].float() for h in ['queued', 'selected_units', 'target_unit',
                                                                  'target_location']], 0)
        R = torch.stack([rewards[k].float() for k in fields], 0)
        WM = torch.stack([masks[k + '_mask'].float() if k in self._PG_MASKED_FIELDS else ones for k in fields], 0)
        atflag = (inputs['step'] < self.action_type_kl_steps).float() * masks['cum_action_mask'].float()
        upgo_f = fields.index('winloss') if 'winloss' in fields else -1
        total, vec = ops.rl_loss_tail(torch.stack(alps, 0), torch.stack(ents, 0), torch.stack(kls, 0), V,
                                      torch.stack(blps, 0).detach(), hm, R, WM, atflag,
                                      self._scalars(fields, V.device), upgo_f, self.only_update_value)
        info: Dict[str, torch.Tensor] = {}
        o = 0
        for f in fields:
            info[f'{f}/total'] = vec[o]
            for i, h in enumerate(HEADS):
                info[f'{f}/{h}'] = vec[o + 1 + i]
            info[f + '/td'], info[f + '/reward'], info[f + '/value'] = vec[o + 7], vec[o + 8], vec[o + 9]
            o += 10
        if 'battle' in rewards:
            info['battle/reward'] = rewards['battle'].float().mean()
        for name in ('upgo', 'entropy', 'kl'):
            for i, h in enumerate(HEADS):
                info[f'{name}/{h}'] = vec[o + i]
            info[f'{name}/total'] = vec[o + 6]
            o += 7
        info['kl/extra_at'] = vec[o]
        info['total_loss'] = total
        return info

    def compute_loss(self, inputs: Dict) -> Dict[str, torch.Tensor]:
        if self._fused_ok(inputs):
            return self._compute_loss_fused(inputs)
        logits = inputs['target_logit']
        values = dict(inputs['value'])
        behaviour_logp = inputs['action_log_prob']
        teacher_logits = inputs['teacher_logit']
        masks = inputs['mask']
        actions = inputs['action']
        rewards = inputs['reward']
        game_steps = inputs['step']
        am = masks['actions_mask']
        su_mask = masks['selected_units_mask'].float()                   # [T,B,64]

        # the winloss bootstrap value is zeroed when the episode ended inside this slice (rl_loss.py:47-49)
        not_done = (rewards['winloss'][-1] == 0).to(values['winloss'].dtype)
        for k in values:
            values[k] = torch.cat([values[k][:-1], values[k][-1:] * not_done], 0).float()

        info: Dict[str, torch.Tensor] = {}
        tgt_logp, rhos, ent_raw, kl_raw = {}, {}, {}, {}
        for h in HEADS:
            alp, ent_raw[h], kl_raw[h] = ops.head_stats(logits[h], teacher_logits.get(h), actions[h])
            with torch.no_grad():
                log_rho = alp - behaviour_logp[h].float()
                if h == 'selected_units':
                    log_rho = (log_rho * su_mask).sum(-1)
                rhos[h] = torch.exp(log_rho).clamp(max=1.0)
            if h == 'selected_units':
                alp = (alp * su_mask).sum(-1)
            tgt_logp[h] = alp
        rho_stack = torch.stack([rhos[h] for h in HEADS], 0)           # [6,T,B]
        logp_stack = torch.stack([tgt_logp[h] for h in HEADS], 0)      # [6,T,B]
        head_mask = torch.stack([torch.ones_like(rhos['action_type']), torch.ones_like(rhos['action_type'])] +
                                [am[h].float() for h in ['queued', 'selected_units', 'target_unit',
                                                         'target_location']], 0)

        # ---------------- V-trace policy gradient, one batched scan per baseline field
        total_pg = 0.0
        pg_w = self._head_weights('pg', rho_stack.device)
        for field, v in values.items():
            wf = self.w.pg.get(field, 0.0)
            with torch.no_grad():
                adv = rl_utils.vtrace_advantages(rho_stack, rho_stack, rewards[field].float(), v.detach(),
                                                 gamma=float(self.gammas.pg.get(field, 1.0)), lambda_=1.0)
            pg = -adv * logp_stack * head_mask
            if field in ('build_order', 'built_unit', 'effect'):
                pg = pg * masks[field + '_mask'].float()
            per_head = pg.mean(dim=(1, 2))
            field_total = (per_head * pg_w).sum()
            total_pg = total_pg + wf * field_total
            info[f'{field}/total'] = field_total.detach()
            for i, h in enumerate(HEADS):
                info[f'{field}/{h}'] = per_head[i].detach()

        # ---------------- UPGO on winloss
        v = values['winloss']
        r = rewards['winloss'].float()
        with torch.no_grad():
            upgo_adv = rho_stack * (rl_utils.upgo_returns(r, v.detach()) - v.detach()[:-1])
        upgo = (-upgo_adv * logp_stack * head_mask).mean(dim=(1, 2))
        upgo_w = self._head_weights('upgo', upgo.device)
        total_upgo = (upgo * upgo_w).sum() * self.w.upgo.winloss
        for i, h in enumerate(HEADS):
            info['upgo/' + h] = upgo[i].detach()
        info['upgo/total'] = total_upgo.detach() / max(self.w.upgo.winloss, 1e-12)

        # ---------------- TD(lambda) critic
        total_critic = 0.0
        for field, vf in values.items():
            wmask = masks[field + '_mask'].float() if field in ('build_order', 'built_unit', 'effect') else None
            c = rl_utils.td_lambda_loss(vf, rewards[field].float(), gamma=float(self.gammas.baseline.get(field, 1.0)),
                                        lambda_=0.8, weight=wmask)
            total_critic = total_critic + self.w.baseline.get(field, 0.0) * c
            info[field + '/td'] = c.detach()
            info[field + '/reward'] = rewards[field].float().mean()
            info[field + '/value'] = vf.detach().mean()
        if 'battle' in rewards:
            info['battle/reward'] = rewards['battle'].float().mean()

        # ---------------- entropy (normalised per head)
        total_ent = 0.0
        for h in HEADS:
            ent = ent_raw[h]
            if h == 'selected_units':
                n_valid = masks['selected_units_logits_mask'].float().sum(-1)
                ent = ent / (1e-9 + torch.log(n_valid + 1).unsqueeze(-1))
                ent = (ent * su_mask).sum(-1) / (su_mask.sum(-1) + 1e-9)
            elif h == 'target_unit':
                n_valid = masks['target_units_logits_mask'].float().sum(-1)
                ent = ent / (1e-9 + torch.log(n_valid + 1))
            else:
                ent = ent / math.log(logits[h].shape[-1])
            if h not in ('action_type', 'delay'):
                ent = ent * am[h].float()
            e = ent.mean()
            info['entropy/' + h] = e.detach()
            total_ent = total_ent - e * self.cfg.entropy_head_weights.get(h, 1.0)
        info['entropy/total'] = total_ent.detach()
        total_ent = total_ent * self.w.entropy

        # ---------------- teacher KL
        total_kl = 0.0
        at_kl_loss = torch.zeros((), device=v.device)
        for h in ['action_type', 'queued', 'delay', 'selected_units', 'target_unit', 'target_location']:
            kl = kl_raw[h]
            if h == 'selected_units':
                kl = (kl * su_mask).sum(-1)
            if h not in ('action_type', 'delay'):
                kl = kl * am[h].float()
            if h == 'action_type':
                flag = (game_steps < self.action_type_kl_steps).float()
                at_kl_loss = (kl * flag * masks['cum_action_mask'].float()).mean()
                info['kl/extra_at'] = at_kl_loss.detach()
            k = kl.mean()
            info['kl/' + h] = k.detach()
            total_kl = total_kl + k * self.cfg.kl_head_weights.get(h, 1.0)
        info['kl/total'] = total_kl.detach()
        total_kl = total_kl * self.w.kl
        at_kl_loss = at_kl_loss * self.w.action_type_kl

        # ---------------- DAPO (distillation from a successive model), only for main players
        total_dapo = 0.0
        if self.use_dapo and 'successive_logit' in inputs:
            flag = (game_steps < self.dapo_steps).float()
            for h in HEADS:
                _, _, kl = ops.head_stats(logits[h], inputs['successive_logit'][h], actions[h])
                if h == 'selected_units':
                    kl = (kl * su_mask).sum(-1)
                if h not in ('action_type', 'delay'):
                    kl = kl * am[h].float()
                d = (kl * flag).mean()
                info['dapo/' + h] = d.detach()
                total_dapo = total_dapo + d * self.cfg.dapo_head_weights.get(h, 1.0)
            total_dapo = total_dapo * self.w.dapo

        if self.only_update_value:
            total = total_critic
        else:
            total = total_pg + total_upgo + total_critic + total_ent + total_kl + at_kl_loss + total_dapo
        info['total_loss'] = total
        return info
