"""Supervised (behaviour-cloning) loss over the six action heads.

Semantics of ``distar/agent/default/sl_training/sl_loss.py:37-286``: per-head cross entropy (or
label smoothing) masked by the action's argument mask and normalised by the number of valid
samples; weights action_type 30, delay 9, queued 1, selected_units 4, target_unit 4,
target_location 8; metrics accuracy / delay L1 / selected-units IoU / location L2.  The ``su_mask``
option masks, at every pointer step, the other *labelled* units except the current one.
Sync-free: ``valid > 0`` branches become clamped divisions, metrics stay on device.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from ..ops.reference import sequence_mask
from ..utils.config import AttrDict, deep_merge_dicts

DEFAULT_SL_LOSS_CONFIG = AttrDict({'loss_weight': {'action_type': 30.0, 'delay': 9.0, 'queued': 1.0,
                                                   'selected_units': 4.0, 'target_unit': 4.0, 'target_location': 8.0},
                                   'su_mask': True, 'label_smooth': False, 'cross_rank_loss': False})


def _ce(logits, labels, smoothing: float = 0.0):
    logp = torch.log_softmax(logits.float(), dim=-1)
    nll = -logp.gather(-1, labels.long().unsqueeze(-1)).squeeze(-1)
    if smoothing > 0:
        return (1 - smoothing) * nll + smoothing * (-logp.mean(-1))
    return nll


def _masked_mean(loss, mask):
    m = mask.float()
    return (loss * m).sum() / m.sum().clamp(min=1.0)


class SupervisedLoss:
    HEADS = ['action_type', 'delay', 'queued', 'selected_units', 'target_unit', 'target_location']

    def __init__(self, learner_cfg: dict | None = None):
        self.cfg = deep_merge_dicts(DEFAULT_SL_LOSS_CONFIG, learner_cfg or {})
        self.w = self.cfg.loss_weight
        self.smooth = 0.1 if self.cfg.get('label_smooth', False) else 0.0
        self.su_mask = bool(self.cfg.su_mask)

    def compute_loss(self, logits: Dict, actions: Dict, actions_mask: Dict, selected_units_num, entity_num,
                     infer_action_info: Dict | None = None) -> Dict[str, torch.Tensor]:
        out = {}
        # action type
        lt = logits['action_type']
        lab = actions['action_type'].long()
        m = actions_mask['action_type']
        out['action_type_loss'] = _masked_mean(_ce(lt, lab, self.smooth), m)
        with torch.no_grad():
            out['action_type_acc'] = (lt.argmax(-1) == lab).float().mean()
        # delay
        ld = logits['delay']
        lab = actions['delay'].long()
        m = actions_mask['delay']
        out['delay_loss'] = _masked_mean(_ce(ld, lab, self.smooth), m)
        with torch.no_grad():
            out['delay_distance_L1'] = ((ld.argmax(-1) - lab).abs().float() * m).sum() / (m.float().sum() + 1e-6)
        # queued
        lq = logits['queued']
        lab = actions['queued'].long()
        m = actions_mask['queued']
        out['queued_loss'] = _masked_mean(_ce(lq, lab, self.smooth), m)
        with torch.no_grad():
            out['queued_acc'] = ((lq.argmax(-1) - lab).abs().float() * m).sum() / (m.float().sum() + 1e-6)
        # selected units
        out.update(self._selected_units(logits['selected_units'], actions['selected_units'].long(),
                                        actions_mask['selected_units'], selected_units_num.long(), entity_num.long(),
                                        None if infer_action_info is None else infer_action_info['selected_units']))
        # target unit
        lu = logits['target_unit']
        lab = actions['target_unit'].long()
        m = actions_mask['target_unit']
        out['target_unit_loss'] = _masked_mean(_ce(lu, lab, self.smooth), m)
        with torch.no_grad():
            out['target_unit_acc'] = ((lu.argmax(-1) == lab).float() * m).sum() / (m.float().sum() + 1e-6)
        # target location
        ll = logits['target_location']
        lab = actions['target_location'].long()
        m = actions_mask['target_location']
        out['target_location_loss'] = _masked_mean(_ce(ll, lab, self.smooth), m)
        with torch.no_grad():
            p = ll.argmax(-1)
            d = torch.stack([(p % 160 - lab % 160), (p // 160 - lab // 160)], -1).float()
            out['target_location_distance_L2'] = (d.pow(2).sum(-1).sqrt() * m).sum() / (m.float().sum() + 1e-6)
        total = 0.0
        for h in self.HEADS:
            total = total + out[h + '_loss'] * self.w[h]
        out['total_loss'] = total
        return out

    def _selected_units(self, logits, labels, mask, lengths, entity_num, selected_units):
        b, s, n = logits.shape
        labels = labels[:, :s]
        if self.su_mask:
            # at each step forbid the *other* labelled units (not the current label)
            no_end = sequence_mask((lengths - 1).clamp(min=0), s)
            lab = torch.where(no_end, labels, torch.full_like(labels, n))
            oh = F.one_hot(lab, n + 1).any(1)                              # [b, n+1] labelled units
            forbid = oh.unsqueeze(1).expand(b, s, n + 1).clone()
            forbid.scatter_(2, lab.unsqueeze(2), False)                    # except this step's own label
            logits = logits.masked_fill(forbid[:, :, :n], -1e9)
        select_mask = sequence_mask(lengths, s)
        loss = _ce(logits.reshape(-1, n), labels.reshape(-1)).view(b, s)
        loss = loss.masked_fill(~select_mask, 0) * mask.float().unsqueeze(1)
        out = {'selected_units_loss': loss.sum() / b,
               'selected_units_loss_norm': loss.sum() / (lengths.sum().float() + 1e-6),
               'selected_units_end_flag_loss': loss[torch.arange(b, device=loss.device),
                                                    (lengths - 1).clamp(min=0)].mean()}
        with torch.no_grad():
            if selected_units is not None:
                preds = selected_units[:, :s].long()
                is_end = preds == entity_num.unsqueeze(1)
                first_end = torch.where(is_end.any(1), is_end.float().argmax(1) + 1, torch.full_like(lengths, s + 1))
                pm = sequence_mask(first_end.clamp(max=s), s)
                P = torch.zeros(b, n + 1, dtype=torch.bool, device=logits.device)
                L = torch.zeros_like(P)
                P.scatter_(1, ((preds + 1) * pm).clamp(max=n), True)
                L.scatter_(1, ((labels + 1) * select_mask).clamp(max=n), True)
                inter = (P & L)[:, 1:].sum(1).float()
                union = (P | L)[:, 1:].sum(1).float()
                out['selected_units_iou'] = (inter / (union + 1e-6) * mask).sum() / (mask.float().sum() + 1e-6)
            else:
                out['selected_units_iou'] = torch.zeros((), device=logits.device)
        return out
