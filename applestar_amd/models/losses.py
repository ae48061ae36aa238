"""Reusable classification losses (``distar/ctools/torch_utils/loss/*.py``).

* :class:`LabelSmoothCELoss` -- CE against (1 - r) on the label and r/(N-1) elsewhere, mean over rows;
* :class:`SoftFocalLoss` -- NLL of (1 - p)^gamma * log p;
* :func:`build_ce_criterion` -- {cross_entropy, label_smooth_ce, soft_focal_loss} from a config;
* :class:`MultiLogitsLoss` -- order-free CE for M predictions vs M labels: the assignment minimising the
  total loss is found with the Hungarian algorithm (scipy's ``linear_sum_assignment``; the reference
  runs a Python Kuhn-Munkres with recursion), then the matched losses are averaged.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _smooth_targets(logits: torch.Tensor, labels: torch.Tensor, ratio: float) -> torch.Tensor:
    n = logits.shape[1]
    val = float(ratio) / (n - 1)
    t = torch.full_like(logits, val, dtype=torch.float32)
    t.scatter_(1, labels.long().unsqueeze(1), 1.0 - val)
    return t


class LabelSmoothCELoss(nn.Module):
    def __init__(self, ratio: float):
        super().__init__()
        self.ratio = ratio

    def forward(self, logits, labels):
        t = _smooth_targets(logits, labels, self.ratio)
        return -(F.log_softmax(logits.float(), 1) * t).sum() / logits.shape[0]


class SoftFocalLoss(nn.Module):
    def __init__(self, gamma: float = 2.0, weight=None, reduction: str = 'mean'):
        super().__init__()
        self.gamma = gamma
        self.weight = weight
        self.reduction = reduction

    def forward(self, inputs, targets):
        logp = F.log_softmax(inputs.float(), 1)
        return F.nll_loss((1 - logp.exp()) ** self.gamma * logp, targets.long(), weight=self.weight,
                          reduction=self.reduction)


def build_ce_criterion(cfg) -> nn.Module:
    typ = cfg['type']
    if typ == 'cross_entropy':
        return nn.CrossEntropyLoss()
    if typ == 'label_smooth_ce':
        return LabelSmoothCELoss(cfg['kwargs']['smooth_ratio'])
    if typ == 'soft_focal_loss':
        return SoftFocalLoss()
    raise ValueError(f'invalid criterion type: {typ}')


class MultiLogitsLoss(nn.Module):
    def __init__(self, criterion: str = 'cross_entropy', smooth_ratio: float = 0.1):
        super().__init__()
        assert criterion in ('cross_entropy', 'label_smooth_ce'), criterion
        self.criterion = criterion
        self.ratio = smooth_ratio

    def metric_matrix(self, logits, labels) -> torch.Tensor:
        """[M(pred), M(label)] matrix of per-pair losses."""
        if self.criterion == 'cross_entropy':
            t = F.one_hot(labels.long(), logits.shape[1]).float()
        else:
            t = _smooth_targets(logits, labels, self.ratio)
        return -(F.log_softmax(logits.float(), 1) @ t.t())

    def forward(self, logits, labels):
        from scipy.optimize import linear_sum_assignment
        assert logits.dim() == 2
        m = self.metric_matrix(logits, labels)
        rows, cols = linear_sum_assignment(m.detach().cpu().numpy())
        r = torch.as_tensor(rows, device=m.device)
        c = torch.as_tensor(cols, device=m.device)
        return m[r, c].mean()
