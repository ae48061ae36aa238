"""Pseudo-reward distances (``distar/ctools/torch_utils/metric.py:4-89``).

``levenshtein_distance`` keeps the reference's DP exactly, including its quirk that a matching pair
with an ``extra_fn`` costs ``dp[i-1][j-1] + extra`` without competing against insert/delete.  The
DP runs over plain Python ints/floats (build orders are <= 20 long), which is ~50x faster than the
reference's per-element tensor indexing.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Sequence

import torch


def _as_list(x) -> list:
    if isinstance(x, torch.Tensor):
        return x.reshape(-1).tolist()
    return list(x)


def l2_distance(a, b, min: float = 0.0, max: float = 0.8, threshold: float = 5.0, spatial_x: int = 160):
    """Clamped, scaled euclidean distance between two flat map locations (y*W + x)."""
    if isinstance(a, torch.Tensor) or isinstance(b, torch.Tensor):
        a = torch.as_tensor(a)
        b = torch.as_tensor(b)
        x0, y0, x1, y1 = a % spatial_x, a // spatial_x, b % spatial_x, b // spatial_x
        l2 = torch.sqrt((torch.square(x1 - x0) + torch.square(y1 - y0)).float())
        return (l2 / threshold).clamp_(min=min, max=max)
    a, b = int(a), int(b)
    d = math.hypot(b % spatial_x - a % spatial_x, b // spatial_x - a // spatial_x)
    return float(min if d / threshold < min else (max if d / threshold > max else d / threshold))


def levenshtein_distance(behaviour, target, behaviour_extra=None, target_extra=None,
                         extra_fn: Optional[Callable] = None) -> torch.Tensor:
    b, t = _as_list(behaviour), _as_list(target)
    be = _as_list(behaviour_extra) if behaviour_extra is not None else None
    te = _as_list(target_extra) if target_extra is not None else None
    n1, n2 = len(b), len(t)
    if n1 == 0 or n2 == 0:
        return torch.tensor(float(max(n1, n2)))
    prev = [float(j) for j in range(n2 + 1)]
    for i in range(1, n1 + 1):
        cur = [float(i)] + [0.0] * n2
        bi = b[i - 1]
        for j in range(1, n2 + 1):
            if bi == t[j - 1]:
                cur[j] = prev[j - 1] + (float(extra_fn(be[i - 1], te[j - 1])) if extra_fn else 0.0)
            else:
                cur[j] = 1.0 + min(prev[j], cur[j - 1], prev[j - 1])
        prev = cur
    return torch.tensor(prev[n2])


def hamming_distance(behaviour: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    assert behaviour.shape == target.shape and behaviour.dtype == target.dtype
    return behaviour.ne(target).sum(dim=-1).float()
