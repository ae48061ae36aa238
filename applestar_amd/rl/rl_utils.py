"""RL return / advantage estimators (V-trace, UPGO, TD(lambda)) as reverse scans over time.

Formulas follow ``distar/agent/default/rl_training/as_rl_utils.py:157-312``.  The reference loops
in Python over T issuing a handful of tiny kernels per step; here the scans are batched over all
heads and baselines at once ([K, T, B] tensors) and, on GPU, run as a single HIP kernel
(``ops.native.reverse_scan``) where one lane owns one (k, b) column.
"""
from __future__ import annotations

import torch

from .. import ops


def reverse_linear_scan(a: torch.Tensor, b: torch.Tensor, init: torch.Tensor) -> torch.Tensor:
    """y[t] = a[t] * y[t+1] + b[t] for t = T-1..0 with y[T] = init.  a,b [..., T, B]; init [..., B].
    Returns y[0..T-1]."""
    n = ops._native(a) if a.is_cuda else None
    if n is not None and n.has('reverse_scan'):
        return n.reverse_scan(a, b, init)
    T = a.shape[-2]
    out = torch.empty_like(b)
    y = init
    for t in range(T - 1, -1, -1):
        y = a[..., t, :] * y + b[..., t, :]
        out[..., t, :] = y
    return out


def vtrace_advantages(clipped_rhos, clipped_cs, rewards, values, gamma: float = 1.0, lambda_: float = 1.0):
    """clipped_rhos/cs [..., T, B], rewards [T, B] (broadcast), values [T+1, B] -> advantages [..., T, B].

    vs[t] - V[t] = delta[t] + gamma*lambda*c[t]*(vs[t+1] - V[t+1]),  delta = rho (r + gamma V' - V)."""
    deltas = clipped_rhos * (rewards + gamma * values[1:] - values[:-1])
    acc = reverse_linear_scan(gamma * lambda_ * clipped_cs, deltas,
                              torch.zeros_like(deltas[..., 0, :]))           # vs - V for t < T
    vs_next = torch.cat([acc[..., 1:, :] + values[1:-1], values[-1:].expand_as(acc[..., -1:, :])], dim=-2)
    return clipped_rhos * (rewards + gamma * vs_next - values[:-1])


def lambda_returns(rewards, values, gamma, lambdas):
    """G[t] = r[t] + gamma*lam[t]*G[t+1] + gamma*(1-lam[t])*V[t+1];  G[T-1] = r[T-1] + gamma V[T]."""
    if not torch.is_tensor(lambdas):
        lambdas = torch.full_like(rewards, float(lambdas))
    lam = lambdas.clone()
    lam[..., -1, :] = 0.0  # last lambda is ignored (forced bootstrap)
    a = gamma * lam
    b = rewards + gamma * (1 - lam) * values[1:]
    return reverse_linear_scan(a, b, torch.zeros_like(rewards[..., 0, :]))


def upgo_returns(rewards, values):
    lam = ((rewards + values[1:]) >= values[:-1]).to(rewards.dtype)
    lam = torch.cat([lam[1:], torch.ones_like(lam[-1:])], 0)
    return lambda_returns(rewards, values, 1.0, lam)


def td_lambda_loss(values, rewards, gamma: float = 1.0, lambda_: float = 0.8, weight=None):
    with torch.no_grad():
        returns = lambda_returns(rewards, values.detach(), gamma, lambda_)
    loss = 0.5 * (returns - values[:-1]) ** 2
    if weight is not None:
        loss = loss * weight
    return loss.mean()
