"""Batching of agent observations / model outputs and of actor trajectories for the learner.

* ``collate_obs`` / ``decollate_output``: the actor-side batch of single-step observations (varlen
  entity tensors padded to the batch max) and the per-env slice of a batched model output, trimmed to
  the env's own ``entity_num`` / ``selected_units_num`` (``agent.py:389-411``).
* ``collate_trajectories``: learner batch from B trajectories of T+1 steps, following
  ``rl_dataloader.collate_fn`` / ``padding_entity_info`` (``rl_dataloader.py:45-76,206-245``):
  entities padded to the max N; SU labels padded to 64; behaviour SU logp padded with -1e9; teacher
  SU / target-unit logits padded with -1e9; SU / logits masks; observations flattened time-major to
  (T+1)*B (index t*B + b); everything else stacked [T, B, ...].  Only step 0's LSTM state is kept
  (the learner unrolls from it), which trims the host->device copy by (T+1)x for that field.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

from ..lib.features import MAX_SELECTED_UNITS_NUM

NEG = -1e9
OBS_KEYS = ('spatial_info', 'entity_info', 'scalar_info', 'entity_num', 'value_feature')


def _stack(xs: Sequence, dim: int = 0):
    x0 = xs[0]
    if isinstance(x0, torch.Tensor):
        return torch.stack(list(xs), dim)
    if isinstance(x0, dict):
        return {k: _stack([x[k] for x in xs], dim) for k in x0}
    if isinstance(x0, (list, tuple)):
        return [_stack([x[i] for x in xs], dim) for i in range(len(x0))]
    if isinstance(x0, (int, float, bool)):
        return torch.tensor(list(xs))
    return list(xs)


def _pad_last(t: torch.Tensor, n: int, value=0) -> torch.Tensor:
    d = n - t.shape[-1]
    return F.pad(t, (0, d), value=value) if d > 0 else t


def collate_obs(obs_list: List[Dict], pad_entities: int = 0) -> Dict:
    """List of single-step agent inputs -> batch (entities padded to the max entity_num, or to
    ``pad_entities`` for a fixed shape, e.g. HIP-graph replay)."""
    n = max(int(o['entity_num']) for o in obs_list)
    n = max(n, max(o['entity_info']['unit_type'].shape[-1] for o in obs_list), pad_entities)
    out = {}
    for k in obs_list[0]:
        vals = [o[k] for o in obs_list]
        if k == 'entity_info':
            out[k] = {f: torch.stack([_pad_last(v[f], n) for v in vals]) for f in vals[0]}
        elif k == 'hidden_state':
            out[k] = [(torch.stack([v[l][0] for v in vals]), torch.stack([v[l][1] for v in vals]))
                      for l in range(len(vals[0]))]
        elif k == 'action_info':
            out[k] = {f: torch.stack([_pad_last(v[f], MAX_SELECTED_UNITS_NUM) if f == 'selected_units' else v[f]
                                      for v in vals]) for f in vals[0]}
        else:
            out[k] = _stack(vals)
    return out


def decollate_output(out: Dict, i: int) -> Dict:
    """Row ``i`` of a batched model output, on the host, trimmed to that sample's sizes."""
    def take(x):
        if isinstance(x, torch.Tensor):
            return x[i].detach().cpu() if x.dim() > 0 else x.detach().cpu()
        if isinstance(x, dict):
            return {k: take(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return [take(v) for v in x]
        return x
    res = {}
    for k, v in out.items():
        if k == 'hidden_state':
            res[k] = [(h[i].detach().cpu(), c[i].detach().cpu()) for h, c in v]
        elif v is None:
            res[k] = None
        else:
            res[k] = take(v)
    n = int(res['entity_num'])
    s = int(res['selected_units_num'])
    lg = res.get('logit')
    if lg is not None:
        if 'selected_units' in lg:
            lg['selected_units'] = lg['selected_units'][:s, :n + 1]
        if 'target_unit' in lg:
            lg['target_unit'] = lg['target_unit'][:n]
    if 'action_info' in res and 'selected_units' in res['action_info']:
        res['action_info']['selected_units'] = res['action_info']['selected_units'][:s]
    if 'action_logp' in res and 'selected_units' in res['action_logp']:
        res['action_logp']['selected_units'] = res['action_logp']['selected_units'][:s]
    if res.get('extra_units') is not None:
        res['extra_units'] = res['extra_units'][:n]
    return res


def _pad_step(step: Dict, n: int) -> Dict:
    """padding_entity_info for one trajectory step (returns a new dict)."""
    s = {k: v for k, v in step.items() if k != 'map_name'}
    s['entity_info'] = {k: _pad_last(v, n) for k, v in step['entity_info'].items()}
    if 'action_info' in step:
        su_num = step['selected_units_num']
        en = int(step['entity_num'])
        s['action_info'] = dict(step['action_info'])
        s['action_info']['selected_units'] = _pad_last(step['action_info']['selected_units'], MAX_SELECTED_UNITS_NUM)
        s['behaviour_logp'] = dict(step['behaviour_logp'])
        s['behaviour_logp']['selected_units'] = _pad_last(step['behaviour_logp']['selected_units'],
                                                          MAX_SELECTED_UNITS_NUM, NEG)
        tl = dict(step['teacher_logit'])
        su = tl['selected_units']
        su = su.reshape(-1, su.shape[-1]) if su.numel() else su.new_zeros(0, en + 1)
        tl['selected_units'] = F.pad(su, (0, n + 1 - su.shape[-1], 0, MAX_SELECTED_UNITS_NUM - su.shape[0]),
                                     value=NEG)
        tl['target_unit'] = _pad_last(tl['target_unit'], n, NEG)
        s['teacher_logit'] = tl
        m = dict(step['mask'])
        ar = torch.arange(MAX_SELECTED_UNITS_NUM)
        m['selected_units_mask'] = ar < int(su_num)
        m['selected_units_logits_mask'] = torch.arange(n + 1) < en + 1
        m['target_units_logits_mask'] = torch.arange(n) < en
        s['mask'] = m
    return s


def collate_trajectories(trajs: List[List[Dict]]) -> Dict:
    """B trajectories of T action steps + 1 bootstrap observation -> learner batch."""
    B = len(trajs)
    T = len(trajs[0]) - 1
    n = max(st['entity_info']['unit_type'].shape[-1] for tr in trajs for st in tr)
    padded = [[_pad_step(st, n) for st in tr] for tr in trajs]
    batch: Dict = {}
    # observations: time-major flatten (T+1)*B
    for k in OBS_KEYS:
        if k not in padded[0][0]:
            continue
        per_t = [_stack([padded[b][t][k] for b in range(B)]) for t in range(T + 1)]
        batch[k] = _flatten_time(_stack(per_t))
    batch['hidden_state'] = [(torch.stack([tr[0]['hidden_state'][l][0] for tr in trajs]),
                              torch.stack([tr[0]['hidden_state'][l][1] for tr in trajs]))
                             for l in range(len(trajs[0][0]['hidden_state']))]
    act_keys = [k for k in padded[0][0] if k not in OBS_KEYS and k not in ('hidden_state', 'map_name')]
    for k in act_keys:
        per_t = [_stack([padded[b][t][k] for b in range(B)]) for t in range(T)]
        batch[k] = _stack(per_t)
    batch['batch_size'] = B
    batch['unroll_len'] = T
    return batch


def _flatten_time(x):
    if isinstance(x, torch.Tensor):
        return x.flatten(0, 1)
    if isinstance(x, dict):
        return {k: _flatten_time(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_flatten_time(v) for v in x]
    return x
