"""Autoregressive action heads: action_type -> delay -> queued -> selected_units -> target_unit ->
target_location (``distar/agent/default/model/head/*.py``, ``policy.py:22-73``).

Two execution modes per head:

* **sampling** (actor inference): draw the action from ``softmax(logits / T)``.  Sampling uses an
  explicit uniform ``u`` (inverse CDF), so given the same noise the native and reference paths pick
  bit-identical actions.
* **teacher-forced** (learner / teacher / SL): the behaviour action is given.  The selected-units
  pointer network is *not* unrolled step by step here: because every step's autoregressive
  embedding depends only on the (known) labels, all 64 steps' inputs are formed in parallel
  (prefix sets of labelled keys), then one batched query MLP, one 32-d LN-LSTM scan and one batched
  logits GEMM.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..lib import game_data as gd
from ..lib.features import MAX_SELECTED_UNITS_NUM, SPATIAL_SIZE, MAX_ENTITY_NUM
from .blocks import FCBlock, ResFCBlock, GLU, GatedResBlock, ConvBlock, glorot_uniform_
from .lstm import StackedLNLSTM

NEG = -1e9


def sample_from_logits(logits: torch.Tensor, u: Optional[torch.Tensor] = None, generator=None) -> torch.Tensor:
    """Inverse-CDF categorical sample over the last dim (rows of ``logits`` are already scaled).
    ``u`` [rows] uniform in [0,1); drawn if not given."""
    p = torch.softmax(logits.float(), dim=-1)
    cdf = torch.cumsum(p, dim=-1)
    if u is None:
        u = torch.rand(p.shape[:-1], device=p.device, generator=generator)
    x = (u.to(cdf.dtype) * cdf[..., -1]).unsqueeze(-1)
    idx = torch.searchsorted(cdf, x, right=True).squeeze(-1)
    return idx.clamp(max=p.shape[-1] - 1)


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _embed_table(module, lin):
    """lin.weight^T [n_in, n_out] contiguous (the one-hot -> fc row table of a head's embedding fc), cached per
    weight version for the fused sampler.  While a HIP graph is being captured the transpose is recorded in
    the graph instead (a cached copy's address would be baked in and go stale after an in-place weight load)."""
    w = lin.weight
    if _capturing():
        return w.detach().t().contiguous()
    tag = (w.data_ptr(), w._version, w.dtype)
    cache = module.__dict__.setdefault('_table_cache', {})
    hit = cache.get(id(lin))
    if hit is None or hit[0] != tag:
        with torch.no_grad():
            hit = cache[id(lin)] = (tag, w.detach().t().contiguous())
    return hit[1]


class ActionTypeHead(nn.Module):
    def __init__(self, input_dim=384, res_dim=256, action_num=gd.NUM_ACTIONS, context_dim=448, gate_dim=1024,
                 action_map_dim=256):
        super().__init__()
        self.action_num = action_num
        self.project = FCBlock(input_dim, res_dim, act=True)
        self.res = nn.Sequential(ResFCBlock(res_dim), ResFCBlock(res_dim))
        self.action_fc = GLU(res_dim, action_num, context_dim)
        self.action_map_fc1 = FCBlock(action_num, action_map_dim, act=True)
        self.action_map_fc2 = FCBlock(action_map_dim, action_map_dim)
        self.glu1 = GLU(action_map_dim, gate_dim, context_dim)
        self.glu2 = GLU(input_dim, gate_dim, context_dim)

    def forward(self, lstm_output, scalar_context, temperature: float = 1.0, action_type=None,
                race_mask: Optional[torch.Tensor] = None, u=None):
        x = self.res(self.project(lstm_output))
        w1 = self.action_map_fc1[0]
        if action_type is None:
            # actor inference: scale, race mask, sample and the action-map row gather in one kernel (heads.hip)
            fused = ops.head_sample(self.action_fc(x, scalar_context), temperature, mask=race_mask, u=u,
                                    table=_embed_table(self, w1), bias=w1.bias)
            if fused is not None:
                logits, action_type, e1 = fused
                e1 = self.action_map_fc2(e1)
                embedding = self.glu1(e1, scalar_context) + self.glu2(lstm_output, scalar_context)
                return logits, action_type, embedding
        logits = self.action_fc(x, scalar_context) / temperature
        if race_mask is not None:
            logits = logits.masked_fill(~race_mask.to(logits.device).unsqueeze(0), NEG)
        if action_type is None:
            action_type = sample_from_logits(logits, u)
        # one-hot(a) @ W^T == column gather of action_map_fc1's weight (index_select: its backward is an
        # index_add of the 384 rows; advanced indexing's is a sort-based index_put, ~0.1 ms per table)
        w1 = self.action_map_fc1[0]
        e1 = F.relu(w1.weight.t().index_select(0, action_type.long().reshape(-1)).view(*action_type.shape, -1)
                    + w1.bias)
        e1 = self.action_map_fc2(e1)
        embedding = self.glu1(e1, scalar_context) + self.glu2(lstm_output, scalar_context)
        return logits, action_type, embedding

    # teacher-forced halves (Policy.train_forward): the logits do not feed the autoregressive embedding, so they can
    # run on a side stream while the embedding chain continues
    def teacher_logits(self, lstm_output, scalar_context, temperature: float = 1.0):
        return self.action_fc(self.res(self.project(lstm_output)), scalar_context) / temperature

    def teacher_embedding(self, lstm_output, scalar_context, action_type):
        w1 = self.action_map_fc1[0]
        e1 = F.relu(w1.weight.t().index_select(0, action_type.long().reshape(-1)).view(*action_type.shape, -1)
                    + w1.bias)
        return self.glu1(self.action_map_fc2(e1), scalar_context) + self.glu2(lstm_output, scalar_context)


class _ArgMLPHead(nn.Module):
    """Shared shape of DelayHead / QueuedHead (action_arg_head.py:27-86)."""

    def __init__(self, n_out: int, input_dim=1024, decode_dim=256, map_dim=256, use_temperature=True):
        super().__init__()
        self.n_out = n_out
        self.use_temperature = use_temperature
        self.fc1 = FCBlock(input_dim, decode_dim, act=True)
        self.fc2 = FCBlock(decode_dim, decode_dim, act=True)
        self.fc3 = FCBlock(decode_dim, n_out)
        self.embed_fc1 = FCBlock(n_out, map_dim, act=True)
        self.embed_fc2 = FCBlock(map_dim, input_dim)

    def forward(self, embedding, temperature: float = 1.0, action=None, u=None):
        logits = self.fc3(self.fc2(self.fc1(embedding)))
        w = self.embed_fc1[0]
        if action is None:
            fused = ops.head_sample(logits, temperature if self.use_temperature else 1.0, u=u,
                                    table=_embed_table(self, w), bias=w.bias)
            if fused is not None:     # actor inference: sample + row-gather embedding in one kernel (heads.hip)
                logits, action, e = fused
                return logits, action, embedding + self.embed_fc2(e)
        if self.use_temperature:
            logits = logits / temperature
        if action is None:
            action = sample_from_logits(logits, u)
        w = self.embed_fc1[0]
        e = F.relu(w.weight.t().index_select(0, action.long().reshape(-1)).view(*action.shape, -1) + w.bias)
        return logits, action, embedding + self.embed_fc2(e)

    def teacher_logits(self, embedding, temperature: float = 1.0):
        logits = self.fc3(self.fc2(self.fc1(embedding)))
        return logits / temperature if self.use_temperature else logits

    def teacher_embedding(self, embedding, action):
        w = self.embed_fc1[0]
        e = F.relu(w.weight.t().index_select(0, action.long().reshape(-1)).view(*action.shape, -1) + w.bias)
        return embedding + self.embed_fc2(e)


class DelayHead(_ArgMLPHead):
    def __init__(self):
        super().__init__(128, use_temperature=False)  # reference never divides delay logits by T


class QueuedHead(_ArgMLPHead):
    def __init__(self):
        super().__init__(2, use_temperature=True)


# teacher-forced split (Policy.train_forward): the earlier steps' embedding update goes with the pointer half (A/B)
SU_AE_SIDE = os.environ.get('APPLESTAR_SU_AE_SIDE', '1') == '1'
# ... and its queries over the earlier steps take query_fc1 folded into embed_fc2 (SelectedUnitsHead._query_in_folded)
SU_FOLD = os.environ.get('APPLESTAR_SU_FOLD', '1') == '1'


class SelectedUnitsHead(nn.Module):
    """Pointer network over entities + end token (action_arg_head.py:89-328)."""

    REDUCE_TYPES = ('selected_units_num', 'attention_pool', 'attention_pool_add_num')

    def __init__(self, input_dim=1024, entity_dim=256, key_dim=32, func_dim=256, hidden_dim=32, num_layers=1,
                 extra_units: bool = False, reduce_type: str = 'selected_units_num'):
        super().__init__()
        # 'entity_num' / 'constant' call an undefined embed_fc in the reference (action_arg_head.py:130-135)
        if reduce_type not in self.REDUCE_TYPES:
            raise NotImplementedError(f'selected-units entity_reduce_type {reduce_type!r}')
        self.reduce_type = reduce_type
        self.key_dim = key_dim
        self.key_fc = FCBlock(entity_dim, key_dim)
        self.query_fc1 = FCBlock(input_dim, func_dim, act=True)
        self.query_fc2 = FCBlock(func_dim, key_dim)
        self.embed_fc1 = FCBlock(key_dim, func_dim, act=True)
        self.embed_fc2 = FCBlock(func_dim, input_dim)
        self.lstm = StackedLNLSTM(key_dim, hidden_dim, num_layers)
        self.end_embedding = nn.Parameter(torch.empty(1, key_dim))
        glorot_uniform_(self.end_embedding)
        self.extra_units = extra_units
        if reduce_type != 'selected_units_num':
            from .optional import AttentionPool
            self.attention_pool = AttentionPool(key_dim, 2, input_dim, max_num=MAX_SELECTED_UNITS_NUM + 1
                                                if reduce_type == 'attention_pool_add_num' else None)

    def keys(self, entity_embedding, entity_num, key=None):
        """key [B,N+1,32] with the learned end embedding at position entity_num; logits mask.  ``key``: the
        key_fc output when the caller already projected the entities (Policy.train_forward)."""
        if key is None:
            key = self.key_fc(entity_embedding)
        B, N, _ = key.shape
        key = F.pad(key, (0, 0, 0, 1))
        ar = torch.arange(N + 1, device=key.device)
        is_end = (ar[None, :] == entity_num[:, None]).unsqueeze(2)
        key = torch.where(is_end, self.end_embedding.to(key.dtype).expand_as(key), key)
        mask = ar[None, :] < (entity_num + 1)[:, None]
        return key, mask

    def _ae_update(self, ae0, emb):
        return ae0 + self.embed_fc2(self.embed_fc1(emb))

    # ------------------------------------------------------------------ teacher forced (parallel)
    def forward_teacher(self, ae0, entity_embedding, entity_num, selected_units_num, selected_units, key=None,
                        split=False):
        key, base_mask = self.keys(entity_embedding, entity_num, key)     # [B,N+1,32], [B,N+1]
        B, N1, C = key.shape
        step_ok = None
        if key.is_cuda:
            # static S = label width (no host sync on max(selected_units_num)); steps at or beyond the
            # batch max are frozen out of the running selection and their logits masked to NEG, which is
            # exactly the dynamic-S result padded to the label width
            S = selected_units.shape[1]
            smax = selected_units_num.max().clamp(min=1)
            step_ok = torch.arange(S, device=key.device) < smax
        else:
            S = max(int(selected_units_num.max()), 1)
        labels = selected_units[:, :S].long()                             # [B,S]
        en = entity_num.long()
        # end_flag after label i; a label is added to the selected set iff no end at or before i
        is_end = labels == en[:, None]
        ended = torch.cumsum(is_end.int(), 1) > 0
        added = ~ended
        # first occurrence among added labels (set semantics of the reference one-hot)
        same = labels[:, :, None] == labels[:, None, :]                   # [B,S(i),S(j)]
        earlier = torch.tril(torch.ones(S, S, dtype=torch.bool, device=key.device), -1)
        dup = (same & earlier[None] & added[:, None, :]).any(-1)
        new = added & ~dup
        if step_ok is not None:
            new = new & step_ok[None, :]
        if self.reduce_type == 'selected_units_num':
            gathered = key.gather(1, labels.clamp(max=N1 - 1).unsqueeze(-1).expand(B, S, C))
            run_sum = torch.cumsum(gathered * new.unsqueeze(-1).to(gathered.dtype), 1)
            run_cnt = torch.cumsum(new.int(), 1)
            div = torch.where((selected_units_num != 0)[:, None], run_cnt.clamp(min=1), torch.ones_like(run_cnt))
            emb = run_sum / div.unsqueeze(-1).to(run_sum.dtype)          # embedding after step i
            if split and SU_AE_SIDE:
                # the caller runs the pointer half (a 32-wide LSTM: latency-bound, a few workgroups) beside the
                # target-unit and location heads, which need only the last step's embedding: the [B, S - 1, 1024]
                # embedding update of the earlier steps (the pointer's queries) moves there too
                ptr = {'ae0': ae0, 'emb_prev': emb[:, :-1], 'key': key, 'labels': labels, 'base_mask': base_mask,
                       'en': en, 'step_ok': step_ok}
                return ptr, self._ae_update(ae0, emb[:, -1]), selected_units_num
            ae_after = self._ae_update(ae0.unsqueeze(1), emb)            # [B,S,1024]
        else:  # attention pooling over the selected set after each step (prefix softmax, all steps at once)
            pooled = self.attention_pool.prefix(key, labels.clamp(max=N1 - 1), new)
            ae_after = ae0.unsqueeze(1) + pooled.to(ae0.dtype)
        ae_in = torch.cat([ae0.unsqueeze(1).to(ae_after.dtype), ae_after[:, :-1]], 1)
        ptr = {'ae_in': ae_in, 'key': key, 'labels': labels, 'base_mask': base_mask, 'en': en, 'step_ok': step_ok}
        if split:
            return ptr, ae_after[:, -1], selected_units_num
        return self.pointer_logits(ptr), None, ae_after[:, -1], selected_units_num

    def pointer_logits(self, ptr):
        """Teacher-forced pointer logits [B,S,N+1] from forward_teacher(split=True)'s inputs."""
        key, labels, base_mask, en, step_ok = (ptr[k] for k in ('key', 'labels', 'base_mask', 'en', 'step_ok'))
        ae_in = ptr.get('ae_in')
        q_h = None
        if ae_in is None:
            ae0 = ptr['ae0']
            if SU_FOLD and not self.query_fc1.norm:
                q_h = self._query_in_folded(ae0, ptr['emb_prev'])            # [B,S,256]
            else:
                ae_prev = self._ae_update(ae0.unsqueeze(1), ptr['emb_prev'])     # [B,S-1,1024]
                ae_in = torch.cat([ae0.unsqueeze(1).to(ae_prev.dtype), ae_prev], 1)
        B, N1, _ = key.shape
        S = labels.shape[1]
        q_in = self.query_fc2(self.query_fc1(ae_in) if q_h is None else q_h)   # [B,S,32]
        state = self.lstm.zero_state(B, q_in.device, torch.float32)
        q, _ = self.lstm(q_in.transpose(0, 1), state)                    # [S,B,32]
        logits = torch.bmm(q.transpose(0, 1).float(), key.float().transpose(1, 2))  # [B,S,N+1]
        # mask: base, end disabled at step 0, labels[:i] masked at step i.  Unit n is masked at step i iff its
        # first label step is < i: one [B, N+1] scatter-min of the label steps and one broadcast compare (a
        # [B,S,N+1] int64 one-hot + cumsum + shifted cat was ~0.2 GB of traffic per step, r2dn)
        steps = torch.arange(S, device=labels.device)
        first = torch.full((B, N1), S, dtype=torch.long, device=labels.device)
        first.scatter_reduce_(1, labels.clamp(max=N1 - 1), steps.expand(B, S), reduce='amin')
        mask = base_mask[:, None, :] & (first[:, None, :] >= steps[None, :, None])
        end_pos = F.one_hot(en.clamp(max=N1 - 1), N1).bool()
        mask[:, 0] &= ~end_pos
        if step_ok is not None:
            mask = mask & step_ok[None, :, None]
        # the reference returns no sampled units in teacher-forced mode (test_iou off)
        return torch.where(mask, logits, NEG)

    def _query_in_folded(self, ae0, emb_prev):
        """relu(query_fc1([ae0, ae0 + embed_fc2(embed_fc1(emb_prev))])) [B,S,256] without the [B, S-1, 1024] embedding
        update: query_fc1 is linear, so Wq (ae0 + We2 h + be2) + bq = (Wq ae0 + bq) + (Wq We2) h + Wq be2 - one
        256 x 256 product over the earlier steps instead of two 1024-wide ones, and neither the 1024-wide
        intermediates nor their gradients reach HBM (the sampler's fold, pointer.hip, in the training graph).
        Same function (fp32 products reassociated); gradients reach Wq, We2, be2 through the fold."""
        q1, e2 = self.query_fc1[0], self.embed_fc2[0]
        h = self.embed_fc1(emb_prev)                                     # [B,S-1,256]
        dt = torch.promote_types(q1.weight.dtype, torch.float32)
        with torch.autocast(ae0.device.type, enabled=False):             # the fold itself in (at least) fp32
            wq = q1.weight.to(dt)
            wf = wq @ e2.weight.to(dt)                                   # [256,256]
            bf = wq @ e2.bias.to(dt)                                     # [256]
        p0 = ops.linear(ae0, q1.weight, q1.bias)                         # [B,256]
        pp = ops.linear(h, wf, bf) + p0.unsqueeze(1)                     # [B,S-1,256]
        return F.relu(torch.cat([p0.unsqueeze(1), pp.to(p0.dtype)], 1))

    # ------------------------------------------------------------------ sampling (actor)
    def _folded_query(self):
        """(Wq1 We2 [256,256] bf16, Wq1 be2 [256]) cached per weight version (pointer.hip fold)."""
        q1, e2 = self.query_fc1[0], self.embed_fc2[0]
        if _capturing():      # recorded in the graph: replays see weights loaded in place later
            wq1 = q1.weight.float()
            return (wq1 @ e2.weight.float()).to(torch.bfloat16).contiguous(), wq1 @ e2.bias.float()
        tag = (q1.weight.data_ptr(), q1.weight._version, e2.weight.data_ptr(), e2.weight._version, e2.bias._version)
        if getattr(self, '_fold_tag', None) != tag:
            with torch.no_grad():
                wq1 = q1.weight.float()
                self._fold = ((wq1 @ e2.weight.float()).to(torch.bfloat16).contiguous(), wq1 @ e2.bias.float())
            self._fold_tag = tag
        return self._fold

    def forward_sample_native(self, native, ae0, entity_embedding, entity_num, su_mask, temperature: float = 1.0,
                              u: Optional[torch.Tensor] = None):
        key, _ = self.keys(entity_embedding, entity_num)
        B, N1, _ = key.shape
        q1 = self.query_fc1[0]
        # fp32 like the sampler's other inputs, on the few-row native GEMM outside autocast (under autocast
        # F.linear re-cast the 256 x 1024 weight to bf16 in every replayed graph: 4 extra launches)
        with torch.autocast('cuda', enabled=False):
            c0 = native.linear_f32_rows(ae0.float(), q1.weight, q1.bias)
        if u is None:
            u = torch.rand(B, MAX_SELECTED_UNITS_NUM, device=key.device)
        wf, bf = self._folded_query()
        logits, results, _, su_num, emb, extra = native.su_sample(
            key, c0, u, entity_num, su_mask, wf, bf, self.query_fc2[0].weight, self.query_fc2[0].bias,
            self.lstm.layers[0].cell, self.embed_fc1[0].weight, self.embed_fc1[0].bias, temperature,
            MAX_SELECTED_UNITS_NUM, self.extra_units)
        ae = self._ae_update(ae0, emb.to(ae0.dtype))
        # the kernel writes the extra-units map at the padded width (zeros past each row's entities)
        ex = extra if self.extra_units else torch.zeros(B, MAX_ENTITY_NUM + 1, device=key.device)
        return logits, results, ae, su_num, ex

    def forward_sample(self, ae0, entity_embedding, entity_num, su_mask, temperature: float = 1.0,
                       u: Optional[torch.Tensor] = None):
        native = ops._native(entity_embedding)
        if native is not None and native.has('su_sample') and not torch.is_grad_enabled() \
                and self.lstm.num_layers == 1 and self.reduce_type == 'selected_units_num':
            return self.forward_sample_native(native, ae0, entity_embedding, entity_num, su_mask, temperature, u)
        key, mask = self.keys(entity_embedding, entity_num)
        B, N1, _ = key.shape
        dev = key.device
        ar_b = torch.arange(B, device=dev)
        en = entity_num.long()
        mask = mask.clone()
        mask[ar_b, en] = False
        end_flag = ~su_mask.bool()
        su_num = torch.where(su_mask.bool(), torch.full_like(en, MAX_SELECTED_UNITS_NUM), torch.zeros_like(en))
        one_hot = torch.zeros(B, N1, device=dev, dtype=key.dtype)
        state = self.lstm.zero_state(B, dev, torch.float32)
        ae = ae0
        results, logits_list = [], []
        result = None
        step_logits = None
        for i in range(MAX_SELECTED_UNITS_NUM):
            if i == 1:
                mask[ar_b, en] = True
            if result is not None:
                mask[ar_b, result] = False
            q_in = self.query_fc2(self.query_fc1(ae)).unsqueeze(0)
            q, state = self.lstm(q_in, state)
            step_logits = torch.einsum('bc,bnc->bn', q[0].float(), key.float()).masked_fill(~mask, NEG) / temperature
            ui = None if u is None else u[:, i]
            result = sample_from_logits(step_logits, ui)
            newly_end = (result == en) & ~end_flag
            su_num = torch.where(newly_end, torch.full_like(su_num, i + 1), su_num)
            end_flag = end_flag | (result == en)
            results.append(result)
            logits_list.append(step_logits)
            keep = ~end_flag
            one_hot[ar_b[keep], result[keep]] = 1
            if self.reduce_type == 'selected_units_num':
                emb = (key * one_hot.unsqueeze(-1)).sum(1)
                cnt = one_hot.sum(1, keepdim=True)
                emb = torch.where(cnt > 0, emb / cnt.clamp(min=1), emb)
                ae = self._ae_update(ae0, emb)
            else:
                ae = ae0 + self.attention_pool(key, num=one_hot.sum(1), mask=one_hot).to(ae0.dtype)
            if bool(end_flag.all()):
                break
        extra = torch.zeros(B, MAX_ENTITY_NUM + 1, device=dev)
        if self.extra_units:
            end_logit = step_logits[ar_b, en]
            ex = (step_logits > end_logit[:, None]) & ~end_flag[:, None]
            extra[:, :N1] = ex.float()
        return torch.stack(logits_list, 1), torch.stack(results, 1), ae, su_num, extra


class TargetUnitHead(nn.Module):
    def __init__(self, input_dim=1024, entity_dim=256, key_dim=32):
        super().__init__()
        self.key_fc = FCBlock(entity_dim, key_dim)
        self.query_fc1 = FCBlock(input_dim, key_dim, act=True)
        self.query_fc2 = FCBlock(key_dim, key_dim)

    def forward(self, embedding, entity_embedding, entity_num, temperature: float = 1.0, target_unit=None, u=None,
                key=None):
        if key is None:
            key = self.key_fc(entity_embedding)
        if target_unit is None:
            fused = ops.target_unit_sample(embedding, self.query_fc1[0], self.query_fc2[0], key, entity_num,
                                           temperature, u)
            if fused is not None:     # actor inference: query MLP + key dot + mask + sample in one kernel
                return fused
        q = self.query_fc2(self.query_fc1(embedding))
        logits = torch.einsum('bc,bnc->bn', q.float(), key.float())
        mask = ops.sequence_mask(entity_num, key.shape[1])
        logits = logits.masked_fill(~mask, NEG) / temperature
        if target_unit is None:
            target_unit = sample_from_logits(logits, u)
        return logits, target_unit


class LocationHead(nn.Module):
    """fc 1024->1520 -> [B,4,19,20] || map_skip[-1] -> 1x1 conv 128 -> 4 gated res-blocks (+skips)
    -> 3 x (bilinear x2, conv3x3) 128->64->32->1 -> 24,320 logits (action_arg_head.py:366-450)."""

    def __init__(self, input_dim=1024, res_dim=128, res_num=4, reshape_channel=4, map_skip_dim=128,
                 upsample_dims=(64, 32, 1)):
        super().__init__()
        self.reshape_channel = reshape_channel
        self.hy, self.hx = SPATIAL_SIZE[0] // 8, SPATIAL_SIZE[1] // 8
        self.conv1 = ConvBlock(map_skip_dim + reshape_channel, res_dim, 1, act=True)
        self.res = nn.ModuleList()  # registered before project_embed, as in the reference
        self.project_embed = FCBlock(input_dim, self.hy * self.hx * reshape_channel, act=True)
        self.res.extend([GatedResBlock(res_dim) for _ in range(res_num)])
        dims = [res_dim] + list(upsample_dims)
        self.upsample = nn.ModuleList([ConvBlock(dims[i], dims[i + 1], 3, 1, 1, act=(i < len(upsample_dims) - 1))
                                       for i in range(len(upsample_dims))])

    def forward(self, embedding, map_skip: List[torch.Tensor], temperature: float = 1.0, location=None, u=None):
        B = embedding.shape[0]
        pf = self.project_embed(embedding)
        skip = map_skip[-1]
        # map_skip[-1] is a ResBlock output (ReLU'd) and pf is ReLU'd: the fused stage skips the cat
        x = ops.location_input(pf, skip, self.conv1[0].weight, self.conv1[0].bias) if self.conv1.act else None
        if x is None:
            p = pf.reshape(B, self.reshape_channel, self.hy, self.hx)
            if skip.is_contiguous(memory_format=torch.channels_last):
                p = p.contiguous(memory_format=torch.channels_last)
            x = F.relu(torch.cat([p.to(skip.dtype), skip], 1))
            x = self.conv1(x)
        # block i's input is the previous output + skip map -1 - i: the adds after the first ride in the blocks'
        # output pass (GatedResBlock post)
        x = x + map_skip[-1]
        for i, blk in enumerate(self.res):
            j = len(map_skip) - 2 - i
            x = blk(x, map_skip[j] if i + 1 < len(self.res) else None)
        for conv in self.upsample[:-1]:
            x = conv(ops.upsample2x(x))
        last = self.upsample[-1][0]  # 32 -> 1: fused upsample + conv, the 32-ch map never hits HBM
        logits = ops.upsample_conv_out(x, last.weight, last.bias) / temperature
        if location is None:
            fused = ops.head_sample(logits, 1.0, u=u)
            location = fused[1] if fused is not None else sample_from_logits(logits, u)
        return logits, location
