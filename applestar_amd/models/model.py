"""AlphaStar policy/value model.

Module tree and parameter names are those of ``distar/agent/default/model/model.py:22-189`` so
released ``rl_model.pth`` / ``sl_model.pth`` state dicts load unchanged.  Public forwards:

* :meth:`Model.compute_logp_action` — actor inference (sample + log-prob)        (model.py:56-74)
* :meth:`Model.compute_teacher_logit` — teacher-forced logits for the KL teacher (model.py:76-93)
* :meth:`Model.rl_learner_forward` — flattened (T+1)*B learner forward          (model.py:95-168)
* :meth:`Model.sl_train` — supervised forward over [B,T] chunks                  (model.py:170-189)
"""
from __future__ import annotations

import os

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..lib import game_data as gd
from ..lib.features import MAX_SELECTED_UNITS_NUM, ACTION_HEADS
from ..utils.config import AttrDict, deep_merge_dicts
from .blocks import FCBlock, ResFCBlock2
from .encoders import Encoder, ValueEncoder
from .heads import (ActionTypeHead, DelayHead, QueuedHead, SelectedUnitsHead, TargetUnitHead, LocationHead,
                    NEG)
from .lstm import StackedLNLSTM

BASELINE_NAMES = ['winloss', 'build_order', 'built_unit', 'effect', 'upgrade', 'battle']

DEFAULT_MODEL_CONFIG = AttrDict({
    'learner': {'use_value_feature': False},
    'agent': {'extra_units': False},
    'common': {'type': 'train'},
    'model': {
        'temperature': 1.0,
        'enable_baselines': list(BASELINE_NAMES),
        'entity_reduce_type': 'selected_units_num',
        'only_update_baseline': False,
        'value': {'res_dim': 256, 'res_num': 16, 'input_dim': 384},
        'lstm': {'input_size': 1536, 'hidden_size': 384, 'num_layers': 3},
    },
})


_SIDE_STREAMS: Dict[tuple, 'torch.cuda.Stream'] = {}
SIDE_STREAMS_ENABLED = True
# the critics on the value encoder's side stream (beside the policy heads): r2 measured no gain (+1.9 ms, noisy); on
# the round-6 tree fp32 53.26 / 53.00 -> 51.98 / 52.07 ms, bf16 neutral to +0.1 ms (profiles/r10j_bench_critic_tu_side.txt,
# r10k_*): APPLESTAR_CRITIC_SIDE_STREAM = fp32 (default: the fp32 step only) | 1 | 0
_CRITIC_SIDE = os.environ.get('APPLESTAR_CRITIC_SIDE_STREAM', 'fp32')
CRITIC_SIDE_STREAM = _CRITIC_SIDE == '1'
CRITIC_SIDE_STREAM_FP32 = _CRITIC_SIDE in ('1', 'fp32')
# the target-unit head behind the selected-units pointer on side stream 2: fp32 -0.07 / bf16 -0.15 ms (same file)
TU_SIDE_STREAM = os.environ.get('APPLESTAR_TU_SIDE_STREAM', '1') == '1'
# teacher-forced action-type / delay / queued logits on side stream 2 beside the embedding chain (A/B switch)
HEAD_LOGITS_SIDE_STREAM = os.environ.get('APPLESTAR_HEAD_LOGITS_SIDE', '1') == '1'
# the heads' joint entity key projection on side stream 2 beside the core LSTM: slower (fp32 52.3 / 53.2 vs 51.2 /
# 51.0 ms, profiles/r10m_bench_keys_side.txt) - a ~200k-row product beside the split recurrence delays the residency
# of its 8-workgroup rows; off (APPLESTAR_KEYS_SIDE=1 turns it on)
KEYS_SIDE = os.environ.get('APPLESTAR_KEYS_SIDE', '0') == '1'
# teacher-forced selected-units pointer (LSTM + logits) on side stream 2 beside the target-unit / location heads
SU_SIDE_STREAM = os.environ.get('APPLESTAR_SU_SIDE_STREAM', '1') == '1'
VE_BWD_OVERLAP = os.environ.get('APPLESTAR_VE_BWD_OVERLAP', '0') == '1'   # A/B r4: 61.6 / 61.7 vs 61.3 / 61.6 ms, off
VE_AFTER_CORE = os.environ.get('APPLESTAR_VE_AFTER_CORE', '1') == '1'   # A/B r4: fp32 61.3 / 60.8 vs 61.8 / 61.6 ms
# selected-units + target-unit key projections as one product before the row slice (APPLESTAR_JOINT_KEYS=0: per head)
JOINT_KEYS = os.environ.get('APPLESTAR_JOINT_KEYS', '1') != '0'
# value baselines' ResFCBlock2 stack as the fused resmlp kernels on the GPU (APPLESTAR_FUSED_RESMLP=0: op by op)
FUSED_RESMLP = __import__('os').environ.get('APPLESTAR_FUSED_RESMLP', '1') == '1'


_DEVICE_TABLES: Dict[tuple, torch.Tensor] = {}


def _device_table(name: str, t: torch.Tensor, device) -> torch.Tensor:
    """Constant lookup table cached per device (a per-call .to(device) is a pageable H2D copy: a host
    sync, and not capturable in a HIP graph)."""
    key = (name, str(device))
    if key not in _DEVICE_TABLES:
        _DEVICE_TABLES[key] = t.to(device)
    return _DEVICE_TABLES[key]


def _side_stream_call(fn, inputs, slot: int = 0, after=None):
    """Run ``fn(inputs)`` on side stream ``slot`` of the device (GPU) and return a handle for
    :func:`_side_stream_join`.  ``after``: an event recorded on the main stream earlier; the side stream waits for
    it instead of for everything issued so far (the inputs were ready at that point)."""
    dev = next((v.device for v in inputs.values() if torch.is_tensor(v)), None) if isinstance(inputs, dict) else None
    if dev is None or dev.type != 'cuda' or not SIDE_STREAMS_ENABLED:
        return fn(inputs), None
    main = torch.cuda.current_stream(dev)
    side = _SIDE_STREAMS.get((dev.index, slot))
    if side is None:
        side = _SIDE_STREAMS[(dev.index, slot)] = torch.cuda.Stream(dev)
    if after is not None:
        side.wait_event(after)
    else:
        side.wait_stream(main)             # inputs were produced on the main stream
    for t in inputs.values():              # ... and are read on the side stream
        if torch.is_tensor(t) and t.is_cuda:
            t.record_stream(side)
    with torch.cuda.stream(side):
        out = fn(inputs)
    return out, side


def _side_stream_join(handle):
    out, side = handle
    if side is not None:
        tensors = [t for t in (out if isinstance(out, (tuple, list)) else (out,)) if torch.is_tensor(t)]
        main = torch.cuda.current_stream(tensors[0].device)
        main.wait_stream(side)
        for t in tensors:
            t.record_stream(main)          # allocated on the side stream, consumed on main
    return out


class _TakeRows(torch.autograd.Function):
    """x[:n] whose backward builds the full-height gradient in x's own memory format (channels_last for
    the spatial skips) with one copy + one tail fill.  The stock SliceBackward materialises an
    NCHW-contiguous zeros tensor, so the autograd engine's sum with the encoder's NHWC gradient of the same
    map ran as a strided elementwise kernel (r2bd: ~0.11 ms per 19x20x128 skip, 4 per step)."""

    @staticmethod
    def forward(ctx, x, n, link=None):
        ctx.shape, ctx.stride, ctx.n = x.shape, x.stride(), n
        ctx.link = link
        return x.narrow(0, 0, n)   # a view: no forward copy

    @staticmethod
    def backward(ctx, g):
        if ctx.link is not None and g.dtype == torch.float32 and not ctx.link.consumed:
            # hand the gradient to the ResBlock consuming this map (ops/native.py SkipLink): it adds it, NHWC,
            # to the first n rows of its input gradient; no full-height gradient here, no autograd add.  A link
            # whose ResBlock backward already ran (consumed) falls through to the ordinary gradient below
            nhwc = g.permute(0, 2, 3, 1)
            ctx.link.g = nhwc if nhwc.is_contiguous() else nhwc.contiguous()
            return None, None, None
        full = torch.empty_strided(ctx.shape, ctx.stride, dtype=g.dtype, device=g.device)
        full[:ctx.n].copy_(g)
        full[ctx.n:].zero_()
        return full, None, None


def _take_rows(x, n):
    if x is None:                 # a skip level the fused encoder never materialises (see SpatialEncoder.trunk)
        return None
    if x.dim() == 4 and x.shape[0] > n and x.is_cuda:
        return _TakeRows.apply(x, n, getattr(x, '_skip_link', None))
    return x[:n]


class ValueBaseline(nn.Module):
    """fc(in->256, ReLU) -> 16 x ResFCBlock2 -> fc(256->1, gain .1) [-> (2/pi) atan(pi/2 x)] (value.py:9-39)."""

    def __init__(self, input_dim: int, res_dim: int = 256, res_num: int = 16, atan: bool = False):
        super().__init__()
        self.input_dim, self.res_dim, self.res_num = input_dim, res_dim, res_num
        self.project = FCBlock(input_dim, res_dim, act=True)
        self.res = nn.Sequential(*[ResFCBlock2(res_dim) for _ in range(res_num)])
        self.value_fc = FCBlock(res_dim, 1, init='xavier_uniform', gain=0.1)
        self.atan = atan

    def fused_params(self):
        """ResFCBlock2 parameters in the fused kernel's order (csrc/kernels/resmlp.hip)."""
        ps = []
        for blk in self.res:
            ps += [blk.fc1[0].weight, blk.fc1[0].bias, blk.fc2[0].weight, blk.fc2[0].bias, blk.norm.weight, blk.norm.bias]
        return ps

    def _fusable(self, x) -> bool:
        if not (x.is_cuda and FUSED_RESMLP and self.res_dim == 256 and 1 <= self.res_num <= 16):
            return False
        n = ops._native(x)
        if n is None or not n.has('resmlp'):
            return False
        return all(p.is_contiguous() and p.dtype == (torch.float32 if i % 6 >= 4 else torch.bfloat16)
                   for i, p in enumerate(self.fused_params()))

    def forward(self, x):
        h = self.project(x)
        if self._fusable(h):
            from ..ops import native
            h = native.resmlp(h.reshape(-1, self.res_dim), self.fused_params()).view(*h.shape[:-1], self.res_dim)
        else:
            h = self.res(h)
        v = self.value_fc(h).squeeze(1).float()
        if self.atan:
            v = (2.0 / torch.pi) * torch.atan((torch.pi / 2.0) * v)
        return v


class Policy(nn.Module):
    def __init__(self, extra_units: bool = False, entity_reduce_type: str = 'selected_units_num'):
        super().__init__()
        self.action_type_head = ActionTypeHead()
        self.delay_head = DelayHead()
        self.queued_head = QueuedHead()
        self.selected_units_head = SelectedUnitsHead(extra_units=extra_units, reduce_type=entity_reduce_type)
        self.target_unit_head = TargetUnitHead()
        self.location_head = LocationHead()

    def forward(self, lstm_output, entity_embeddings, map_skip, scalar_context, entity_num, temperature=1.0,
                race_mask=None, noise: Optional[Dict[str, torch.Tensor]] = None):
        if noise is None and lstm_output.is_cuda:
            # every head's sampling uniforms in two launches (was one torch.rand per head, six launches per step)
            B = lstm_output.shape[0]
            u5 = torch.rand(5, B, device=lstm_output.device)
            noise = {'action_type': u5[0], 'delay': u5[1], 'queued': u5[2], 'target_unit': u5[3],
                     'target_location': u5[4],
                     'selected_units': torch.rand(B, MAX_SELECTED_UNITS_NUM, device=lstm_output.device)}
        noise = noise or {}
        logit, action = {}, {}
        logit['action_type'], action['action_type'], emb = self.action_type_head(
            lstm_output, scalar_context, temperature, race_mask=race_mask, u=noise.get('action_type'))
        logit['delay'], action['delay'], emb = self.delay_head(emb, temperature, u=noise.get('delay'))
        logit['queued'], action['queued'], emb = self.queued_head(emb, temperature, u=noise.get('queued'))
        su_mask = _device_table('su_mask', gd.SELECTED_UNITS_MASK, action['action_type'].device)[action['action_type']]
        logit['selected_units'], action['selected_units'], emb, su_num, extra = \
            self.selected_units_head.forward_sample(emb, entity_embeddings, entity_num, su_mask, temperature,
                                                    u=noise.get('selected_units'))
        logit['target_unit'], action['target_unit'] = self.target_unit_head(
            emb, entity_embeddings, entity_num, temperature, u=noise.get('target_unit'))
        logit['target_location'], action['target_location'] = self.location_head(
            emb, map_skip, temperature, u=noise.get('target_location'))
        return action, su_num, logit, extra

    def joint_keys(self, entity_embeddings, rows: Optional[int] = None):
        """The selected-units and target-unit key projections (both 256 -> 32 over every entity) as ONE
        256 -> 64 product over the full padded batch, sliced to ``rows`` afterwards: the backward is one input
        gradient of the entity embeddings (no sum of two, no full-size zero-padded slice gradient)."""
        su, tu = self.selected_units_head.key_fc[0], self.target_unit_head.key_fc[0]
        k = ops.linear(entity_embeddings, torch.cat([su.weight, tu.weight], 0), torch.cat([su.bias, tu.bias], 0))
        if rows is not None:
            k = k[:rows]
        return k.split(su.weight.shape[0], dim=-1)

    def train_forward(self, lstm_output, entity_embeddings, map_skip, scalar_context, entity_num, action_info,
                      selected_units_num, temperature=1.0, keys=None):
        """``keys``: (selected-units, target-unit) key projections from :meth:`joint_keys` (else per head)."""
        logit, action = {}, {}
        su_key, tu_key = keys if keys is not None else (None, None)
        if HEAD_LOGITS_SIDE_STREAM and lstm_output.is_cuda and SU_SIDE_STREAM and \
                not torch.cuda.is_current_stream_capturing():
            # teacher forcing: the action-type / delay / queued logits branches do not feed the autoregressive
            # embedding chain - they run on side stream 2 (before the selected-units pointer) while the chain continues
            at, dh, qh = self.action_type_head, self.delay_head, self.queued_head
            heads_h = [('action_type', _side_stream_call(
                lambda d: at.teacher_logits(d['x'], d['c'], temperature), {'x': lstm_output, 'c': scalar_context},
                slot=2))]
            emb = at.teacher_embedding(lstm_output, scalar_context, action_info['action_type'])
            heads_h.append(('delay', _side_stream_call(lambda d: dh.teacher_logits(d['e'], temperature), {'e': emb},
                                                       slot=2)))
            emb = dh.teacher_embedding(emb, action_info['delay'])
            heads_h.append(('queued', _side_stream_call(lambda d: qh.teacher_logits(d['e'], temperature), {'e': emb},
                                                        slot=2)))
            emb = qh.teacher_embedding(emb, action_info['queued'])
            for k, _ in heads_h:
                action[k] = action_info[k]
        else:
            heads_h = []
            logit['action_type'], action['action_type'], emb = self.action_type_head(
                lstm_output, scalar_context, temperature, action_type=action_info['action_type'])
            logit['delay'], action['delay'], emb = self.delay_head(emb, temperature, action=action_info['delay'])
            logit['queued'], action['queued'], emb = self.queued_head(emb, temperature, action=action_info['queued'])
        su = self.selected_units_head
        if SU_SIDE_STREAM and emb.is_cuda and not torch.cuda.is_current_stream_capturing():
            # the pointer half of the selected-units head (its 32-wide LSTM + logits: latency-bound) on side stream 2,
            # beside the target-unit and location heads, which need only the head's output embedding; autograd
            # replays its backward on that stream as well
            ptr, emb, su_num = su.forward_teacher(emb, entity_embeddings, entity_num, selected_units_num,
                                                  action_info['selected_units'], key=su_key, split=True)
            su_h = _side_stream_call(su.pointer_logits, ptr, slot=2)
        else:
            su_logit, _, emb, su_num = su.forward_teacher(emb, entity_embeddings, entity_num, selected_units_num,
                                                          action_info['selected_units'], key=su_key)
            su_h = (su_logit, None)
        action['selected_units'] = None
        tu_in = {'emb': emb, 'ee': entity_embeddings, 'en': entity_num, 'tu': action_info['target_unit'],
                 'key': tu_key}
        tu_head = lambda d: self.target_unit_head(d['emb'], d['ee'], d['en'], temperature, target_unit=d['tu'],
                                                  key=d['key'])
        if TU_SIDE_STREAM and su_h[1] is not None:
            tu_h = _side_stream_call(tu_head, tu_in, slot=2)
        else:
            tu_h = (tu_head(tu_in), None)
        logit['target_location'], action['target_location'] = self.location_head(
            emb, map_skip, temperature, location=action_info['target_location'])
        logit['target_unit'], action['target_unit'] = _side_stream_join(tu_h)
        logit['selected_units'] = _side_stream_join(su_h)
        for k, h in heads_h:
            logit[k] = _side_stream_join(h)
        logit = {k: logit[k] for k in ('action_type', 'delay', 'queued', 'selected_units', 'target_unit',
                                       'target_location')}
        action = {k: action[k] for k in ('action_type', 'delay', 'queued', 'selected_units', 'target_unit',
                                         'target_location')}
        return action, su_num, logit


class Model(nn.Module):
    def __init__(self, cfg: Optional[dict] = None, use_value_network: bool = False, temperature: Optional[float] = None):
        super().__init__()
        self.whole_cfg = deep_merge_dicts(DEFAULT_MODEL_CONFIG, cfg or {})
        mcfg = self.whole_cfg.model
        if temperature is not None:
            mcfg.temperature = temperature
        self.cfg = mcfg
        self.temperature = float(mcfg.temperature)
        self.encoder = Encoder(mcfg.entity_reduce_type)
        self.policy = Policy(extra_units=bool(self.whole_cfg.get('agent', {}).get('extra_units', False)),
                             entity_reduce_type=mcfg.entity_reduce_type)
        self._use_value_feature = bool(self.whole_cfg.learner.get('use_value_feature', False))
        self.use_value_network = use_value_network
        if use_value_network:
            if self._use_value_feature:
                self.value_encoder = ValueEncoder()
            self.value_networks = nn.ModuleDict()
            in_dim = mcfg.value.input_dim + (1056 if self._use_value_feature else 0)
            for name in BASELINE_NAMES:
                if name in mcfg.enable_baselines:
                    self.value_networks[name] = ValueBaseline(in_dim, mcfg.value.res_dim, mcfg.value.res_num,
                                                              atan=(name == 'winloss'))
        self.only_update_baseline = bool(mcfg.get('only_update_baseline', False))
        lc = mcfg.lstm
        self.core_lstm = StackedLNLSTM(lc.input_size, lc.hidden_size, lc.num_layers)
        self.race_mask: Optional[torch.Tensor] = None  # set by the agent in play mode (action_type_head.py:52)

    # ------------------------------------------------------------------ helpers
    def _graphed(self, name: str, module: nn.Module):
        """HIP-graph-captured (forward + backward) view of a static-shape section (runtime/graphs.py);
        kept outside the module tree so state_dict keys are unchanged."""
        from ..runtime.graphs import GraphedSection
        cache = self.__dict__.setdefault('_graph_sections', {})
        if name not in cache:
            cache[name] = GraphedSection(module)
        return cache[name]

    def _encode(self, spatial_info, entity_info, scalar_info, entity_num, entity_total=None, entity_pad=None):
        out = self.encoder(spatial_info, entity_info, scalar_info, entity_num, entity_total, entity_pad)
        if getattr(self, 'phase_cut', False) and torch.is_grad_enabled() and \
                not (out[0].is_cuda and torch.cuda.is_current_stream_capturing()):
            # the two-phase backward (parallel/dp.py backward_phased): everything downstream of the encoders (core
            # LSTM, heads, critics) reads detached leaf copies of the encoders' outputs, so backward phase 1 stops at
            # them; phase 2 runs the encoders' backward from the (encoder output, leaf gradient) pairs in ONE
            # autograd call (the outputs are not independent: each skip map feeds the next, the entity embeddings feed
            # the spatial scatter).  A skip map's SkipLink rides along on its leaf.
            pairs = []

            def cut(t):
                if not torch.is_tensor(t) or not t.requires_grad:
                    return t
                leaf = t.detach().requires_grad_()
                if getattr(t, '_skip_link', None) is not None:
                    leaf._skip_link = t._skip_link
                pairs.append((t, leaf))
                return leaf
            lstm_input, scalar_context, baseline_feature, entity_embeddings, map_skip = out
            out = (cut(lstm_input), cut(scalar_context), cut(baseline_feature), cut(entity_embeddings),
                   [cut(m) for m in map_skip])
            self.encoder_boundary = pairs
        return out

    def _core(self, lstm_input_seq, hidden_state):
        state = [(h.float(), c.float()) for h, c in hidden_state]
        return self.core_lstm(lstm_input_seq, state)

    # ------------------------------------------------------------------ actor inference
    @torch.no_grad()
    def compute_logp_action(self, spatial_info, entity_info, scalar_info, entity_num, hidden_state,
                            noise: Optional[Dict[str, torch.Tensor]] = None, **kwargs):
        lstm_input, scalar_context, _, entity_embeddings, map_skip = self._encode(
            spatial_info, entity_info, scalar_info, entity_num)
        out, out_state = self._core(lstm_input.unsqueeze(0), hidden_state)
        action, su_num, logit, extra = self.policy(out[0], entity_embeddings, map_skip, scalar_context, entity_num,
                                                   self.temperature, self.race_mask, noise)
        logp = ops.action_logp(logit, action)
        return {'action_info': action, 'action_logp': logp, 'selected_units_num': su_num,
                'entity_num': entity_num, 'hidden_state': out_state, 'logit': logit, 'extra_units': extra}

    @torch.no_grad()
    def compute_teacher_logit(self, spatial_info, entity_info, scalar_info, entity_num, hidden_state,
                              selected_units_num, action_info, **kwargs):
        lstm_input, scalar_context, _, entity_embeddings, map_skip = self._encode(
            spatial_info, entity_info, scalar_info, entity_num)
        out, out_state = self._core(lstm_input.unsqueeze(0), hidden_state)
        _, su_num, logit = self.policy.train_forward(out[0], entity_embeddings, map_skip, scalar_context,
                                                     entity_num, action_info, selected_units_num, self.temperature)
        return {'logit': logit, 'hidden_state': out_state, 'entity_num': entity_num, 'selected_units_num': su_num}

    # ------------------------------------------------------------------ learners
    def rl_learner_forward(self, spatial_info, entity_info, scalar_info, entity_num, hidden_state, action_info,
                           selected_units_num, batch_size: int, unroll_len: int, behaviour_logp=None,
                           teacher_logit=None, mask=None, reward=None, step=None, value_feature=None, **kwargs):
        """Observations are flattened time-major: index t*B + b for t in [0, T] (T+1 steps)."""
        B, T = batch_size, unroll_len
        flat_action = {k: v.flatten(0, 1) for k, v in action_info.items()}
        flat_su_num = selected_units_num.flatten(0, 1)
        # The opponent-aware value encoder depends only on its own inputs: on the GPU it runs on a side HIP
        # stream, overlapping the policy encoders and the latency-bound core LSTM (which occupies a handful
        # of CUs); autograd replays its backward on the same side stream, so that overlaps as well.
        vf = None
        if self._use_value_feature and not VE_AFTER_CORE:
            vf = _side_stream_call(self.value_encoder, value_feature)
        lstm_input, scalar_context, baseline_feature, entity_embeddings, map_skip = self._encode(
            spatial_info, entity_info, scalar_info, entity_num, kwargs.get('entity_total'), kwargs.get('entity_pad'))
        H = hidden_state[0][0].shape[-1]
        h0 = [(h.view(-1, B, H)[0], c.view(-1, B, H)[0]) for h, c in hidden_state]
        ev = None
        if self._use_value_feature and VE_AFTER_CORE and lstm_input.is_cuda and VE_BWD_OVERLAP and \
                SIDE_STREAMS_ENABLED and not torch.cuda.is_current_stream_capturing():
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(lstm_input.device))
        elif self._use_value_feature and VE_AFTER_CORE and lstm_input.is_cuda:
            # issued right behind the core LSTM's inputs: the value encoder's forward runs on its side stream
            # while the latency-bound recurrence occupies a few dozen CUs (A/B switch)
            vf = _side_stream_call(self.value_encoder, value_feature)
        ev_keys = None
        if KEYS_SIDE and JOINT_KEYS and lstm_input.is_cuda and SIDE_STREAMS_ENABLED and \
                not torch.cuda.is_current_stream_capturing():
            ev_keys = torch.cuda.Event()
            ev_keys.record(torch.cuda.current_stream(lstm_input.device))
        out, _ = self._core(lstm_input.view(T + 1, B, -1), h0)
        if self._use_value_feature and vf is None:
            # VE_BWD_OVERLAP: created AFTER the core LSTM (so autograd issues its backward before the LSTM's: the
            # side-stream backward then runs beside the recurrence's backward), but ordered on the GPU only
            # behind the event recorded before the LSTM (its forward still overlaps the recurrence)
            vf = _side_stream_call(self.value_encoder, value_feature, after=ev)
        lstm_output = out.reshape((T + 1) * B, -1)
        n = T * B
        critic_input = lstm_output
        if self.only_update_baseline:
            critic_input = critic_input.detach()
            baseline_feature = baseline_feature.detach()

        def critic(inp):
            ci = inp['lstm']
            if self._use_value_feature:
                v = inp['vf']
                ci = torch.cat([ci.to(v.dtype), v, inp['bf'].to(v.dtype)], 1)
            return [self._graphed(k, m)(ci).view(T + 1, B) for k, m in self.value_networks.items()]

        # the critic MLPs depend only on the LSTM output (+ value features): they run on the value encoder's
        # side stream (which already holds vf) while the policy heads run on the main stream
        # join the value encoder's side stream here (after the encoders and the LSTM were issued on the main
        # stream, so the overlap is kept): the critic below reads vf on the main stream
        vf_out = _side_stream_join(vf) if isinstance(vf, tuple) else vf
        critic_in = {'lstm': critic_input, 'vf': vf_out, 'bf': baseline_feature}
        critic_side = CRITIC_SIDE_STREAM or (CRITIC_SIDE_STREAM_FP32 and not torch.is_autocast_enabled())
        values_h = _side_stream_call(critic, critic_in) if critic_side else (critic(critic_in), None)
        if ev_keys is not None:
            # the heads' entity key projections depend only on the encoders: issued after the core LSTM (autograd
            # then runs their backward before the recurrence's, beside it) on side stream 2, ordered on the GPU only
            # behind the event recorded before the LSTM - the product runs beside the recurrence
            keys = _side_stream_join(_side_stream_call(lambda d: self.policy.joint_keys(d['ee'], n),
                                                       {'ee': entity_embeddings}, slot=2, after=ev_keys))
        else:
            keys = self.policy.joint_keys(entity_embeddings, n) if JOINT_KEYS else None
        _, _, logits = self.policy.train_forward(
            lstm_output[:n], entity_embeddings[:n], [_take_rows(m, n) for m in map_skip], scalar_context[:n],
            entity_num[:n], flat_action, flat_su_num, self.temperature, keys=keys)
        values = dict(zip(self.value_networks.keys(), _side_stream_join(values_h)))
        for k in list(logits):
            logits[k] = logits[k].view(T, B, *logits[k].shape[1:])
        su = logits['selected_units']
        logits['selected_units'] = F.pad(su, (0, 0, 0, MAX_SELECTED_UNITS_NUM - su.shape[2]), value=NEG)
        return {'unroll_len': T, 'batch_size': B, 'selected_units_num': selected_units_num,
                'target_logit': logits, 'value': values, 'action_log_prob': behaviour_logp,
                'teacher_logit': teacher_logit, 'mask': mask, 'action': action_info, 'reward': reward,
                'step': step}

    def sl_train(self, spatial_info, entity_info, scalar_info, entity_num, selected_units_num, traj_lens,
                 hidden_state, action_info, **kwargs):
        """Inputs flattened batch-major [B*T]; hidden_state per layer [B,H]."""
        B = len(traj_lens)
        lstm_input, scalar_context, _, entity_embeddings, map_skip = self._encode(
            spatial_info, entity_info, scalar_info, entity_num)
        T = lstm_input.shape[0] // B
        seq = lstm_input.view(B, T, -1).transpose(0, 1)
        out, out_state = self._core(seq, hidden_state)
        lstm_output = out.transpose(0, 1).reshape(B * T, -1)
        action, su_num, logits = self.policy.train_forward(lstm_output, entity_embeddings, map_skip, scalar_context,
                                                           entity_num, action_info, selected_units_num,
                                                           self.temperature)
        return logits, action, out_state

    def policy_state_dict(self):
        """Actor-facing weights (everything except value networks / value encoder)."""
        return {k: v for k, v in self.state_dict().items() if 'value_networks' not in k and 'value_encoder' not in k}


def _install_fast_apply():
    from ..ops.native import install_fast_apply
    install_fast_apply(globals(), __name__)


_install_fast_apply()
