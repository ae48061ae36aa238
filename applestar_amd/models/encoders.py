"""Observation encoders: scalar (+ build-order transformer), entity, spatial, value-feature.

Parameter names/shapes match ``distar/agent/default/model/obs_encoder/*.py`` and
``model/encoder.py``.  The compute graph is restructured for MI355X:

* entity one-hot/binary/scalar fields are never concatenated into a 997-wide tensor on the GPU:
  ``ops.entity_embed`` sums the selected weight rows (one-hot @ W == row gather);
* the entity transformer runs on packed real entities (no padding work);
* the spatial one-hot planes + effect points + entity scatter are assembled by
  ``ops.spatial_embed`` directly into the 1x1-projected 32-channel map.
"""
from __future__ import annotations

import math
import os
import weakref

from typing import Dict, List, Tuple, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..lib import game_data as gd
from ..lib.features import (MAX_ENTITY_NUM, ENTITY_FIELDS, SPATIAL_ONE_HOT, EFFECT_KEYS, SPATIAL_SIZE, ENTITY_EMBED_DIM,
                            BEGINNING_ORDER_LENGTH)
from .blocks import FCBlock, ConvBlock, ResBlock, MaxPool2x2, OneHotTable, binary_table, eye_table
from .transformer import Transformer, dense_segments

SPATIAL_Y, SPATIAL_X = SPATIAL_SIZE


def _denominator(dim: int) -> torch.Tensor:
    x = torch.arange(dim, dtype=torch.float)
    x = torch.div(x, 2, rounding_mode='floor') * 2
    return 1.0 / torch.pow(10000.0, x / dim)


class BeginningBuildOrderEncoder(nn.Module):
    """20-token pre-LN transformer over (action one-hot 174 | position one-hot 20 | 2x10-bit location)
    -> mean -> fc 64 (scalar_encoder.py:19-53)."""

    def __init__(self, output_dim: int = 64, head_dim: int = 8, binary_dim: int = 10):
        super().__init__()
        self.action_dim = gd.NUM_BEGINNING_ORDER_ACTIONS
        in_dim = self.action_dim + BEGINNING_ORDER_LENGTH + 2 * binary_dim
        self.transformer = Transformer(in_dim, head_dim=head_dim, hidden_dim=output_dim * 2, output_dim=output_dim,
                                       ln_type='pre')
        self.embedd_fc = FCBlock(output_dim, output_dim, act=True)
        self.action_one_hot = OneHotTable(eye_table(self.action_dim))
        self.order_one_hot = OneHotTable(eye_table(BEGINNING_ORDER_LENGTH))
        self.location_binary = OneHotTable(binary_table(binary_dim))

    def fused_params(self):
        """Parameters in the order of the fused kernel (csrc/kernels/bo_encoder.hip)."""
        t = self.transformer
        ps = [t.embedding[0].weight, t.embedding[0].bias]
        for layer in t.layers:
            a = layer.attention
            ps += [layer.layernorm1.weight, layer.layernorm1.bias, a.attention_pre[0].weight, a.attention_pre[0].bias,
                   a.project[0].weight, a.project[0].bias, layer.layernorm2.weight, layer.layernorm2.bias,
                   layer.mlp[0][0].weight, layer.mlp[0][0].bias, layer.mlp[1][0].weight, layer.mlp[1][0].bias]
        return ps

    def _fusable(self, bo) -> bool:
        if not bo.is_cuda or bo.shape[1] != BEGINNING_ORDER_LENGTH or not FUSED_BO:
            return False
        n = ops._native(bo)
        if n is None or not n.has('bo_encoder'):
            return False
        ps = self.fused_params()
        lin = ps[0].dtype
        return lin in (torch.float32, torch.bfloat16) and all(
            p.is_contiguous() and p.dtype == (torch.float32 if i >= 2 and (i - 2) % 12 in (0, 1, 6, 7) else lin)
            for i, p in enumerate(ps))

    def forward(self, bo: torch.Tensor, bo_location: torch.Tensor) -> torch.Tensor:
        if self._fusable(bo):
            from ..ops import native
            mean = native.bo_encoder(bo, bo_location, self.fused_params())          # fp32 [B, 64]
            return self.embedd_fc(mean)
        return self.forward_torch(bo, bo_location)

    def forward_torch(self, bo: torch.Tensor, bo_location: torch.Tensor) -> torch.Tensor:
        """The op-by-op path (CPU, and the reference the fused kernel is tested against)."""
        B, L = bo.shape
        dev = bo.device
        act = F.one_hot(bo.long().clamp(0, self.action_dim - 1), self.action_dim).float()
        pos = torch.eye(L, device=dev).expand(B, L, L)
        loc = bo_location.long()
        lx = self.location_binary.weight[loc % SPATIAL_X]
        ly = self.location_binary.weight[torch.div(loc, SPATIAL_X, rounding_mode='floor').clamp(max=1023)]
        x = torch.cat([act, pos, lx, ly], dim=2)
        x = self.transformer.forward_dense(x)
        return self.embedd_fc(x.mean(dim=1))


# fused build-order transformer kernel on the GPU (tools/ab_bench / APPLESTAR_FUSED_BO=0 for the op-by-op path)
FUSED_BO = __import__('os').environ.get('APPLESTAR_FUSED_BO', '1') == '1'


# (name, kind, in_dim/num, out_dim, scalar_context, baseline_feature) in reference module order
SCALAR_MODULES = [
    ('agent_statistics', 'fc', 10, 64, False, True),
    ('home_race', 'emb', 5, 32, True, False),
    ('away_race', 'emb', 5, 32, True, False),
    ('upgrades', 'fc', gd.NUM_UPGRADES, 128, False, True),
    ('unit_counts_bow', 'fc', gd.NUM_UNIT_TYPES, 128, False, True),
    ('last_delay', 'emb', 128, 64, False, False),
    ('last_queued', 'emb', 2, 32, False, False),
    ('last_action_type', 'emb', gd.NUM_ACTIONS, 128, False, False),
    ('cumulative_stat', 'fc', gd.NUM_CUMULATIVE_STAT_ACTIONS, 128, True, True),
    ('beginning_order', 'bo', 0, 64, True, True),
    ('unit_type_bool', 'fc', gd.NUM_UNIT_TYPES, 64, True, False),
    ('enemy_unit_type_bool', 'fc', gd.NUM_UNIT_TYPES, 64, True, False),
    ('unit_order_type', 'fc', gd.NUM_UNIT_MIX_ABILITIES, 64, True, False),
]
TIME_DIM = 32
_TIME_PHASE = {}      # (device, dim) -> the sine phase row (0, pi/2, 0, pi/2, ...) of the bf16 time encoding


class ScalarEncoder(nn.Module):
    """13 scalar fields -> embedded_scalar [B,1024], scalar_context [B,448], baseline_feature [B,512]."""

    def __init__(self):
        super().__init__()
        self.encode_modules = nn.ModuleDict()
        for name, kind, n_in, n_out, _, _ in SCALAR_MODULES:
            if kind == 'fc':
                self.encode_modules[name] = FCBlock(n_in, n_out, act=True)
            elif kind == 'emb':
                emb = nn.Embedding(n_in, n_out)
                nn.init.xavier_uniform_(emb.weight)
                self.encode_modules[name] = emb
        self.position_array = nn.Parameter(_denominator(TIME_DIM), requires_grad=False)
        # the reference registers the build-order transformer after the loop -> last in state_dict
        self.encode_modules['beginning_order'] = BeginningBuildOrderEncoder(64)

    def time_encoder(self, t: torch.Tensor, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        pos = self.position_array
        if out_dtype is not None and out_dtype != torch.float32:
            # bf16 inference: cos(a) = sin(a + pi/2), so one multiply-add and one sine that writes bf16 (was mul,
            # sin, cos, two strided copies and a cast: 6 launches); the fp32 phase add rounds far below bf16's step
            key = (pos.device, pos.shape[-1])
            ph = _TIME_PHASE.get(key)
            if ph is None:
                ph = _TIME_PHASE[key] = torch.zeros(pos.shape[-1], device=pos.device)
                ph[1::2] = math.pi / 2
            out = torch.empty(t.shape[0], pos.shape[-1], dtype=out_dtype, device=t.device)
            return torch.sin(torch.addcmul(ph, t.float().unsqueeze(1), pos), out=out)
        ang = t.float().unsqueeze(1) * pos
        out = torch.empty_like(ang)
        out[:, 0::2] = torch.sin(ang[:, 0::2])
        out[:, 1::2] = torch.cos(ang[:, 1::2])
        return out

    def forward(self, x: Dict[str, torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        embedded, context, baseline = [], [], []
        # actor inference under bf16 autocast: every piece in bf16 before the three concatenations (mixed fp32 / bf16
        # pieces made torch.cat promote all ~16 of them to fp32 - a cast launch each, profiles/r6m_timeline_*)
        lowp_inf = SCALAR_BF16_INFERENCE and torch.is_autocast_enabled() and not torch.is_grad_enabled() and \
            self.position_array.is_cuda
        if lowp_inf:
            from ..ops import native
        # the integer feature columns of the fc modules cast to the compute dtype in ONE multi-tensor launch (was a
        # cast launch per module: 6-7 per forward, in the actor's graph and in the learner step alike)
        pre = _cast_int_features(x, [name for name, kind, *_ in SCALAR_MODULES if kind not in ('emb', 'bo')])
        for name, kind, n_in, n_out, is_ctx, is_base in SCALAR_MODULES:
            m = self.encode_modules[name]
            if kind == 'emb':
                # row gather + ReLU: one native launch per direction for the small tables (the index in its stored
                # dtype, LDS-accumulated masked backward); last_action_type's 327 x 128 table gathers with
                # index_select - torch's embedding_dense_backward took 0.9 ms for 390 rows of last_delay
                e = ops.embed_relu(native._bf16w(m.weight) if lowp_inf else m.weight, x[name])
            elif kind == 'bo':
                e = m(x['beginning_order'], x['bo_location'])
                if lowp_inf:
                    e = e.to(torch.bfloat16)
            elif name in pre:
                e = m(pre[name])
            else:
                v = x[name]
                # integer feature columns: straight to the bf16 compute dtype under autocast (one cast; via fp32 it was
                # two launches per module - the linear casts its input anyway, and uint8 / int16 -> fp32 is exact)
                e = m(v.to(torch.bfloat16) if v.is_cuda and torch.is_autocast_enabled() and not v.is_floating_point()
                      else v.float())
            embedded.append(e)
            if is_ctx:
                context.append(e)
            if is_base:
                baseline.append(e)
        embedded.append(self.time_encoder(x['time'], torch.bfloat16) if lowp_inf else
                        self.time_encoder(x['time']).to(embedded[0].dtype))
        n = ops._native(embedded[0])
        if n is not None and n.has('col_assemble'):
            # the three concatenations in one launch, each module's gradient summed from its slices in one
            flags = [(True, c, b) for *_, c, b in SCALAR_MODULES] + [(True, False, False)]
            out = n.col_assemble(embedded, [[f[k] for f in flags] for k in range(3)])
            if out is not None:
                return out
        return torch.cat(embedded, 1), torch.cat(context, 1), torch.cat(baseline, 1)


def _cast_int_features(x: Dict[str, torch.Tensor], names) -> Dict[str, torch.Tensor]:
    """{name: x[name] in the compute dtype} for the integer (uint8 / int16) GPU feature columns among ``names``:
    bf16 under autocast, else fp32 (both exact for these ranges), all in one native multi-tensor copy; {} off the
    GPU or without the extension (the per-module casts stay)."""
    names = [n for n in names if n in x and x[n].is_cuda and x[n].dtype in (torch.uint8, torch.int16)
             and x[n].is_contiguous()]
    if len(names) < 2:
        return {}
    n = ops._native(x[names[0]])
    if n is None:
        return {}
    dt = torch.bfloat16 if torch.is_autocast_enabled() else torch.float32
    dst = [torch.empty(x[k].shape, dtype=dt, device=x[k].device) for k in names]
    n.ensure_loaded().multi_copy(dst, [x[k] for k in names])
    return dict(zip(names, dst))


def entity_field_layout() -> List[Tuple[str, str, int, int]]:
    """[(name, encoding, column offset into the 997-wide input, width)]."""
    out, off = [], 0
    for name, _, enc, width in ENTITY_FIELDS:
        out.append((name, enc, off, width))
        off += width
    return out


ENTITY_LAYOUT = entity_field_layout()


def entity_one_hot_input(entity_info: Dict[str, torch.Tensor], index: torch.Tensor, dtype) -> torch.Tensor:
    """Reference construction of the 997-wide entity input for the selected (packed) entity rows."""
    T = index.numel()
    x = torch.zeros(T, ENTITY_EMBED_DIM, dtype=dtype, device=index.device)
    rows = torch.arange(T, device=index.device)
    for name, enc, off, width in ENTITY_LAYOUT:
        v = entity_info[name].reshape(-1)[index]
        if enc == 'one_hot':
            x[rows, off + v.long().clamp(0, width - 1)] = 1
        elif enc == 'binary':
            bits = (v.long().unsqueeze(1) >> torch.arange(width - 1, -1, -1, device=v.device)) & 1
            x[:, off:off + width] = bits.to(dtype)
        else:
            x[:, off] = v.to(dtype)
    return x


class EntityEncoder(nn.Module):
    """Entity transformer (entity_encoder.py:20-96): 997 -> 256, 3 post-LN layers, 2 heads x 128."""

    def __init__(self, reduce_type: str = 'selected_units_num'):
        super().__init__()
        self.encode_modules = nn.ModuleDict()
        for name, enc, _, width in ENTITY_LAYOUT:
            if enc == 'one_hot':
                self.encode_modules[name] = OneHotTable(eye_table(width))
            elif enc == 'binary':
                self.encode_modules[name] = OneHotTable(binary_table(width))
        self.transformer = Transformer(ENTITY_EMBED_DIM, head_dim=128, hidden_dim=1024, output_dim=256, head_num=2,
                                       mlp_num=2, layer_num=3, ln_type='post')
        self.entity_fc = FCBlock(256, 256, act=True)
        self.embed_fc = FCBlock(256, 256, act=True)
        self.reduce_type = reduce_type
        if reduce_type.startswith('attention_pool'):  # entity_encoder.py:54-57
            from .optional import AttentionPool
            self.attention_pool = AttentionPool(256, 2, 256, max_num=MAX_ENTITY_NUM + 1
                                                if reduce_type == 'attention_pool_add_num' else None)
        elif reduce_type not in ('entity_num', 'selected_units_num', 'constant'):
            raise NotImplementedError(f'entity_reduce_type {reduce_type!r}')

    def embed(self, entity_info, flat_index):
        lin = self.transformer.embedding[0]
        n = ops._native(lin.weight) if flat_index.is_cuda else None
        if n is not None and n.has('entity_embed'):
            return n.entity_embed(entity_info, flat_index, lin.weight, lin.bias)
        x = entity_one_hot_input(entity_info, flat_index, lin.weight.dtype)
        return ops.linear(x, lin.weight, lin.bias, act='relu')

    def forward(self, entity_info: Dict[str, torch.Tensor], entity_num: torch.Tensor,
                entity_total: Optional[int] = None, entity_pad: Optional[int] = None):
        """``entity_total`` (optional host int = sum(min(entity_num, N))) lets the packing skip the
        host<->device sync of a data-dependent ``nonzero``; ``entity_pad`` (host int, a multiple of
        ``PAD_SEGMENTS * N`` at least the real count) packs to that fixed row count instead, so the
        step's shapes do not depend on the data (HIP-graph capture of the learner step)."""
        B, N = entity_info['unit_type'].shape
        padded = entity_pad is not None and not self.reduce_type.startswith('attention_pool')
        n = ops._native(entity_num) if entity_total is not None and not padded and \
            not (STATIC_SHAPES and entity_num.is_cuda) else None
        if n is not None and n.has('entity_pack'):
            # valid / packed -> padded rows / segments / offsets in one launch
            valid, flat_index, seg, cu = n.entity_pack(entity_num, N, int(entity_total))
        else:
            valid = ops.sequence_mask(entity_num, N)                     # [B,N]
            if STATIC_SHAPES and valid.is_cuda:
                return self._forward_static(entity_info, entity_num, valid)
            if padded:
                return self._forward_padded(entity_info, entity_num, valid, int(entity_pad))
            seg = None
            if entity_total is not None and valid.is_cuda:
                flat_index = torch.nonzero_static(valid.reshape(-1), size=int(entity_total)).squeeze(1)
            else:
                flat_index = valid.reshape(-1).nonzero().squeeze(1)     # packed row -> padded row
            lens = entity_num.clamp(max=N).to(torch.int32)
            cu = F.pad(torch.cumsum(lens, 0, dtype=torch.int32), (1, 0))
        x = self.embed(entity_info, flat_index)                      # [T,256]
        # the reference's inplace ReLU (entity_encoder.py:84), which also rectifies x used by the mean below,
        # applied by the transformer's closing LayerNorm kernel (no separate pass / mask pass over [T,256])
        x = self.transformer.forward_packed_embedded(x, cu, N, final_act='relu')      # [T,256]
        ee = self.entity_fc(x)
        entity_embeddings = ee.new_zeros(B * N, ee.shape[-1])
        entity_embeddings = entity_embeddings.index_copy(0, flat_index, ee).view(B, N, -1)
        # the packed rows behind the padded output, for a consumer that projects them directly (Encoder.forward)
        self._packed = (weakref.ref(entity_embeddings), ee, flat_index)
        if self.reduce_type.startswith('attention_pool'):
            xp = x.new_zeros(B * N, x.shape[-1]).index_copy(0, flat_index, x).view(B, N, -1)
            pooled = self.attention_pool(xp, num=entity_num, mask=valid)
            return entity_embeddings, self.embed_fc(pooled.to(x.dtype)), valid
        # masked mean of relu(transformer output) over real entities (entity_encoder.py:85-87)
        if seg is None:
            seg = torch.repeat_interleave(torch.arange(B, device=x.device), lens.long(), output_size=x.shape[0])
        summed = ops.segment_sum(x, cu, seg).to(x.dtype)
        if self.reduce_type == 'constant':
            mean = summed / 512
        else:
            mean = summed / entity_num.clamp(min=1).unsqueeze(1).to(summed.dtype)
        embedded_entity = self.embed_fc(mean)
        return entity_embeddings, embedded_entity, valid


    def _forward_padded(self, entity_info, entity_num, valid, T_pad: int):
        """Packed path at a fixed row count ``T_pad``: the real entities first (same order as the
        data-dependent packing), then ``T_pad - total`` padding rows that ride along as PAD_SEGMENTS
        extra attention segments of <= N rows each (so every row the kernels touch is a well-formed
        token and stays finite).  Padding rows gather entity row 0, scatter into a trash row and are
        dropped from the per-observation mean, so they receive zero gradient; real rows see exactly
        the packed path's math."""
        B, N = valid.shape
        P = PAD_SEGMENTS
        dev = valid.device
        gidx = torch.nonzero_static(valid.reshape(-1), size=T_pad, fill_value=0).squeeze(1)
        lens = entity_num.clamp(max=N).to(torch.int32)
        total = lens.sum()
        pad_lens = ((T_pad - total) - N * torch.arange(P, device=dev, dtype=torch.int32)).clamp(0, N)
        all_lens = torch.cat([lens, pad_lens.to(torch.int32)])
        cu = F.pad(torch.cumsum(all_lens, 0, dtype=torch.int32), (1, 0))
        rows = torch.arange(T_pad, device=dev)
        sidx = torch.where(rows < total, gidx, torch.full_like(gidx, B * N))
        x = self.embed(entity_info, gidx)                            # [T_pad,256]
        x = self.transformer.forward_packed_embedded(x, cu, N, final_act='relu')
        ee = self.entity_fc(x)
        entity_embeddings = ee.new_zeros(B * N + 1, ee.shape[-1]).index_copy(0, sidx, ee)[:B * N].view(B, N, -1)
        seg = torch.repeat_interleave(torch.arange(B + P, device=dev), all_lens.long(), output_size=T_pad)
        summed = ops.segment_sum(x, cu, seg)[:B].to(x.dtype)
        if self.reduce_type == 'constant':
            mean = summed / 512
        else:
            mean = summed / entity_num.clamp(min=1).unsqueeze(1).to(summed.dtype)
        return entity_embeddings, self.embed_fc(mean), valid

    def _forward_static(self, entity_info, entity_num, valid):
        """Shape-static variant for HIP-graph capture (inference): every padded slot is embedded and
        the transformer runs dense with a key mask (no data-dependent packing, no host sync).  Valid
        rows get the packed path's values; padded rows are zeroed like the packed path leaves them."""
        B, N = valid.shape
        flat_index = torch.arange(B * N, device=valid.device)
        h = self.embed(entity_info, flat_index).view(B, N, -1)
        # the native varlen attention over 2B segments (real rows | padding rows) instead of dense masked scores
        n = ops._native(h)
        cu = dense_segments(entity_num, N) if n is not None and n.has('varlen_attention') and DENSE_VARLEN and \
            self.transformer.layers[0].ln_type == 'post' else None
        for layer in self.transformer.layers:
            h = layer.forward_dense(h, valid, cu)
        x = F.relu(h)
        vm = valid.unsqueeze(-1).to(x.dtype)
        ee = self.entity_fc(x)
        entity_embeddings = ee * vm.to(ee.dtype)
        if self.reduce_type.startswith('attention_pool'):
            pooled = self.attention_pool(x * vm, num=entity_num, mask=valid)
            return entity_embeddings, self.embed_fc(pooled.to(x.dtype)), valid
        if n is not None and n.has('entity_mean_pool') and self.reduce_type != 'constant' and \
                not (torch.is_grad_enabled() and x.requires_grad):
            mean = n.entity_mean_pool(x, valid, entity_num)     # mask + sum + count + divide + cast in one launch
            if mean is not None:
                return entity_embeddings, self.embed_fc(mean), valid
        summed = (x * vm).sum(1, dtype=torch.float32)      # fp32 accumulation inside the reduce (no fp32 copy)
        if self.reduce_type == 'constant':
            mean = summed / 512
        else:
            mean = summed / entity_num.clamp(min=1).unsqueeze(1).to(summed.dtype)
        return entity_embeddings, self.embed_fc(mean.to(x.dtype)), valid


class SpatialEncoder(nn.Module):
    """spatial_encoder.py:9-90: 56 input planes -> 1x1 conv 32 -> 3x[maxpool2, conv3x3] (64,128,128)
    -> 4 ResBlocks(128) @19x20 -> fc 48640 -> 256. Returns (embedding, map_skip[7])."""

    def __init__(self):
        super().__init__()
        self.project = ConvBlock(56, 32, 1, act=True)
        self.encode_modules = nn.ModuleDict({k: OneHotTable(eye_table(n)) for k, n in SPATIAL_ONE_HOT})
        dims = [32, 64, 128, 128]
        self.downsample = nn.ModuleList([ConvBlock(dims[i], dims[i + 1], 3, 1, 1, act=True) for i in range(3)])
        self.res = nn.ModuleList([ResBlock(128) for _ in range(4)])
        self.fc = FCBlock(128 * (SPATIAL_Y // 8) * (SPATIAL_X // 8), 256, act=True)

    @staticmethod
    def input_planes(spatial_info, scatter_map):
        """Reference assembly of the 56 input planes [B,56,H,W] (spatial_encoder.py:51-70)."""
        planes = [spatial_info['height_map'].unsqueeze(1).float() / 256]
        for k, n in SPATIAL_ONE_HOT:
            planes.append(F.one_hot(spatial_info[k].long().clamp(0, n - 1), n).permute(0, 3, 1, 2).float())
        B = scatter_map.shape[0]
        for k in EFFECT_KEYS:
            m = torch.zeros(B, SPATIAL_Y * SPATIAL_X, device=scatter_map.device)
            m.scatter_(1, spatial_info[k].long().clamp(0, SPATIAL_Y * SPATIAL_X - 1), 1.0)
            planes.append(m.view(B, 1, SPATIAL_Y, SPATIAL_X))
        planes.append(scatter_map.float())
        return torch.cat(planes, 1)

    def forward(self, spatial_info, scatter_map):
        x = self.input_planes(spatial_info, scatter_map).to(self.project[0].weight.dtype)
        x = self.project(x)
        return self.trunk(x)

    def forward_native(self, spatial_info, proj, entity_x, entity_y, entity_num, native):
        """GPU path: input planes + entity scatter + 1x1 projection fused (ops.native.spatial_embed).
        The 1x1 conv is linear, so its 32 scatter-map columns are applied per entity *before* the
        scatter-add (W_s . sum_e p_e == sum_e W_s . p_e) and no 32-channel scatter map is built."""
        w = self.project[0].weight[:, :, 0, 0]                        # [32, 56]
        rows = ops.linear(proj, w[:, 24:])                            # [B,N,32]
        pooled = native.spatial_embed_pool(spatial_info, rows, entity_x, entity_y, entity_num, w[:, :24],
                                           self.project[0].bias) if native.has('spatial_embed_pool') else None
        if pooled is not None:
            return self.trunk(pooled, pooled_first=True)
        x = native.spatial_embed(spatial_info, rows, entity_x, entity_y, entity_num, w[:, :24], self.project[0].bias)
        return self.trunk(x)

    def trunk(self, x, pooled_first: bool = False):
        """``pooled_first``: x is already relu(embed) -> max_pool2x2 (the fused GPU stage), so the
        full-resolution map is never built and skip level 0 is None — no consumer reads levels 0-2 (the
        location head takes the last four)."""
        map_skip = []
        for i, conv in enumerate(self.downsample):
            if i == 0 and pooled_first:
                map_skip.append(None)
                x = conv(x)
                continue
            map_skip.append(x)
            x = conv(ops.max_pool2x2(x))
        for block in self.res:
            map_skip.append(x)
            x = block(x)
        x = self.fc(x.reshape(x.shape[0], -1))
        return x, map_skip


SCALAR_SIDE_STREAM = True
# the spatial scatter projection over the packed entity rows (APPLESTAR_PACKED_SCATTER=0: over the padded rows + mask);
# fp32 only: fp32 49.25 / 48.92 vs 49.23 / 49.31 ms, bf16 neutral within its noise (profiles/r10zm_bench_packed_scatter.txt)
PACKED_SCATTER = os.environ.get('APPLESTAR_PACKED_SCATTER', '1') == '1'
# bf16 inference: the scalar encoder's concatenated pieces kept in bf16 (APPLESTAR_SCALAR_BF16_INFERENCE=0: as trained)
SCALAR_BF16_INFERENCE = os.environ.get('APPLESTAR_SCALAR_BF16_INFERENCE', '1') == '1'
# set by runtime.graphs.GraphedPolicy while capturing / replaying: shape-static entity path
STATIC_SHAPES = False
# static (graph-captured) entity path: attention on the native varlen kernel over 2B segments
DENSE_VARLEN = os.environ.get('APPLESTAR_DENSE_VARLEN', '1') == '1'
# padded packing (EntityEncoder._forward_padded): the padding rows form this many extra segments
PAD_SEGMENTS = 8


def entity_pad_for(total: int, n: int) -> int:
    """Fixed packed row count for ``total`` real entities at padded width ``n``: the next multiple of
    PAD_SEGMENTS * n (so the padding always fits the PAD_SEGMENTS extra segments of <= n rows)."""
    g = PAD_SEGMENTS * max(int(n), 1)
    return max(1, (int(total) + g - 1) // g) * g


class Encoder(nn.Module):
    def __init__(self, reduce_type: str = 'selected_units_num'):
        super().__init__()
        self.scalar_encoder = ScalarEncoder()
        self.spatial_encoder = SpatialEncoder()
        self.entity_encoder = EntityEncoder(reduce_type)
        self.scatter_project = FCBlock(256, 32, act=True)

    def forward(self, spatial_info, entity_info, scalar_info, entity_num, entity_total: Optional[int] = None,
                entity_pad: Optional[int] = None):
        # the scalar encoder (incl. the 20-token build-order transformer: many small kernels) is independent
        # of the entity / spatial path: side stream 1 on the GPU (its backward follows it there)
        from .model import _side_stream_call, _side_stream_join
        scalar_h = _side_stream_call(self.scalar_encoder, scalar_info, slot=1) if SCALAR_SIDE_STREAM else \
            (self.scalar_encoder(scalar_info), None)
        entity_embeddings, embedded_entity, entity_mask = self.entity_encoder(entity_info, entity_num, entity_total,
                                                                              entity_pad)
        pk, self.entity_encoder._packed = getattr(self.entity_encoder, '_packed', None), None
        if PACKED_SCATTER and pk is not None and pk[0]() is entity_embeddings and not torch.is_autocast_enabled():
            # the scatter projection over the packed entity rows, zero-padded afterwards (its padded rows were masked
            # to zero anyway): half the rows of the GEMMs, and the padded 256-wide embeddings then have one consumer
            # in training (the heads' keys), so autograd sums no two [B * N, 256] input gradients
            B, N = entity_embeddings.shape[:2]
            p = self.scatter_project(pk[1])
            proj = p.new_zeros(B * N, p.shape[-1]).index_copy(0, pk[2], p).view(B, N, -1)
        else:
            proj = self.scatter_project(entity_embeddings) * entity_mask.unsqueeze(2).to(entity_embeddings.dtype)
        n = ops._native(proj) if proj.is_cuda else None
        if n is not None and n.has('spatial_embed'):
            embedded_spatial, map_skip = self.spatial_encoder.forward_native(
                spatial_info, proj, entity_info['x'], entity_info['y'], entity_num, n)
        else:
            scatter_map = ops.scatter_connection(proj, entity_info['x'], entity_info['y'], SPATIAL_Y, SPATIAL_X)
            embedded_spatial, map_skip = self.spatial_encoder(spatial_info, scatter_map)
        embedded_scalar, scalar_context, baseline_feature = _side_stream_join(scalar_h)
        lstm_input = torch.cat([embedded_scalar, embedded_entity.to(embedded_scalar.dtype),
                                embedded_spatial.to(embedded_scalar.dtype)], dim=-1)
        return lstm_input, scalar_context, baseline_feature, entity_embeddings, map_skip


VALUE_FC_MODULES = [('enemy_unit_counts_bow', gd.NUM_UNIT_TYPES, 64), ('enemy_unit_type_bool', gd.NUM_UNIT_TYPES, 64),
                    ('enemy_agent_statistics', 10, 64), ('enemy_upgrades', gd.NUM_UPGRADES, 32),
                    ('cumulative_stat', gd.NUM_CUMULATIVE_STAT_ACTIONS, 128)]


class ValueEncoder(nn.Module):
    """Opponent-aware critic features -> [B,544] (value_encoder.py:12-74)."""

    def __init__(self):
        super().__init__()
        self.encode_modules = nn.ModuleDict()
        for name, n_in, n_out in VALUE_FC_MODULES[:4]:
            self.encode_modules[name] = FCBlock(n_in, n_out, act=True)
        self.encode_modules['unit_alliance'] = nn.Embedding(2, 16)
        self.encode_modules['unit_type'] = nn.Embedding(gd.NUM_UNIT_TYPES, 48)
        self.encode_modules['beginning_order'] = BeginningBuildOrderEncoder(64)
        name, n_in, n_out = VALUE_FC_MODULES[4]
        self.encode_modules[name] = FCBlock(n_in, n_out, act=True)
        self.scatter_project = FCBlock(64, 8, act=True)
        self.project = ConvBlock(10, 16, 1, act=True)
        dims = [16, 16, 32, 32]
        layers = []
        for i in range(3):
            layers += [MaxPool2x2(), ConvBlock(dims[i], dims[i + 1], 3, 1, 1, act=True)]
        self.downsample = nn.Sequential(*layers)
        self.res = nn.ModuleList([ResBlock(32) for _ in range(4)])
        self.spatial_fc = FCBlock(32 * (SPATIAL_Y // 8) * (SPATIAL_X // 8), 128, act=True)

    def forward(self, x):
        fc = [self.encode_modules[n](x[n].float()) for n, _, _ in VALUE_FC_MODULES]
        bo = self.encode_modules['beginning_order'](x['beginning_order'], x['bo_location'])
        # scatter_project(cat(E_a[alliance], E_t[type])) == relu(T_a[alliance] + T_t[type] + b) with the
        # per-table projections T = E @ W_slice^T folded first: the gather (and its backward, an index_add
        # of 8-wide rows instead of a sort-based 64-wide embedding backward over ~2e5 units) shrinks 8x
        lin = self.scatter_project[0]
        ea, et = self.encode_modules['unit_alliance'].weight, self.encode_modules['unit_type'].weight
        ta = ea @ lin.weight[:, :ea.shape[1]].t()
        tt = et @ lin.weight[:, ea.shape[1]:].t()
        ia = x['unit_alliance'].long().reshape(-1)
        it = x['unit_type'].long().clamp(0, gd.NUM_UNIT_TYPES - 1).reshape(-1)
        pre = ops.gather_rows(tt, it) + ops.gather_rows(ta, ia) + lin.bias.to(tt.dtype)
        proj = torch.relu(pre).view(*x['unit_type'].shape, -1)
        U = proj.shape[1]
        mask = ops.sequence_mask(x['total_unit_count'], U)
        proj = proj * mask.unsqueeze(2).to(proj.dtype)
        H, W = x['own_units_spatial'].shape[-2:]
        sc = ops.scatter_connection(proj, x['unit_x'], x['unit_y'], H, W)
        c = self.project[0]
        pooled = ops.value_spatial_proj_pool(sc, x['own_units_spatial'], x['enemy_units_spatial'], c.weight, c.bias) \
            if sc.is_cuda and isinstance(self.downsample[0], MaxPool2x2) else None
        fused = None if pooled is not None or not sc.is_cuda else \
            ops.value_spatial_proj(sc, x['own_units_spatial'], x['enemy_units_spatial'], c.weight, c.bias)
        if pooled is not None:
            sp = pooled          # = downsample[0](projection): the first pool is fused into the projection
        elif fused is not None:
            sp = fused
        elif sc.is_cuda:
            # assembled directly in NHWC, zero-padded 10 -> 16 channels (with a zero-padded 1x1 weight) so
            # the 9.5M-row 1x1 conv's weight gradient takes the split-R MFMA kernel (K % 8 == 0)
            B_ = sc.shape[0]
            own = x['own_units_spatial'].to(proj.dtype).reshape(B_, H, W, 1)
            enemy = x['enemy_units_spatial'].to(proj.dtype).reshape(B_, H, W, 1)
            pad = own.new_zeros(B_, H, W, 6)
            sp = torch.cat([sc.to(proj.dtype).permute(0, 2, 3, 1), own, enemy, pad], -1).permute(0, 3, 1, 2)
            sp = ops.conv2d(sp, torch.nn.functional.pad(c.weight, (0, 0, 0, 0, 0, 6)), c.bias, 1, 0, act='relu')
        else:
            sp = torch.cat([sc.to(proj.dtype), x['own_units_spatial'].to(proj.dtype),
                            x['enemy_units_spatial'].to(proj.dtype)], 1)
            sp = self.project(sp)
        sp = self.downsample[1:](sp) if pooled is not None else self.downsample(sp)
        for blk in self.res:
            sp = blk(sp)
        sp = self.spatial_fc(sp.reshape(sp.shape[0], -1))
        fc_cat = torch.cat(fc, -1)
        return torch.cat([fc_cat, sp.to(fc_cat.dtype), bo.to(fc_cat.dtype)], -1)
