"""Native HIP kernels vs plain-PyTorch fp32 references (run on an MI355X)."""
import os

import pytest
import torch

from applestar_amd.ops import reference as R
from applestar_amd.ops import native as N

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(scope='module', autouse=True)
def _load():
    N.ensure_loaded()


def _err(a, b):
    return (a.float() - b.float()).abs().max().item()


@pytest.mark.parametrize('cols', [64, 256, 384, 1536])
@pytest.mark.parametrize('x_dtype,res_dtype', [(torch.float32, None), (torch.bfloat16, torch.float32),
                                               (torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32)])
@pytest.mark.parametrize('act', [None, 'relu'])
def test_layer_norm_matches_reference(cols, x_dtype, res_dtype, act):
    torch.manual_seed(0)
    rows = 1031
    x = torch.randn(rows, cols, device=DEV).to(x_dtype).requires_grad_()
    res = torch.randn(rows, cols, device=DEV).to(res_dtype).requires_grad_() if res_dtype else None
    w = (1 + 0.1 * torch.randn(cols, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(cols, device=DEV)).requires_grad_()
    y = N.layer_norm(x, w, b, residual=res, act=act)
    xr = x.detach().float().requires_grad_()
    rr = res.detach().float().requires_grad_() if res is not None else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = R.layer_norm(xr, wr, br, rr, act)
    assert _err(y, yr) < 2e-5 * 10
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g)
    tol = 3e-2 if x_dtype == torch.bfloat16 else 1e-4
    assert _err(x.grad, xr.grad) < tol * max(1.0, xr.grad.abs().max().item())
    if res is not None:
        assert _err(res.grad, rr.grad) < tol * max(1.0, rr.grad.abs().max().item())
    assert _err(w.grad, wr.grad) < 1e-3 * max(1.0, wr.grad.abs().max().item())
    assert _err(b.grad, br.grad) < 1e-3 * max(1.0, br.grad.abs().max().item())


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_gated_residual(dtype):
    torch.manual_seed(1)
    shape = (5, 128, 19, 20)
    y, g, x = (torch.randn(shape, device=DEV).to(dtype).requires_grad_() for _ in range(3))
    sp = torch.full((1,), 0.1, device=DEV, requires_grad=True)
    out = N.gated_residual(y, g, sp, x)
    ys, gs, xs = (t.detach().float().requires_grad_() for t in (y, g, x))
    sps = sp.detach().clone().requires_grad_()
    ref = R.gated_residual(ys, gs, sps, xs)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _err(out, ref) < tol
    d = torch.randn_like(ref).to(dtype)
    out.backward(d)
    ref.backward(d.float())
    for a, b in ((y.grad, ys.grad), (g.grad, gs.grad), (x.grad, xs.grad)):
        assert _err(a, b) < tol * 4
    # d(sp) is a sum of ~2.4e5 signed terms: bound the error by the sum of |terms|
    mag = (d.float().abs() * torch.tanh(ys * torch.sigmoid(gs)).abs()).sum().item()
    assert abs(sp.grad.item() - sps.grad.item()) < 1e-3 * mag


def test_reverse_scan():
    torch.manual_seed(2)
    K, T, B = 6, 64, 6
    a = torch.rand(K, T, B, device=DEV)
    b = torch.randn(K, T, B, device=DEV)
    init = torch.randn(K, B, device=DEV)
    y = N.reverse_scan(a, b, init)
    ref = torch.empty_like(b)
    acc = init.clone()
    for t in range(T - 1, -1, -1):
        acc = a[:, t] * acc + b[:, t]
        ref[:, t] = acc
    assert _err(y, ref) < 1e-5


@pytest.mark.parametrize('H,I,T,B', [(384, 1536, 9, 6), (384, 384, 65, 16), (384, 1536, 3, 20), (32, 32, 13, 37)])
@pytest.mark.parametrize('autocast', [False, True])
def test_lnlstm_layer_matches_reference(H, I, T, B, autocast):
    # H = 384, B <= 16 runs the split (8 workgroups per row, cross-workgroup all-reduce) recurrence;
    # B = 20 the one-workgroup-per-row kernel
    if autocast and T > 16:
        pytest.skip('bf16 weights vs the fp32 oracle diverge chaotically over long sequences; fp32 covers T=65')
    torch.manual_seed(3)
    x = torch.randn(T, B, I, device=DEV, requires_grad=True)
    h0 = (0.5 * torch.randn(B, H, device=DEV)).requires_grad_()
    c0 = (0.5 * torch.randn(B, H, device=DEV)).requires_grad_()
    params = [torch.randn(4 * H, I, device=DEV) / I ** 0.5, torch.randn(4 * H, H, device=DEV) / H ** 0.5,
              1 + 0.1 * torch.randn(4 * H, device=DEV), 0.1 * torch.randn(4 * H, device=DEV),
              1 + 0.1 * torch.randn(4 * H, device=DEV), 0.1 * torch.randn(4 * H, device=DEV),
              1 + 0.1 * torch.randn(H, device=DEV), 0.1 * torch.randn(H, device=DEV)]
    params = [p.requires_grad_() for p in params]
    ref_in = [t.detach().clone().requires_grad_() for t in [x, h0, c0] + params]
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        out, hT, cT = N.lnlstm_layer(x, h0, c0, *params)
    r_out, r_h, r_c = R.lnlstm_layer(*ref_in)
    tol = 5e-2 if autocast else 2e-4
    assert _err(out, r_out) < tol
    assert _err(cT, r_c) < tol * 4
    g = torch.randn_like(r_out)
    gh = torch.randn_like(r_h)
    (out * g).sum().add_((hT * gh).sum()).backward()
    (r_out * g).sum().add_((r_h * gh).sum()).backward()
    for a, b in zip([x, h0, c0] + params, ref_in):
        scale = max(1.0, b.grad.abs().max().item())
        assert _err(a.grad, b.grad) < tol * 4 * scale
    torch.cuda.synchronize()
    assert int(N.ensure_loaded().lstm_split_error(0).item()) == 0, 'split LSTM exchange timed out'


@pytest.mark.parametrize('autocast', [False, True])
def test_entity_embed_matches_one_hot_linear(autocast):
    from applestar_amd.lib.features import random_obs
    from applestar_amd.models.encoders import entity_one_hot_input
    torch.manual_seed(4)
    obs = random_obs(5, max_entities=70, generator=torch.Generator().manual_seed(4))
    info = {k: v.cuda() for k, v in obs['entity_info'].items()}
    en = obs['entity_num'].cuda()
    n_ent = info['unit_type'].shape[1]
    idx = (torch.arange(n_ent, device=DEV)[None] < en[:, None]).reshape(-1).nonzero().squeeze(1)
    w = (torch.randn(256, 997, device=DEV) * 0.05).requires_grad_()
    b = (torch.randn(256, device=DEV) * 0.1).requires_grad_()
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        out = N.entity_embed(info, idx, w, b)
    X = entity_one_hot_input(info, idx, torch.float32)
    ref = torch.relu(X @ wr.t() + br)
    tol = 3e-2 if autocast else 1e-4
    assert _err(out, ref) < tol * max(1, ref.abs().max().item())
    g = torch.randn_like(ref)
    out.backward(g.to(out.dtype))
    # relu-boundary flips between bf16 and fp32 pre-activations are not kernel errors: take the
    # mask from the native output and check dW = dpre^T X, db = sum dpre exactly against fp32
    dpre = g * (out.float() > 0)
    assert _err(w.grad, dpre.t() @ X) < tol * max(1, (dpre.t() @ X).abs().max().item())
    assert _err(b.grad, dpre.sum(0)) < tol * max(1, dpre.sum(0).abs().max().item())


@pytest.mark.parametrize('C,H,W', [(128, 19, 20), (32, 76, 80), (4, 3, 5)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_upsample2x_matches_interpolate(C, H, W, dtype):
    torch.manual_seed(5)
    x = torch.randn(3, C, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    xr = x.detach().float().requires_grad_()
    y = N.upsample2x(x)
    yr = torch.nn.functional.interpolate(xr, scale_factor=2.0, mode='bilinear', align_corners=False)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _err(y, yr) < tol
    g = torch.randn_like(yr).to(dtype)
    y.backward(g)
    yr.backward(g.float())
    assert _err(x.grad, xr.grad) < tol * 4


@pytest.mark.parametrize('autocast', [False, True])
def test_spatial_embed_matches_reference_planes(autocast):
    from applestar_amd.lib.features import random_obs
    from applestar_amd.models.encoders import SpatialEncoder
    from applestar_amd.ops.reference import scatter_connection
    torch.manual_seed(6)
    obs = random_obs(3, max_entities=40, generator=torch.Generator().manual_seed(6))
    sp = {k: v.cuda() for k, v in obs['spatial_info'].items()}
    ent = {k: v.cuda() for k, v in obs['entity_info'].items()}
    en = obs['entity_num'].cuda()
    B, Nn = ent['x'].shape
    proj = torch.relu(torch.randn(B, Nn, 32, device=DEV))
    proj = proj * (torch.arange(Nn, device=DEV)[None] < en[:, None]).unsqueeze(2)
    w = (torch.randn(32, 56, device=DEV) * 0.2).requires_grad_()
    b = (torch.randn(32, device=DEV) * 0.1).requires_grad_()
    proj = proj.requires_grad_()
    wr, br, pr = (t.detach().clone().requires_grad_() for t in (w, b, proj))
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
        rows = torch.nn.functional.linear(proj, w[:, 24:])
        out = N.spatial_embed(sp, rows, ent['x'], ent['y'], en, w[:, :24], b)
    smap = scatter_connection(pr, ent['x'], ent['y'], 152, 160)
    planes = SpatialEncoder.input_planes(sp, smap)
    pre = torch.nn.functional.conv2d(planes, wr[:, :, None, None], br)
    ref = torch.relu(pre)
    tol = 5e-2 if autocast else 1e-4
    assert _err(out, ref) < tol * max(1, ref.abs().max().item())
    g = torch.randn_like(ref)
    out.backward(g.to(out.dtype))
    # gradients through the ReLU mask the kernel actually applied (bf16 flips values near 0)
    (pre * (out.detach().float() > 0)).backward(g)
    # padded entity rows are never scattered by the native kernel (the model masks them before the
    # projection anyway), so only the valid rows carry a gradient
    valid = (torch.arange(Nn, device=DEV)[None] < en[:, None]).unsqueeze(2)
    for a, r in ((w.grad, wr.grad), (b.grad, br.grad), (proj.grad, pr.grad * valid)):
        assert _err(a, r) < tol * max(1, r.abs().max().item()) * 2


@pytest.mark.parametrize('fp32', [False, True], ids=['bf16', 'fp32'])
@pytest.mark.parametrize('crowded', [False, True])
def test_spatial_embed_partial_tile(crowded, fp32):
    """Map sizes that are not a multiple of the kernels' 256-pixel tile (odd pixel count: the last
    tile is partial and its pixel pairs straddle the end) against an fp32 reference of the planes.
    crowded: 300 entities inside the first tile (more than its 256-entry compacted list).  fp32: the fp32 step's
    kernels (the weight gradient on three exact bf16 parts of dpre against the exact-in-bf16 planes), held to 1e-5."""
    from applestar_amd.lib.features import SPATIAL_ONE_HOT, EFFECT_KEYS
    torch.manual_seed(11)
    B, H, W, Nn, L = 3, 37, 45, (300 if crowded else 9), 5
    sp = {'height_map': torch.randint(0, 256, (B, H, W), device=DEV, dtype=torch.uint8)}
    for k, n in SPATIAL_ONE_HOT:
        sp[k] = torch.randint(0, n + 1, (B, H, W), device=DEV, dtype=torch.uint8)   # n -> clamped to n-1
    for k in EFFECT_KEYS:
        sp[k] = torch.randint(0, H * W, (B, L), device=DEV, dtype=torch.int16)
    ex = torch.randint(0, 8 if crowded else W, (B, Nn), device=DEV)
    ey = torch.randint(0, 3 if crowded else H, (B, Nn), device=DEV)
    en = torch.tensor([Nn, 4, 0], device=DEV)
    rows = torch.randn(B, Nn, 32, device=DEV) * (torch.arange(Nn, device=DEV)[None] < en[:, None]).unsqueeze(2)
    w = (torch.randn(32, 24, device=DEV) * 0.3).requires_grad_()
    b = (torch.randn(32, device=DEV) * 0.1).requires_grad_()
    if fp32:
        out = N.spatial_embed(sp, rows, ex, ey, en, w, b)
    else:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = N.spatial_embed(sp, rows.to(torch.bfloat16), ex, ey, en, w, b)
    rows_ref = rows if fp32 else rows.to(torch.bfloat16).float()
    tol = 1e-5 if fp32 else 2e-2
    planes = [sp['height_map'].float().unsqueeze(1) / 256]
    for k, n in SPATIAL_ONE_HOT:
        planes.append(torch.nn.functional.one_hot(sp[k].long().clamp(0, n - 1), n).permute(0, 3, 1, 2).float())
    for k in EFFECT_KEYS:
        m = torch.zeros(B, H * W, device=DEV)
        m.scatter_(1, sp[k].long(), 1.0)
        planes.append(m.view(B, 1, H, W))
    X = torch.cat(planes, 1)                                                      # [B,24,H,W]
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    pre = torch.einsum('bkhw,nk->bnhw', X, wr) + br[None, :, None, None]
    ent = torch.zeros(B, 32, H, W, device=DEV)
    for i in range(B):
        for j in range(int(en[i])):
            ent[i, :, ey[i, j], ex[i, j]] += rows_ref[i, j]
    pre = pre + ent
    ref = torch.relu(pre)
    assert _err(out, ref) < tol * max(1, ref.abs().max().item())
    # channels_last gradient: the NHWC-contiguous dout takes the fused ReLU-gate path of the backward
    # (the NCHW gradient of test_spatial_embed_matches_reference_planes takes the act_grad path)
    g = torch.randn_like(ref).contiguous(memory_format=torch.channels_last)
    out.backward(g.to(out.dtype))
    (pre * (out.detach().float() > 0)).backward(g if fp32 else g.to(torch.bfloat16).float())
    assert _err(w.grad, wr.grad) < tol * max(1, wr.grad.abs().max().item())
    assert _err(b.grad, br.grad) < tol * max(1, br.grad.abs().max().item())


@pytest.mark.parametrize('lens', [[1, 64, 65, 200, 511], [37], [128, 3, 300]])
def test_varlen_attention_matches_reference(lens):
    torch.manual_seed(7)
    H, Dh = 2, 128
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    qkv = (torch.randn(T, 3 * H * Dh, device=DEV) * 0.5).to(torch.bfloat16).requires_grad_()
    ref_in = qkv.detach().float().requires_grad_()
    out = N.varlen_attention(qkv, cu, max(lens), H, Dh)
    ref = R.varlen_attention(ref_in, cu, max(lens), H, Dh)
    assert _err(out, ref) < 2e-2
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    scale = ref_in.grad.abs().max().item()
    assert _err(qkv.grad, ref_in.grad) < 3e-2 * max(1.0, scale)


@pytest.fixture(params=[23, 0, 1, 9], ids=['img_default', 'perwave', 'img_pf_rawv', 'img_dq_nopf'])
def attn_variant(request):
    """fp32 attention split-path variant (attention_f32.hip attn_f32_variant): pre-split LDS images (default) and
    its forward / dQ forms, or the per-wave split kernels"""
    C = N.ensure_loaded()
    old = C.attn_f32_variant(request.param)
    yield request.param
    C.attn_f32_variant(old)


@pytest.mark.parametrize('lens', [[1, 64, 65, 200, 511], [37], [128, 3, 300]])
@pytest.mark.parametrize('score_scale', [0.5, 2.0])
def test_varlen_attention_fp32_matches_fp64(lens, score_scale, f32_mfma, attn_variant):
    """fp32 operands take the f32-MFMA kernel (attention_f32.hip), never a bf16 copy: forward and all three
    input gradients within fp32 rounding of a float64 reference."""
    torch.manual_seed(11)
    H, Dh = 2, 128
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    qkv = (torch.randn(T, 3 * H * Dh, device=DEV) * score_scale).requires_grad_()
    ref_in = qkv.detach().double().cpu().requires_grad_()
    out = N.varlen_attention(qkv, cu, max(lens), H, Dh)
    assert out.dtype == torch.float32
    ref = R.varlen_attention(ref_in, cu.cpu(), max(lens), H, Dh)
    assert _err(out.cpu(), ref) < 2e-5 * max(1.0, ref.abs().max().item())
    g = torch.randn(ref.shape, dtype=torch.float64)
    out.backward(g.float().to(DEV))
    ref.backward(g)
    scale = ref_in.grad.abs().max().item()
    err = (qkv.grad.double().cpu() - ref_in.grad).abs()
    assert err.max().item() < 5e-5 * max(1.0, scale), err.max().item()
    # relative Frobenius over each of q / k / v
    for part in range(3):
        sl = slice(part * H * Dh, (part + 1) * H * Dh)
        rel = err[:, sl].norm() / ref_in.grad[:, sl].norm().clamp_min(1e-30)
        assert rel.item() < 1e-5, (part, rel.item())


def test_su_sample_kernel_matches_teacher_forcing_and_torch_sampler():
    """Persistent pointer-network sampler: its logits must equal the teacher-forced logits of the
    units it picked, its picks must follow inverse-CDF sampling of those logits, and (fp32) it should
    pick the same units as the step-by-step torch loop given the same uniforms."""
    from applestar_amd import ops
    from applestar_amd.models.heads import SelectedUnitsHead, sample_from_logits
    torch.manual_seed(11)
    head = SelectedUnitsHead(extra_units=True).to(DEV).eval()
    B, N = 12, 70
    ae0 = torch.randn(B, 1024, device=DEV)
    ent = torch.randn(B, N, 256, device=DEV)
    en = torch.tensor([70, 1, 5, 33, 64, 69, 2, 40, 10, 70, 17, 50], device=DEV)
    su_mask = torch.tensor([1, 1, 1, 1, 0, 1, 1, 1, 1, 1, 0, 1], device=DEV).bool()
    u = torch.rand(B, 64, device=DEV)
    with torch.no_grad():
        lg, res, ae, su_num, extra = head.forward_sample(ae0, ent, en, su_mask, 1.0, u=u)
        assert lg.shape == (B, 64, N + 1) and res.shape == (B, 64)
        assert (su_num[~su_mask] == 0).all() and (su_num[su_mask] >= 2).all()
        for b in range(B):
            s = int(su_num[b])
            if s:
                assert int(res[b, s - 1]) == int(en[b])            # ended with the end token
                assert len(set(res[b, :s - 1].tolist())) == s - 1  # no unit twice
                # each pick is the inverse-CDF sample of its own logits row
                pick = sample_from_logits(lg[b, :s, :int(en[b]) + 1], u[b, :s])
                assert torch.equal(pick, res[b, :s])
        lt, _, ae_t, _ = head.forward_teacher(ae0, ent, en, su_num, res)
        for b in range(B):
            s, n1 = int(su_num[b]), int(en[b]) + 1
            if s:
                a, r = lg[b, :s, :n1], lt[b, :s, :n1]
                valid = r > -1e8
                assert torch.equal(valid, a > -1e8)
                assert (a[valid] - r[valid]).abs().max() < 2e-2 * max(1.0, r[valid].abs().max().item())
        rows = su_num > 0  # rows without a unit selection keep ae0 + embed(0) (not teacher-forced labels)
        assert (ae[rows] - ae_t[rows]).abs().max() < 2e-2 * ae_t[rows].abs().max()
        # step-by-step torch loop with the same noise
        ops.set_native(False)
        try:
            lg2, res2, ae2, su2, _ = head.forward_sample(ae0, ent, en, su_mask, 1.0, u=u)
        finally:
            ops.set_native(True)
        same = sum(int(torch.equal(res[b, :int(su_num[b])], res2[b, :int(su2[b])])) for b in range(B))
        assert same >= B - 1, (same, B)


@pytest.mark.parametrize('H,W,dtype', [(76, 80, torch.float32), (76, 80, torch.bfloat16), (5, 9, torch.float32),
                                       (1, 1, torch.float32)])
def test_upsample_conv_out_matches_interpolate_conv(H, W, dtype):
    """Fused bilinear x2 + conv3x3 (32 -> 1) vs F.interpolate + F.conv2d in fp32: output, dx, dw, db."""
    torch.manual_seed(11)
    B = 3
    x = torch.randn(B, 32, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    w = (torch.randn(1, 32, 3, 3, device=DEV) * 0.2).requires_grad_()
    b = (torch.randn(1, device=DEV) * 0.1).requires_grad_()
    xr, wr, br = (t.detach().float().clone().requires_grad_() for t in (x, w, b))
    y = N.upsample_conv_out(x, w, b)
    up = torch.nn.functional.interpolate(xr, scale_factor=2.0, mode='bilinear', align_corners=False)
    yr = torch.nn.functional.conv2d(up, wr, br, padding=1).reshape(B, -1)
    assert y.shape == yr.shape and y.dtype == torch.float32
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    assert _err(y, yr) < tol
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    rel = lambda a, r: _err(a, r) / max(1.0, r.abs().max().item())
    assert rel(x.grad.float(), xr.grad) < tol * 10
    assert rel(w.grad, wr.grad) < tol * 10
    assert rel(b.grad, br.grad) < tol * 10


@pytest.mark.parametrize('C,H,W', [(32, 152, 160), (128, 38, 40), (16, 19, 21)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_maxpool2x2_matches_torch(C, H, W, dtype):
    torch.manual_seed(5)
    x = torch.randn(3, C, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    x[0, :, :2, :2] = 0.5  # ties resolve to the first window position, like torch
    xr = x.detach().clone().requires_grad_()
    x.requires_grad_()
    y = N.maxpool2x2(x)
    yr = torch.nn.functional.max_pool2d(xr, 2, 2)
    assert torch.equal(y, yr)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    assert torch.equal(x.grad, xr.grad)


def test_segment_sum_and_gather_rows():
    torch.manual_seed(6)
    lens = torch.tensor([5, 0, 300, 1, 77], device=DEV)
    cu = torch.nn.functional.pad(torch.cumsum(lens, 0), (1, 0)).int()
    T = int(lens.sum())
    seg = torch.repeat_interleave(torch.arange(5, device=DEV), lens)
    for dtype in (torch.float32, torch.bfloat16):
        x = torch.randn(T, 256, device=DEV).to(dtype).requires_grad_()
        out = N.segment_sum(x, cu, seg)
        ref = torch.zeros(5, 256, device=DEV).index_add(0, seg, x.float())
        assert _err(out, ref) < 1e-3
        g = torch.randn_like(out)
        out.backward(g)
        assert _err(x.grad, g[seg]) < 1e-2
    for V, D, U in [(260, 8, 200000), (2, 8, 200000), (7, 3, 11)]:
        table = torch.randn(V, D, device=DEV, requires_grad=True)
        idx = torch.randint(0, V, (U,), device=DEV)
        y = N.gather_rows(table, idx)
        assert torch.equal(y, table[idx])
        g = torch.randn(U, D, device=DEV)
        y.backward(g)
        ref = torch.zeros(V, D, device=DEV, dtype=torch.float64).index_add(0, idx, g.double())
        assert (table.grad.double() - ref).abs().max().item() < 1e-3 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize('cin,cout,H,W', [(128, 128, 19, 20), (32, 64, 76, 80), (64, 128, 38, 40),
                                          (128, 64, 38, 40), (64, 32, 19, 21), (32, 32, 7, 5), (256, 128, 9, 9),
                                          (16, 16, 38, 40), (16, 32, 19, 20), (32, 16, 11, 13), (16, 64, 7, 9),
                                          (64, 32, 76, 80), (64, 32, 19, 20), (64, 64, 30, 62)])
@pytest.mark.parametrize('act,res', [(None, False), ('relu', False), ('relu', True)])
def test_conv3x3_mfma_matches_fp32(cin, cout, H, W, act, res):
    from applestar_amd import ops
    torch.manual_seed(7)
    B = 3
    cl = torch.channels_last
    x = torch.randn(B, cin, H, W, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl).requires_grad_()
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (3 * cin ** 0.5)).to(torch.bfloat16)
    w = w.contiguous(memory_format=cl).requires_grad_()
    b = (0.1 * torch.randn(cout, device=DEV)).to(torch.bfloat16).requires_grad_()
    r = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl).requires_grad_() \
        if res else None
    y = ops.conv2d(x, w, b, 1, 1, act=act, residual=r)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=cl)
    xs, ws, bs = (t.detach().float().requires_grad_() for t in (x, w, b))
    rs = r.detach().float().requires_grad_() if res else None
    yr = torch.nn.functional.conv2d(xs, ws, bs, 1, 1)
    if res:
        yr = yr + rs
    if act == 'relu':
        yr = torch.relu(yr)
    assert _err(y, yr) < 2e-2 * max(1.0, yr.abs().max().item())
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    for a, ref in ((x.grad, xs.grad), (w.grad, ws.grad), (b.grad, bs.grad)) + (((r.grad, rs.grad),) if res else ()):
        assert _err(a, ref) < 3e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize('cin,cout,H,W', [(128, 128, 19, 20), (64, 128, 38, 40), (32, 32, 38, 40), (128, 64, 9, 9)])
def test_conv3x3_few_tiles(cin, cout, H, W):
    """The actor's B = 1 convs (few output tiles: 32-wide N tiles, 128-wide K-steps when Cin % 128 == 0) against
    an fp32 conv with bias + residual + ReLU; repeated calls give identical outputs."""
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(3)
    x = torch.randn(1, H, W, cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, 3, 3, cin, device=DEV) / (3 * cin ** 0.5)).to(torch.bfloat16)
    b = 0.1 * torch.randn(cout, device=DEV)
    r = torch.randn(1, H, W, cout, device=DEV).to(torch.bfloat16)
    y = C.conv3x3_fwd(x, w, b, r, 1)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    ref = torch.relu(ref.permute(0, 2, 3, 1) + r.float())
    assert _err(y, ref) < 2e-2 * max(1.0, ref.abs().max().item())
    for _ in range(3):
        assert torch.equal(C.conv3x3_fwd(x, w, b, r, 1), y)


@pytest.mark.parametrize('cin,cout,H,W', [(128, 128, 19, 20), (64, 128, 38, 40), (128, 64, 38, 40),
                                          (256, 128, 9, 9), (32, 32, 7, 5), (128, 128, 76, 80)])
def test_conv3x3_drelu_epilogue(cin, cout, H, W):
    """act mode 4: out = conv(x) * (res > 0) - the input gradient gated by the ReLU output it flows into
    (window / halo / implicit-GEMM kernels all share the epilogue)."""
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(9)
    B = 3
    x = torch.randn(B, H, W, cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, 3, 3, cin, device=DEV) / (3 * cin ** 0.5)).to(torch.bfloat16)
    y = torch.relu(torch.randn(B, H, W, cout, device=DEV)).to(torch.bfloat16)
    y[0, 0, 0, :] = -0.0   # negative zero gates like zero
    out = C.conv3x3_fwd(x, w, None, y, 4)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 1, 1)
    ref = ref.permute(0, 2, 3, 1) * (y.float() > 0)
    assert _err(out, ref) < 2e-2 * max(1.0, ref.abs().max().item())
    assert bool((out[y <= 0] == 0).all())


def test_conv1x1_gemm_path_matches_conv():
    from applestar_amd import ops
    torch.manual_seed(8)
    x = torch.randn(4, 132, 19, 20, device=DEV).contiguous(memory_format=torch.channels_last)
    w = torch.randn(128, 132, 1, 1, device=DEV) / 12
    b = torch.randn(128, device=DEV)
    y = ops.conv2d(x, w, b, 1, 0, act='relu')
    yr = torch.relu(torch.nn.functional.conv2d(x, w, b))
    assert _err(y, yr) < 1e-3


def _wgrad_tiles(N, K):
    """(BN, BK) chosen by wgrad.hip for an N x K gradient (pick_bn / pick_bk)."""
    bn = 32 if N <= 32 else (64 if N <= 64 else 128)
    bk, best = 128, (K + 127) // 128 * 128
    for c in (96, 64):
        if (K + c - 1) // c * c < best:
            bk, best = c, (K + c - 1) // c * c
    return bn, bk


def _check_wgrad(got, ref64, ref_gpu, tol, rerun):
    """Compare against a CPU float64 reference; on a miss, say where (n, k, tile), whether the GPU fp32
    torch reference is itself off, and whether a second launch reproduces the result (round-1
    intermittent: docs/OPEN_ISSUES.md)."""
    d = (got.double().cpu() - ref64).abs()
    err = float(torch.nan_to_num(d, nan=float('inf')).max())
    if err < tol:
        return
    N, K = ref64.shape
    n, k = divmod(int(torch.nan_to_num(d, nan=float('inf')).argmax()), K)
    bn, bk = _wgrad_tiles(N, K)
    again = rerun().double().cpu()
    raise AssertionError(
        f'wgrad max err {err:.4g} (tol {tol:.4g}) at n={n} k={k} tile=({n // bn},{k // bk}) '
        f'got={float(got[n, k]):.6g} ref={float(ref64[n, k]):.6g}; elements over tol: {int((d >= tol).sum())}; '
        f'gpu fp32 torch ref err vs f64: {float((ref_gpu.double().cpu() - ref64).abs().max()):.4g}; '
        f'rerun identical: {torch.equal(again, got.double().cpu())}, rerun err {float((again - ref64).abs().max()):.4g}')


@pytest.mark.parametrize('R,N,K', [(5000, 128, 128), (100003, 256, 768), (70001, 32, 56), (4097, 1024, 256),
                                   (300, 64, 64), (145920, 128, 128), (20000, 24, 288), (3000, 40, 200)])
def test_wgrad_dense_matches_fp32(R, N, K):
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(11)
    dy = torch.randn(R, N, device=DEV).to(torch.bfloat16)
    x = torch.randn(R, K, device=DEV).to(torch.bfloat16)
    dw, db = C.wgrad(dy, x, 0, True)
    assert dw.dtype == torch.float32 and dw.shape == (N, K) and db.shape == (N,)
    dy64, x64 = dy.double().cpu(), x.double().cpu()
    scale = R ** 0.5
    _check_wgrad(dw, dy64.t() @ x64, dy.float().t() @ x.float(), 1e-3 * scale,
                 lambda: C.wgrad(dy, x, 0, True)[0])
    assert float((db.double().cpu() - dy64.sum(0)).abs().max()) < 1e-3 * scale
    dw2, db2 = C.wgrad(dy, x, 0, False)
    assert db2 is None
    assert torch.equal(dw2, dw)            # deterministic (fixed split, ordered partial sum)
    # bf16 output: the cast is fused into the split reduction -> exactly the rounded fp32 result
    dw3, db3 = C.wgrad(dy, x, 0, True, True)
    assert dw3.dtype == torch.bfloat16 and db3.dtype == torch.bfloat16
    assert torch.equal(dw3, dw.to(torch.bfloat16)) and torch.equal(db3, db.to(torch.bfloat16))


@pytest.mark.parametrize('B,H,W,cin,cout', [(5, 19, 20, 128, 128), (2, 76, 80, 32, 64), (3, 7, 5, 64, 32),
                                            (4, 38, 40, 64, 128)])
def test_wgrad_conv3x3_matches_fp32(B, H, W, cin, cout):
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(12)
    x = torch.randn(B, H, W, cin, device=DEV).to(torch.bfloat16)
    dy = torch.randn(B, H, W, cout, device=DEV).to(torch.bfloat16)
    dw, db = C.wgrad(dy.view(-1, cout), x, cin, True)
    ref64 = torch.nn.grad.conv2d_weight(x.double().cpu().permute(0, 3, 1, 2), (cout, cin, 3, 3),
                                        dy.double().cpu().permute(0, 3, 1, 2), padding=1)   # [Cout,Cin,3,3]
    ref_gpu = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (cout, cin, 3, 3),
                                          dy.float().permute(0, 3, 1, 2), padding=1)
    as_k = lambda w: w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)    # noqa: E731  [Cout, 3, 3, Cin] order
    scale = (B * H * W) ** 0.5
    _check_wgrad(dw, as_k(ref64), as_k(ref_gpu), 1e-3 * scale, lambda: C.wgrad(dy.view(-1, cout), x, cin, True)[0])
    assert float((db.double().cpu() - dy.double().cpu().sum((0, 1, 2))).abs().max()) < 1e-3 * scale
    dw3, db3 = C.wgrad(dy.view(-1, cout), x, cin, True, True)
    assert torch.equal(dw3, dw.to(torch.bfloat16)) and torch.equal(db3, db.to(torch.bfloat16))


def test_native_linear_autocast_grads_match_fp32():
    from applestar_amd import ops
    torch.manual_seed(13)
    x = torch.randn(9000, 256, device=DEV, requires_grad=True)
    w = (torch.randn(128, 256, device=DEV) / 16).requires_grad_()
    b = torch.randn(128, device=DEV, requires_grad=True)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = ops.linear(x, w, b)     # (no ReLU: bf16 vs fp32 mask flips near 0 would dominate the dX error)
    assert y.dtype == torch.bfloat16
    g = torch.randn(9000, 128, device=DEV)
    y.float().backward(g)
    xs, ws, bs = (t.detach().clone().requires_grad_() for t in (x, w, b))
    (xs @ ws.t() + bs).backward(g)
    assert w.grad.dtype == torch.float32 and b.grad.dtype == torch.float32
    for a, r in ((x.grad, xs.grad), (w.grad, ws.grad), (b.grad, bs.grad)):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize('K', [256, 32])
def test_native_linear_thin_output_dx(K):
    """N = 32 outputs: the input gradient runs the K = 32 MFMA kernel (gemm_k32.hip); R not a multiple
    of its 64-row block."""
    from applestar_amd import ops
    from applestar_amd.ops import native
    torch.manual_seed(17)
    R = 5003
    x = torch.randn(R, K, device=DEV, requires_grad=True)
    w = (torch.randn(32, K, device=DEV) / K ** 0.5).requires_grad_()
    b = torch.randn(32, device=DEV, requires_grad=True)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = ops.linear(x, w, b)
    g = torch.randn(R, 32, device=DEV)
    y.float().backward(g)
    xs, ws, bs = (t.detach().clone().requires_grad_() for t in (x, w, b))
    (xs @ ws.t() + bs).backward(g)
    for a, r in ((x.grad, xs.grad), (w.grad, ws.grad), (b.grad, bs.grad)):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())
    C = native.ensure_loaded()
    a = torch.randn(130, 32, device=DEV).to(torch.bfloat16)
    wt = torch.randn(48, 32, device=DEV).to(torch.bfloat16)
    assert _err(C.mm_k32(a, wt), a.float() @ wt.float().t()) < 2e-2 * 8


def test_native_linear_pads_odd_k():
    """K = 132 (not a multiple of 8): the reduction dim is zero-padded so the native weight-gradient
    kernel runs; grads of x, w (original shapes) and b must match fp32."""
    from applestar_amd import ops
    torch.manual_seed(16)
    x = torch.randn(5000, 132, device=DEV, requires_grad=True)
    w = (torch.randn(128, 132, device=DEV) / 12).requires_grad_()
    b = torch.randn(128, device=DEV, requires_grad=True)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = ops.linear(x, w, b)
    assert y.shape == (5000, 128)
    g = torch.randn(5000, 128, device=DEV)
    y.float().backward(g)
    xs, ws, bs = (t.detach().clone().requires_grad_() for t in (x, w, b))
    (xs @ ws.t() + bs).backward(g)
    assert x.grad.shape == x.shape and w.grad.shape == w.shape
    for a, r in ((y.float(), xs.detach() @ ws.detach().t() + bs.detach()), (x.grad, xs.grad), (w.grad, ws.grad),
                 (b.grad, bs.grad)):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize('layout', ['nhwc', 'nchw', 'strided'])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('relu', [False, True])
def test_act_grad_nhwc(layout, dtype, relu):
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(14)
    B, H, W, Ch = 3, 19, 21, 64
    out = torch.randn(B, H, W, Ch, device=DEV).to(torch.bfloat16)
    g = torch.randn(B, Ch, H, W, device=DEV).to(dtype)
    if layout == 'nhwc':
        dout = g.permute(0, 2, 3, 1).contiguous()
    elif layout == 'nchw':
        dout = g.permute(0, 2, 3, 1)                     # NCHW-contiguous underneath
    else:
        dout = g.permute(0, 2, 3, 1)[:, :, ::1, :].transpose(1, 2).contiguous().transpose(1, 2)
    got = C.act_grad_nhwc(dout, out, relu)
    ref = dout.float() * (out > 0) if relu else dout.float()
    assert got.dtype == torch.bfloat16 and got.is_contiguous()
    assert _err(got, ref) <= 1e-2 * ref.abs().max().item()


def test_native_linear_relu_epilogue_grads():
    from applestar_amd import ops
    torch.manual_seed(15)
    x = torch.randn(6000, 256, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(1024, 256, device=DEV) / 16).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(1024, device=DEV)).to(torch.bfloat16).requires_grad_()
    y = ops.linear(x, w, b, act='relu')
    yr = torch.relu(x.float() @ w.float().t() + b.float())
    assert y.dtype == torch.bfloat16 and _err(y, yr) < 3e-2 * yr.abs().max().item()
    g = torch.randn(6000, 1024, device=DEV)
    y.backward(g)
    dpre = g * (y.detach() > 0)                          # same mask as the bf16 forward
    for a, r in ((x.grad, dpre @ w.float()), (w.grad, dpre.t() @ x.float()), (b.grad, dpre.sum(0))):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())


def test_multi_copy_converts_and_handles_many_tensors():
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(16)
    srcs, dsts = [], []
    flat = torch.zeros(4 * 10 ** 6, device=DEV)
    off = 0
    for i in range(150):                              # > kCopyMaxT tensors -> several launches
        shape = (int(torch.randint(1, 40, ()).item()), int(torch.randint(1, 700, ()).item()))
        n = shape[0] * shape[1]
        s = torch.randn(shape, device=DEV).to(torch.bfloat16 if i % 2 else torch.float32)
        d = flat[off:off + n].view(shape) if i % 3 else torch.empty(shape, device=DEV, dtype=torch.bfloat16)
        off += n
        srcs.append(s)
        dsts.append(d)
    conv_w = torch.randn(64, 32, 3, 3, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv_d = torch.empty(64, 32, 3, 3, device=DEV).contiguous(memory_format=torch.channels_last)
    srcs.append(conv_w)
    dsts.append(conv_d)
    srcs.append(torch.randn(3, 5, device=DEV).t())     # stride mismatch -> copy_ fallback
    dsts.append(torch.empty(5, 3, device=DEV))
    C.multi_copy(dsts, srcs)
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s.to(d.dtype)), (d.shape, d.dtype, s.dtype)


def test_copy_into_strided_sources_without_copy_launches():
    """parallel/dp.py copy_into (the gradient -> bucket copy): sources whose strides differ from the contiguous
    destination (channels_last conv-weight gradients, transposed views) take ONE strided multi-tensor launch, equal
    strides the raw / converting multi-copy - exact values, and no aten copy_ dispatched."""
    from torch.utils._python_dispatch import TorchDispatchMode
    from applestar_amd.parallel.dp import copy_into
    torch.manual_seed(4)
    srcs = [torch.randn(64, 32, 3, 3, device=DEV).contiguous(memory_format=torch.channels_last),
            torch.randn(48, 80, device=DEV).t(),
            torch.randn(7, 5, 3, device=DEV).permute(2, 0, 1),
            torch.randn(1000, device=DEV),
            torch.randn(33, 17, device=DEV).bfloat16().t(),
            torch.randn(20, 30, device=DEV)]
    dsts = [torch.empty(s.shape, device=DEV, dtype=torch.float32) for s in srcs]
    seen = []

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, a=(), kw=None):
            seen.append(str(func.overloadpacket.__name__))
            return func(*a, **(kw or {}))
    with Rec():
        copy_into(dsts, srcs)
    torch.cuda.synchronize()
    assert 'copy_' not in seen, seen
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s.float())


def test_multi_copy_integer_sources_convert_exactly():
    """uint8 / int16 feature columns -> bf16 / fp32 in one launch (the scalar encoder's casts), values exact;
    int32 falls back to copy_."""
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(19)
    srcs = [torch.randint(0, 256, (1, 260), device=DEV, dtype=torch.uint8),
            torch.randint(-300, 300, (390, 90), device=DEV, dtype=torch.int16),
            torch.randint(0, 256, (9000,), device=DEV, dtype=torch.uint8),
            torch.randint(-200, 200, (17, 5), device=DEV, dtype=torch.int32)]
    for dt in (torch.bfloat16, torch.float32):
        dsts = [torch.empty(s.shape, device=DEV, dtype=dt) for s in srcs]
        C.multi_copy(dsts, srcs)
        for d, s in zip(dsts, srcs):
            assert torch.equal(d, s.to(dt)), (dt, s.dtype)


def test_multi_copy_raw_bytes_any_dtype():
    """Equal-dtype pairs travel as raw bytes (the graph step's batch refresh): int64 / int32 / bool / uint8 /
    fp16 / fp32 leaves, odd byte counts and views at unaligned offsets (byte path), > 64 MB leaves (many
    chunks), one launch per 64 leaves."""
    from applestar_amd.ops import native
    from applestar_amd.runtime.step_graph import _tree_copy_
    C = native.ensure_loaded()
    torch.manual_seed(18)
    srcs, dsts = [], []
    big = torch.randint(-2 ** 40, 2 ** 40, (9 * 10 ** 6,), device=DEV)      # 72 MB
    srcs.append(big)
    dsts.append(torch.empty_like(big))
    base_u8 = torch.randint(0, 255, (10 ** 5,), device=DEV, dtype=torch.uint8)
    dst_u8 = torch.zeros(10 ** 5 + 64, device=DEV, dtype=torch.uint8)
    for i in range(140):
        kind = i % 6
        n = int(torch.randint(1, 3000, ()).item())
        if kind == 0:
            s = torch.randint(-10 ** 9, 10 ** 9, (n,), device=DEV)
        elif kind == 1:
            s = torch.randint(-10 ** 6, 10 ** 6, (n, 3), device=DEV, dtype=torch.int32)
        elif kind == 2:
            s = torch.rand(n, device=DEV) > 0.5
        elif kind == 3:                                  # unaligned source and destination views
            o = int(torch.randint(1, 15, ()).item())
            s = base_u8[o:o + n]
            dsts.append(dst_u8[o + 3:o + 3 + n])
            srcs.append(s)
            continue
        elif kind == 4:
            s = torch.randn(n, device=DEV).half()
        else:
            s = torch.randn(n, 2, device=DEV)
        srcs.append(s)
        dsts.append(torch.empty_like(s))
    C.multi_copy(dsts, srcs)
    torch.cuda.synchronize()
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s), (d.shape, d.dtype)
    # the graph step's tree refresh: nested dict/list of device leaves + a host leaf
    src = {'a': [torch.arange(7, device=DEV), torch.ones(3, 4, device=DEV, dtype=torch.bool)],
           'b': {'c': torch.randn(5, device=DEV)}, 'h': torch.arange(3)}
    dst = {'a': [torch.zeros(7, device=DEV, dtype=torch.long), torch.zeros(3, 4, device=DEV, dtype=torch.bool)],
           'b': {'c': torch.zeros(5, device=DEV)}, 'h': torch.zeros(3, dtype=torch.long)}
    _tree_copy_(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst['a'][0], src['a'][0]) and torch.equal(dst['a'][1], src['a'][1])
    assert torch.equal(dst['b']['c'], src['b']['c']) and torch.equal(dst['h'], src['h'])


@pytest.mark.parametrize('cin,cout,act', [(16, 16, 'relu'), (32, 8, None), (8, 32, 'relu')])
def test_pointwise_conv1x1_matches_fp32(cin, cout, act):
    from applestar_amd import ops
    torch.manual_seed(17)
    x = torch.randn(3, cin, 37, 41, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    w = (torch.randn(cout, cin, 1, 1, device=DEV) / cin ** 0.5).requires_grad_()
    b = (0.1 * torch.randn(cout, device=DEV)).requires_grad_()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = ops.conv2d(x, w, b, 1, 0, act=act)
    assert y.dtype == torch.bfloat16
    xs, ws, bs = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv2d(xs, ws, bs)
    if act == 'relu':
        yr = torch.relu(yr)
    assert _err(y, yr) < 3e-2 * max(1.0, yr.abs().max().item())
    g = torch.randn_like(yr)
    y.float().backward(g)
    dpre = g * (y.detach().float() > 0) if act == 'relu' else g    # the bf16 forward's mask
    dx = torch.nn.grad.conv2d_input(xs.shape, ws, dpre)
    dw = torch.nn.grad.conv2d_weight(xs, ws.shape, dpre)
    for a, r in ((x.grad, dx), (w.grad, dw), (b.grad, dpre.sum((0, 2, 3)))):
        assert _err(a, r) < 3e-2 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize('C,H,W', [(128, 19, 20), (32, 19, 20)])
def test_fused_resblock_matches_unfused(C, H, W):
    """The one-node ResBlock (skip gradient fused into the dX conv epilogue) vs the two-conv native path
    (each conv checked against fp32 above): same bf16 forward, so same ReLU masks, and the gradients
    agree up to bf16 rounding of the separate add."""
    from applestar_amd import ops
    from applestar_amd.models.blocks import ResBlock
    torch.manual_seed(18)
    blk = ResBlock(C).to(DEV).to(memory_format=torch.channels_last)
    c1, c2 = blk.conv1[0], blk.conv2[0]
    x = torch.randn(3, C, H, W, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        y = blk(x)
        yu = ops.conv2d(ops.conv2d(x2, c1.weight, c1.bias, 1, 1, act='relu'), c2.weight, c2.bias, 1, 1,
                        act='relu', residual=x2)
    assert torch.equal(y, yu)
    g = torch.randn_like(y.float())
    gx, gw1, gb2 = torch.autograd.grad(y.float(), [x, c1.weight, c2.bias], g)
    ux, uw1, ub2 = torch.autograd.grad(yu.float(), [x2, c1.weight, c2.bias], g)
    for a, r in ((gx, ux), (gw1, uw1), (gb2, ub2)):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize('P', [1520, 128, 77])
def test_gate_chain_matches_fp32(P):
    """Four chained 128x128 pointwise layers in one launch (gate_chain.hip), forward form (bias + ReLU on
    the first three) and backward form (transposed operands, ReLU masks of saved activations, residual
    gradient added to the last output), vs fp32 torch of the same chain on the same bf16 inputs."""
    torch.manual_seed(23)
    C = 128
    x = torch.randn(P, C, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn(C, C, device=DEV) / C ** 0.5).to(torch.bfloat16) for _ in range(4)]
    bs = [0.1 * torch.randn(C, device=DEV) for _ in range(4)]
    outs = N._C.gate_chain(x, ws, bs, [None] * 4, [None] * 4, 0b0111)
    h = x.float()
    for i in range(4):
        h = h @ ws[i].float().t() + bs[i]
        if i < 3:
            h = torch.relu(h)
        assert _err(outs[i], h) < 2e-2 * max(1.0, h.abs().max().item())
        h = outs[i].float()                      # continue from the kernel's bf16 rows (mask agreement)
    a1, a2, a3 = outs[:3]
    dg = torch.randn(P, C, device=DEV).to(torch.bfloat16)
    dres = torch.randn(P, C, device=DEV).to(torch.bfloat16)
    wt = [ws[i].t().contiguous() for i in (3, 2, 1, 0)]
    d3, d2, d1, dx = N._C.gate_chain(dg, wt, [None] * 4, [a3, a2, a1, None], [None, None, None, dres], 0)
    d = dg.float()
    for got, w, m, res in ((d3, ws[3], a3, None), (d2, ws[2], a2, None), (d1, ws[1], a1, None),
                           (dx, ws[0], None, dres)):
        r = d @ w.float()
        if m is not None:
            r = r * (m.float() > 0)
        if res is not None:
            r = r + res.float()
        assert _err(got, r) < 2e-2 * max(1.0, r.abs().max().item())
        d = got.float()


@pytest.mark.parametrize('gate_chain', [True, False])
def test_fused_gated_resblock_matches_unfused(gate_chain, monkeypatch):
    """One-node GatedResBlock vs the per-op native path (conv / 1x1 GEMM / gated-residual kernels, each
    checked against fp32 elsewhere), with the gate path as one gate_chain launch or as four GEMMs."""
    from applestar_amd import ops
    from applestar_amd.models.blocks import GatedResBlock
    monkeypatch.setattr(N, 'GATE_CHAIN', gate_chain)
    torch.manual_seed(19)
    C = 128
    blk = GatedResBlock(C).to(DEV).to(memory_format=torch.channels_last)
    with torch.no_grad():
        blk.UpdateSP.fill_(0.7)
    # bf16 input (as in the model): an fp32 skip would make the per-op path evaluate the gated residual in
    # fp32 and flip ReLU masks relative to the bf16 fused node
    x = torch.randn(4, C, 19, 20, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    params = list(blk.parameters())
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = blk(x)
        y = blk.conv2(blk.conv1(x2))
        g = blk.GateWeightG(x2)
        ref = ops.gated_residual(y, g, blk.UpdateSP, x2)
    assert _err(out, ref) < 3e-2 * max(1.0, ref.float().abs().max().item())
    gout = torch.randn_like(out.float())
    ga = torch.autograd.grad(out.float(), [x] + params, gout)
    gb = torch.autograd.grad(ref.float(), [x2] + params, gout)
    for a, b in zip(ga, gb):
        assert _err(a, b) < 5e-2 * max(1.0, b.float().abs().max().item())


@pytest.mark.parametrize('cout,cin', [(128, 128), (64, 32), (1, 32), (33, 7)])
@pytest.mark.parametrize('channels_last', [False, True])
def test_conv_wt_matches_flip_permute(cout, cin, channels_last):
    """One-launch flipped/transposed conv3x3 weight == w.flip(2,3).permute(1,2,3,0), bit-exact."""
    w = torch.randn(cout, cin, 3, 3, device=DEV).to(torch.bfloat16)
    if channels_last:
        w = w.contiguous(memory_format=torch.channels_last)
    got = N._C.conv_wt(w)
    ref = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
    assert got.shape == ref.shape and got.is_contiguous()
    assert torch.equal(got, ref)


@pytest.mark.parametrize('C', [2, 128, 327, 513, 4097, 24320])
@pytest.mark.parametrize('ldt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('with_teacher', [True, False])
def test_head_stats_matches_reference(C, ldt, with_teacher):
    """Fused (logp_a, entropy, KL) rows and their one-pass backward vs log_softmax chains in fp32,
    including -1e9-masked columns and fully masked rows (padded selected-units steps)."""
    torch.manual_seed(21)
    R = 37
    logits = (3 * torch.randn(R, C, device=DEV)).to(ldt)
    teacher = 3 * torch.randn(R, C, device=DEV) if with_teacher else None
    if C > 4:
        logits[:, C // 2:] = -1e9                   # masked tail
        if teacher is not None:
            teacher[:, C // 2:] = -1e9
        logits[3] = -1e9                            # fully masked row
        if teacher is not None:
            teacher[3] = -1e9
    act = torch.randint(0, max(1, C // 2), (R,), device=DEV)
    l1 = logits.detach().clone().requires_grad_()
    got = N.head_stats(l1, teacher, act)
    l2 = logits.detach().float().clone().requires_grad_()
    ref = R_head_stats(l2, teacher, act)
    for a, b in zip(got, ref):
        assert a.dtype == torch.float32
        assert _err(a, b) < 1e-3 * max(1.0, b.abs().max().item()), (_err(a, b))
    gs = [torch.randn(R, device=DEV) for _ in range(3)]
    sum((x * g).sum() for x, g in zip(got, gs)).backward()
    sum((x * g).sum() for x, g in zip(ref, gs)).backward()
    assert l1.grad.dtype == ldt
    tol = 2e-2 if ldt == torch.bfloat16 else 1e-4
    assert _err(l1.grad, l2.grad) < tol * max(1.0, l2.grad.abs().max().item()), _err(l1.grad, l2.grad)


def R_head_stats(logits, teacher, act):
    return R.head_stats(logits, teacher, act)


@pytest.mark.parametrize('wdtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('idx_dtype', [torch.int16, torch.int64])
def test_bo_encoder_fused_matches_torch(wdtype, idx_dtype):
    """Fused build-order transformer (one kernel per direction) vs the op-by-op module in fp32:
    output and every parameter gradient, with bf16 or fp32 linear weights."""
    from applestar_amd.models.encoders import BeginningBuildOrderEncoder
    torch.manual_seed(31)
    enc = BeginningBuildOrderEncoder(64).to(DEV)
    ref = BeginningBuildOrderEncoder(64).to(DEV)
    ref.load_state_dict(enc.state_dict())
    if wdtype == torch.bfloat16:
        for ps in (enc.fused_params(),):
            for i, p in enumerate(ps):
                if not (i >= 2 and (i - 2) % 12 in (0, 1, 6, 7)):
                    p.data = p.data.to(torch.bfloat16)
        with torch.no_grad():   # the reference sees the same bf16-rounded values in fp32
            for pe, pr in zip(enc.fused_params(), ref.fused_params()):
                pr.copy_(pe.float())
    B = 97
    bo = torch.randint(0, 174, (B, 20), device=DEV).to(idx_dtype)
    loc = torch.randint(0, 152 * 160, (B, 20), device=DEV).to(idx_dtype)
    bo[5, 3:] = 0
    assert enc._fusable(bo)
    n_before = len(enc.fused_params())
    out = enc(bo, loc)
    out_ref = ref.forward_torch(bo, loc)
    scale = out_ref.abs().max().item()
    tol = 2e-3 if wdtype == torch.float32 else 2e-2
    assert _err(out, out_ref) < tol * max(1.0, scale), _err(out, out_ref)
    g = torch.randn_like(out_ref)
    out.float().backward(g)
    out_ref.backward(g)
    for (pe, pr) in zip(enc.parameters(), ref.parameters()):
        if pr.grad is None:
            continue
        assert pe.grad is not None and pe.grad.dtype == pe.dtype
        s = pr.grad.abs().max().item()
        assert _err(pe.grad, pr.grad) < tol * max(1e-3, s), (pe.shape, _err(pe.grad, pr.grad), s)
    assert n_before == 38


def test_resmlp_fused_matches_op_by_op():
    """Value baseline with the fused 16 x ResFCBlock2 kernels vs the op-by-op blocks (same bf16 weights,
    autocast), both against an fp32 golden run of the same weights: the fused path must be as close to
    fp32 as the op-by-op bf16 path (16 residual blocks amplify bf16 rounding, so the two bf16 paths are
    compared through the golden, not with each other)."""
    import copy
    from applestar_amd.models import model as M
    torch.manual_seed(41)
    vb = M.ValueBaseline(1440, 256, 16, atan=True).to(DEV)
    for blk in vb.res:
        for lin in (blk.fc1[0], blk.fc2[0]):
            lin.weight.data = lin.weight.data.to(torch.bfloat16)
            lin.bias.data = lin.bias.data.to(torch.bfloat16)
    ref = copy.deepcopy(vb)
    gold = copy.deepcopy(vb).float()
    x = torch.randn(390, 1440, device=DEV)
    xa, xb, xg = (x.clone().requires_grad_() for _ in range(3))
    with torch.autocast('cuda', dtype=torch.bfloat16):
        assert vb._fusable(torch.empty(1, 256, device=DEV, dtype=torch.bfloat16))
        out = vb(xa)
        M.FUSED_RESMLP = False
        try:
            out_ref = ref(xb)
        finally:
            M.FUSED_RESMLP = True
    M.FUSED_RESMLP = False
    try:
        out_g = gold(xg)
    finally:
        M.FUSED_RESMLP = True
    e_f, e_r = _err(out, out_g), _err(out_ref, out_g)
    assert e_f < 2 * e_r + 1e-3, (e_f, e_r)
    g = torch.randn_like(out_g)
    out.backward(g)
    out_ref.backward(g)
    out_g.backward(g)
    e_f, e_r = _err(xa.grad, xg.grad), _err(xb.grad, xg.grad)
    assert e_f < 2 * e_r + 1e-4, ('input grad', e_f, e_r)
    for (na, pa), (_, pb), (_, pg) in zip(vb.named_parameters(), ref.named_parameters(), gold.named_parameters()):
        assert pa.grad is not None and pa.grad.dtype == pa.dtype, na
        # relative Frobenius error: a max-abs error over a weight gradient behind 16 bf16 residual blocks is set by
        # single ReLU-mask flips (a 2^-9 perturbation flips pre-activations within that margin of zero, see
        # test_model_parity_gpu.py::test_bf16_head_grad_error_is_weight_rounding_sensitivity), in either bf16 path
        rel = lambda a, r: ((a.float() - r.float()).norm() / r.float().norm().clamp_min(1e-30)).item()
        e_f, e_r = rel(pa.grad, pg.grad), rel(pb.grad, pg.grad)
        assert e_f < 2 * e_r + 1e-3, (na, e_f, e_r)


@pytest.mark.parametrize('B', [6, 5])
def test_location_input_matches_cat_path(B):
    """locin.hip: relu(conv1x1(relu(cat([fc output as [B,4,H,W], skip])))) without the concat vs the fp32
    torch cat + conv path, forward and all four gradients (skip gradient where skip > 0: the fused stage
    leaves the skip map's own ReLU mask to its producer)."""
    import torch.nn.functional as F
    torch.manual_seed(0)
    H, W, C, P = 19, 20, 128, 4
    pf = torch.relu(torch.randn(B, P * H * W, device=DEV)).bfloat16().requires_grad_()
    skip = torch.relu(torch.randn(B, C, H, W, device=DEV)).bfloat16()
    skip = skip.contiguous(memory_format=torch.channels_last).requires_grad_()
    w = (0.1 * torch.randn(C, P + C, 1, 1, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=DEV)).bfloat16().requires_grad_()
    y = N.location_input(pf, skip, w, b)
    assert y is not None and y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, C, H, W, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    pr, sr, wr, br = (t.detach().float().requires_grad_() for t in (pf, skip, w, b))
    x = torch.relu(torch.cat([pr.view(B, P, H, W), sr], 1))
    z = F.conv2d(x, wr, br)
    yr = torch.relu(z)
    # the output ReLU's mask is taken from the kernel's own output: pre-activations within bf16 rounding of
    # zero may flip sign between the bf16 and the fp32 paths, and one flipped entry moves dP by |dy w|
    (z * (y.detach().float() > 0)).backward(dy.float())

    def rel(a, r):
        return _err(a, r) / max(r.abs().max().item(), 1e-6)

    assert rel(y, yr) < 1e-2
    assert rel(pf.grad, pr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    assert rel(b.grad, br.grad) < 2e-2
    assert rel(skip.grad * (skip > 0), sr.grad) < 2e-2


@pytest.mark.parametrize('B,H,W', [(3, 152, 160), (2, 7, 9)])
def test_value_spatial_proj_matches_cat_path(B, H, W):
    """value_spatial.hip: relu(conv1x1(cat([scatter map (8 ch), own, enemy]))) without the cat vs fp32
    torch, forward and the scatter-map / weight / bias gradients (output ReLU mask from the kernel's own
    output, as in the location-input test)."""
    import torch.nn.functional as F
    torch.manual_seed(0)
    sc = torch.zeros(B * H * W, 8, device=DEV)
    hot = torch.rand(B * H * W, device=DEV) < 0.05          # a sparse unit scatter, like the real map
    sc[hot] = torch.randn(int(hot.sum()), 8, device=DEV)
    sc = sc.bfloat16().view(B, H, W, 8).permute(0, 3, 1, 2).requires_grad_()
    own = torch.rand(B, 1, H, W, device=DEV) < 0.1
    enemy = torch.rand(B, 1, H, W, device=DEV) < 0.1
    w = (0.3 * torch.randn(16, 10, 1, 1, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(16, device=DEV)).bfloat16().requires_grad_()
    y = N.value_spatial_proj(sc, own, enemy, w, b)
    assert y is not None and y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, 16, H, W, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    sr, wr, br = (t.detach().float().requires_grad_() for t in (sc, w, b))
    z = F.conv2d(torch.cat([sr, own.float(), enemy.float()], 1), wr, br)
    (z * (y.detach().float() > 0)).backward(dy.float())

    def rel(a, r):
        return _err(a, r) / max(r.abs().max().item(), 1e-6)

    assert rel(y, torch.relu(z)) < 1e-2
    assert rel(sc.grad, sr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    assert rel(b.grad, br.grad) < 2e-2


@pytest.mark.parametrize('pooled', [True, False])
def test_value_spatial_proj_fp32_matches_fp64(pooled):
    """fp32 step: the value-encoder projection (pooled and plain) keeps fp32 maps (no bf16 copy) - forward and the
    scatter-map / weight / bias gradients vs float64 torch (cat + 1x1 conv + ReLU (+ max_pool2x2))."""
    import torch.nn.functional as F
    torch.manual_seed(43)
    B, H, W = 3, 38, 40
    sc0 = torch.zeros(B * H * W, 8, device=DEV)
    hot = torch.rand(B * H * W, device=DEV) < 0.2
    sc0[hot] = torch.randn(int(hot.sum()), 8, device=DEV)
    own = torch.rand(B, 1, H, W, device=DEV) < 0.1
    enemy = torch.rand(B, 1, H, W, device=DEV) < 0.1
    sc = sc0.view(B, H, W, 8).permute(0, 3, 1, 2).requires_grad_()
    w = (0.3 * torch.randn(16, 10, 1, 1, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(16, device=DEV)).requires_grad_()
    y = N.value_spatial_proj_pool(sc, own, enemy, w, b) if pooled else N.value_spatial_proj(sc, own, enemy, w, b)
    assert y is not None and y.dtype == torch.float32
    g = torch.randn(y.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV).contiguous(memory_format=torch.channels_last))
    sr, wr, br = (_f64(t) for t in (sc, w, b))
    z = torch.relu(F.conv2d(torch.cat([sr, own.double().cpu(), enemy.double().cpu()], 1), wr, br))
    if pooled:
        z = F.max_pool2d(z, 2, 2)
    z.backward(g)
    assert _err(y.cpu(), z) < 1e-5 * max(1.0, z.abs().max().item())
    for name, a, r in (('dsc', sc.grad, sr.grad), ('dw', w.grad, wr.grad), ('db', b.grad, br.grad)):
        assert _err(a.cpu(), r) < 2e-5 * max(1.0, r.abs().max().item()), name


@pytest.mark.parametrize('R,K,N,relu', [(390, 48640, 256, True), (5000, 256, 1024, False)])
def test_native_linear_reformulated_gemms(R, K, N, relu):
    """The library-GEMM reformulations in _Linear: a few rows over a huge K run as a 32-chunk split-K batched
    GEMM (the spatial fc, 48640 -> 256), and large dX products use a transposed weight copy; values and all
    gradients vs fp32 (ReLU mask from the bf16 output)."""
    from applestar_amd import ops
    from applestar_amd.ops import native
    assert native.GEMM_REFORM
    torch.manual_seed(23)
    x = torch.randn(R, K, device=DEV).bfloat16().requires_grad_()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16().requires_grad_()
    b = torch.randn(N, device=DEV).bfloat16().requires_grad_()
    y = ops.linear(x, w, b, act='relu' if relu else None)
    g = torch.randn(R, N, device=DEV).bfloat16()
    y.backward(g)
    xs, ws, bs = (t.detach().float().requires_grad_() for t in (x, w, b))
    z = xs @ ws.t() + bs
    ref = torch.relu(z) if relu else z
    assert _err(y, ref) < 2e-2 * max(1.0, ref.abs().max().item())
    (z * (y.detach().float() > 0) if relu else z).backward(g.float())
    for a, r in ((x.grad, xs.grad), (w.grad, ws.grad), (b.grad, bs.grad)):
        assert _err(a, r) < 2e-2 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize('fp32', [False, True], ids=['bf16', 'fp32'])
@pytest.mark.parametrize('HW', [(38, 40), (152, 160)])
@pytest.mark.parametrize('crowded', [False, True])
def test_spatial_embed_pool_matches_unfused(HW, crowded, fp32):
    """Fused relu(embed) -> max_pool2x2 (pixel-row-pair tiles) vs the unfused native embed + maxpool:
    bf16: pooled output bit-equal (same arithmetic, same argmax rule) and the rows / dense-weight / bias
    gradients equal up to summation order.  fp32 (the fp32 step: the projection on three bf16 parts of W, fp32
    entity rows; backward through the fp32 maxpool2_bwd_relu and the MFMA weight gradient without a gate): within
    fp32 rounding of the unfused fp32 kernels."""
    from applestar_amd.lib.features import SPATIAL_ONE_HOT, EFFECT_KEYS
    from applestar_amd import ops
    torch.manual_seed(31)
    B, (H, W), L = 3, HW, 5
    Nn = 400 if crowded else 37
    sp = {'height_map': torch.randint(0, 256, (B, H, W), device=DEV, dtype=torch.uint8)}
    for k, n in SPATIAL_ONE_HOT:
        sp[k] = torch.randint(0, n + 1, (B, H, W), device=DEV, dtype=torch.uint8)
    for k in EFFECT_KEYS:
        sp[k] = torch.randint(0, H * W, (B, L), device=DEV, dtype=torch.int16)
    ex = torch.randint(0, 6 if crowded else W, (B, Nn), device=DEV)
    ey = torch.randint(0, 2 if crowded else H, (B, Nn), device=DEV)
    en = torch.tensor([Nn, 4, 0], device=DEV)
    rows0 = (torch.randn(B, Nn, 32, device=DEV) * (torch.arange(Nn, device=DEV)[None] < en[:, None]).unsqueeze(2))
    w0 = torch.randn(32, 24, device=DEV) * 0.3
    b0 = torch.randn(32, device=DEV) * 0.1
    outs, grads = [], []
    for fused in (True, False):
        rows = (rows0.clone() if fp32 else rows0.to(torch.bfloat16)).requires_grad_()
        w, b = w0.clone().requires_grad_(), b0.clone().requires_grad_()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=not fp32):
            if fused:
                y = N.spatial_embed_pool(sp, rows, ex, ey, en, w, b)
                assert y is not None and y.shape == (B, 32, H // 2, W // 2)
                assert y.dtype == (torch.float32 if fp32 else torch.bfloat16)
            else:
                y = ops.max_pool2x2(N.spatial_embed(sp, rows, ex, ey, en, w, b))
        g = torch.randn(B, 32, H // 2, W // 2, device=DEV, generator=torch.Generator(DEV).manual_seed(5))
        y.backward(g.to(y.dtype).contiguous(memory_format=torch.channels_last))
        outs.append(y.detach().float())
        grads.append((rows.grad.float(), w.grad, b.grad))
    if fp32:
        assert _err(outs[0], outs[1]) < 1e-5 * max(1, outs[1].abs().max().item())
    else:
        assert torch.equal(outs[0], outs[1])
    for a, r in zip(grads[0], grads[1]):
        assert _err(a, r) < (1e-5 if fp32 else 1e-2) * max(1, r.abs().max().item())


@pytest.mark.parametrize('B,H,W', [(3, 152, 160), (2, 6, 10)])
def test_value_spatial_proj_pool_matches_unfused(B, H, W):
    """Pooled value-encoder projection (value_spatial.hip vsp_pool_*) vs value_spatial_proj followed by the
    native max_pool2x2: pooled output bit-equal, scatter-map / weight / bias gradients equal up to order."""
    from applestar_amd import ops
    torch.manual_seed(41)
    sc0 = torch.zeros(B * H * W, 8, device=DEV)
    hot = torch.rand(B * H * W, device=DEV) < 0.05
    sc0[hot] = torch.randn(int(hot.sum()), 8, device=DEV)
    own = torch.rand(B, 1, H, W, device=DEV) < 0.1
    enemy = torch.rand(B, 1, H, W, device=DEV) < 0.1
    w0 = 0.3 * torch.randn(16, 10, 1, 1, device=DEV)
    b0 = 0.1 * torch.randn(16, device=DEV)
    g = torch.randn(B, 16, H // 2, W // 2, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    res = []
    for fused in (True, False):
        sc = sc0.bfloat16().view(B, H, W, 8).permute(0, 3, 1, 2).requires_grad_()
        w, b = w0.bfloat16().requires_grad_(), b0.bfloat16().requires_grad_()
        y = N.value_spatial_proj_pool(sc, own, enemy, w, b) if fused else \
            ops.max_pool2x2(N.value_spatial_proj(sc, own, enemy, w, b))
        assert y is not None and y.shape == (B, 16, H // 2, W // 2)
        y.backward(g)
        res.append((y.detach().float(), sc.grad.float(), w.grad.float(), b.grad.float()))
    assert torch.equal(res[0][0], res[1][0])
    for a, r in zip(res[0][1:], res[1][1:]):
        assert _err(a, r) < 1e-2 * max(1, r.abs().max().item())


# ------------------------------------------------------------------ fp32 step kernels (f32 MFMA), vs float64
@pytest.fixture(params=['split', 'exact'])
def f32_mfma(request):
    """Both product modes of the fp32 kernels (csrc/split_mfma.h): the bf16x6 split (default) and the exact-f32
    MFMA; every fp32 kernel test holds both to the same float64 bound."""
    C = N.ensure_loaded()
    old = C.f32_mfma_mode()
    C.set_f32_mfma_mode(1 if request.param == 'split' else 0)
    yield request.param
    C.set_f32_mfma_mode(old)


def _f64(t):
    return t.detach().double().cpu().requires_grad_()


@pytest.mark.parametrize('cin,cout,H,W,act,res', [(128, 128, 19, 20, 'relu', True), (32, 64, 21, 17, 'relu', False),
                                                  (64, 128, 10, 12, None, False), (16, 16, 9, 11, 'relu', False),
                                                  (16, 32, 8, 8, None, True), (128, 64, 5, 7, 'relu', False),
                                                  (32, 32, 19, 20, 'relu', True), (32, 16, 7, 9, None, False)])
def test_conv3x3_f32_matches_fp64(cin, cout, H, W, act, res, f32_mfma):
    """fp32 operands take conv3x3_f32.hip (forward, dX with the flipped weight, split-R dW / db): within fp32
    rounding of a float64 reference - no bf16 anywhere.  Cin = Cout = 16 takes the narrow direct-conv kernel in
    split mode (forward and dX), the others the LDS-DMA ring (test_conv3x3_f32_narrow_all_shapes: every narrow
    shape on the direct kernel)."""
    from applestar_amd import ops
    torch.manual_seed(21)
    B, cl = 3, torch.channels_last
    x = torch.randn(B, cin, H, W, device=DEV).contiguous(memory_format=cl).requires_grad_()
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (3 * cin ** 0.5)).contiguous(memory_format=cl).requires_grad_()
    b = (0.1 * torch.randn(cout, device=DEV)).requires_grad_()
    r = torch.randn(B, cout, H, W, device=DEV).contiguous(memory_format=cl).requires_grad_() if res else None
    y = ops.conv2d(x, w, b, 1, 1, act=act, residual=r)
    assert y.dtype == torch.float32
    xs, ws, bs = _f64(x), _f64(w), _f64(b)
    rs = _f64(r) if res else None
    yr = torch.nn.functional.conv2d(xs, ws, bs, 1, 1)
    if res:
        yr = yr + rs
    if act == 'relu':
        yr = torch.relu(yr)
    assert _err(y.cpu(), yr) < 1e-5 * max(1.0, yr.abs().max().item())
    g = torch.randn(yr.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV).contiguous(memory_format=cl))
    yr.backward(g)
    for name, a, ref in (('dx', x.grad, xs.grad), ('dw', w.grad, ws.grad), ('db', b.grad, bs.grad)) + \
            ((('dres', r.grad, rs.grad),) if res else ()):
        e = _err(a.cpu(), ref)
        assert e < 2e-5 * max(1.0, ref.abs().max().item()), (name, e, ref.abs().max().item())


@pytest.mark.parametrize('R,N,K', [(4096, 768, 256), (1000, 256, 1024), (390, 128, 48640 // 64), (100003, 32, 16),
                                   (390, 256, 256), (384, 1024, 384), (7800, 64, 128)])
def test_linear_f32_grads_match_fp64(R, N, K, f32_mfma):
    """The fp32 step's linear (gemm_f32.hip forward / dX, wgrad_f32.hip dW / db) vs float64."""
    from applestar_amd.ops import native as NN
    torch.manual_seed(5)
    x = torch.randn(R, K, device=DEV).requires_grad_()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).requires_grad_()
    b = (0.1 * torch.randn(N, device=DEV)).requires_grad_()
    y = NN.linear(x, w, b, act='relu')
    xs, ws, bs = _f64(x), _f64(w), _f64(b)
    yr = torch.relu(xs @ ws.t() + bs)
    assert _err(y.cpu(), yr) < 1e-5 * max(1.0, yr.abs().max().item())
    g = torch.randn(yr.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV))
    yr.backward(g)
    for name, a, ref in (('dx', x.grad, xs.grad), ('dw', w.grad, ws.grad), ('db', b.grad, bs.grad)):
        e = _err(a.cpu(), ref)
        assert e < 2e-5 * max(1.0, ref.abs().max().item()), (name, e)


@pytest.mark.parametrize('R,H', [(6000, 512), (390, 256)])
@pytest.mark.parametrize('extra_consumer', [False, True])
def test_linear_f32_relu_handoff_matches_fp64(extra_consumer, R, H, f32_mfma, monkeypatch):
    """Chained fp32 linears: the second layer's dX epilogue applies the first layer's ReLU mask and the first
    layer's backward skips its threshold pass (native._premasked); with a second consumer of the hidden
    activation the summed gradient must take the mask as usual.  Both vs float64.  The few-row case runs its
    products on the small-product kernel (gemm_f32_small_kernel), so the hand-off is exercised there too."""
    from applestar_amd.ops import native as NN
    monkeypatch.setattr(NN, 'F32_SMALL', True)
    torch.manual_seed(6)
    K, O = 256, 256
    x = torch.randn(R, K, device=DEV).requires_grad_()
    w1 = (torch.randn(H, K, device=DEV) / K ** 0.5).requires_grad_()
    b1 = (0.1 * torch.randn(H, device=DEV)).requires_grad_()
    w2 = (torch.randn(O, H, device=DEV) / H ** 0.5).requires_grad_()
    b2 = (0.1 * torch.randn(O, device=DEV)).requires_grad_()
    h = NN.linear(x, w1, b1, act='relu')
    assert NN._relu_src(h)
    y = NN.linear(h, w2, b2, act='relu')
    if extra_consumer:
        y = y.sum(1, keepdim=True) + (h * h).sum(1, keepdim=True)
    xs, w1s, b1s, w2s, b2s = (_f64(t) for t in (x, w1, b1, w2, b2))
    hs = torch.relu(xs @ w1s.t() + b1s)
    ys = torch.relu(hs @ w2s.t() + b2s)
    if extra_consumer:
        ys = ys.sum(1, keepdim=True) + (hs * hs).sum(1, keepdim=True)
    g = torch.randn(ys.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV))
    ys.backward(g)
    assert not NN._MASKED_DX, 'the producer did not consume the hand-off'
    for name, a, ref in (('dx', x.grad, xs.grad), ('dw1', w1.grad, w1s.grad), ('db1', b1.grad, b1s.grad),
                         ('dw2', w2.grad, w2s.grad), ('db2', b2.grad, b2s.grad)):
        e = _err(a.cpu(), ref)
        assert e < 2e-5 * max(1.0, ref.abs().max().item()), (name, e)


@pytest.mark.parametrize('gated', [False, True])
def test_fused_resblocks_f32_match_torch_fp64(gated, f32_mfma):
    """The one-node fp32 ResBlock / GatedResBlock (skip gradients fused into the dX conv epilogue) vs the same
    module on float64 CPU weights (plain PyTorch path)."""
    import copy
    from applestar_amd.models.blocks import ResBlock, GatedResBlock
    torch.manual_seed(8)
    C, H, W = 128, 19, 20
    blk = GatedResBlock(C) if gated else ResBlock(C)
    ref = copy.deepcopy(blk).double()
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(2, C, H, W, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_()
    xr = _f64(x)
    y = blk(x)
    yr = ref(xr)
    assert _err(y.cpu(), yr) < 1e-5 * max(1.0, yr.abs().max().item())
    g = torch.randn(yr.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV).contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    assert _err(x.grad.cpu(), xr.grad) < 2e-5 * max(1.0, xr.grad.abs().max().item())
    for (n, p), (_, pr) in zip(blk.named_parameters(), ref.named_parameters()):
        e = _err(p.grad.cpu(), pr.grad)
        assert e < 3e-5 * max(1.0, pr.grad.abs().max().item()), (n, e)


@pytest.mark.parametrize('cin,cout', [(16, 16), (16, 32), (32, 16), (32, 32)])
def test_conv3x3_f32_narrow_all_shapes(cin, cout):
    """The narrow direct-conv kernel (conv3x3_f32.hip conv3x3_f32_narrow_kernel) on every shape it implements,
    in a child process with APPLESTAR_CONV_F32_NARROW=all (the mode is read once per process): forward with bias +
    residual + ReLU and the DReLU-masked form against float64."""
    import subprocess
    import sys
    code = f'''
import torch
from applestar_amd.ops import native as N
C = N.ensure_loaded()
C.set_f32_mfma_mode(1)
torch.manual_seed(5)
B, H, W = 3, 13, 11
x = torch.randn(B, H, W, {cin}, device="cuda")
w = torch.randn({cout}, 3, 3, {cin}, device="cuda") / 12
b = torch.randn({cout}, device="cuda")
r = torch.randn(B, H, W, {cout}, device="cuda")
ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(), 1, 1)
ref = ref.permute(0, 2, 3, 1)
for act, res, want in ((1, r, torch.relu(ref + r.double())), (4, r, ref * (r.double() > 0)), (0, None, ref)):
    y = C.conv3x3_f32(x, w, b, res, act)
    err = (y.double() - want).abs().max().item()
    assert err < 1e-5 * max(1.0, want.abs().max().item()), (act, err)
print("ok")
'''
    env = dict(os.environ, APPLESTAR_CONV_F32_NARROW='all')
    out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0 and out.stdout.strip().endswith('ok'), out.stderr[-2000:]


@pytest.mark.parametrize('linked', [False, True])
def test_residual_ln_relu_mask_handoff_f32(linked):
    """Transformer FFN shape: x -> relu(x W1^T + b1) -> relu(. W2^T + b2) = m -> LN(m + x).  The residual LayerNorm's
    backward writes m's gradient masked by (m > 0) as a second output (ops/native.py LN_RELU_MASK) and the second
    linear skips its threshold pass; the residual gradient stays unmasked (through autograd, or handed to the first
    linear's dX GEMM with a GradLink).  Every gradient vs float64."""
    from applestar_amd import ops
    torch.manual_seed(14)
    R, C, Hd = 3000, 256, 512
    x = torch.randn(R, C, device=DEV).requires_grad_()
    w1 = (torch.randn(Hd, C, device=DEV) / C ** 0.5).requires_grad_()
    b1 = (0.1 * torch.randn(Hd, device=DEV)).requires_grad_()
    w2 = (torch.randn(C, Hd, device=DEV) / Hd ** 0.5).requires_grad_()
    b2 = (0.1 * torch.randn(C, device=DEV)).requires_grad_()
    lw = (1 + 0.1 * torch.randn(C, device=DEV)).requires_grad_()
    lb = (0.1 * torch.randn(C, device=DEV)).requires_grad_()
    ts = [_f64(t) for t in (x, w1, b1, w2, b2, lw, lb)]
    link = ops.grad_link(x) if linked else None
    h = N.linear(x, w1, b1, act='relu', grad_link=link)
    m = N.linear(h, w2, b2, act='relu')
    assert N._relu_src(m)
    y = N.layer_norm(m, lw, lb, residual=x, grad_link=link)
    xs, w1s, b1s, w2s, b2s, lws, lbs = ts
    ms = torch.relu(torch.relu(xs @ w1s.t() + b1s) @ w2s.t() + b2s)
    ys = torch.nn.functional.layer_norm(ms + xs, (C,), lws, lbs)
    g = torch.randn(R, C, dtype=torch.float64)
    y.backward(g.float().to(DEV))
    ys.backward(g)
    assert not N._MASKED_DX, 'the producer did not consume the hand-off'
    for name, a, r in zip(('dx', 'dw1', 'db1', 'dw2', 'db2', 'dlw', 'dlb'), (x, w1, b1, w2, b2, lw, lb), ts):
        e = _err(a.grad.cpu(), r.grad)
        assert e < 3e-5 * max(1.0, r.grad.abs().max().item()), (name, e)


@pytest.mark.parametrize('between', ['maxpool', 'upsample', 'upconv'])
@pytest.mark.parametrize('extra_consumer', [False, True])
def test_conv_relu_mask_handoff_f32(between, extra_consumer):
    """fp32 conv(ReLU) -> maxpool / bilinear x2 -> conv (or the fused bilinear x2 + conv 32 -> 1, upconv1): the pool /
    upsample / upconv backward applies the first conv's ReLU mask and the conv backward skips its threshold pass
    (ops/native.py _premasked); with a second consumer of the ReLU output the summed gradient takes the mask as
    usual.  Both vs float64."""
    from applestar_amd import ops
    torch.manual_seed(12)
    cl = torch.channels_last
    x = torch.randn(3, 16, 20, 24, device=DEV).contiguous(memory_format=cl).requires_grad_()
    w1 = (torch.randn(32, 16, 3, 3, device=DEV) / 12).contiguous(memory_format=cl).requires_grad_()
    b1 = (0.1 * torch.randn(32, device=DEV)).requires_grad_()
    w2 = (torch.randn(32, 32, 3, 3, device=DEV) / 17).contiguous(memory_format=cl).requires_grad_()
    ts = [_f64(t) for t in (x, w1, b1, w2)]

    def net(x, w1, b1, w2, ref):
        h = ops.conv2d(x, w1, b1, 1, 1, act='relu') if not ref else torch.relu(torch.nn.functional.conv2d(x, w1, b1, 1, 1))
        if between == 'upconv':
            if not ref:
                y = N.upsample_conv_out(h, w2[:1], None)
            else:
                up = torch.nn.functional.interpolate(h, scale_factor=2.0, mode='bilinear', align_corners=False)
                y = torch.nn.functional.conv2d(up, w2[:1], None, 1, 1)
            out = (y * y).sum()
            return out + (h * h).sum() if extra_consumer else out
        if between == 'maxpool':
            m = N.maxpool2x2(h) if not ref else torch.nn.functional.max_pool2d(h, 2, 2)
        else:
            m = N.upsample2x(h) if not ref else torch.nn.functional.interpolate(h, scale_factor=2.0, mode='bilinear',
                                                                                align_corners=False)
        y = ops.conv2d(m, w2, None, 1, 1) if not ref else torch.nn.functional.conv2d(m, w2, None, 1, 1)
        out = (y * y).sum()
        return out + (h * h).sum() if extra_consumer else out
    net(x, w1, b1, w2, False).backward()
    net(*ts, True).backward()
    assert not N._MASKED_DX, 'the producer did not consume the hand-off'
    for name, a, r in zip(('dx', 'dw1', 'db1', 'dw2'), (x, w1, b1, w2), ts):
        e = _err(a.grad.cpu(), r.grad)
        assert e < 3e-5 * max(1.0, r.grad.abs().max().item()), (name, e)


@pytest.mark.parametrize('chain', [True, False], ids=['chain_f32', 'gemm_f32'])
def test_gated_resblock_f32_gemm_gate_path(f32_mfma, monkeypatch, chain):
    """At 12 x 38 x 40 pixels the fp32 GatedResBlock's four gate layers take the one-launch fp32 chain
    (gate_chain_f32: split activation tile resident in LDS) or four f32 GEMMs (bias + ReLU forward, the ReLU masks
    and the skip gradient in the dX epilogues).  Against the same block with the gate layers on the
    library fp32 GEMM, same inputs: every gradient within 1e-5 (relative Frobenius).  The gate layers get small
    weights and +-1 biases (half the channels on, half off, none near zero): with random ones a few of the 7 M ReLU
    decisions sit within fp32 rounding of zero and flip between any two fp32 implementations (and against
    float64), moving the first gate layer's weight gradient by ~1e-3 - tools/diag/gated_block_f32.py,
    profiles/r3y_gated_block_diag.txt."""
    import copy
    from applestar_amd.models.blocks import GatedResBlock
    torch.manual_seed(9)
    blk0 = GatedResBlock(128)
    with torch.no_grad():
        for m in blk0.GateWeightG:
            m[0].weight.mul_(0.01)
            m[0].bias.copy_(torch.where(torch.arange(128) % 2 == 0, 1.0, -1.0))
    x = torch.randn(12, 128, 38, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    g = torch.randn(12, 128, 38, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    assert N._gemm_f32_ok(12 * 38 * 40, 128, 128)
    monkeypatch.setattr(N, 'GATE_CHAIN_F32', chain)
    C = N.ensure_loaded()
    calls = []
    if chain:
        real = C.gate_chain_f32
        monkeypatch.setattr(C, 'gate_chain_f32', lambda *a: calls.append(1) or real(*a), raising=False)
    grads = []
    for lib in (False, True):
        if lib:
            monkeypatch.setattr(N, 'GATE_CHAIN_F32', False)
            monkeypatch.setattr(N, '_gemm_f32_ok', lambda *a: False)
        blk = copy.deepcopy(blk0).to(DEV).to(memory_format=torch.channels_last)
        xg = x.clone().requires_grad_()
        blk(xg).backward(g)
        grads.append([xg.grad] + [p.grad for p in blk.parameters()])
    assert len(calls) == (2 if chain else 0)   # one launch per direction
    for i, (a, r) in enumerate(zip(*grads)):
        fro = ((a - r).norm() / r.norm()).item()
        assert fro < 1e-5, (i, fro)


@pytest.mark.parametrize('max_norm,wd', [(1.0, 0.0), (1e6, 0.0), (1.0, 1e-4)])
def test_fused_clip_adam_matches_torch(max_norm, wd):
    """optim.hip (two launches: chunked sum of squares, then clip-scaled Adam) == pytorch_norm clip + torch Adam
    over 4 steps on tensors of mixed sizes / layouts, sharing the torch optimizer's state tensors."""
    from applestar_amd.utils.fused_optim import FusedClipAdam
    from applestar_amd.utils.grad_clip import GradClip
    torch.manual_seed(3)
    shapes = [(64, 32, 3, 3), (100003,), (256,), (7, 5), (40000, 33)]

    def make():
        ps = []
        for i, s in enumerate(shapes):
            p = torch.nn.Parameter(torch.randn(*s, device=DEV))
            if len(s) == 4:
                p.data = p.data.contiguous(memory_format=torch.channels_last)
            p.grad = torch.zeros_like(p)
            ps.append(p)
        return ps
    pa, pb = make(), make()
    for a, b in zip(pa, pb):
        b.data.copy_(a.data)
    oa = torch.optim.Adam(pa, lr=1e-3, betas=(0.0, 0.99), eps=1e-5, weight_decay=wd)
    ob = torch.optim.Adam(pb, lr=1e-3, betas=(0.0, 0.99), eps=1e-5, weight_decay=wd)
    clip = GradClip('pytorch_norm', max_norm)
    fused = FusedClipAdam(ob, max_norm)
    for step in range(4):
        for a, b in zip(pa, pb):
            g = torch.randn_like(a) * (step + 1)
            a.grad.copy_(g)
            b.grad.copy_(g)
        na = clip.apply(pa)
        oa.step()
        nb = fused.step()
        assert abs(float(na) - float(nb)) <= 1e-5 * float(na)
        for a, b in zip(pa, pb):
            assert _err(a, b) < 1e-6 * max(1.0, a.abs().max().item()), step
    ob.state_dict()                  # the fused step's per-parameter counters are written lazily, before a state read
    for a, b in zip(pa, pb):
        assert torch.allclose(oa.state[a]['exp_avg_sq'], ob.state[b]['exp_avg_sq'], rtol=1e-5, atol=1e-12)
        assert float(oa.state[a]['step']) == float(ob.state[b]['step']) == 4.0


@pytest.mark.parametrize('segmented', [False, True])
def test_fused_momentum_norm_adam_matches_torch(segmented):
    """optim.hip momentum_norm (per-tensor norm vs the EMA of past clipped norms, three launches) + Adam(0.9,
    0.999, L2 decay) == GradClip('momentum_norm') + torch Adam over 5 steps.  ``segmented``: the same tensors as
    pieces of ONE flat parameter (the bf16 learner's fp32 master), split back by the chunk table."""
    from applestar_amd.utils.fused_optim import FusedClipAdam
    from applestar_amd.utils.grad_clip import GradClip
    torch.manual_seed(5)
    shapes = [(64, 32, 3, 3), (100003,), (256,), (7, 5), (40000, 33)]
    pa = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in shapes]
    for p in pa:
        p.grad = torch.zeros_like(p)
    n = [p.numel() for p in pa]
    if segmented:
        flat = torch.nn.Parameter(torch.cat([p.detach().reshape(-1) for p in pa]))
        flat.grad = torch.zeros_like(flat)
        pb = [flat]
        offs = [sum(n[:i]) for i in range(len(n))]
        segments = {flat: list(zip(offs, n))}
    else:
        pb = [torch.nn.Parameter(p.detach().clone()) for p in pa]
        for p in pb:
            p.grad = torch.zeros_like(p)
        segments = None
    oa = torch.optim.Adam(pa, lr=1e-3, weight_decay=1e-5)
    ob = torch.optim.Adam(pb, lr=1e-3, weight_decay=1e-5)
    ca, cb = GradClip('momentum_norm', 1.0, momentum_mode='ema'), GradClip('momentum_norm', 1.0, momentum_mode='ema')
    fused = FusedClipAdam(ob, None, clip=cb, segments=segments)
    for step in range(5):
        gs = [torch.randn_like(a) * (1 + 3 * (step % 2)) for a in pa]     # alternating scale: the clip engages
        for a, g in zip(pa, gs):
            a.grad.copy_(g)
        if segmented:
            pb[0].grad.copy_(torch.cat([g.reshape(-1) for g in gs]))
        else:
            for b, g in zip(pb, gs):
                b.grad.copy_(g)
        na = ca.apply(pa)
        oa.step()
        nb = fused.step()
        assert abs(float(na) - float(nb)) <= 1e-5 * float(na), step
        assert torch.allclose(ca.norm_mom, cb.norm_mom, rtol=1e-5), step
        got = pb[0].detach().split(n) if segmented else [b.detach().reshape(-1) for b in pb]
        for a, b in zip(pa, got):
            assert _err(a.detach().reshape(-1), b) < 1e-6 * max(1.0, a.abs().max().item()), step


def test_fused_momentum_norm_gated_first_step_and_cpu_resume():
    """(1) a gated-off FIRST fused momentum_norm step leaves the EMA uninitialised (the device flag),
    so the next kept step initialises it and updates normally (a host flag would pin every scale to 0);
    (2) a clip state loaded with map_location='cpu' is moved to the device, not re-zeroed: the fused step then
    matches the torch GradClip continuing from the same state."""
    from applestar_amd.utils.fused_optim import FusedClipAdam
    from applestar_amd.utils.grad_clip import GradClip
    torch.manual_seed(7)
    ps = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in [(300, 17), (4097,)]]
    for p in ps:
        p.grad = torch.full_like(p, float('nan'))
    opt = torch.optim.Adam(ps, lr=1e-3)
    clip = GradClip('momentum_norm', 1.0, momentum_mode='ema')
    fused = FusedClipAdam(opt, None, clip=clip)
    snap = [p.detach().clone() for p in ps]
    fused.step(torch.zeros((), device=DEV))
    torch.cuda.synchronize()
    assert float(clip.mom_init) == 0.0 and all(torch.equal(p.detach(), s) for p, s in zip(ps, snap))
    gs = [torch.randn_like(p) for p in ps]
    for p, g in zip(ps, gs):
        p.grad.copy_(g)
    fused.step(torch.ones((), device=DEV))
    torch.cuda.synchronize()
    assert float(clip.mom_init) == 1.0
    assert torch.allclose(clip.norm_mom, torch.stack([g.norm() for g in gs]), rtol=1e-5)
    assert all(not torch.equal(p.detach(), s) for p, s in zip(ps, snap))
    # resume from a CPU-mapped clip state
    sd = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in clip.state_dict().items()}
    a = GradClip('momentum_norm', 1.0, momentum_mode='ema')
    a.load_state_dict({k: (v.clone() if torch.is_tensor(v) else v) for k, v in sd.items()})
    b = GradClip('momentum_norm', 1.0, momentum_mode='ema')
    b.load_state_dict(sd)
    assert b.norm_mom.device.type == 'cpu'
    qa = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    qb = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    oa, ob = torch.optim.Adam(qa, lr=1e-3), torch.optim.Adam(qb, lr=1e-3)
    fb = FusedClipAdam(ob, None, clip=b)
    spike = [torch.randn_like(p) * 50 for p in ps]
    for x, y, g in zip(qa, qb, spike):
        x.grad, y.grad = g.clone(), g.clone()
    a.norm_mom, a.mom_init = a.norm_mom.to(DEV), a.mom_init.to(DEV)
    na = a.apply(qa)
    oa.step()
    nb = fb.step()
    assert b.norm_mom.is_cuda and abs(float(na) - float(nb)) <= 1e-5 * float(na)
    assert float(nb) < 0.1 * float(torch.stack([g.norm() for g in spike]).norm())    # the spike was clipped
    for x, y in zip(qa, qb):
        assert _err(x.detach().reshape(-1), y.detach().reshape(-1)) < 1e-6 * max(1.0, x.abs().max().item())


@pytest.mark.parametrize('clip_type', ['pytorch_norm', 'momentum_norm'])
def test_fused_adam_gate_skips_update(clip_type):
    """A zero health gate (timed-out LSTM exchange) with NaN gradients leaves the parameters, both Adam moments
    and the momentum EMA bit-identical; the next step with the gate open updates normally."""
    from applestar_amd.utils.fused_optim import FusedClipAdam
    from applestar_amd.utils.grad_clip import GradClip
    torch.manual_seed(6)
    ps = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in [(300, 17), (70001,)]]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = torch.optim.Adam(ps, lr=1e-3, betas=(0.5, 0.99), weight_decay=1e-4)
    clip = GradClip(clip_type, 1.0, momentum_mode='ema')
    fused = FusedClipAdam(opt, 1.0 if clip_type == 'pytorch_norm' else None, clip=clip)
    fused.step(torch.ones((), device=DEV))                                # state exists, EMA initialised
    snap = [t.clone() for p in ps for t in (p.detach(), opt.state[p]['exp_avg'], opt.state[p]['exp_avg_sq'])]
    mom = clip.norm_mom.clone() if clip.norm_mom is not None else None
    for p in ps:
        p.grad.fill_(float('nan'))
    fused.step(torch.zeros((), device=DEV))
    torch.cuda.synchronize()
    now = [t for p in ps for t in (p.detach(), opt.state[p]['exp_avg'], opt.state[p]['exp_avg_sq'])]
    assert all(torch.equal(a, b) for a, b in zip(snap, now))
    if mom is not None:
        assert torch.equal(mom, clip.norm_mom)
    for p in ps:
        p.grad.copy_(torch.randn_like(p))
    fused.step(torch.ones((), device=DEV))
    assert all(torch.isfinite(p).all() and not torch.equal(p.detach(), s) for p, s in zip(ps, snap[::3]))


def test_fused_adam_device_hparams_in_graph():
    """The update captured in a HIP graph reads lr / bias corrections from the device buffer that prepare()
    refreshes before each replay: 4 replays == 4 eager fused steps."""
    from applestar_amd.utils.fused_optim import FusedClipAdam
    torch.manual_seed(8)
    shapes = [(513, 9), (4096,)]
    pa = [torch.nn.Parameter(torch.randn(*s, device=DEV)) for s in shapes]
    pb = [torch.nn.Parameter(p.detach().clone()) for p in pa]
    for p in pa + pb:
        p.grad = torch.zeros_like(p)
    oa = torch.optim.Adam(pa, lr=1e-2, betas=(0.0, 0.99), eps=1e-5)
    ob = torch.optim.Adam(pb, lr=1e-2, betas=(0.0, 0.99), eps=1e-5)
    fa, fb = FusedClipAdam(oa, 1.0), FusedClipAdam(ob, 1.0, device_hparams=True)
    grads = [[torch.randn_like(p) for p in pa] for _ in range(5)]

    def load(ps, i):
        for p, g in zip(ps, grads[i]):
            p.grad.copy_(g)
    load(pa, 0); fa.step()
    load(pb, 0); fb.step()                 # eager first step (creates the state)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            fb.step()
    torch.cuda.current_stream().wait_stream(s)
    for i in range(1, 5):
        load(pa, i); fa.step()
        load(pb, i); fb.prepare(); g.replay()
    torch.cuda.synchronize()
    for a, b in zip(pa, pb):
        assert torch.equal(a.detach(), b.detach())
    ob.state_dict()
    assert float(ob.state[pb[0]]['step']) == 5.0


@pytest.mark.parametrize('M,Nc,K', [(390, 256, 256), (384, 1024, 448), (33, 70, 1020), (2047, 130, 4096), (1, 327, 64)])
@pytest.mark.parametrize('mode', ['bias_relu', 'res_add', 'drelu'])
def test_gemm_f32_small_epilogues_match_fp64(M, Nc, K, mode, f32_mfma):
    """gemm_f32 on few-row products (< 128 pipe tiles: one wave per 32 x 32 tile, operands from L2, K tails,
    ragged M / N edges, K up to 4096) with each epilogue vs float64, in both f32 MFMA modes."""
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(Nc, K, device=DEV) / K ** 0.5
    bias = 0.1 * torch.randn(Nc, device=DEV)
    res = torch.randn(M, Nc, device=DEV)
    C = N.ensure_loaded()
    ref = a.double() @ b.double().t() + bias.double()
    if mode == 'bias_relu':
        got, ref = C.gemm_f32(a, b, bias, None, 1), torch.relu(ref)
    elif mode == 'res_add':
        got, ref = C.gemm_f32(a, b, bias, res, 0), ref + res.double()
    else:
        got, ref = C.gemm_f32(a, b, bias, res, 4), ref * (res.double() > 0)
    assert (got.double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize('M,Nc,K', [(390, 256, 256), (384, 1024, 448), (33, 72, 1024), (1, 328, 64)])
@pytest.mark.parametrize('mode', ['bias_relu', 'res_add', 'drelu'])
def test_gemm_bf16_small_epilogues(M, Nc, K, mode):
    """gemm_bf16_small (the bf16 step's few-row products): bf16 operands, fp32 accumulation + epilogue, bf16 out,
    vs float64 of the same bf16 inputs within one bf16 rounding of the result."""
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(Nc, K, device=DEV) / K ** 0.5).bfloat16()
    bias = 0.1 * torch.randn(Nc, device=DEV)
    res = torch.randn(M, Nc, device=DEV).bfloat16()
    C = N.ensure_loaded()
    ref = a.double() @ b.double().t() + bias.double()
    if mode == 'bias_relu':
        got, ref = C.gemm_bf16_small(a, b, bias, None, 1), torch.relu(ref)
    elif mode == 'res_add':
        got, ref = C.gemm_bf16_small(a, b, bias, res, 0), ref + res.double()
    else:
        got, ref = C.gemm_bf16_small(a, b, bias, res, 4), ref * (res.double() > 0)
    assert got.dtype == torch.bfloat16
    err = (got.double() - ref).abs()
    assert (err <= 2 ** -7 * ref.abs() + 1e-3 * max(1.0, ref.abs().max().item())).all(), err.max().item()


def test_bf16_linear_small_path_matches_library(monkeypatch):
    """A few-row bf16 linear (+ ReLU) through _Linear on the small-tile kernels vs the library path (switch off):
    forward and all three gradients within bf16 rounding."""
    from applestar_amd.ops import native as NN
    torch.manual_seed(7)
    x0 = torch.randn(384, 448, device=DEV).bfloat16()
    w0 = (torch.randn(256, 448, device=DEV) / 448 ** 0.5).bfloat16()
    b0 = (0.1 * torch.randn(256, device=DEV)).bfloat16()
    g = torch.randn(384, 256, device=DEV).bfloat16()
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(NN, 'BF16_SMALL', on)
        x, w, b = (t.clone().requires_grad_() for t in (x0, w0, b0))
        y = NN.linear(x, w, b, act='relu')
        y.backward(g)
        outs[on] = [t.float() for t in (y, x.grad, w.grad, b.grad)]
    for name, a, r in zip(('y', 'dx', 'dw', 'db'), outs[True], outs[False]):
        assert (a - r).norm() <= 1e-2 * r.norm(), (name, float((a - r).norm() / r.norm()))


_SMALL_SHAPES = [(390, 128, 167, 'relu'), (390, 64, 10, 'relu'), (384, 327, 256, None), (384, 2, 256, None),
                 (390, 1, 256, None), (384, 256, 448, 'sigmoid'), (100, 77, 33, 'relu'), (1, 5, 7, None),
                 (3000, 129, 131, 'sigmoid'), (390, 64, 269, 'relu')]


def _count_small(monkeypatch):
    from applestar_amd.ops import native as NN
    C = NN.ensure_loaded()
    calls = {'nt': 0, 'tn': 0}

    class _Wrap:
        def __getattr__(self, k):
            return getattr(C, k)

        def small_gemm(self, *a):
            calls['nt'] += 1
            return C.small_gemm(*a)

        def small_wgrad(self, *a):
            calls['tn'] += 1
            return C.small_wgrad(*a)
    monkeypatch.setattr(NN, '_C', _Wrap())
    return calls


@pytest.mark.parametrize('R,Nc,K,act', _SMALL_SHAPES)
def test_small_linear_native_fp32_matches_fp64(R, Nc, K, act, f32_mfma, monkeypatch):
    """Few-row fp32 linears of any shape (odd K / N, sigmoid gates) on gemm_small.hip: forward (bias + act in the
    epilogue), dX (activation gradient applied as dY is loaded) and the TN dW + db kernel, vs float64."""
    from applestar_amd.ops import native as NN
    calls = _count_small(monkeypatch)
    torch.manual_seed(R + K)
    x = torch.randn(R, K, device=DEV).requires_grad_()
    w = (torch.randn(Nc, K, device=DEV) / K ** 0.5).requires_grad_()
    b = (0.1 * torch.randn(Nc, device=DEV)).requires_grad_()
    y = NN.linear(x, w, b, act=act)
    xs, ws, bs = _f64(x), _f64(w), _f64(b)
    yr = xs @ ws.t() + bs
    yr = torch.relu(yr) if act == 'relu' else (torch.sigmoid(yr) if act == 'sigmoid' else yr)
    assert _err(y.cpu(), yr) < 1e-5 * max(1.0, yr.abs().max().item())
    g = torch.randn(yr.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV))
    yr.backward(g)
    for name, a, ref in (('dx', x.grad, xs.grad), ('dw', w.grad, ws.grad), ('db', b.grad, bs.grad)):
        e = _err(a.cpu(), ref)
        assert e < 2e-5 * max(1.0, ref.abs().max().item()), (name, e)
    assert calls == {'nt': 2, 'tn': 1}, calls


@pytest.mark.parametrize('R,Nc,K,act', _SMALL_SHAPES)
def test_small_linear_native_bf16_matches_fp64(R, Nc, K, act, monkeypatch):
    """The bf16 step's form of the same layers: bf16 operands / outputs / gradients, fp32 accumulation, vs float64
    of the same bf16 inputs within bf16 rounding (relative Frobenius error)."""
    from applestar_amd.ops import native as NN
    calls = _count_small(monkeypatch)
    torch.manual_seed(R + K + 1)
    x = torch.randn(R, K, device=DEV).bfloat16().requires_grad_()
    w = (torch.randn(Nc, K, device=DEV) / K ** 0.5).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(Nc, device=DEV)).bfloat16().requires_grad_()
    y = NN.linear(x, w, b, act=act)
    assert y.dtype == torch.bfloat16
    xs, ws, bs = _f64(x), _f64(w), _f64(b)
    yr = xs @ ws.t() + bs
    yr = torch.relu(yr) if act == 'relu' else (torch.sigmoid(yr) if act == 'sigmoid' else yr)
    g = torch.randn(yr.shape, dtype=torch.float64).bfloat16().double()
    y.backward(g.to(DEV).bfloat16())
    yr.backward(g)
    for name, a, ref in (('y', y, yr), ('dx', x.grad, xs.grad), ('dw', w.grad, ws.grad), ('db', b.grad, bs.grad)):
        assert a.dtype == torch.bfloat16, name
        e = float((a.double().cpu() - ref.detach()).norm() / max(ref.detach().norm().item(), 1e-30))
        assert e < 1e-2, (name, e)
    assert calls == {'nt': 2, 'tn': 1}, calls


@pytest.mark.parametrize('M,Nc,K,act', [(390, 256, 48640, 1), (390, 128, 12160, 0), (17, 40, 9001, 2)])
@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_small_gemm_splitk_matches_fp64(M, Nc, K, act, dt, f32_mfma):
    """Split-K few-row product (the spatial encoder's 48,640-wide fc): slices + ordered sum + epilogue vs float64."""
    C = N.ensure_loaded()
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=DEV).to(dt)
    b = (torch.randn(Nc, K, device=DEV) / K ** 0.5).to(dt)
    bias = 0.1 * torch.randn(Nc, device=DEV)
    ref = a.double() @ b.double().t() + bias.double()
    ref = torch.relu(ref) if act == 1 else (torch.sigmoid(ref) if act == 2 else ref)
    got = C.small_gemm_splitk(a, b, bias, act)
    assert got.dtype == dt
    err = (got.double() - ref).abs().max().item()
    tol = (2e-5 if dt == torch.float32 else 1e-2) * max(1.0, ref.abs().max().item())
    assert err < tol, err


def test_linear_f32_long_k_grads_match_fp64(f32_mfma):
    """A few-row fp32 linear with K > 4096 (split-K forward, native dX / dW) vs float64."""
    from applestar_amd.ops import native as NN
    torch.manual_seed(41)
    R, Nc, K = 390, 256, 16640
    x = torch.randn(R, K, device=DEV).requires_grad_()
    w = (torch.randn(Nc, K, device=DEV) / K ** 0.5).requires_grad_()
    b = (0.1 * torch.randn(Nc, device=DEV)).requires_grad_()
    y = NN.linear(x, w, b, act='relu')
    xs, ws, bs = _f64(x), _f64(w), _f64(b)
    yr = torch.relu(xs @ ws.t() + bs)
    assert _err(y.cpu(), yr) < 1e-5 * max(1.0, yr.abs().max().item())
    g = torch.randn(yr.shape, dtype=torch.float64)
    y.backward(g.float().to(DEV))
    yr.backward(g)
    for name, a, ref in (('dx', x.grad, xs.grad), ('dw', w.grad, ws.grad), ('db', b.grad, bs.grad)):
        e = _err(a.cpu(), ref)
        assert e < 2e-5 * max(1.0, ref.abs().max().item()), (name, e)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_small_gemm_residual_epilogues(dt, f32_mfma):
    """small_gemm's residual add and residual ReLU-mask epilogues (odd K / N) vs float64."""
    C = N.ensure_loaded()
    torch.manual_seed(31)
    a = torch.randn(77, 45, device=DEV).to(dt)
    b = (torch.randn(39, 45, device=DEV) / 7).to(dt)
    res = torch.randn(77, 39, device=DEV).to(dt)
    ref = a.double() @ b.double().t()
    tol = 2e-5 if dt == torch.float32 else 1e-2
    got = C.small_gemm(a, b, None, res, None, 0, 0)
    assert (got.double() - (ref + res.double())).abs().max().item() < tol * 4
    got = C.small_gemm(a, b, None, res, None, 0, 4)
    assert (got.double() - ref * (res.double() > 0)).abs().max().item() < tol * 4


@pytest.mark.parametrize('M,Nc,K', [(5000, 768, 256), (3001, 256, 1024), (20000, 32, 24), (2500, 96, 136),
                                    (9000, 1024, 256), (390, 12160, 128)])
@pytest.mark.parametrize('mode', ['bias_relu', 'res_add', 'drelu'])
def test_gemm_bf16_pipe_epilogues(M, Nc, K, mode):
    """gemm_bf16 (the bf16 step's large products on the LDS-DMA ring): bf16 operands, fp32 accumulation and
    epilogue, bf16 out, vs float64 of the same bf16 inputs within one bf16 rounding of the result."""
    torch.manual_seed(M + K + 3)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(Nc, K, device=DEV) / K ** 0.5).bfloat16()
    bias = 0.1 * torch.randn(Nc, device=DEV)
    res = torch.randn(M, Nc, device=DEV).bfloat16()
    C = N.ensure_loaded()
    ref = a.double() @ b.double().t() + bias.double()
    if mode == 'bias_relu':
        got, ref = C.gemm_bf16(a, b, bias, None, 1), torch.relu(ref)
    elif mode == 'res_add':
        got, ref = C.gemm_bf16(a, b, bias, res, 0), ref + res.double()
    else:
        got, ref = C.gemm_bf16(a, b, bias, res, 4), ref * (res.double() > 0)
    assert got.dtype == torch.bfloat16
    err = (got.double() - ref).abs()
    assert (err <= 2 ** -7 * ref.abs() + 1e-3 * max(1.0, ref.abs().max().item())).all(), err.max().item()


def test_bf16_linear_pipe_path_matches_library(monkeypatch):
    """A many-row bf16 linear (+ ReLU) through _Linear on gemm_bf16 (forward and dX) vs the library path (switch
    off): forward and all three gradients within bf16 rounding."""
    from applestar_amd.ops import native as NN
    torch.manual_seed(8)
    x0 = torch.randn(6000, 256, device=DEV).bfloat16()
    w0 = (torch.randn(1024, 256, device=DEV) / 16).bfloat16()
    b0 = (0.1 * torch.randn(1024, device=DEV)).bfloat16()
    g = torch.randn(6000, 1024, device=DEV).bfloat16()
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(NN, 'BF16_PIPE', on)
        x, w, b = (t.clone().requires_grad_() for t in (x0, w0, b0))
        y = NN.linear(x, w, b, act='relu')
        y.backward(g)
        outs[on] = [t.float() for t in (y, x.grad, w.grad, b.grad)]
    for name, a, r in zip(('y', 'dx', 'dw', 'db'), outs[True], outs[False]):
        assert (a - r).norm() <= 1e-2 * r.norm(), (name, float((a - r).norm() / r.norm()))


@pytest.mark.parametrize('M,Nc,K', [(5000, 768, 256), (3001, 256, 1024), (20000, 32, 20), (2500, 96, 132)])
@pytest.mark.parametrize('mode', ['bias_relu', 'res_add', 'drelu'])
def test_gemm_f32_epilogues_match_fp64(M, Nc, K, mode, f32_mfma):
    """gemm_f32.hip: A [M,K] . B [Nc,K]^T with each epilogue (bias + ReLU; + residual; ReLU-output mask) vs float64."""
    torch.manual_seed(M)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(Nc, K, device=DEV) / K ** 0.5
    bias = 0.1 * torch.randn(Nc, device=DEV)
    res = torch.randn(M, Nc, device=DEV)
    C = N.ensure_loaded()
    ref = a.double().cpu() @ b.double().cpu().t() + bias.double().cpu()
    if mode == 'bias_relu':
        out = C.gemm_f32(a, b, bias, None, 1)
        ref = ref.clamp_min(0)
    elif mode == 'res_add':
        out = C.gemm_f32(a, b, bias, res, 0)
        ref = ref + res.double().cpu()
    else:
        out = C.gemm_f32(a, b, bias, res, 4)
        ref = ref * (res.double().cpu() > 0)
    assert _err(out.cpu(), ref) < 1e-5 * max(1.0, ref.abs().max().item())


def _same_or_boundary(a, b, logits, u):
    """Sampled indices agree, except where u sits within float rounding of a CDF boundary."""
    p = torch.softmax(logits.double(), -1)
    cdf = torch.cumsum(p, -1)
    for i in torch.nonzero(a != b).flatten().tolist():
        lo = min(int(a[i]), int(b[i]))
        assert abs(float(cdf[i, lo]) - float(u[i])) < 1e-5, (i, int(a[i]), int(b[i]))


@pytest.mark.parametrize('B,C,dtype,masked', [(16, 327, torch.bfloat16, 'shared'), (3, 128, torch.float32, None),
                                              (64, 2, torch.bfloat16, None), (2, 24320, torch.float32, None),
                                              (5, 513, torch.float32, 'lens')])
def test_head_sample_matches_reference_sampler(B, C, dtype, masked):
    """heads.hip head_sample: same scaled / masked logits, same inverse-CDF draw as sample_from_logits for the same
    uniforms, and the row-gathered embedding relu(W^T[a] + b)."""
    from applestar_amd import ops
    from applestar_amd.models.heads import sample_from_logits, NEG
    torch.manual_seed(B * C)
    logits = (torch.randn(B, C, device=DEV) * 3).to(dtype)
    u = torch.rand(B, device=DEV)
    mask = lens = None
    ref = logits.float() / 0.8
    if masked == 'shared':
        mask = torch.rand(C, device=DEV) > 0.3
        ref = ref.masked_fill(~mask, NEG)
    elif masked == 'lens':
        lens = torch.randint(1, C + 1, (B,), device=DEV)
        ref = ref.masked_fill(torch.arange(C, device=DEV)[None] >= lens[:, None], NEG)
    table = torch.randn(C, 256, device=DEV).to(dtype)
    bias = torch.randn(256, device=DEV)
    with torch.no_grad():
        out, act, emb = ops.head_sample(logits, 0.8, mask=mask, lens=lens, u=u, table=table, bias=bias)
    assert _err(out, ref) < 1e-5 * ref.abs().clamp(max=1e3).max().item() + 1e-6
    ra = sample_from_logits(ref, u)
    _same_or_boundary(act.cpu(), ra.cpu(), ref.cpu(), u.cpu())
    assert torch.equal(emb, torch.relu(table.float()[act] + bias))
    if mask is not None:
        assert bool(mask[act].all())
    if lens is not None:
        assert bool((act < lens).all())


@pytest.mark.parametrize('edtype', [torch.float32, torch.bfloat16])
def test_target_unit_fused_matches_torch(edtype):
    """heads.hip target_unit_sample == TargetUnitHead's torch path (query MLP, key dot, mask, 1/T, sample)."""
    from applestar_amd import ops
    from applestar_amd.models.heads import TargetUnitHead
    torch.manual_seed(9)
    B, N = 6, 300
    head = TargetUnitHead().to(DEV)
    emb = torch.randn(B, 1024, device=DEV).to(edtype)
    ent = torch.randn(B, N, 256, device=DEV).to(edtype)
    en = torch.randint(1, N + 1, (B,), device=DEV)
    u = torch.rand(B, device=DEV)
    with torch.no_grad():
        key = head.key_fc(ent.float()).to(edtype)
        lf, af = head(emb, ent, en, 0.7, u=u, key=key)
        ops.set_native(False)
        try:
            lr_, ar_ = head(emb.float(), ent.float(), en, 0.7, u=u, key=key.float())
        finally:
            ops.set_native(True)
    valid = lr_ > -1e8
    assert torch.equal(valid, lf > -1e8)
    assert _err(lf[valid], lr_[valid]) < 2e-4 * max(1.0, lr_[valid].abs().max().item())
    _same_or_boundary(af.cpu(), ar_.cpu(), lr_.cpu(), u.cpu())


def test_wgrad_f32_long_reduction_is_deterministic():
    """A split-R fp32 weight gradient with more than 1,024 slices takes the two-pass chunked column reduction
    (pool_reduce.hip column_reduce_chunk_kernel): fixed summation order - bit-identical across launches (the former
    zero fill + atomicAdd pass was not) - and within the usual bound of float64."""
    from applestar_amd.ops import native
    C = native.ensure_loaded()
    torch.manual_seed(3)
    R, N, K = 300000, 128, 128
    dy = torch.randn(R, N, device=DEV)
    x = torch.randn(R, K, device=DEV)
    dw1, db1 = C.wgrad_f32(dy, x, 0, True)
    dw2, db2 = C.wgrad_f32(dy, x, 0, True)
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    ref = dy[:20000].double().cpu().t() @ x[:20000].double().cpu()
    part = C.wgrad_f32(dy[:20000].contiguous(), x[:20000].contiguous(), 0, False)[0]
    assert float((part.double().cpu() - ref).abs().max()) < 1e-3 * 20000 ** 0.5
    assert float((db1.double().cpu() - dy.double().cpu().sum(0)).abs().max()) < 1e-3 * R ** 0.5
