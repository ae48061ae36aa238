"""Optional network blocks (models/optional.py): numerics vs the reference modules where the reference
tree is present (CPU, fp32), plus self-consistency checks that always run."""
import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.models import optional as O

needs_ref = pytest.mark.skipif(not reference_available(), reason='reference tree not available')


def _ref_module_utils():
    import_reference()
    import distar.agent.default.model.module_utils as mu
    return mu


def _ref_lstm():
    import_reference()
    import distar.agent.default.model.lstm as rl
    return rl


def test_attention_pool_prefix_matches_sequential_masks():
    torch.manual_seed(0)
    for max_num in (None, 65):
        ap = O.AttentionPool(32, 2, 64, max_num=max_num)
        B, N, S = 3, 9, 5
        key = torch.randn(B, N, 32)
        labels = torch.stack([torch.randperm(N)[:S] for _ in range(B)])  # distinct, as in the head
        new = torch.rand(B, S) > 0.3
        new[0] = False  # an empty selection: uniform softmax over all tokens
        got = ap.prefix(key, labels, new)
        for i in range(S):
            m = torch.zeros(B, N)
            for b in range(B):
                for j in range(i + 1):
                    if new[b, j]:
                        m[b, labels[b, j]] = 1
            exp = ap(key, num=m.sum(1), mask=m.unsqueeze(2))
            torch.testing.assert_close(got[:, i], exp, atol=1e-5, rtol=1e-5)


@needs_ref
@pytest.mark.parametrize('max_num', [None, 20])
def test_attention_pool_matches_reference(max_num):
    mu = _ref_module_utils()
    torch.manual_seed(1)
    ref = mu.AttentionPool(16, 2, 24, max_num=max_num)
    ours = O.AttentionPool(16, 2, 24, max_num=max_num)
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randn(4, 7, 16)
    mask = (torch.rand(4, 7, 1) > 0.4)
    num = torch.randint(0, 20, (4,))
    kw = {'num': num} if max_num else {}
    torch.testing.assert_close(ours(x, mask=mask, **kw), ref(x, mask=mask.clone(), **kw), atol=1e-5, rtol=1e-5)


@needs_ref
@pytest.mark.parametrize('method', ['conv-film', 'block-input-film', 'bn-film', 'relu-film', 'block-output-film'])
def test_filmed_resblock_matches_reference(method):
    mu = _ref_module_utils()
    torch.manual_seed(2)
    kw = dict(with_cond=[True], with_batchnorm=True, condition_method=method, num_extra_channels=2,
              extra_channel_freq=2, num_cond_maps=3)
    ref = mu.FiLMedResBlock(8, **kw).eval()
    ours = O.FiLMedResBlock(8, **kw).eval()
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randn(2, 8, 5, 6)
    g, b = torch.randn(2, 8), torch.randn(2, 8)
    ex, cm = torch.randn(2, 2, 5, 6), torch.randn(2, 3, 5, 6)
    torch.testing.assert_close(ours(x, g, b, ex, cm), ref(x, g, b, ex, cm), atol=1e-5, rtol=1e-5)


@needs_ref
def test_norm_lstm_matches_reference():
    mu = _ref_module_utils()
    torch.manual_seed(3)
    ref = mu.LSTM(12, 16, 2, norm_type='LN')
    ours = O.NormLSTM(12, 16, 2, norm_type='LN')
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randn(5, 3, 12)
    h0, c0 = torch.randn(2, 3, 16), torch.randn(2, 3, 16)
    ro, rs = ref(x, (h0, c0))
    oo, (oh, oc) = ours(x, (h0, c0))
    torch.testing.assert_close(oo, ro, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(oh, torch.stack([s[0] for s in rs]), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(oc, torch.stack([s[1] for s in rs]), atol=1e-5, rtol=1e-5)


def test_pytorch_lstm_state_formats():
    torch.manual_seed(4)
    m = O.get_lstm('pytorch', 6, 8, 2)
    x = torch.randn(4, 3, 6)
    out, (h, c) = m(x, None)
    assert out.shape == (4, 3, 8) and h.shape == (2, 3, 8)
    per_sample = [None, (h[:, 1:2], c[:, 1:2]), None]
    out2, listed = m(x, per_sample, list_next_state=True)
    assert len(listed) == 3 and listed[0][0].shape == (2, 1, 8)


@needs_ref
@pytest.mark.parametrize('bidirectional', [False, True])
def test_script_lstm_matches_reference(bidirectional):
    rl = _ref_lstm()
    torch.manual_seed(5)
    ref = rl.script_lstm(6, 8, 2, bidirectional=bidirectional)
    ours = O.script_lstm(6, 8, 2, bidirectional=bidirectional)
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randn(4, 3, 6)
    z = torch.zeros(3, 8)
    st = [[(z, z), (z, z)] if bidirectional else (z, z) for _ in range(2)]
    ro, _ = ref(x, st)
    oo, _ = ours(x, st)
    torch.testing.assert_close(oo, ro, atol=1e-5, rtol=1e-5)


@needs_ref
def test_bidirectional_lnlstm_matches_reference():
    rl = _ref_lstm()
    torch.manual_seed(6)
    ref = rl.script_lnlstm(6, 8, 2, bidirectional=True)
    ours = O.script_lnlstm(6, 8, 2, bidirectional=True)
    ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randn(4, 3, 6)
    z = torch.zeros(3, 8)
    st = [[(z, z), (z, z)] for _ in range(2)]
    ro, _ = ref(x, st)
    oo, _ = ours(x, st)
    torch.testing.assert_close(oo, ro, atol=1e-4, rtol=1e-4)


def test_block_builders_key_layout():
    blk = O.conv2d_block(4, 8, 3, 1, 1, activation='relu', norm_type='BN')
    assert list(blk.state_dict())[:2] == ['0.weight', '0.bias']
    assert blk(torch.randn(2, 4, 5, 5)).shape == (2, 8, 5, 5)
    blk = O.conv2d_block(4, 8, 3, 1, 1, pad_type='reflect')
    assert blk(torch.randn(2, 4, 5, 5)).shape == (2, 8, 5, 5)
    d = O.deconv2d_block(8, 4, 4, 2, 1, activation='relu')
    assert d(torch.randn(2, 8, 5, 5)).shape == (2, 4, 10, 10)
    f = O.fc_block2(16, 1, gain=0.1, norm_type='LN')
    assert float(f[0].bias.detach().abs().sum()) == 0.0
    assert O.build_normalization('BN', 2) is torch.nn.BatchNorm2d
    assert O.build_normalization('LN', 1) is torch.nn.LayerNorm
    sbn = O.build_normalization('SyncBN', 2)(8)
    assert sbn(torch.randn(3, 8, 4, 4)).shape == (3, 8, 4, 4)  # no process group -> plain BN
    with pytest.raises(KeyError):
        O.build_normalization('XX')
