"""Shape-static learner step pieces (CPU): the fixed-row-count entity packing used by the graph-captured
step must give the data-dependent packing's outputs and gradients."""
import torch

from applestar_amd.lib.features import random_obs
from applestar_amd.models import encoders
from applestar_amd.models.encoders import EntityEncoder, entity_pad_for


def _grads(m):
    return {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}


def test_entity_pad_for_is_bucketed():
    assert entity_pad_for(1, 64) == 8 * 64
    assert entity_pad_for(8 * 64, 64) == 8 * 64
    assert entity_pad_for(8 * 64 + 1, 64) == 16 * 64
    for total in (1, 100, 4095, 4096, 4097, 100000):
        p = entity_pad_for(total, 512)
        assert p >= total and p % (encoders.PAD_SEGMENTS * 512) == 0
        assert p - total < encoders.PAD_SEGMENTS * 512      # padding fits the extra segments


def test_padded_entity_packing_matches_packed():
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(3)
    en = torch.tensor([5, 1, 17, 9, 12, 3])
    obs = random_obs(6, entity_num=en, generator=g)
    ei, N = obs['entity_info'], int(en.max())
    enc = EntityEncoder()
    total = int(en.clamp(max=N).sum())
    ref_e, ref_m, ref_v = enc(ei, en, total)
    (ref_e.square().sum() + ref_m.square().sum()).backward()
    ref_g = _grads(enc)
    enc.zero_grad()
    pad = entity_pad_for(total, N)
    assert pad > total
    e, m, v = enc(ei, en, total, pad)
    (e.square().sum() + m.square().sum()).backward()
    got_g = _grads(enc)
    assert torch.equal(v, ref_v)
    assert torch.allclose(e, ref_e, atol=1e-5, rtol=1e-5)
    assert torch.allclose(m, ref_m, atol=1e-5, rtol=1e-5)
    assert ref_g.keys() == got_g.keys()
    for k in ref_g:
        assert torch.allclose(got_g[k], ref_g[k], atol=1e-4, rtol=1e-4), k
