"""utils/serialize.py frames: the native codec (csrc/codec.cpp) and the Python codec produce and read the same
frames (byte-identical encodes, cross-decodes), for every supported dtype and leaf kind."""
import math

import pytest
import torch

from applestar_amd.utils import serialize

NATIVE = serialize._native()
needs_native = pytest.mark.skipif(not NATIVE, reason='native extension not built')


def _tree():
    g = torch.Generator().manual_seed(0)
    t = {
        'f32': torch.randn(3, 5, generator=g), 'f16': torch.randn(7, generator=g).half(),
        'bf16': torch.randn(2, 2, generator=g).bfloat16(), 'f64': torch.randn(4, generator=g).double(),
        'i64': torch.arange(9).view(3, 3), 'i32': torch.arange(5, dtype=torch.int32),
        'i16': torch.tensor([-3, 7], dtype=torch.int16), 'i8': torch.tensor([-1, 2], dtype=torch.int8),
        'u8': torch.tensor([0, 255], dtype=torch.uint8), 'b': torch.tensor([True, False, True]),
        'empty': torch.zeros(0, 4), 'scalar_t': torch.tensor(3.5), 'noncontig': torch.randn(4, 6, generator=g).t(),
        'nested': {'l': [torch.ones(2), 1, 2.5, None, True, 'x"y\\z\né\U0001F600'],
                   'tu': (torch.zeros(1, dtype=torch.long), -7, 2 ** 70, float('inf'), -float('inf'), 1.0, 1e-300)},
        7: 'int key', 'nan': float('nan'),
    }
    return t


def _eq(a, b):
    if torch.is_tensor(a):
        assert torch.is_tensor(b) and a.dtype == b.dtype and a.shape == b.shape
        assert torch.equal(a.contiguous().view(-1).view(torch.uint8) if a.dtype != torch.bool else a,
                           b.contiguous().view(-1).view(torch.uint8) if b.dtype != torch.bool else b)
    elif isinstance(a, dict):
        assert sorted(map(str, a)) == sorted(map(str, b))
        for k in a:
            _eq(a[k], b[str(k)] if str(k) in b else b[k])
    elif isinstance(a, (list, tuple)):
        assert type(a) == type(b) and len(a) == len(b)
        for x, y in zip(a, b):
            _eq(x, y)
    elif isinstance(a, float) and math.isnan(a):
        assert isinstance(b, float) and math.isnan(b)
    else:
        assert a == b and type(a) == type(b), (a, b)


def test_python_codec_roundtrip():
    t = _tree()
    _eq(t, serialize.loads_py(serialize.dumps_py(t)))


@needs_native
def test_native_matches_python_codec():
    t = _tree()
    nat = NATIVE.tree_dumps(t)
    py = serialize.dumps_py(t)
    assert nat == py                                    # same header text and body layout
    _eq(t, NATIVE.tree_loads(py, True))
    _eq(t, serialize.loads_py(nat))
    _eq(t, serialize.loads(nat))


@needs_native
def test_native_alias_mode_and_fallback():
    t = {'a': torch.arange(10, dtype=torch.float32), 'b': [torch.ones(3, dtype=torch.int16)]}
    buf = bytearray(serialize.dumps(t))
    out = serialize.loads(buf, copy=False)
    _eq(t, out)
    del buf
    assert out['a'].sum().item() == 45.0               # the aliased tensors keep the buffer alive
    import numpy as np
    mixed = {'np': np.arange(4), 'npf': np.float32(2.5)}   # numpy leaves: the Python encoder takes over
    back = serialize.loads(serialize.dumps(mixed))
    assert torch.equal(back['np'], torch.arange(4)) and back['npf'] == 2.5
    with pytest.raises(ValueError):
        serialize.loads(b'NOTAFRAME' + bytes(20))
    z = serialize.dumps(t, compress=True)               # compressed frames stay on the Python codec
    _eq(t, serialize.loads(z))


@needs_native
def test_native_collate_frames_matches_collate_obs():
    """collate_frames (native: B request frames -> one staged batch) == collate_obs over the decoded requests:
    entity leaves padded to the entity bucket, action_info selected_units to 64, hidden states stacked."""
    from applestar_amd.agent.collate import collate_obs
    from applestar_amd.lib.features import random_obs
    g = torch.Generator().manual_seed(3)
    obs = random_obs(3, entity_num=torch.tensor([12, 200, 77]), generator=g)
    reqs = []
    for i in range(3):
        n = int(obs['entity_num'][i])
        r = {k: ({kk: (vv[i, :n] if k == 'entity_info' else vv[i]) for kk, vv in v.items()} if isinstance(v, dict)
                 else v[i]) for k, v in obs.items()}
        r['hidden_state'] = [(torch.randn(384, generator=g), torch.randn(384, generator=g)) for _ in range(3)]
        r['action_info'] = {'action_type': torch.tensor(i), 'selected_units': torch.arange(i + 2)}
        r['flag'] = i
        reqs.append(r)
    for pad in (0, 256):
        ref = collate_obs(reqs, pad_entities=pad)
        got = NATIVE.collate_frames([serialize.dumps(r) for r in reqs], pad)
        _eq(ref, got)
    with pytest.raises(ValueError):
        bad = dict(reqs[1])
        bad.pop('flag')
        NATIVE.collate_frames([serialize.dumps(reqs[0]), serialize.dumps(bad)], 0)


def _patched_header(frame: bytes, old: bytes, new: bytes) -> bytes:
    """The frame with one header substring replaced (hlen re-stamped, body re-aligned as the encoder would)."""
    import struct
    pre = len(serialize.MAGIC) + 9
    hlen = struct.unpack('<Q', frame[len(serialize.MAGIC):len(serialize.MAGIC) + 8])[0]
    header = frame[pre:pre + hlen]
    pad = (-(pre + hlen)) % 64
    body = frame[pre + hlen + pad:]
    assert old in header
    header = header.replace(old, new, 1)
    npad = (-(pre + len(header))) % 64
    return serialize.MAGIC + struct.pack('<QB', len(header), 0) + header + b'\0' * npad + body


@needs_native
def test_native_decoders_reject_malformed_frames():
    """a frame whose tensor descriptor disagrees with its bytes, a huge / truncated header
    length, or a header cut mid-token must raise ValueError in BOTH native decoders (tree_loads and the inference
    server's collate_frames) - never read outside the frame."""
    import struct
    t = {'a': torch.arange(12, dtype=torch.int32).reshape(3, 4), 'b': 1.5}
    good = serialize.dumps(t)
    assert serialize.loads(good)['a'].shape == (3, 4)
    nb = str(12 * 4).encode()
    bad_frames = [
        _patched_header(good, b'[3, 4]', b'[300, 4]'),            # shape larger than nbytes
        _patched_header(good, b'[3, 4]', b'[-3, -4]'),            # negative dims (product matches)
        _patched_header(good, b', ' + nb + b']', b', -48]'),       # negative nbytes
        _patched_header(good, b', ' + nb + b']', b', 0]'),         # zero nbytes for a non-empty shape
        _patched_header(good, b'[3, 4]', b'[3, 99999999999999999999]'),   # overflowing dim
        good[:len(serialize.MAGIC)] + struct.pack('<Q', 2 ** 63 + 5) + good[len(serialize.MAGIC) + 8:],  # huge hlen
        good[:len(serialize.MAGIC)] + struct.pack('<Q', len(good)) + good[len(serialize.MAGIC) + 8:],    # hlen > frame
        good[:len(serialize.MAGIC) + 9 + 20],                     # truncated mid-header
    ]
    for i, f in enumerate(bad_frames):
        with pytest.raises(ValueError):
            NATIVE.tree_loads(f, True)
        with pytest.raises(ValueError):
            NATIVE.collate_frames([f], 0)
    # a descriptor pointing past the body
    with pytest.raises(ValueError):
        NATIVE.tree_loads(_patched_header(good, b'0, ' + nb, b'64, ' + nb) if b'0, ' + nb in good else good[:-8], True)
    # literal scanning stops at the header end: a header ending in a bare 'tru' prefix
    with pytest.raises(ValueError):
        NATIVE.tree_loads(_patched_header(good, b'1.5', b'tru'), True)
