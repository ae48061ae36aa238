"""utils/data.py helpers; parity with the reference where its code runs here."""
import collections

import numpy as np
import pytest
import torch

from refutil import reference_available, import_reference
from applestar_amd.utils import data as D
from applestar_amd.models.optional import SoftArgmax, ScatterConnection, build_activation

needs_ref = pytest.mark.skipif(not reference_available(), reason='reference tree not available')


def test_conversions_round_trip():
    item = {'a': np.arange(6).reshape(2, 3), 'b': [1.5, 2.5], 'c': 'name', 'd': (np.float32(3.0), None)}
    t = D.to_tensor(item)
    assert torch.is_tensor(t['a']) and t['a'].shape == (2, 3) and t['c'] == 'name'
    assert torch.equal(t['b'], torch.tensor([1.5, 2.5]))
    back = D.to_ndarray(t)
    assert np.array_equal(back['a'], item['a'])
    assert D.tensor_to_list({'x': torch.tensor([1, 2])}) == {'x': [1, 2]}
    assert D.to_dtype({'x': torch.ones(2)}, torch.float16)['x'].dtype == torch.float16
    assert D.same_shape([torch.zeros(2), torch.ones(2)]) and not D.same_shape([torch.zeros(2), torch.ones(3)])
    x = torch.ones(2, requires_grad=True)
    d = D.detach_grad({'x': [x * 2]})
    assert not d['x'][0].requires_grad


def test_collate_decollate():
    Pair = collections.namedtuple('Pair', 'p q')
    batch = [{'x': torch.full((3,), float(i)), 'n': i, 'f': 0.5 * i, 'pair': Pair(torch.tensor([i]), i)}
             for i in range(4)]
    c = D.default_collate(batch)
    assert c['x'].shape == (4, 3) and c['n'].dtype == torch.int64 and c['f'].dtype == torch.float32
    assert c['pair'].p.shape == (4, 1)
    dc = D.default_decollate({'x': c['x'], 'n': c['n']})
    assert len(dc) == 4 and torch.equal(dc[2]['x'], batch[2]['x'])
    cd = D.default_collate_with_dim([torch.zeros(2, 5), torch.ones(2, 5)], dim=1)
    assert cd.shape == (2, 2, 5)
    back = D.default_decollate_with_dim(cd, dim=1)
    assert torch.equal(back[1], torch.ones(2, 5))
    ds = D.diff_shape_collate([torch.zeros(2), torch.zeros(3)])
    assert isinstance(ds, list)
    ts = D.timestep_collate([{'obs': [torch.zeros(2), torch.ones(2)], 'prev_state': (0, 1)} for _ in range(3)])
    assert ts['obs'].shape == (2, 3, 2) and ts['prev_state'] == [(0, 0, 0), (1, 1, 1)]


def test_defaults_and_locks():
    assert D.lists_to_dicts([{'a': 1, 'b': 2}, {'a': 3, 'b': 4}]) == {'a': [1, 3], 'b': [2, 4]}
    assert D.dicts_to_lists({'a': [1, 3], 'b': [2, 4]}) == [{'a': 1, 'b': 2}, {'a': 3, 'b': 4}]
    assert D.squeeze([5]) == 5 and D.squeeze({'k': 1}) == 1
    assert D.default_get({'a': 1}, 'b', default_fn=lambda: 3, judge_fn=lambda v: v > 0) == 3
    assert D.list_split([1, 2, 3, 4, 5], 2) == ([[1, 2], [3, 4]], [5])
    f = D.error_wrapper(lambda: 1 / 0, default_ret=-1)
    assert f() == -1
    with D.LockContext(D.LockContextType.THREAD_LOCK):
        pass
    with D.LockContext(D.LockContextType.PROCESS_LOCK):
        pass


def test_prefetcher_cpu():
    items = [{'x': torch.full((2,), float(i))} for i in range(5)]
    got = [int(b['x'][0]) for b in D.DevicePrefetcher(items, 'cpu')]
    assert got == list(range(5))


def test_network_misc():
    x = torch.zeros(2, 1, 4, 5)
    x[0, 0, 1, 3] = 50.0
    loc = SoftArgmax()(x)
    assert torch.allclose(loc[0], torch.tensor([1.0, 3.0]), atol=1e-3)
    feats = torch.arange(2 * 3 * 2, dtype=torch.float32).view(2, 3, 2)
    where = torch.tensor([[[0, 0], [1, 2], [0, 0]], [[2, 1], [2, 1], [0, 4]]])
    out = ScatterConnection('add')(feats, (3, 5), where)
    assert out.shape == (2, 2, 3, 5)
    assert torch.equal(out[0, :, 0, 0], feats[0, 0] + feats[0, 2])
    assert torch.equal(out[1, :, 2, 1], feats[1, 0] + feats[1, 1])
    assert isinstance(build_activation('relu'), torch.nn.ReLU)
    with pytest.raises(KeyError):
        build_activation('nope')


@pytest.mark.parametrize('fs_type', ['applestar', 'torch', 'numpy', 'nppickle'])
@pytest.mark.parametrize('compress', [False, True])
def test_file_helper_round_trip(tmp_path, fs_type, compress):
    from applestar_amd.utils import file_helper as F
    tree = {'obs': {'x': torch.arange(6, dtype=torch.float32).view(2, 3)}, 'steps': [1, 2], 'name': 'traj'}
    back = F.loads(F.dumps(tree, fs_type, compress), fs_type, compress)
    x = back['obs']['x']
    assert np.array_equal(np.asarray(x), np.arange(6, dtype=np.float32).reshape(2, 3))
    assert list(back['steps']) == [1, 2] and back['name'] == 'traj'
    if not compress:
        p = str(tmp_path / f'f.{fs_type}')
        F.save_file(p, tree, fs_type)
        assert F.read_file(p, fs_type)['name'] == 'traj'
        F.remove_file(p)


def test_file_helper_refuses_pickle_by_default():
    from applestar_amd.utils import file_helper as F
    raw = F.dumps({'a': 1}, 'pickle')
    with pytest.raises(PermissionError):
        F.loads(raw, 'pickle')
    assert F.loads(raw, 'pickle', allow_pickle=True) == {'a': 1}


def test_packed_batch_roundtrip():
    """pack_tree: every tensor of an RL batch becomes a view of one byte buffer with the same values;
    to_device rebuilds the same structure (here on the CPU) from one copy of the buffer."""
    from applestar_amd.rl.synthetic import rl_batch
    from applestar_amd.runtime.prefetch import pack_tree, PackedBatch

    b = rl_batch(2, 3, max_entities=16, seed=0)
    pk = pack_tree(b, pin=False)
    assert isinstance(pk, PackedBatch)

    def leaves(x, out):
        if torch.is_tensor(x):
            out.append(x)
        elif isinstance(x, dict):
            for v in x.values():
                leaves(v, out)
        elif isinstance(x, (list, tuple)):
            for v in x:
                leaves(v, out)
        return out

    ref, got, dev = leaves(b, []), leaves(dict(pk), []), leaves(pk.to_device('cpu'), [])
    assert len(ref) == len(got) == len(dev) > 50
    base = pk.buffer.data_ptr()
    for r, g, d in zip(ref, got, dev):
        assert g.dtype == r.dtype and g.shape == r.shape and torch.equal(g, r) and torch.equal(d, r)
        assert base <= g.data_ptr() < base + pk.buffer.numel()
    assert pk['batch_size'] == b['batch_size'] and pk.to_device('cpu')['unroll_len'] == b['unroll_len']
