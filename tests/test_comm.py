"""Data plane extras: coordinator metadata shards (start_worker) and stream channels (legacy put/get)."""
import threading

import torch

from applestar_amd.comm.adapter import Adapter, Coordinator, serve_coordinator
from applestar_amd.comm.stream import StreamChannel


def _coord():
    coord = Coordinator()
    srv = serve_coordinator(coord, host='127.0.0.1', port=0)
    return coord, srv, srv.server_address[1]


def test_sharded_push_pull():
    coord, srv, port = _coord()
    try:
        prod, cons = Adapter('127.0.0.1', port), Adapter('127.0.0.1', port)
        for i in range(12):
            prod.push({'i': torch.tensor([i])}, 'traj', worker_num=3)
        shards = coord.start_worker('traj', 3)
        assert len(shards) == 3 and coord.stats()['queued'] == {}  # nothing on the main broker
        got = cons.pull('traj', size=12, worker_num=3, timeout=10)
        assert sorted(int(d['i']) for d in got) == list(range(12))
        assert cons.pull('traj', size=1, worker_num=3, block=False) == []
        prod.close()
    finally:
        coord.close_workers()
        srv.shutdown()


def test_stream_channel_get_server():
    coord, srv, port = _coord()
    try:
        getter = StreamChannel('sl_data', 'get', coordinator_port=port)            # consumer listens
        putter = StreamChannel('sl_data', 'put', coordinator_port=port, server=False)
        for i in range(3):
            putter.put({'x': torch.full((2,), float(i))}, timeout=10)
        vals = sorted(float(getter.get(timeout=10)['x'][0]) for _ in range(3))
        assert vals == [0.0, 1.0, 2.0]
        getter.close()
    finally:
        srv.shutdown()


def test_stream_channel_put_server_and_dead_server_removal():
    coord, srv, port = _coord()
    try:
        putter = StreamChannel('model', 'put', coordinator_port=port, server=True)  # producer listens
        getter = StreamChannel('model', 'get', coordinator_port=port, server=False)
        t = threading.Thread(target=lambda: [putter.put({'v': torch.tensor([7])}) for _ in range(2)])
        t.start()
        assert int(getter.get(timeout=10)['v']) == 7
        assert int(getter.get(timeout=10)['v']) == 7
        t.join()
        # a server that went away is dropped after repeated reports
        coord.register({'token': 'model', 'type': 'put', 'server': True, 'ip': '127.0.0.1', 'port': 1})
        for _ in range(6):
            coord.remove_server({'token': 'model', 'type': 'get', 'ip': '127.0.0.1', 'port': 1})
        assert {'ip': '127.0.0.1', 'port': 1} not in coord.register({'token': 'model', 'type': 'get',
                                                                     'server': False})
        putter.close()
    finally:
        srv.shutdown()


def test_wire_codec_and_import_helper():
    """The data plane's tensor wire codec (the reference's coordinator/protocol.py encode / decode) is
    utils/serialize's frame format."""
    import torch
    from applestar_amd.utils import import_helper, serialize
    tree = {'a': torch.arange(10, dtype=torch.int16), 'b': [1.5, 'x', None, {'c': torch.ones(2, 3)}]}
    out = serialize.loads(serialize.dumps(tree, compress=True))
    assert torch.equal(out['a'], tree['a']) and out['b'][:3] == [1.5, 'x', None]
    assert torch.equal(out['b'][3]['c'], tree['b'][3]['c'])
    assert import_helper.try_import_link() is not None
    assert import_helper.try_import_mc() is None
    import_helper.import_module(['applestar_amd.utils.config'])
