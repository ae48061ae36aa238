"""Native shared-memory request/response channel (csrc/host/shm_channel.cpp): multi-process
correctness, zero-copy server view, timeouts, dead-client detection and slot takeover."""
import multiprocessing as mp
import os
import time

import pytest

from applestar_amd.runtime import shm

pytestmark = pytest.mark.skipif(not shm.available(), reason='host runtime not built')


def _client(name, slot, n, q):
    c = shm.ShmClient(name, slot, tag=100 + slot)
    out = []
    for i in range(n):
        payload = bytes([slot]) * (1000 + i) + i.to_bytes(4, 'little')
        out.append(c.request(payload, timeout_ms=20000))
    q.put((slot, out))


def test_many_clients_round_trip():
    srv = shm.ShmServer(4, 64 * 1024)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    n = 25
    procs = [ctx.Process(target=_client, args=(srv.name, s, n, q)) for s in range(4)]
    for p in procs:
        p.start()
    served = 0
    t0 = time.time()
    while served < 4 * n and time.time() - t0 < 60:
        for s in srv.wait(200):
            req = srv.request(s)
            assert req.readonly and srv.tag(s) == 100 + s
            data = bytes(req)
            assert data[0] == s
            i = int.from_bytes(data[-4:], 'little')
            assert len(data) == 1000 + i + 4
            srv.respond(s, (b'ok' + bytes([s]) + i.to_bytes(4, 'little')))
            served += 1
    res = dict(q.get(timeout=30) for _ in range(4))
    for p in procs:
        p.join(timeout=30)
    assert served == 4 * n
    for s, outs in res.items():
        assert [int.from_bytes(o[3:], 'little') for o in outs] == list(range(n))
        assert all(o[:3] == b'ok' + bytes([s]) for o in outs)
    srv.close()


def _hold_slot(name, slot, q, release):
    c = shm.ShmClient(name, slot)  # noqa: F841 (held until exit)
    q.put(os.getpid())
    release.wait(30)
    os._exit(0)  # die without releasing the slot


def test_timeout_dead_client_and_takeover():
    srv = shm.ShmServer(2, 4096)
    c = shm.ShmClient(srv.name, 1)
    with pytest.raises(RuntimeError, match='timed out'):
        c.request(b'x', timeout_ms=50)
    assert srv.pending() == [1]
    srv.respond(1, b'late')  # answers the abandoned request; the next one must not see it
    assert srv.pending() == []
    ctx = mp.get_context('spawn')
    q, release = ctx.Queue(), ctx.Event()
    p = ctx.Process(target=_hold_slot, args=(srv.name, 0, q, release))
    p.start()
    q.get(timeout=30)
    with pytest.raises(RuntimeError, match='owned by live pid'):
        shm.ShmClient(srv.name, 0)
    release.set()
    p.join(timeout=30)
    assert srv.dead_slots() == [0]
    c0 = shm.ShmClient(srv.name, 0)  # owner is dead -> takeover
    assert srv.dead_slots() == []
    del c0


def test_oversized_and_closed():
    srv = shm.ShmServer(1, 4096)
    c = shm.ShmClient(srv.name, 0)
    with pytest.raises(ValueError):
        c.request(b'y' * (srv.slot_bytes + 1))
    srv.close()
    with pytest.raises(RuntimeError, match='closed'):
        c.request(b'z', timeout_ms=1000)


@pytest.mark.parametrize('sanitizer', ['thread', 'address'])
def test_native_stress_under_sanitizer(tmp_path, sanitizer):
    """Host sanitizers on the native protocol: TSan checks the acquire/release pairing of
    the sequence words against the plain-memory payload copies; ASan checks the slot arithmetic."""
    import shutil
    import subprocess
    if shutil.which('g++') is None:
        pytest.skip('no host compiler')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / f'shm_stress_{sanitizer}')
    subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-pthread', f'-fsanitize={sanitizer}',
                    os.path.join(root, 'tests', 'native', 'shm_stress.cpp'), '-o', exe, '-lrt'], check=True)
    r = subprocess.run([exe, '4', '300'], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'OK served=1200' in r.stdout
    assert 'ThreadSanitizer' not in r.stderr and 'AddressSanitizer' not in r.stderr, r.stderr
