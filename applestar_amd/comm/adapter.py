"""Data plane: coordinator (metadata broker) + adapter (producer-side payload server, consumer pull).

Same topology as ``distar/ctools/worker/coordinator/{coordinator,adapter}.py``: producers keep the
serialized payload locally and publish only ``{token, ip, port, key}`` to the coordinator; consumers
pop metadata (LIFO, newest first, bounded deques) and fetch the bytes directly from the producer, so
the coordinator never touches trajectory/model bytes.

Differences (by design):
* one persistent listening socket per adapter (the reference binds a fresh port per payload);
* payloads use :mod:`applestar_amd.utils.serialize` (safe, 64 B-aligned raw tensor frames; no
  pickle), so the learner can ``frombuffer`` the bytes straight into pinned memory;
* "broadcast" tokens (model weights) are *peeked*, not popped: every actor reads the newest model
  and the producer replaces it in place (the reference's ``maxlen 1`` model deque + re-push).
"""
from __future__ import annotations

import http.client
import json
import socket
import struct
import threading
import time
import uuid
from collections import defaultdict, deque
from functools import partial
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

from ..utils import serialize

_LEN = struct.Struct('<Q')


# ----------------------------------------------------------------------------- coordinator
class Coordinator:
    def __init__(self, maxlen: int = 1000, host: str = '127.0.0.1'):
        self._lock = threading.Lock()
        self._meta: Dict[str, deque] = defaultdict(partial(deque, maxlen=maxlen))
        self._broadcast: Dict[str, dict] = {}
        self.push_count = defaultdict(int)
        self.pull_count = defaultdict(int)
        self._host = host
        # metadata shards ("workers", coordinator.py:20-57,156-165) and stream-server registry
        self._workers: Dict[str, List[dict]] = defaultdict(list)
        self._worker_servers = []
        self._servers = {'put': defaultdict(list), 'get': defaultdict(list)}
        self._remove_count = defaultdict(int)

    def push(self, info: dict) -> bool:
        token = info['token']
        with self._lock:
            if info.get('broadcast'):
                self._broadcast[token] = info
            else:
                self._meta[token].append(info)
            self.push_count[token] += 1
        return True

    def pull(self, token: str, size: int = 1) -> List[dict]:
        with self._lock:
            if token in self._broadcast:
                return [self._broadcast[token]]
            q = self._meta.get(token)
            out = []
            while q and len(out) < size:
                out.append(q.pop())
            self.pull_count[token] += len(out)
            return out

    def start_worker(self, token: str, worker_num: int) -> List[dict]:
        """Shard ``token``'s metadata over ``worker_num`` extra brokers (maxlen 256 each, as the
        reference's workers); idempotent per token.  Each shard is its own HTTP server thread."""
        with self._lock:
            if not self._workers[token]:
                for _ in range(int(worker_num)):
                    srv = serve_coordinator(Coordinator(maxlen=256), host=self._host, port=0)
                    self._worker_servers.append(srv)
                    self._workers[token].append({'ip': self._host, 'port': srv.server_address[1]})
            return list(self._workers[token])

    def register(self, info: dict):
        """Stream-channel registry (coordinator.py:75-109): a server registers itself under
        (token, type); a client asks for the servers of the opposite type."""
        info = dict(info)
        typ, token = info.pop('type'), info.pop('token')
        server = info.pop('server', typ == 'get')
        with self._lock:
            if server:
                entry = {'ip': info['ip'], 'port': int(info['port'])}
                if entry not in self._servers[typ][token]:
                    self._servers[typ][token].append(entry)
                return True
            other = 'get' if typ == 'put' else 'put'
            return list(self._servers[other][token]) or False

    def remove_server(self, info: dict) -> bool:
        """A client reports an unreachable server; it is dropped after 5 reports (coordinator.py:111-124)."""
        typ = 'put' if info['type'] == 'get' else 'get'
        entry = {'ip': info['ip'], 'port': int(info['port'])}
        with self._lock:
            lst = self._servers[typ][info['token']]
            if entry in lst:
                key = f"{entry['ip']}:{entry['port']}"
                self._remove_count[key] += 1
                if self._remove_count[key] > 5:
                    lst.remove(entry)
                    self._remove_count.pop(key)
                    return True
        return False

    def close_workers(self):
        for srv in self._worker_servers:
            srv.shutdown()
            srv.server_close()
        self._worker_servers = []

    def stats(self) -> dict:
        with self._lock:
            return {'queued': {k: len(v) for k, v in self._meta.items()},
                    'broadcast': sorted(self._broadcast), 'push': dict(self.push_count),
                    'pull': dict(self.pull_count)}


def serve_coordinator(coord: Coordinator, host: str = '0.0.0.0', port: int = 0) -> ThreadingHTTPServer:
    if host not in ('0.0.0.0', ''):
        coord._host = host
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _reply(self, obj):
            body = json.dumps({'code': 0, 'info': obj}).encode()
            self.send_response(200)
            self.send_header('Content-Type', 'application/json')
            self.send_header('Content-Length', str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_POST(self):
            n = int(self.headers.get('Content-Length', 0))
            req = json.loads(self.rfile.read(n) or b'{}')
            if self.path == '/coordinator/push':
                self._reply(coord.push(req))
            elif self.path == '/coordinator/pull':
                self._reply(coord.pull(req['token'], int(req.get('size', 1))))
            elif self.path == '/coordinator/start_worker':
                self._reply(coord.start_worker(req['token'], int(req['worker_num'])))
            elif self.path == '/coordinator/register':
                self._reply(coord.register(req))
            elif self.path == '/coordinator/remove_server':
                self._reply(coord.remove_server(req))
            else:
                self.send_error(404)

        def do_GET(self):
            if self.path == '/coordinator/stats':
                self._reply(coord.stats())
            else:
                self.send_error(404)

    srv = ThreadingHTTPServer((host, port), Handler)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True, name='coordinator').start()
    return srv


def _post_json(ip: str, port: int, path: str, obj: dict, timeout: float = 30.0):
    conn = http.client.HTTPConnection(ip, port, timeout=timeout)
    try:
        body = json.dumps(obj)
        conn.request('POST', path, body=body, headers={'Content-Type': 'application/json'})
        r = conn.getresponse()
        data = json.loads(r.read())
        if data.get('code', 0) != 0:
            raise RuntimeError(data)
        return data['info']
    finally:
        conn.close()


# ----------------------------------------------------------------------------- payload server
def _recv_into_all(sock: socket.socket, view, n: int, timeout: Optional[float] = None) -> None:
    """Fill view[:n] from the socket in (usually) ONE blocking ``recv(MSG_WAITALL)``: the kernel copies the whole
    payload while the GIL stays released.  The chunked loop of a socket with a Python timeout (non-blocking fd,
    ~64 KB per call, the GIL re-taken for every chunk) starved the learner's launch thread of the GIL while a
    trajectory was arriving: its step took 280 ms instead of 55 (profiles/r5v_pipeline_learner_threads.txt).
    ``timeout``: an OS-level receive timeout (SO_RCVTIMEO) instead of Python's, so a dead peer still raises."""
    prev = sock.gettimeout()
    if timeout is None:
        timeout = prev
    sock.settimeout(None)
    if timeout:
        sec = int(timeout)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVTIMEO, struct.pack('ll', sec, int((timeout - sec) * 1e6)))
    try:
        got = 0
        while got < n:
            k = sock.recv_into(view[got:n], n - got, socket.MSG_WAITALL)
            if k == 0:
                raise ConnectionError('peer closed')
            got += k
    finally:
        sock.settimeout(prev)


def _recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    _recv_into_all(sock, memoryview(buf), n)
    return buf


class _PayloadServer:
    def __init__(self, host: str, max_items: int = 4096):
        self._items: Dict[str, bytes] = {}
        self._keep = set()
        self._order = deque()
        self._max = max_items
        self._lock = threading.Lock()
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._sock.bind((host, 0))
        self._sock.listen(64)
        self.port = self._sock.getsockname()[1]
        self._closed = False
        threading.Thread(target=self._accept_loop, daemon=True, name='payload-server').start()

    def put(self, key: str, data: bytes, keep: bool = False) -> None:
        with self._lock:
            self._items[key] = data
            if keep:
                self._keep.add(key)
            else:
                self._order.append(key)
                while len(self._order) > self._max:  # bounded: drop the oldest unread payload
                    self._items.pop(self._order.popleft(), None)

    def drop(self, key: str) -> None:
        with self._lock:
            self._items.pop(key, None)
            self._keep.discard(key)

    def _accept_loop(self):
        while not self._closed:
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn: socket.socket):
        with conn:
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            try:
                while True:
                    (klen,) = _LEN.unpack(_recv_exact(conn, 8))
                    key = bytes(_recv_exact(conn, klen)).decode()
                    with self._lock:
                        data = self._items.get(key) if key in self._keep else self._items.pop(key, None)
                    if data is None:
                        conn.sendall(_LEN.pack(0))
                    else:
                        conn.sendall(_LEN.pack(len(data)))
                        conn.sendall(data)
            except (ConnectionError, OSError, struct.error):
                return

    def close(self):
        self._closed = True
        try:
            self._sock.close()
        except OSError:
            pass


def fetch(ip: str, port: int, key: str, timeout: float = 60.0, alloc=None):
    """Receive one payload.  ``alloc(n)`` may supply the destination (e.g. a pinned staging buffer
    of the trajectory ring) so the bytes land where the H2D copy reads them, with no extra copy."""
    with socket.create_connection((ip, port), timeout=timeout) as s:
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        k = key.encode()
        s.sendall(_LEN.pack(len(k)) + k)
        (n,) = _LEN.unpack(_recv_exact(s, 8))
        if not n:
            return None
        if alloc is None:
            return _recv_exact(s, n)
        buf = alloc(n)
        view = memoryview(buf)[:n]
        _recv_into_all(s, view, n, timeout)
        return view


# ----------------------------------------------------------------------------- adapter
class Adapter:
    """``push(obj, token)`` / ``pull(token, size)`` against a coordinator."""

    def __init__(self, coordinator_ip: str = '127.0.0.1', coordinator_port: int = 0, host_ip: Optional[str] = None,
                 compress: bool = False):
        self._cip, self._cport = coordinator_ip, int(coordinator_port)
        self._ip = host_ip or self._local_ip()
        self._compress = compress
        self._server: Optional[_PayloadServer] = None
        self._broadcast_keys: Dict[str, str] = {}
        self._worker_addr: Dict[str, List[tuple]] = {}

    def _local_ip(self) -> str:
        if self._cip in ('127.0.0.1', 'localhost'):
            return '127.0.0.1'
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect((self._cip, self._cport or 80))
            return s.getsockname()[0]
        finally:
            s.close()

    def _shards(self, token: str, worker_num: Optional[int]) -> List[tuple]:
        """Metadata brokers for ``token``: the coordinator itself, or its ``worker_num`` shards."""
        if not worker_num:
            return [(self._cip, self._cport)]
        if token not in self._worker_addr:
            ws = _post_json(self._cip, self._cport, '/coordinator/start_worker',
                            {'token': token, 'worker_num': int(worker_num)})
            self._worker_addr[token] = [(w['ip'], int(w['port'])) for w in ws]
        return self._worker_addr[token]

    def push(self, data: Any, token: str, broadcast: bool = False, retries: int = 20,
             worker_num: Optional[int] = None) -> str:
        if self._server is None:
            self._server = _PayloadServer('0.0.0.0' if self._ip != '127.0.0.1' else '127.0.0.1')
        payload = data if isinstance(data, (bytes, bytearray)) else serialize.dumps(data, compress=self._compress)
        key = f'{token}/{uuid.uuid4().hex}'
        self._server.put(key, bytes(payload), keep=broadcast)
        meta = {'token': token, 'ip': self._ip, 'port': self._server.port, 'key': key, 'size': len(payload),
                'broadcast': broadcast, 'time': time.time()}
        shards = self._shards(token, None if broadcast else worker_num)
        cip, cport = shards[hash(key) % len(shards)]
        for i in range(retries + 1):
            try:
                _post_json(cip, cport, '/coordinator/push', meta)
                break
            except (ConnectionError, OSError):
                if i == retries:
                    raise
                time.sleep(min(2 ** i * 0.1, 5.0))
        if broadcast:
            old = self._broadcast_keys.get(token)
            self._broadcast_keys[token] = key
            if old is not None:
                # keep the previous version briefly for readers that already hold its metadata
                threading.Timer(30.0, self._server.drop, args=(old,)).start()
        return key

    def pull(self, token: str, size: int = 1, block: bool = True, sleep_time: float = 0.05,
             timeout: Optional[float] = None, raw: bool = False, alloc=None,
             worker_num: Optional[int] = None) -> List[Any]:
        out: List[Any] = []
        t0 = time.time()
        shards = self._shards(token, worker_num)
        turn = 0
        while len(out) < size:
            cip, cport = shards[turn % len(shards)]
            turn += 1
            metas = _post_json(cip, cport, '/coordinator/pull', {'token': token, 'size': size - len(out)})
            for m in metas:
                try:
                    data = fetch(m['ip'], m['port'], m['key'], alloc=alloc)
                except OSError:
                    data = None
                if data is not None:
                    out.append(data if raw else serialize.loads(data))
                if m.get('broadcast'):
                    return out
            if len(out) >= size or (timeout is not None and time.time() - t0 > timeout):
                break
            if turn % len(shards) == 0:  # every shard visited once this round
                if not block:
                    break
                time.sleep(sleep_time)
        return out

    def stats(self) -> dict:
        conn = http.client.HTTPConnection(self._cip, self._cport, timeout=10)
        try:
            conn.request('GET', '/coordinator/stats')
            return json.loads(conn.getresponse().read())['info']
        finally:
            conn.close()

    def close(self):
        if self._server is not None:
            self._server.close()
