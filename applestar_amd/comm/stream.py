"""Point-to-point stream channels brokered by the coordinator: the reference adapter's legacy
``put``/``get`` API (``adapter.py:248-412``, ``coordinator.py:75-124``).

A channel is (token, side).  One side runs *servers* that listen on a socket and register with the
coordinator; the other side's *clients* ask the coordinator for the server list and connect to a random
server per message.  Either side may be the server:

* ``StreamChannel(token, 'put', server=True)``: producers listen; each ``put`` is handed to the next
  consumer that connects;
* ``StreamChannel(token, 'get', server=True)`` (default for getters): consumers listen; producers
  connect and deliver.

Frames are ``u64 length + payload`` (our :mod:`serialize` format unless bytes are given; no pickle).
Unreachable servers are reported to the coordinator, which drops them after repeated reports.  The
server list is refreshed every ``refresh_s`` seconds.
"""
from __future__ import annotations

import random
import socket
import struct
import threading
import time
from collections import deque
from typing import Any, Optional

from ..utils import serialize
from .adapter import _post_json, _recv_exact

_LEN = struct.Struct('<Q')


class StreamChannel:
    def __init__(self, token: str, type: str, coordinator_ip: str = '127.0.0.1', coordinator_port: int = 0,
                 server: Optional[bool] = None, host_ip: str = '127.0.0.1', refresh_s: float = 120.0,
                 connect_timeout: float = 0.5):
        assert type in ('put', 'get'), type
        self.token, self.type = token, type
        self.server = (type == 'get') if server is None else bool(server)
        self._cip, self._cport = coordinator_ip, int(coordinator_port)
        self._refresh_s = refresh_s
        self._connect_timeout = connect_timeout
        self._peers = []
        self._peers_time = 0.0
        self._queue = deque()
        self._cv = threading.Condition()
        self._closed = False
        if self.server:
            self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            self._sock.bind((host_ip, 0))
            self._sock.listen(64)
            self.ip, self.port = host_ip, self._sock.getsockname()[1]
            self._register({'ip': self.ip, 'port': self.port, 'server': True})
            threading.Thread(target=self._accept_loop, daemon=True, name=f'stream-{type}-{token}').start()

    # ---------------------------------------------------------------- coordinator
    def _register(self, extra: dict):
        req = {'token': self.token, 'type': self.type}
        req.update(extra)
        while True:
            try:
                return _post_json(self._cip, self._cport, '/coordinator/register', req)
            except RuntimeError:  # no servers of the other side yet
                return False
            except OSError:
                if self._closed:
                    return False
                time.sleep(0.5)

    def _servers(self, force: bool = False):
        if force or not self._peers or time.time() - self._peers_time > self._refresh_s:
            res = self._register({'server': False})
            self._peers = [(d['ip'], int(d['port'])) for d in res] if res else []
            self._peers_time = time.time()
        return self._peers

    def _report_dead(self, ip, port):
        try:
            _post_json(self._cip, self._cport, '/coordinator/remove_server',
                       {'token': self.token, 'type': self.type, 'ip': ip, 'port': port})
        except (OSError, RuntimeError):
            pass

    # ---------------------------------------------------------------- server side
    def _accept_loop(self):
        while not self._closed:
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve_one, args=(conn,), daemon=True).start()

    def _serve_one(self, conn: socket.socket):
        with conn:
            try:
                if self.type == 'put':           # hand the next queued payload to the connecting getter
                    with self._cv:
                        while not self._queue and not self._closed:
                            self._cv.wait(0.5)
                        if self._closed:
                            return
                        data = self._queue.popleft()
                    conn.sendall(_LEN.pack(len(data)) + data)
                else:                            # receive one payload from the connecting putter
                    (n,) = _LEN.unpack(_recv_exact(conn, 8))
                    data = bytes(_recv_exact(conn, n))
                    conn.sendall(b'\x01')        # ack: delivered
                    with self._cv:
                        self._queue.append(data)
                        self._cv.notify()
            except (OSError, ConnectionError, struct.error):
                return

    # ---------------------------------------------------------------- API
    def put(self, data: Any, timeout: Optional[float] = None) -> None:
        assert self.type == 'put'
        payload = data if isinstance(data, (bytes, bytearray)) else serialize.dumps(data)
        if self.server:
            with self._cv:
                self._queue.append(bytes(payload))
                self._cv.notify()
            return
        t0 = time.time()
        while True:
            peers = self._servers()
            if peers:
                ip, port = random.choice(peers)
                try:
                    with socket.create_connection((ip, port), timeout=self._connect_timeout) as s:
                        s.settimeout(None)
                        s.sendall(_LEN.pack(len(payload)) + bytes(payload))
                        if _recv_exact(s, 1) == b'\x01':
                            return
                except (ConnectionRefusedError, socket.timeout):
                    self._report_dead(ip, port)
                    self._servers(force=True)
                except (OSError, ConnectionError):
                    pass
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(f'no get-server accepted {self.token!r}')
            time.sleep(0.05)
            if not peers:
                self._servers(force=True)

    def get(self, timeout: Optional[float] = None, raw: bool = False) -> Any:
        assert self.type == 'get'
        t0 = time.time()
        if self.server:
            with self._cv:
                while not self._queue:
                    left = None if timeout is None else timeout - (time.time() - t0)
                    if left is not None and left <= 0:
                        raise TimeoutError(f'nothing received on {self.token!r}')
                    self._cv.wait(0.5 if left is None else min(left, 0.5))
                data = self._queue.popleft()
            return data if raw else serialize.loads(data)
        while True:
            peers = self._servers()
            if peers:
                ip, port = random.choice(peers)
                try:
                    with socket.create_connection((ip, port), timeout=self._connect_timeout) as s:
                        s.settimeout(None if timeout is None else max(timeout - (time.time() - t0), 0.1))
                        (n,) = _LEN.unpack(_recv_exact(s, 8))
                        data = bytes(_recv_exact(s, n))
                        return data if raw else serialize.loads(data)
                except (ConnectionRefusedError,):
                    self._report_dead(ip, port)
                    self._servers(force=True)
                except (OSError, ConnectionError, struct.error):
                    pass
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(f'no put-server delivered {self.token!r}')
            time.sleep(0.05)
            if not peers:
                self._servers(force=True)

    def close(self):
        self._closed = True
        if self.server:
            try:
                self._sock.close()
            except OSError:
                pass
        with self._cv:
            self._cv.notify_all()
