"""SC2 API client: a minimal RFC 6455 websocket + protobuf request/response RPC
(``pysc2/lib/protocol.py:72-192`` + ``remote_controller.py:127-386``).

Only the message classes come from ``s2clientprotocol`` (imported lazily); the websocket framing is
implemented here so the client has no other third-party dependency.  Requests are written as one
binary frame, responses may span continuation frames; pings are answered.
"""
from __future__ import annotations

import base64
import os
import socket
import struct
import time
from typing import Optional


def _pb():
    from s2clientprotocol import sc2api_pb2, common_pb2, raw_pb2  # noqa: F401
    return sc2api_pb2


class WebSocket:
    def __init__(self, host: str, port: int, path: str = '/sc2api', timeout: float = 120.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        key = base64.b64encode(os.urandom(16)).decode()
        req = (f'GET {path} HTTP/1.1\r\nHost: {host}:{port}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n'
               f'Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\n\r\n')
        self.sock.sendall(req.encode())
        head = b''
        while b'\r\n\r\n' not in head:
            chunk = self.sock.recv(4096)
            if not chunk:
                raise ConnectionError('websocket handshake failed')
            head += chunk
        if b' 101 ' not in head.split(b'\r\n', 1)[0]:
            raise ConnectionError(f'websocket upgrade refused: {head[:80]!r}')
        self._buf = head.split(b'\r\n\r\n', 1)[1]

    def _recv_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise ConnectionError('websocket closed')
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def send(self, payload: bytes, opcode: int = 0x2) -> None:
        mask = os.urandom(4)
        n = len(payload)
        if n < 126:
            hdr = struct.pack('!BB', 0x80 | opcode, 0x80 | n)
        elif n < 65536:
            hdr = struct.pack('!BBH', 0x80 | opcode, 0x80 | 126, n)
        else:
            hdr = struct.pack('!BBQ', 0x80 | opcode, 0x80 | 127, n)
        import numpy as np
        p = np.frombuffer(payload, dtype=np.uint8)
        m = np.frombuffer(mask * ((n + 3) // 4), dtype=np.uint8)[:n]
        self.sock.sendall(hdr + mask + (p ^ m).tobytes())

    def recv(self) -> bytes:
        parts = []
        while True:
            b0, b1 = self._recv_exact(2)
            fin, opcode = b0 & 0x80, b0 & 0x0F
            n = b1 & 0x7F
            if n == 126:
                n = struct.unpack('!H', self._recv_exact(2))[0]
            elif n == 127:
                n = struct.unpack('!Q', self._recv_exact(8))[0]
            data = self._recv_exact(n)
            if opcode == 0x9:  # ping -> pong
                self.send(data, 0xA)
                continue
            if opcode == 0x8:
                raise ConnectionError('websocket closed by peer')
            parts.append(data)
            if fin:
                return b''.join(parts)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


class RemoteController:
    """Blocking RPC client for one SC2 instance."""

    def __init__(self, host: str, port: int, timeout: float = 120.0, retries: int = 60):
        self._pb = _pb()
        err = None
        for _ in range(retries):
            try:
                self._ws = WebSocket(host, port, timeout=timeout)
                break
            except OSError as e:
                err = e
                time.sleep(1)
        else:
            raise ConnectionError(f'cannot connect to SC2 at {host}:{port}: {err}')
        self.status_ended = False
        self._last_status = None

    def _call(self, **kw):
        req = self._pb.Request(**kw)
        self._ws.send(req.SerializeToString())
        res = self._pb.Response()
        res.ParseFromString(self._ws.recv())
        if res.error:
            raise RuntimeError(f'SC2 error on {list(kw)}: {list(res.error)}')
        self._last_status = res.status
        self.status_ended = res.status == self._pb.Status.Value('ended')
        field = list(kw)[0]
        return getattr(res, field)

    # --- game lifecycle
    def create_game(self, req):
        return self._call(create_game=req)

    def join_game(self, req):
        return self._call(join_game=req)

    def restart(self):
        return self._call(restart_game=self._pb.RequestRestartGame())

    def leave(self):
        return self._call(leave_game=self._pb.RequestLeaveGame())

    def quit(self):
        try:
            self._call(quit=self._pb.RequestQuit())
        except (ConnectionError, OSError):
            pass
        self._ws.close()

    # --- stepping
    def game_info(self):
        return self._call(game_info=self._pb.RequestGameInfo())

    def data(self):
        return self._call(data=self._pb.RequestData(ability_id=True, unit_type_id=True))

    def observe(self, disable_fog: bool = False, target_game_loop: int = 0):
        obs = self._call(observation=self._pb.RequestObservation(game_loop=target_game_loop,
                                                                 disable_fog=disable_fog))
        if obs.observation.game_loop == 2 ** 32 - 1:  # stub observation after the game ended
            obs.observation.game_loop = 0
        return obs

    def step(self, count: int = 1):
        return self._call(step=self._pb.RequestStep(count=count))

    def actions(self, req_action):
        return self._call(action=req_action)

    def act(self, action):
        if action and action.ListFields():
            return self.actions(self._pb.RequestAction(actions=[action]))
        return None

    # --- replays
    def save_replay(self) -> bytes:
        return self._call(save_replay=self._pb.RequestSaveReplay()).data

    def replay_info(self, replay_data: bytes):
        return self._call(replay_info=self._pb.RequestReplayInfo(replay_data=replay_data))

    def start_replay(self, req):
        return self._call(start_replay=req)

    def ping(self):
        return self._call(ping=self._pb.RequestPing())
