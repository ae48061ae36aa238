"""Env layer without SC2: websocket framing of the SC2 RPC client, SC2 install discovery, fake env
contract (scheduling by skip_steps, episode end, random maps)."""
import base64
import hashlib
import os
import socket
import struct
import threading

import numpy as np
import pytest

from applestar_amd.envs.fake_env import FakeSC2Env
from applestar_amd.envs.sc2.controller import WebSocket
from applestar_amd.envs.sc2 import launcher


def _ws_echo_server():
    srv = socket.socket()
    srv.bind(('127.0.0.1', 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def run():
        conn, _ = srv.accept()
        data = b''
        while b'\r\n\r\n' not in data:
            data += conn.recv(4096)
        key = [l.split(b': ')[1] for l in data.split(b'\r\n') if l.lower().startswith(b'sec-websocket-key')][0]
        acc = base64.b64encode(hashlib.sha1(key + b'258EAFA5-E914-47DA-95CA-C5AB0DC85B11').digest())
        conn.sendall(b'HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n'
                     b'Sec-WebSocket-Accept: ' + acc + b'\r\n\r\n')
        buf = b''

        def need(n):
            nonlocal buf
            while len(buf) < n:
                buf += conn.recv(1 << 20)
            out, buf = buf[:n], buf[n:]
            return out
        def frame():
            b0, b1 = need(2)
            n = b1 & 0x7F
            if n == 126:
                n = struct.unpack('!H', need(2))[0]
            elif n == 127:
                n = struct.unpack('!Q', need(8))[0]
            mask = np.frombuffer(need(4) * ((n + 3) // 4), np.uint8)[:n]
            return b0 & 0x0F, (np.frombuffer(need(n), np.uint8) ^ mask).tobytes()
        served = 0
        while served < 2:
            op, payload = frame()
            if op == 0xA:  # the client's pong
                assert payload == b'hi'
                continue
            served += 1
            conn.sendall(bytes([0x89, 2]) + b'hi')  # a ping the client must answer transparently
            # echo back unmasked, split into two fragments
            half = len(payload) // 2
            for fin, op, part in ((0, 0x2, payload[:half]), (1, 0x0, payload[half:])):
                m = len(part)
                hdr = bytes([(0x80 if fin else 0) | op])
                hdr += bytes([m]) if m < 126 else (bytes([126]) + struct.pack('!H', m) if m < 65536 else
                                                   bytes([127]) + struct.pack('!Q', m))
                conn.sendall(hdr + part)
        assert frame() == (0xA, b'hi')  # last pong
        conn.close()
    threading.Thread(target=run, daemon=True).start()
    return port


def test_websocket_roundtrip_fragments_and_ping():
    port = _ws_echo_server()
    ws = WebSocket('127.0.0.1', port, timeout=10)
    for payload in (os.urandom(100), os.urandom(300000)):
        ws.send(payload)
        assert ws.recv() == payload
    ws.close()


def test_sc2_binary_discovery(tmp_path, monkeypatch):
    exe = tmp_path / 'Versions' / 'Base75689' / 'SC2_x64'
    exe.parent.mkdir(parents=True)
    exe.write_text('')
    monkeypatch.setenv('SC2PATH', str(tmp_path))
    assert launcher.find_sc2_binary('4.10.0') == str(exe)
    assert launcher.VERSIONS['4.10.0'].build_version == 75689
    assert launcher.map_path('Ladder2019Season2\\KairosJunctionLE.SC2Map').endswith(
        os.path.join('Maps', 'Ladder2019Season2', 'KairosJunctionLE.SC2Map'))


def test_fake_env_contract():
    env = FakeSC2Env({'env': {'player_ids': ['agent1', 'agent2'], 'game_steps_per_episode': 500,
                              'random_seed': 3, 'map_name': 'random'}})
    obs, gi, m = env.reset()
    assert m in ('KairosJunction', 'KingsCove', 'NewRepugnancy') and set(obs) == {0, 1}
    a = {'func_id': 0, 'skip_steps': 20, 'queued': 0, 'unit_tags': [], 'target_unit_tag': 0, 'location': (0, 0)}
    b = dict(a, skip_steps=50)
    nobs, rew, done = env.step({0: [a], 1: [b]})
    assert set(nobs) == {0} and not done      # agent 1 is still waiting for its delay
    loops = [nobs[0]['raw_obs'].observation.game_loop]
    while not done:
        nobs, rew, done = env.step({i: [a] for i in nobs})
    assert sorted(rew) == [-1, 1] and set(nobs) == {0, 1}
    # bot games have a single agent slot
    env = FakeSC2Env({'env': {'player_ids': ['agent1', 'bot7'], 'game_steps_per_episode': 100}})
    obs, _, _ = env.reset()
    assert set(obs) == {0} and obs[0]['opponent_obs'] is not None


def test_fake_env_learnable_mode_rewards_the_action_set(tmp_path):
    """Learnable FakeSC2Env: the result depends on the share of rewarded action types; each
    finished episode is logged to fake_stats_path."""
    import json
    from applestar_amd.envs.fake_env import REWARDED_ACTION_TYPES
    from applestar_amd.lib.game_data import ACTIONS
    plain = [a for a in range(1, len(ACTIONS)) if not ACTIONS[a]['target_unit'] and not ACTIONS[a]['target_location']]
    good = next(a for a in plain if a in REWARDED_ACTION_TYPES)
    bad = next(a for a in plain if a not in REWARDED_ACTION_TYPES)
    stats = tmp_path / 'stats.jsonl'
    wins = {}
    for name, at in (('good', good), ('bad', bad)):
        env = FakeSC2Env({'env': {'player_ids': ['agent1', 'bot7'], 'fake_learnable': True,
                                  'fake_episode_agent_steps': 8, 'random_seed': 0, 'fake_stats_path': str(stats)}})
        n = 0
        for ep in range(40):
            env.reset()
            done, steps = False, 0
            while not done:
                _, reward, done = env.step({0: [{'func_id': ACTIONS[at]['func_id'], 'skip_steps': 4,
                                                 'unit_tags': [], 'queued': 0}]})
                steps += 1
            assert steps == 8
            n += reward[0] > 0
        wins[name] = n / 40
    # rate 1 vs the bot's ~0.25: p(win) = 1; rate 0: p(win) = 0.25
    assert wins['good'] == 1.0 and wins['bad'] < 0.5, wins
    lines = [json.loads(x) for x in stats.read_text().splitlines()]
    assert len(lines) == 80 and lines[0]['rate'] == [1.0] and lines[-1]['rate'] == [0.0]
