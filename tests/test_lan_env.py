"""LAN / remote env plumbing on CPU: settings channel, UDP<->TCP bridge, run_loop over the fake env.
(The SC2-process halves of LanGameHost / LanSC2Env need the game binary; parity unpinned here.)"""
import socket
import threading

from applestar_amd.envs import lan
from applestar_amd.envs.fake_env import FakeSC2Env


def _free_port(kind=socket.SOCK_STREAM):
    s = socket.socket(socket.AF_INET, kind)
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_settings_roundtrip():
    port = _free_port()
    ready = threading.Event()
    settings = {'map_name': 'KairosJunction', 'map_data': bytes(range(256)) * 40, 'game_version': '4.10.0',
                'ports': {'server': {'game': 1, 'base': 2}, 'client': {'game': 3, 'base': 4}}}
    box = {}
    t = threading.Thread(target=lambda: box.setdefault('conn', lan.serve_settings(lan.Addr('127.0.0.1', port),
                                                                                  settings, ready, timeout=20)))
    t.start()
    ready.wait(10)
    got = lan.fetch_settings(lan.Addr('127.0.0.1', port))
    t.join(10)
    box['conn'].close()
    assert got == settings
    assert str(lan.Addr('::1', 5)) == '[::1]:5'


def test_udp_over_tcp_bridge_both_directions():
    a, b = socket.socketpair()
    pa, pb = _free_port(socket.SOCK_DGRAM), _free_port(socket.SOCK_DGRAM)
    dest = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    dest.bind(('127.0.0.1', 0))
    dest.settimeout(5)
    # side A listens on pa and forwards to side B, which re-emits to dest
    ua = lan.forward_ports(a, lan.Addr('127.0.0.1', pa))
    ub = lan.forward_ports(b, lan.Addr('127.0.0.1', pb), lan.Addr(*dest.getsockname()))
    client = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    client.settimeout(5)
    client.sendto(b'hello-sc2', ('127.0.0.1', pa))
    data, src = dest.recvfrom(100)
    assert data == b'hello-sc2'
    dest.sendto(b'reply', ('127.0.0.1', pb))              # back through B -> TCP -> A -> last sender
    data, _ = client.recvfrom(100)
    assert data == b'reply'
    for s in (ua, ub, a, b, client, dest):
        s.close()


class _NoopAgent:
    def __init__(self):
        self.resets = 0
        self.steps = 0

    def reset(self, map_name, race, game_info, obs):
        self.resets += 1

    def step(self, obs):
        self.steps += 1
        return []


def test_run_loop_over_fake_env():
    env = FakeSC2Env({'env': {'player_ids': ['agent1', 'bot7'], 'game_steps_per_episode': 200,
                              'map_name': 'KairosJunction'}})
    agent = _NoopAgent()
    out = lan.run_loop([agent], lan.EnvWrapper(env), max_episodes=2)
    assert out['episodes'] == 2 and out['frames'] > 0
    assert agent.resets == 2 and agent.steps >= out['frames']


def test_sc2_tools_offline_commands():
    from applestar_amd.bin import sc2_tools
    maps = sc2_tools.map_list()
    assert 'KairosJunction' in maps and len(maps['KairosJunction']['cropped_size']) == 2
    allv = sc2_tools.valid_actions()
    assert allv['count'] == 327
    zerg = sc2_tools.valid_actions('zerg')
    assert 0 < zerg['count'] < 327
    bench = sc2_tools.benchmark_observe(fake=True, steps=50, steps_per_episode=100)
    assert bench['steps'] == 50 and bench['steps_per_s'] > 0 and 'p90_ms' in bench
    mem = sc2_tools.mem_leak_check(fake=True, episodes=2, steps_per_episode=50)
    assert len(mem['rss_mb']) == 2 and mem['rss_mb'][0] > 0
