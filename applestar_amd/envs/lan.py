"""LAN / remote StarCraft II games and the generic env loop (the upstream pysc2 ``env`` layer:
``lan_sc2_env.py``, ``remote_sc2_env.py``, ``host_remote_agent.py``, ``run_loop.py``).

Three pieces, all on top of this package's own SC2 stack (``envs/sc2``: process launcher + websocket RPC):

* :class:`LanGameHost` - the hosting side.  Launches SC2, creates a two-participant game on a local map
  and publishes a small **settings record** (map name + bytes, game version, the LAN port set) over a
  one-shot TCP server, so a second machine can join (host_remote_agent.py:25-143).
* :class:`LanSC2Env` - the joining side as an ordinary :class:`SC2Env` with one agent slot: it fetches
  the settings record from ``host:config_port``, launches (or, :class:`RemoteSC2Env`, connects to an
  already running) local SC2 and joins with the published ports (lan_sc2_env.py:199-363,
  remote_sc2_env.py:32-213).
* :func:`forward_ports` - UDP<->TCP bridges for SC2's LAN traffic when the two machines only share a TCP
  path (e.g. an SSH tunnel): every UDP datagram is framed onto the TCP stream and re-emitted on the
  other side (lan_sc2_env.py:105-193).

Wire format of the settings channel and of the bridged datagrams: ``uint32 little-endian length`` +
payload; the settings record is the map bytes followed by a JSON document of the remaining keys.
"""
from __future__ import annotations

import json
import socket
import struct
import threading
from collections import namedtuple
from typing import Callable, Dict, List, Optional, Sequence

from .sc2_env import SC2Env

__all__ = ['Addr', 'write_msg', 'read_msg', 'serve_settings', 'fetch_settings', 'forward_ports', 'LanGameHost',
           'LanSC2Env', 'RemoteSC2Env', 'run_loop', 'EnvWrapper']

_LEN = struct.Struct('<I')


class Addr(namedtuple('Addr', ['ip', 'port'])):
    def __str__(self):
        return f'[{self.ip}]:{self.port}' if ':' in self.ip else f'{self.ip}:{self.port}'


def _family(ip: str):
    return socket.AF_INET6 if ':' in ip else socket.AF_INET


def write_msg(conn: socket.socket, payload: bytes) -> None:
    conn.sendall(_LEN.pack(len(payload)) + payload)


def _read_exact(conn: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = conn.recv(n - len(buf))
        if not chunk:
            raise ConnectionError('peer closed the connection')
        buf += chunk
    return bytes(buf)


def read_msg(conn: socket.socket) -> bytes:
    (n,) = _LEN.unpack(_read_exact(conn, _LEN.size))
    return _read_exact(conn, n)


# ---------------------------------------------------------------------------- settings channel
def serve_settings(addr: Addr, settings: Dict, ready: Optional[threading.Event] = None,
                   timeout: Optional[float] = None) -> socket.socket:
    """Accept ONE joiner on ``addr`` and send it ``settings`` (must hold ``map_data`` bytes).  Returns the
    open connection (kept by the host for the game's lifetime, like the reference's tcp_server)."""
    srv = socket.socket(_family(addr.ip), socket.SOCK_STREAM)
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(tuple(addr))
    srv.listen(1)
    srv.settimeout(timeout)
    if ready is not None:
        ready.set()
    try:
        conn, _ = srv.accept()
    finally:
        srv.close()
    write_msg(conn, bytes(settings['map_data']))
    write_msg(conn, json.dumps({k: v for k, v in settings.items() if k != 'map_data'}).encode())
    return conn


def fetch_settings(addr: Addr, timeout: float = 60.0) -> Dict:
    conn = socket.create_connection(tuple(addr), timeout=timeout)
    try:
        map_data = read_msg(conn)
        settings = json.loads(read_msg(conn).decode())
    finally:
        conn.close()
    settings['map_data'] = map_data
    return settings


# ---------------------------------------------------------------------------- UDP <-> TCP bridge
def _udp_to_tcp(udp: socket.socket, tcp: socket.socket, peer: List):
    try:
        while True:
            data, src = udp.recvfrom(65535)
            peer[0] = src                      # reply path for datagrams coming back over TCP
            write_msg(tcp, data)
    except OSError:
        return


def _tcp_to_udp(tcp: socket.socket, udp: socket.socket, dest: Callable[[], Optional[tuple]]):
    try:
        while True:
            data = read_msg(tcp)
            d = dest()
            if d is not None:
                udp.sendto(data, d)
    except (OSError, ConnectionError):
        return


def forward_ports(tcp_conn: socket.socket, udp_listen: Addr, udp_target: Optional[Addr] = None) -> socket.socket:
    """Bridge one UDP port over an established TCP connection (both directions, daemon threads).

    Datagrams arriving at ``udp_listen`` go out on ``tcp_conn``; frames read from ``tcp_conn`` are sent to
    ``udp_target`` (or, when None, back to the last local UDP sender).  Returns the UDP socket."""
    udp = socket.socket(_family(udp_listen.ip), socket.SOCK_DGRAM)
    udp.bind(tuple(udp_listen))
    peer = [None]
    target = (lambda: tuple(udp_target)) if udp_target is not None else (lambda: peer[0])
    for fn, args in ((_udp_to_tcp, (udp, tcp_conn, peer)), (_tcp_to_udp, (tcp_conn, udp, target))):
        threading.Thread(target=fn, args=args, daemon=True).start()
    return udp


# ---------------------------------------------------------------------------- SC2 host / joiners
def _lan_ports(ports: Sequence[int]):
    """[server game, server base, client game, client base] -> RequestJoinGame port fields."""
    return {'server_ports': {'game_port': ports[0], 'base_port': ports[1]},
            'client_ports': [{'game_port': ports[2], 'base_port': ports[3]}]}


class LanGameHost:
    """Host a two-participant LAN game (host_remote_agent.py VsAgent): ``start`` creates the game on the
    host's SC2, joins the host player and serves the settings record to the remote player."""

    def __init__(self, map_name: str, race: str = 'zerg', name: str = 'host', version: Optional[str] = None,
                 host_ip: str = '127.0.0.1', config_port: int = 14380, realtime: bool = False):
        self.map_name, self.race, self.name, self.version = map_name, race, name, version
        self.host_ip, self.config_port, self.realtime = host_ip, config_port, realtime
        self._proc = self._ctrl = self._conn = None

    def settings(self, ports: Sequence[int], map_data: bytes, game_version: str) -> Dict:
        return {'map_name': self.map_name, 'map_data': map_data, 'game_version': game_version,
                'ports': {'server': {'game': ports[0], 'base': ports[1]},
                          'client': {'game': ports[2], 'base': ports[3]}},
                'realtime': self.realtime, 'host_race': self.race}

    def start(self, interface_options=None):
        from .sc2.launcher import SC2Process, pick_ports, map_path
        from .sc2.controller import RemoteController
        from .sc2_env import _pb
        from .map_info import MAPS
        sc_pb, common_pb, _ = _pb()
        ports = pick_ports(4)
        self._proc = SC2Process(self.version, host=self.host_ip)
        self._ctrl = RemoteController(self._proc.host, self._proc.port)
        path = map_path(MAPS[self.map_name][1])
        with open(path, 'rb') as f:
            map_data = f.read()
        create = sc_pb.RequestCreateGame(realtime=self.realtime)
        create.local_map.map_path = path
        create.local_map.map_data = map_data
        create.player_setup.add(type=sc_pb.Participant)
        create.player_setup.add(type=sc_pb.Participant)
        self._ctrl.create_game(create)
        version = self._ctrl.ping().game_version
        self._conn = serve_settings(Addr(self.host_ip, self.config_port), self.settings(ports, map_data, version))
        join = sc_pb.RequestJoinGame(race=common_pb.Race.Value(self.race.capitalize()), player_name=self.name)
        if interface_options is not None:
            join.options.CopyFrom(interface_options)
        else:
            join.options.raw = True
        lp = _lan_ports(ports)
        join.server_ports.game_port = lp['server_ports']['game_port']
        join.server_ports.base_port = lp['server_ports']['base_port']
        join.client_ports.add(**lp['client_ports'][0])
        self._ctrl.join_game(join)
        return self._ctrl

    def close(self):
        for obj, fn in ((self._conn, 'close'), (self._ctrl, 'quit'), (self._proc, 'close')):
            if obj is not None:
                try:
                    getattr(obj, fn)()
                except Exception:  # noqa: BLE001 - best-effort teardown
                    pass
        self._proc = self._ctrl = self._conn = None


class LanSC2Env(SC2Env):
    """Join a LAN game hosted elsewhere as the (single) agent slot of an :class:`SC2Env`.

    ``cfg.env`` keys on top of SC2Env's: ``lan_host`` (host address), ``lan_config_port``."""

    def __init__(self, cfg):
        env = cfg['env'] if 'env' in cfg else cfg
        env = dict(env)
        env.setdefault('player_ids', ['agent1', 'human'])
        super().__init__({'env': env} if 'env' in cfg else env)
        self._lan_host = env.get('lan_host', '127.0.0.1')
        self._lan_config_port = int(env.get('lan_config_port', 14380))
        self._num_agents = 1
        self._agent_slots = [0]
        self._settings = None

    def _launch(self):
        from .sc2.launcher import SC2Process
        from .sc2.controller import RemoteController
        self._settings = fetch_settings(Addr(self._lan_host, self._lan_config_port))
        self._procs = [SC2Process(self._version)]
        self._controllers = [RemoteController(self._procs[0].host, self._procs[0].port)]

    def _join_request(self):
        from .sc2_env import _pb
        sc_pb, common_pb, _ = _pb()
        s = self._settings
        self._map_name = s['map_name']
        join = sc_pb.RequestJoinGame(options=self._interface(0), host_ip=self._lan_host)
        join.race = common_pb.Race.Value(self._races[0].capitalize())
        join.player_name = self._player_ids[0][:32]
        join.server_ports.game_port = s['ports']['server']['game']
        join.server_ports.base_port = s['ports']['server']['base']
        join.client_ports.add(game_port=s['ports']['client']['game'], base_port=s['ports']['client']['base'])
        return join

    def _create_join(self):
        self._controllers[0].join_game(self._join_request())
        self._game_info = [self._controllers[0].game_info()]


class RemoteSC2Env(LanSC2Env):
    """Like :class:`LanSC2Env`, but drives an SC2 instance that is already running at
    ``cfg.env.remote_host:remote_port`` (e.g. started by a launcher on another node) instead of
    launching one."""

    def __init__(self, cfg):
        super().__init__(cfg)
        env = cfg['env'] if 'env' in cfg else cfg
        self._remote = Addr(env.get('remote_host', '127.0.0.1'), int(env.get('remote_port', 5000)))

    def _launch(self):
        from .sc2.controller import RemoteController
        self._settings = fetch_settings(Addr(self._lan_host, self._lan_config_port))
        self._procs = []
        self._controllers = [RemoteController(self._remote.ip, self._remote.port)]


# ---------------------------------------------------------------------------- generic loop / wrapper
class EnvWrapper:
    """Transparent wrapper base (base_env_wrapper.py): forwards everything to ``env``."""

    def __init__(self, env):
        self._env = env

    def __getattr__(self, name):
        return getattr(self._env, name)

    def reset(self, *a, **kw):
        return self._env.reset(*a, **kw)

    def step(self, *a, **kw):
        return self._env.step(*a, **kw)

    def close(self, *a, **kw):
        return self._env.close(*a, **kw)

    @property
    def unwrapped(self):
        return self._env.unwrapped if isinstance(self._env, EnvWrapper) else self._env


def run_loop(agents: Sequence, env, max_frames: int = 0, max_episodes: int = 0) -> Dict[str, int]:
    """Drive ``agents`` (objects with ``reset(map_name, race, game_info, obs)`` optional and
    ``step(obs) -> [action dict]``) through ``env`` (reset() -> (obs, game_info, map_name),
    step(actions) -> (obs, reward, done)) for ``max_frames`` env steps / ``max_episodes`` episodes
    (0 = unbounded) - run_loop.py:19-43 with this package's env contract."""
    frames = episodes = 0
    try:
        while not max_episodes or episodes < max_episodes:
            obs, game_info, map_name = env.reset()
            for i, a in enumerate(agents):
                if hasattr(a, 'reset') and i in obs:
                    a.reset(map_name, None, game_info.get(i) if isinstance(game_info, dict) else None, obs[i])
            episodes += 1
            done = False
            while not done:
                actions = {i: agents[i].step(o) for i, o in obs.items() if i < len(agents)}
                obs, _, done = env.step(actions)
                frames += 1
                if max_frames and frames >= max_frames:
                    return {'frames': frames, 'episodes': episodes}
    finally:
        if hasattr(env, 'close'):
            env.close()
    return {'frames': frames, 'episodes': episodes}
