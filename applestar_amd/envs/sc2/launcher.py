"""Locate and launch StarCraft II (``pysc2/run_configs`` + ``pysc2/lib/sc_process.py``).

* install discovery: ``$SC2PATH``, then the platform defaults (``~/StarCraftII`` on Linux,
  ``/Applications/StarCraft II``, ``C:/Program Files (x86)/StarCraft II``);
* version table (game version -> build / data hash) extracted from the reference into
  ``lib/data/game_data.json``; replay-version selection via ``SC2PATH<ver>`` env overrides;
* :class:`SC2Process` spawns ``Versions/Base<build>/SC2_x64 -listen -port -dataDir -tempDir
  -displayMode 0`` (``sc_process.py:59-143``), waits for the websocket port, and kills the process
  group on close.
"""
from __future__ import annotations

import glob
import os
import platform
import shutil
import signal
import socket
import subprocess
import tempfile
import time
from collections import namedtuple
from typing import List, Optional

from ...lib.game_data import _RAW

Version = namedtuple('Version', ['game_version', 'build_version', 'data_version', 'binary'])
VERSIONS = {v[0]: Version(*v) for v in _RAW['sc2_versions']}
DEFAULT_VERSION = '4.10.0'


def sc2_path(version: Optional[str] = None) -> Optional[str]:
    if version:
        p = os.environ.get('SC2PATH' + version)
        if p and os.path.isdir(p):
            return p
    p = os.environ.get('SC2PATH')
    if p and os.path.isdir(p):
        return p
    for cand in (os.path.expanduser('~/StarCraftII'), '/Applications/StarCraft II',
                 'C:/Program Files (x86)/StarCraft II'):
        if os.path.isdir(cand):
            return cand
    return None


def find_sc2_binary(version: Optional[str] = None) -> Optional[str]:
    base = sc2_path(version)
    if base is None:
        return None
    exe = 'SC2_x64' if platform.system() == 'Linux' else ('SC2_x64.exe' if platform.system() == 'Windows' else
                                                          'SC2.app/Contents/MacOS/SC2')
    if version and version in VERSIONS:
        p = os.path.join(base, 'Versions', f'Base{VERSIONS[version].build_version}', exe)
        if os.path.exists(p):
            return p
    builds = sorted(glob.glob(os.path.join(base, 'Versions', 'Base*', exe)),
                    key=lambda x: int(os.path.basename(os.path.dirname(x))[4:] or 0))
    return builds[-1] if builds else None


def map_path(map_rel: str) -> str:
    """Absolute path of a map given its ``Ladder2019Season2\\X.SC2Map`` style relative path."""
    base = sc2_path() or ''
    return os.path.join(base, 'Maps', *map_rel.replace('\\', '/').split('/'))


def install_maps(src_dir: str) -> None:
    """Copy the bundled ladder maps into ``$SC2PATH/Maps`` if missing (``rl_train.py:115-116``)."""
    base = sc2_path()
    if base is None or not os.path.isdir(src_dir):
        return
    dst = os.path.join(base, 'Maps', os.path.basename(src_dir))
    if not os.path.exists(dst):
        shutil.copytree(src_dir, dst)


def pick_port(host: str = '127.0.0.1') -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def pick_ports(n: int) -> List[int]:
    return [pick_port() for _ in range(n)]


class SC2Process:
    def __init__(self, version: Optional[str] = None, host: str = '127.0.0.1', port: Optional[int] = None,
                 timeout: float = 120.0, extra_args: Optional[List[str]] = None, full_screen: bool = False):
        exe = find_sc2_binary(version or DEFAULT_VERSION)
        if exe is None:
            raise FileNotFoundError('StarCraft II binary not found (set SC2PATH)')
        self.host, self.port = host, port or pick_port(host)
        self._tmp = tempfile.mkdtemp(prefix='sc-')
        data_dir = sc2_path(version) + os.sep
        args = [exe, '-listen', host, '-port', str(self.port), '-dataDir', data_dir, '-tempDir', self._tmp]
        if not full_screen:
            args += ['-displayMode', '0']
        args += list(extra_args or [])
        cwd = os.path.join(sc2_path(version), 'Support64') if platform.system() == 'Windows' else None
        self._proc = subprocess.Popen(args, cwd=cwd, start_new_session=True,
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        self._wait_port(timeout)

    def _wait_port(self, timeout: float):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self._proc.poll() is not None:
                raise RuntimeError(f'SC2 exited with code {self._proc.returncode}')
            try:
                with socket.create_connection((self.host, self.port), timeout=1):
                    return
            except OSError:
                time.sleep(0.5)
        self.close()
        raise TimeoutError('SC2 did not open its websocket port')

    @property
    def running(self) -> bool:
        return self._proc is not None and self._proc.poll() is None

    def close(self):
        if self._proc is not None and self._proc.poll() is None:
            try:
                os.killpg(self._proc.pid, signal.SIGTERM)
                self._proc.wait(timeout=10)
            except (ProcessLookupError, subprocess.TimeoutExpired):
                try:
                    os.killpg(self._proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        self._proc = None
        shutil.rmtree(self._tmp, ignore_errors=True)
