"""Liveness tracking for the control plane (the reference has no heartbeat / failure
detector).  Every learner rank and actor reports ``(role, id)`` heartbeats; the league serves them
and marks members dead after ``timeout`` seconds of silence so operators / supervisors can react."""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, Optional


class HeartbeatRegistry:
    def __init__(self, timeout: float = 120.0, clock: Callable[[], float] = time.time):
        self.timeout = timeout
        self._clock = clock
        self._lock = threading.Lock()
        self._seen: Dict[str, dict] = {}

    def beat(self, role: str, member_id: str, info: Optional[dict] = None) -> None:
        key = f'{role}/{member_id}'
        with self._lock:
            e = self._seen.setdefault(key, {'role': role, 'id': member_id, 'first_seen': self._clock(), 'beats': 0})
            e['last_seen'] = self._clock()
            e['beats'] += 1
            if info:
                e['info'] = dict(info)

    def status(self) -> Dict[str, dict]:
        now = self._clock()
        with self._lock:
            return {k: dict(v, age=now - v['last_seen'], alive=now - v['last_seen'] <= self.timeout)
                    for k, v in self._seen.items()}

    def dead(self, role: Optional[str] = None):
        return sorted(k for k, v in self.status().items() if not v['alive'] and (role is None or v['role'] == role))

    def forget(self, role: str, member_id: str) -> None:
        with self._lock:
            self._seen.pop(f'{role}/{member_id}', None)


class HeartbeatSender:
    """Background thread posting ``/league/heartbeat`` every ``interval`` seconds."""

    def __init__(self, client, role: str, member_id: str, interval: float = 10.0, info_fn=None):
        self._client, self._role, self._id = client, role, member_id
        self._interval = interval
        self._info_fn = info_fn
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True, name=f'heartbeat-{role}')
        self._t.start()

    def _loop(self):
        while not self._stop.is_set():
            try:
                self._client.post('/league/heartbeat', {'role': self._role, 'id': self._id,
                                                        'info': self._info_fn() if self._info_fn else {}})
            except Exception:  # noqa: BLE001 - the league may be restarting; keep beating
                pass
            self._stop.wait(self._interval)

    def stop(self):
        self._stop.set()
