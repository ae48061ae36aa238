"""Restart-on-failure supervisor for framework roles (SURVEY §5.3 MI355X plan).

``Supervisor(cmd)`` runs a role as a child process (never exec-replacing itself) and restarts it
with exponential back-off when it exits non-zero, up to ``max_restarts``.  Learners restart from
their newest checkpoint: :func:`latest_checkpoint` is passed through ``APPLESTAR_RESUME_PATH`` and
the learner's ``load_ckpt`` hook picks it up, so a crash costs at most ``save_ckpt`` freq iterations.
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import time
from typing import List, Optional


def latest_checkpoint(exp_dir: str, player_id: Optional[str] = None) -> Optional[str]:
    d = os.path.join(exp_dir, player_id, 'checkpoint') if player_id else os.path.join(exp_dir, 'checkpoint')
    files = glob.glob(os.path.join(d, '*_iteration_*.pth.tar'))
    if not files:
        return None
    it = lambda p: int(re.search(r'_iteration_(\d+)\.pth\.tar$', p).group(1))
    return max(files, key=it)


class Supervisor:
    def __init__(self, cmd: List[str], max_restarts: int = 5, backoff: float = 1.0, max_backoff: float = 60.0,
                 env: Optional[dict] = None, resume_dir: Optional[str] = None, player_id: Optional[str] = None):
        self.cmd = list(cmd)
        self.max_restarts = max_restarts
        self.backoff, self.max_backoff = backoff, max_backoff
        self.env = dict(os.environ if env is None else env)
        self.resume_dir, self.player_id = resume_dir, player_id
        self.restarts = 0
        self.exit_codes: List[int] = []

    def run(self) -> int:
        delay = self.backoff
        while True:
            env = dict(self.env)
            if self.resume_dir:
                ck = latest_checkpoint(self.resume_dir, self.player_id)
                if ck:
                    env['APPLESTAR_RESUME_PATH'] = ck
            rc = subprocess.call(self.cmd, env=env)
            self.exit_codes.append(rc)
            if rc == 0:
                return 0
            if self.restarts >= self.max_restarts:
                print(f'[supervisor] {self.cmd[:3]} failed {self.restarts + 1}x, giving up (rc={rc})',
                      file=sys.stderr)
                return rc
            self.restarts += 1
            print(f'[supervisor] exit {rc}; restart {self.restarts}/{self.max_restarts} in {delay:.1f}s',
                  file=sys.stderr)
            time.sleep(delay)
            delay = min(delay * 2, self.max_backoff)
