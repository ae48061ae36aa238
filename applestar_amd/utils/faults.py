"""Fault injection for recovery tests (the reference has none).

``APPLESTAR_FAULT="<point>:<n>[:<action>]"`` (comma separated for several) triggers ``action`` the
n-th time ``inject('<point>')`` is reached in this process: ``exit`` (os._exit(17), default),
``raise`` (RuntimeError), ``hang`` (sleep forever).  Points wired in the framework:
``learner_iter`` (after each learner iteration), ``actor_step`` (each env step of an env worker),
``env_reset`` (each episode start); ``actor_step@<env_id>`` targets one env worker.  With
``APPLESTAR_FAULT_ONCE=<file>`` a fault fires only if the file does not exist yet (and creates it),
so a supervised restart is not killed again.  Zero cost when the variable is unset.
"""
from __future__ import annotations

import os
import time
from collections import Counter

_counts: Counter = Counter()
_spec = None


def _parse():
    global _spec
    if _spec is None:
        _spec = {}
        for item in filter(None, os.environ.get('APPLESTAR_FAULT', '').split(',')):
            parts = item.split(':')
            _spec[parts[0]] = (int(parts[1]), parts[2] if len(parts) > 2 else 'exit')
    return _spec


def reset():
    global _spec
    _spec = None
    _counts.clear()


def inject(point: str) -> None:
    spec = _parse()
    if point not in spec:
        return
    _counts[point] += 1
    n, action = spec[point]
    if _counts[point] != n:
        return
    once = os.environ.get('APPLESTAR_FAULT_ONCE')
    if once:
        if os.path.exists(once):
            return
        open(once, 'w').close()
    if action == 'raise':
        raise RuntimeError(f'injected fault at {point}#{n}')
    if action == 'hang':
        while True:
            time.sleep(3600)
    os._exit(17)
