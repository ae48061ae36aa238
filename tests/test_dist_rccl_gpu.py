"""RCCL (backend ``nccl``) on the GPU box: the nccl-only branches of parallel/dist.py and the bucketed reducer's
async AVG all-reduce, executed for real at world size 1 (a 1-GPU box cannot host two RCCL ranks: RCCL refuses
two ranks on one device).  Multi-rank numerics are covered by the gloo rehearsals (tests/test_dp.py,
tests/test_model_gpu.py 2-rank test); this pins that the RCCL calls themselves run on MI355X."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_rccl_world1_collectives_and_reducer():
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', MASTER_ADDR='127.0.0.1')
    env.pop('APPLESTAR_DIST_BACKEND', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'helpers', 'rccl_world1.py'), str(_free_port())],
                       env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith('{')][-1])
    assert rec['backend'] == 'nccl', rec
    for k in ('avg_ok', 'min_ok', 'all_gather_ok', 'broadcast_ok', 'reducer_ok'):
        assert rec[k], (k, rec)
    assert rec['reducer_buckets'] >= 2, rec
