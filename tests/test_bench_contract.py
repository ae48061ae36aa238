"""bench.py driver contract on CPU: launched by torch.distributed.run with two ranks (gloo), every rank
runs the learner step, rank 0 alone prints ONE JSON line whose value is the whole-job aggregate and whose
config names the data-parallel degree (the driver's N = 1, 2, 4, 8 scaling runs use this path with RCCL)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_bench_two_ranks_prints_one_aggregate_line(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', '29657', os.path.join(ROOT, 'bench.py'),
           '--gpus', '2', '--steps', '2', '--warmup', '1', '--batch', '1', '--unroll', '4', '--max-entities', '24']
    res = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=500)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config'):
        assert k in out, k
    assert out['n_gpus'] == 2 and out['steps'] == 2 and out['warmup'] == 1
    assert out['config']['parallelism'] == 'dp2' and out['config']['samples_per_step'] == 2 * 1 * 4
    # value = total samples over all ranks / the slowest rank's wall time
    assert abs(out['value'] - out['config']['samples_per_step'] / (out['ms_per_step'] / 1000.0)) < 0.02 * out['value']
    assert out['value'] > 0 and out['scaling'] == 'weak' and out['higher_is_better'] is True
