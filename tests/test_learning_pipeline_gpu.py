"""The production RL pipeline learns: a bounded ``tools/learn_pipeline.py`` run on one GPU -
league, coordinator, actor env workers on the LEARNABLE FakeSC2Env, GPU batched inference server, data plane, HBM
trajectory ring, RL learner, flat model push back into the inference server - and the ACTOR-side curve must rise:
the share of rewarded action types the agents pick and their win rate against the bot, first 30-s bin vs last.

Slow (~2.5 min per precision): runs only with APPLESTAR_RUN_SLOW=1.  Both learners: fp32 and the bf16 one.
The full-length curves are kept in profiles/ (``r8b_learn_pipeline_*.json``)."""
import json
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow,
              pytest.mark.skipif(os.environ.get('APPLESTAR_RUN_SLOW') != '1', reason='slow: APPLESTAR_RUN_SLOW=1')]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(420)
@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_pipeline_learns_rewarded_actions(precision, tmp_path):
    out = tmp_path / f'learn_{precision}.json'
    cmd = [sys.executable, '-u', os.path.join(ROOT, 'tools', 'learn_pipeline.py'), '--envs', '24', '--seconds', '120',
           '--precision', precision, '--lr', '1e-4', '--report', '30', '--workdir', str(tmp_path / 'work'),
           '--out', str(out)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=400, text=True)
    progress = [ln for ln in r.stdout.splitlines() if ln.startswith('{"progress"')]
    print('\n'.join(progress))
    assert out.exists(), r.stdout[-3000:]
    d = json.loads(out.read_text())
    if os.path.isdir(os.path.join(ROOT, 'gpurun_out')):
        shutil.copy(out, os.path.join(ROOT, 'gpurun_out', f'learn_pipeline_test_{precision}.json'))
    first, last = d['first_bin'], d['last_bin']
    assert d['learner_iterations'] > 500 and d['episodes'] > 2000, d
    # chance: a quarter of the action types is rewarded; the untrained policy picks them ~25 % of the time
    assert d['rate_before_training'] is None or d['rate_before_training'] < 0.35, d
    assert last['rewarded_rate'] >= first['rewarded_rate'] + 0.2, (first, last)
    assert last['win_rate'] >= first['win_rate'] + 0.1 and last['win_rate'] > 0.8, (first, last)
