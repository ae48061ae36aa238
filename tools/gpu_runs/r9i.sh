set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_cu_mask.py -q --timeout 120 --timeout-method thread > gpurun_out/r9i_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r9i_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r9i_pytest.txt | head; exit 1; }
for R in 16 32; do
APPLESTAR_LEARNER_CU_RESERVE=$R timeout -k 10 300 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32r$R > gpurun_out/r9i_pipeline_envs32_reserve$R.json 2> gpurun_out/r9i_pipeline_envs32_reserve$R.log || { tail -20 gpurun_out/r9i_pipeline_envs32_reserve$R.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r9i_pipeline_envs32_reserve$R.json')); s=d['inference_server']
print('reserve $R', d['actor_agent_steps_per_s'], d['learner_iters_per_s'], d['learner_train_ms_mean'], s['ms_per_group'])"
done
