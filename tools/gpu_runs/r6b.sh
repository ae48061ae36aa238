set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "ring or graphed_policy" > gpurun_out/r6b_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r6b_pytest.txt; [ $rc -eq 0 ] || exit 1
for E in 32 64; do
APPLESTAR_PIPE_PROFILE_AT=25 APPLESTAR_PIPE_PROFILE_N=5 APPLESTAR_PIPE_PROFILE_OUT=$PWD/gpurun_out/r6b_learner_profile_envs$E.txt timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_$E > gpurun_out/r6b_pipeline_envs$E.json 2> gpurun_out/r6b_pipeline_envs$E.log || { tail -20 gpurun_out/r6b_pipeline_envs$E.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6b_pipeline_envs$E.json'));print($E, {k: d[k] for k in ('learner_iters_per_s','learner_samples_per_s_fed','learner_train_ms_mean','learner_train_main_thread_cpu_ms_mean','fresh_samples_per_s','cgroup_cpu')})"
head -8 gpurun_out/r6b_learner_profile_envs$E.txt
done
