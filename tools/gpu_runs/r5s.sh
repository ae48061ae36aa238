set -o pipefail
mkdir -p gpurun_out
for E in 32 8; do
  timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_$E > gpurun_out/r5s_pipeline_envs$E.json 2> gpurun_out/r5s_pipeline_envs$E.log || { tail -20 gpurun_out/r5s_pipeline_envs$E.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5s_pipeline_envs$E.json'));print($E, {k: d[k] for k in ('learner_iters_per_s','learner_train_ms_mean','learner_train_host_ms_mean','learner_train_cpu_ms_mean','learner_train_stream_ms_mean','fresh_samples_per_s','cgroup_cpu','affinity_cpus','loadavg')})"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5s_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/r5s_pytest_gpu.txt; exit $rc
