set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_derived_weights_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "su_sample or fused_gated or cached_forms" > gpurun_out/r5t_pytest_focus.txt 2>&1; rc=$?
tail -3 gpurun_out/r5t_pytest_focus.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 > gpurun_out/r5t_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5t_bench_inference.jsonl | cut -c1-400
APPLESTAR_GRAPH_SIDE_STREAMS=1 timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "graphed_policy or inference_server_graphed" > gpurun_out/r5t_pytest_sidestream.txt 2>&1; rc=$?
tail -2 gpurun_out/r5t_pytest_sidestream.txt; [ $rc -eq 0 ] || exit 1
APPLESTAR_GRAPH_SIDE_STREAMS=1 timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 --modes policy_graph > gpurun_out/r5t_bench_inference_side.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5t_bench_inference_side.jsonl | cut -c1-400
APPLESTAR_PIPE_PROFILE_AT=25 APPLESTAR_PIPE_PROFILE_N=5 APPLESTAR_PIPE_PROFILE_OUT=$PWD/gpurun_out/r5t_learner_cprofile.txt timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32 > gpurun_out/r5t_pipeline_envs32.json 2> gpurun_out/r5t_pipeline_envs32.log || { tail -20 gpurun_out/r5t_pipeline_envs32.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5t_pipeline_envs32.json'));print({k: d[k] for k in ('learner_iters_per_s','learner_train_ms_mean','learner_train_cpu_ms_mean','learner_train_main_thread_cpu_ms_mean','fresh_samples_per_s')})"
head -60 gpurun_out/r5t_learner_cprofile.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5t_pytest_gpu.txt 2>&1; rc=$?
tail -8 gpurun_out/r5t_pytest_gpu.txt; exit $rc
