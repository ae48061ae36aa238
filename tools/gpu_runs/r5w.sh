set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_glue_fusions_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "head_sample or multi_logp or su_sample or target_unit or graphed_policy or inference_server_graphed" > gpurun_out/r5w_pytest_focus.txt 2>&1; rc=$?
tail -3 gpurun_out/r5w_pytest_focus.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_small_gemm.py > gpurun_out/r5w_small_gemm.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5w_small_gemm.jsonl
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r5w_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5w_bench_inference.jsonl | cut -c1-300
APPLESTAR_GRAPH_SIDE_STREAMS=1 timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph > gpurun_out/r5w_bench_inference_side.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5w_bench_inference_side.jsonl | cut -c1-300
for E in 32 64; do
APPLESTAR_PIPE_PROFILE_AT=25 APPLESTAR_PIPE_PROFILE_N=5 APPLESTAR_PIPE_PROFILE_OUT=$PWD/gpurun_out/r5w_learner_profile_envs$E.txt timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_$E > gpurun_out/r5w_pipeline_envs$E.json 2> gpurun_out/r5w_pipeline_envs$E.log || { tail -20 gpurun_out/r5w_pipeline_envs$E.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5w_pipeline_envs$E.json'));print($E, {k: d[k] for k in ('learner_iters_per_s','learner_samples_per_s_fed','learner_train_ms_mean','learner_train_cpu_ms_mean','learner_train_main_thread_cpu_ms_mean','fresh_samples_per_s','cgroup_cpu')})"
head -8 gpurun_out/r5w_learner_profile_envs$E.txt
done
