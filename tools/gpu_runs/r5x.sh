set -o pipefail
mkdir -p gpurun_out
run() {  # name, extra env, args
  N=$1; shift
  env "$@" timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 30 --precision fp32 --workdir /tmp/pipe_$N $PIPE_ARGS > gpurun_out/r5x_pipeline_$N.json 2> gpurun_out/r5x_pipeline_$N.log || { tail -20 gpurun_out/r5x_pipeline_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5x_pipeline_$N.json'));print('$N', {k: d[k] for k in ('learner_iters_per_s','learner_train_ms_mean','learner_train_main_thread_cpu_ms_mean','fresh_samples_per_s')})"
}
PIPE_ARGS="--max-reuse 1000000000" run noingest A=1 || exit 1
PIPE_ARGS="" run switch05 APPLESTAR_PIPE_SWITCH=0.0005 || exit 1
PIPE_ARGS="" run base A=1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "graphed_policy or small" > gpurun_out/r5x_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r5x_pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r5x_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5x_bench_inference.jsonl | cut -c1-300
timeout -k 10 200 python -u tools/inference_casts.py --batch 1 --top 50 > gpurun_out/r5x_inference_ops_b1.txt 2>&1 || exit 1
head -30 gpurun_out/r5x_inference_ops_b1.txt
