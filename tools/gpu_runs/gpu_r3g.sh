# new kernel tests (gemm_f32 epilogues, head sampling) + graphed policy / inference tests + fp32 steady profile
O=gpurun_out/r3g; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_new 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm_f32 or head_sample or target_unit or graphed_policy or inference_server or linear_f32" -v --timeout 120 --timeout-method thread > $O/pytest_new.txt 2>&1
step bench_infer 300 python -u bench.py --precision bf16 --steps 5 --warmup 3 > $O/bench_bf16_infer.json 2> $O/bench_bf16_infer.err
TAG=r3g_fp32 ITERS=7 STEADY=3 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 4 --warmup 3 --inference 0" step prof_fp32 560 bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
step pipeline 300 python -u tools/bench_pipeline.py --envs 12 --seconds 60 --batch 6 --traj-len 64 > $O/pipeline.json 2> $O/pipeline.err
echo done >> $O/progress.txt
