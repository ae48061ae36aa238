# round-3 GPU session d: fp32 conv / wgrad / linear kernels vs float64, whole-model parity, fp32 bench + steady profile
O=gpurun_out/r3d; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_f32 300 python -u -m pytest tests/test_kernels_gpu.py -k "f32 or fp32" -v --timeout 120 --timeout-method thread > $O/pytest_f32.txt 2>&1
step pytest_parity 600 python -u -m pytest tests/test_model_parity_gpu.py -v --timeout 400 --timeout-method thread > $O/pytest_parity.txt 2>&1
step bench_fp32 400 python -u bench.py --precision fp32 --steps 10 --warmup 3 --inference 0 > $O/bench_fp32.json 2> $O/bench_fp32.err
TAG=r3d_fp32 ITERS=7 STEADY=3 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 4 --warmup 3 --inference 0" step prof_fp32 560 bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
echo done >> $O/progress.txt
