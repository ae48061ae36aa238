# headline numbers for the docs: default bench (fp32 + bf16 + inference) first on the box, SL bench, shared-batch
# test; then the effective-clock pass on the MFMA probe and the fp32 conv / gemm microbenchmarks
O=gpurun_out/r3r; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step bench_default 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
step bench_sl 400 python -u bench.py --mode sl --inference 0 > $O/bench_sl.json 2> $O/bench_sl.err
step pytest_shared 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "shared_batch" > $O/pytest_shared.txt 2>&1
step clock_probe 150 env TAG=r3r_clock_probe bash tools/gpu_clock.sh ./tools/mfma_peak
step clock_conv 150 env TAG=r3r_clock_conv FILTER=f32 bash tools/gpu_clock.sh python3 tools/bench_f32_kernels.py conv
step clock_gemm 150 env TAG=r3r_clock_gemm bash tools/gpu_clock.sh python3 tools/bench_f32_kernels.py gemm
rm -rf gpurun_out/r3r_clock_*/ 2>/dev/null
echo done >> $O/progress.txt
