# round-3 GPU session c: steady-state fp32 + bf16 kernel tables, fp32 row diag
O=gpurun_out/r3c; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step row_diag 200 python -u tools/diag/fp32_row_diag.py > $O/fp32_row_diag.txt 2>&1
TAG=r3c_fp32 ITERS=7 STEADY=3 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 4 --warmup 3 --inference 0" step prof_fp32 560 bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
TAG=r3c_bf16 ITERS=15 STEADY=5 BENCH_ARGS="--precision bf16 --steps 10 --warmup 5 --inference 0" step prof_bf16 400 bash tools/gpu_prof.sh > $O/prof_bf16.out 2>&1
echo done >> $O/progress.txt
