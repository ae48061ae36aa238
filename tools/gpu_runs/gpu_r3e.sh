# round-3 GPU session e: full GPU suite, both-precision bench (fused clip+Adam), bf16 steady profile
O=gpurun_out/r3e; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
step bench_both 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_both.json 2> $O/bench_both.err
TAG=r3e_bf16 ITERS=15 STEADY=5 BENCH_ARGS="--precision bf16 --steps 10 --warmup 5 --inference 0" step prof_bf16 400 bash tools/gpu_prof.sh > $O/prof_bf16.out 2>&1
echo done >> $O/progress.txt
