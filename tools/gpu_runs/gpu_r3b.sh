# round-3 GPU session b: parity tests (with torch-bf16 / fp32 controls), per-op layer diag, fp32 + bf16 kernel profiles
O=gpurun_out/r3b; mkdir -p $O
step() {  # name timeout cmd...  (test failures rc 1 continue; faults / timeouts stop the session)
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_parity 600 python -u -m pytest tests/test_model_parity_gpu.py -v --timeout 400 --timeout-method thread > $O/pytest_parity.txt 2>&1
cp gpurun_out/*.json $O/ 2>/dev/null
step layer_diag 300 python -u tools/diag/layer_grad_diag.py > $O/layer_grad_diag.txt 2>&1
TAG=r3b_fp32 ITERS=6 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 3 --warmup 3 --inference 0" step prof_fp32 560 bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
TAG=r3b_bf16 ITERS=15 BENCH_ARGS="--precision bf16 --steps 10 --warmup 5 --inference 0" step prof_bf16 400 bash tools/gpu_prof.sh > $O/prof_bf16.out 2>&1
echo done >> $O/progress.txt
