# side-stream weight gradients (A/B), attention swizzle without prefetch, gemm BK16 default; numerics + fp32 bench
O=gpurun_out/r3j; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step bench_fp32 300 python -u bench.py --precision fp32 --steps 10 --warmup 3 > $O/bench_fp32.json 2> $O/bench_fp32.err
step bench_fp32_noside 300 env APPLESTAR_SIDE_WGRAD=0 python -u bench.py --precision fp32 --steps 10 --warmup 3 > $O/bench_fp32_noside.json 2> $O/bench_fp32_noside.err
step bench_bf16 300 python -u bench.py --precision bf16 --steps 10 --warmup 3 > $O/bench_bf16.json 2> $O/bench_bf16.err
step bench_bf16_noside 300 env APPLESTAR_SIDE_WGRAD=0 python -u bench.py --precision bf16 --steps 10 --warmup 3 > $O/bench_bf16_noside.json 2> $O/bench_bf16_noside.err
step micro_attn_f32 120 env PREC=fp32 python -u tools/bench_attention.py > $O/micro_attn_f32.jsonl 2>&1
step pytest_k 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "f32 or fp32 or handoff or varlen or resblock" > $O/pytest_k.txt 2>&1
step pytest_model 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_parity_gpu.py tests/test_model_gpu.py > $O/pytest_model.txt 2>&1
echo done >> $O/progress.txt
