# fp32 kernel round: attention LDS swizzle + prefetch, incremental conv-wgrad coordinates, 32-deep gemm_f32 stages,
# ReLU-mask hand-off; numerics, microbenchmarks (BK 32 vs 16), fp32 bench + steady profile
O=gpurun_out/r3i; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_f32 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "f32 or fp32 or handoff or varlen" > $O/pytest_f32.txt 2>&1
step micro_f32 200 python -u tools/bench_f32_kernels.py all > $O/micro_f32.jsonl 2>&1
step micro_gemm_bk16 120 env APPLESTAR_GEMM_F32_BK=16 python -u tools/bench_f32_kernels.py gemm > $O/micro_gemm_bk16.jsonl 2>&1
step micro_attn_f32 120 env PREC=fp32 python -u tools/bench_attention.py > $O/micro_attn_f32.jsonl 2>&1
step bench_fp32 400 python -u bench.py --precision fp32 --steps 10 --warmup 3 > $O/bench_fp32.json 2> $O/bench_fp32.err
step prof_fp32 560 env TAG=r3i_fp32 ITERS=7 STEADY=3 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 4 --warmup 3 --inference 0" bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
echo done >> $O/progress.txt
