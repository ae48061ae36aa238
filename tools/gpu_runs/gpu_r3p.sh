# conflict-free staging writes (conv3x3_f32 / gemm_f32 / attention_f32): numerics, microbench, LDS counters, fp32 bench
O=gpurun_out/r3p; mkdir -p $O
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
step micro_attn_f32 120 env PREC=fp32 python -u tools/bench_attention.py > $O/micro_attn_f32.jsonl 2>&1
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY"
step pmc_conv_f32 150 env TAG=r3p_pmc_conv_f32 FILTER=conv3x3_f32 COUNTERS="$C" bash tools/gpu_pmc.sh python3 tools/bench_f32_kernels.py conv
step pmc_attn_f32 150 env TAG=r3p_pmc_attn_f32 FILTER=attn COUNTERS="$C" PREC=fp32 bash tools/gpu_pmc.sh python3 tools/bench_attention.py child
step bench_fp32 300 python -u bench.py --precision fp32 --steps 10 --warmup 3 > $O/bench_fp32.json 2> $O/bench_fp32.err
rm -rf gpurun_out/r3p_pmc_*/ 2>/dev/null
echo done >> $O/progress.txt
