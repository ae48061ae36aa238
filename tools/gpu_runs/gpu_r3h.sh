# fp32 kernel microbenchmarks + PMC passes (MFMA busy, waits, LDS conflicts) on fp32 and bf16 conv / attention kernels
O=gpurun_out/r3h; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step micro_f32 200 python -u tools/bench_f32_kernels.py all > $O/micro_f32.jsonl 2>&1
step micro_attn_f32 120 env PREC=fp32 python -u tools/bench_attention.py > $O/micro_attn_f32.jsonl 2>&1
step micro_attn_bf16 120 python -u tools/bench_attention.py > $O/micro_attn_bf16.jsonl 2>&1
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU"
step pmc_conv_f32 150 env TAG=r3h_pmc_conv_f32 FILTER=conv3x3_f32 COUNTERS="$C" bash tools/gpu_pmc.sh python3 tools/bench_f32_kernels.py conv
step pmc_gemm_f32 150 env TAG=r3h_pmc_gemm_f32 FILTER=gemm_f32 COUNTERS="$C" bash tools/gpu_pmc.sh python3 tools/bench_f32_kernels.py gemm
step pmc_wgrad_f32 150 env TAG=r3h_pmc_wgrad_f32 FILTER=wgrad_f32 COUNTERS="$C" bash tools/gpu_pmc.sh python3 tools/bench_f32_kernels.py wgrad
step pmc_attn_f32 150 env TAG=r3h_pmc_attn_f32 FILTER=attn COUNTERS="$C" PREC=fp32 bash tools/gpu_pmc.sh python3 tools/bench_attention.py child
step pmc_attn_bf16 150 env TAG=r3h_pmc_attn_bf16 FILTER=attn COUNTERS="$C" bash tools/gpu_pmc.sh python3 tools/bench_attention.py child
step pmc_conv_bf16 150 env TAG=r3h_pmc_conv_bf16 FILTER=conv3x3 COUNTERS="$C" APPLESTAR_CONV_HALO=1 bash tools/gpu_pmc.sh python3 tools/bench_conv3x3.py child
rm -rf gpurun_out/r3h_pmc_*/ 2>/dev/null
echo done >> $O/progress.txt
