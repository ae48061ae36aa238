set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gemm_variants.py 0,5 5 > gpurun_out/r5c_gemm_variants.jsonl 2>&1 || { tail -20 gpurun_out/r5c_gemm_variants.jsonl; exit 1; }
cat gpurun_out/r5c_gemm_variants.jsonl
timeout -k 10 300 python tools/bench_conv_variants.py 0,3 5 > gpurun_out/r5c_conv_variants.jsonl 2>&1 || { tail -20 gpurun_out/r5c_conv_variants.jsonl; exit 1; }
cat gpurun_out/r5c_conv_variants.jsonl
TAG=r5c_pmc_gemm FILTER=gemm_f32_pipe bash tools/gpu_pmc.sh python3 tools/bench_gemm_variants.py 0 1
TAG=r5c_pmc_gemm2 FILTER=gemm_f32_pipe COUNTERS="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh python3 tools/bench_gemm_variants.py 0 1
timeout -k 10 500 python -u tools/learn_curves.py --rl-only --no-control --rl-lrs 1e-4,3e-4,1e-3 --rl-iters 150 --out gpurun_out/r5c_learn_sweep.json > gpurun_out/r5c_learn.log 2>&1 || { tail -20 gpurun_out/r5c_learn.log; exit 1; }
grep run gpurun_out/r5c_learn.log | cut -c1-1200
