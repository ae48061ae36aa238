set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_flat_model.py tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "glue or skip or defer or epi2 or flat or resblock or conv3x3_f32 or fp32 or fused" > gpurun_out/r5d_pytest.txt 2>&1 || { tail -40 gpurun_out/r5d_pytest.txt; exit 1; }
tail -2 gpurun_out/r5d_pytest.txt
for v in default nodefer noskip; do
  case $v in default) E="";; nodefer) E="APPLESTAR_DEFER_WGRAD=0";; noskip) E="APPLESTAR_SKIP_LINK=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5d_bench_$v.json 2> gpurun_out/r5d_bench_$v.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5d_bench_$v.json'));print('$v', d['ms_per_step'])"
done
timeout -k 10 300 python tools/bench_gemm_variants.py 0,5 5 > gpurun_out/r5d_gemm_variants.jsonl 2>&1 || exit 1
cat gpurun_out/r5d_gemm_variants.jsonl
timeout -k 10 300 python tools/bench_conv_variants.py 0,3 5 > gpurun_out/r5d_conv_variants.jsonl 2>&1 || exit 1
cat gpurun_out/r5d_conv_variants.jsonl
TAG=r5d_pmc_gemm FILTER=gemm_f32_pipe bash tools/gpu_pmc.sh python3 tools/bench_gemm_variants.py 0 1
timeout -k 10 500 python -u tools/learn_curves.py --rl-only --no-control --rl-lrs 1e-4,3e-4,1e-3 --rl-iters 150 --out gpurun_out/r5d_learn_sweep.json > gpurun_out/r5d_learn.log 2>&1 || { tail -20 gpurun_out/r5d_learn.log; exit 1; }
grep run gpurun_out/r5d_learn.log | cut -c1-1200
TAG=r5d_fp32 ITERS=5 STEADY=3 BENCH_ARGS="--precision fp32 --steps 3 --warmup 2 --inference 0" bash tools/gpu_prof.sh
