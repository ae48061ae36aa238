set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_flat_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or flat" > gpurun_out/r5a_pytest.txt 2>&1 || { tail -40 gpurun_out/r5a_pytest.txt; exit 1; }
tail -1 gpurun_out/r5a_pytest.txt
timeout -k 10 300 python tools/bench_gemm_variants.py 0,3,4 5 > gpurun_out/r5a_gemm_variants.jsonl 2>&1 || { tail -20 gpurun_out/r5a_gemm_variants.jsonl; exit 1; }
cat gpurun_out/r5a_gemm_variants.jsonl
timeout -k 10 300 python tools/bench_conv_variants.py 0,1,2 5 > gpurun_out/r5a_conv_variants.jsonl 2>&1 || { tail -20 gpurun_out/r5a_conv_variants.jsonl; exit 1; }
cat gpurun_out/r5a_conv_variants.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5a_bench_fp32.json 2> gpurun_out/r5a_bench_fp32.log || exit 1
cat gpurun_out/r5a_bench_fp32.json | cut -c1-300
timeout -k 10 400 python -u tools/learn_curves.py --out gpurun_out/r5a_learn_curves.json > gpurun_out/r5a_learn.log 2>&1 || { tail -20 gpurun_out/r5a_learn.log; exit 1; }
cat gpurun_out/r5a_learn.log | cut -c1-700
TAG=r5a_fp32 ITERS=5 STEADY=3 BENCH_ARGS="--precision fp32 --steps 3 --warmup 2 --inference 0" bash tools/gpu_prof.sh
timeout -k 10 300 python tools/glue_sites.py --steps 2 --precision fp32 --shapes > gpurun_out/r5a_glue_sites_fp32.txt 2>&1 || exit 1
head -5 gpurun_out/r5a_glue_sites_fp32.txt
