set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused" > gpurun_out/r5a_pytest.txt 2>&1 || { tail -40 gpurun_out/r5a_pytest.txt; exit 1; }
tail -1 gpurun_out/r5a_pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5a_bench_fp32.json 2> gpurun_out/r5a_bench_fp32.log || exit 1
cat gpurun_out/r5a_bench_fp32.json | cut -c1-300
TAG=r5a_fp32 ITERS=5 STEADY=3 BENCH_ARGS="--precision fp32 --steps 3 --warmup 2 --inference 0" bash tools/gpu_prof.sh
timeout -k 10 400 python -u tools/learn_curves.py --out gpurun_out/r5a_learn_curves.json > gpurun_out/r5a_learn.log 2>&1 || { tail -20 gpurun_out/r5a_learn.log; exit 1; }
cat gpurun_out/r5a_learn.log | cut -c1-600
