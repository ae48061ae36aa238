set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small" > gpurun_out/s5_pytest.txt 2>&1 || { tail -30 gpurun_out/s5_pytest.txt; exit 1; }
timeout -k 10 300 python -u tools/bench_f32_kernels.py smallnative > gpurun_out/s5_small.jsonl 2>&1 || exit 1
