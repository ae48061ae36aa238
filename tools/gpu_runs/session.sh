set -o pipefail
mkdir -p gpurun_out
APPLESTAR_F32_STAGED=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_f32 or conv3x3_f32 or linear_f32" > gpurun_out/x_pytest_staged.txt 2>&1 || { tail -30 gpurun_out/x_pytest_staged.txt; exit 1; }
timeout -k 10 200 python -u tools/bench_f32_kernels.py bf16 > gpurun_out/x_bf16_micro.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_f32_kernels.py conv > gpurun_out/x_conv_f32_unstaged.jsonl 2>&1 || exit 1
APPLESTAR_F32_STAGED=1 timeout -k 10 200 python -u tools/bench_f32_kernels.py conv > gpurun_out/x_conv_f32_staged.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_f32_kernels.py gemm > gpurun_out/x_gemm_f32_unstaged.jsonl 2>&1 || exit 1
APPLESTAR_F32_STAGED=1 timeout -k 10 200 python -u tools/bench_f32_kernels.py gemm > gpurun_out/x_gemm_f32_staged.jsonl 2>&1 || exit 1
timeout -k 10 200 python bench.py --precision bf16 --steps 20 --warmup 5 > gpurun_out/x_bench_bf16.json 2> gpurun_out/x_bf16.err || exit 1
APPLESTAR_BF16_GEMM=0 timeout -k 10 200 python bench.py --precision bf16 --steps 20 --warmup 5 > gpurun_out/x_bench_bf16_off.json 2> gpurun_out/x_bf16_off.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/x_bench_fp32.json 2> gpurun_out/x_fp32.err || exit 1
APPLESTAR_F32_STAGED=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/x_bench_fp32_staged.json 2> gpurun_out/x_fp32_staged.err || exit 1
