#!/bin/bash
# residual-gradient link: test (native vs plain vs torch-bf16 / fp64), full GPU suite, smoke, driver-shaped bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2dx_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2dx_pytest_gpu.log | cut -c1-400; exit 1; }
tail -1 gpurun_out/r2dx_pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/r2dx_smoke.log 2>&1 || { tail -20 gpurun_out/r2dx_smoke.log; exit 1; }
tail -1 gpurun_out/r2dx_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2dx_bench.jsonl 2>gpurun_out/r2dx_bench.err || { tail -20 gpurun_out/r2dx_bench.err; exit 1; }
cut -c1-300 gpurun_out/r2dx_bench.jsonl
