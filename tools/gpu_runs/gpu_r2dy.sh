#!/bin/bash
# in-place residual-gradient addmm: full GPU suite, smoke, bench, A/B/A/B of the link
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2dy_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2dy_pytest_gpu.log | cut -c1-400; exit 1; }
tail -1 gpurun_out/r2dy_pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py > gpurun_out/r2dy_smoke.log 2>&1 || { tail -20 gpurun_out/r2dy_smoke.log; exit 1; }
tail -1 gpurun_out/r2dy_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2dy_bench.jsonl 2>gpurun_out/r2dy_bench.err || { tail -20 gpurun_out/r2dy_bench.err; exit 1; }
cut -c1-300 gpurun_out/r2dy_bench.jsonl
VAR=APPLESTAR_RESID_LINK bash tools/gpu_ab3.sh | tee gpurun_out/r2dy_ab_resid_link.txt || exit 1
