#!/bin/bash
# r5: GPU tests, bench, op-level profile, inference latency
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r5_pytest_gpu.log 2>&1; echo "pytest exit $?" | tee -a gpurun_out/r5_pytest_gpu.log
tail -3 gpurun_out/r5_pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r5_bench.log 2>&1 || { tail -30 gpurun_out/r5_bench.log; exit 1; }
tail -1 gpurun_out/r5_bench.log
timeout -k 10 600 python tools/op_profile.py --out gpurun_out/r5_op_profile.txt > gpurun_out/r5_op_profile.log 2>&1; echo "op_profile exit $?"
timeout -k 10 600 python tools/bench_inference.py > gpurun_out/r5_infer.log 2>&1; echo "infer exit $?"
cat gpurun_out/r5_infer.log | tail -5
timeout -k 10 600 python tools/phase_timing.py > gpurun_out/r5_phases.log 2>&1; echo "phases exit $?"
