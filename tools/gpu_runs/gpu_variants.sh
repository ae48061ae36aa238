#!/bin/bash
# bench variants: MIOpen find-mode autotune, TunableOp GEMM tuning
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --conv-benchmark 0 > gpurun_out/v_base.log 2>&1; echo "base $?"; tail -1 gpurun_out/v_base.log | cut -c1-200
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --conv-benchmark 1 > gpurun_out/v_convbench.log 2>&1; echo "convbench $?"; tail -1 gpurun_out/v_convbench.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop.csv timeout -k 10 900 python bench.py --steps 10 --warmup 5 --conv-benchmark 1 > gpurun_out/v_tunable.log 2>&1; echo "tunable $?"; tail -1 gpurun_out/v_tunable.log | cut -c1-200
