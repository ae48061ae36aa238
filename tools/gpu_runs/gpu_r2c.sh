#!/bin/bash
# Overlapped master-gradient DP path: 2-rank gloo rehearsal on one GPU, GPU suite, 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
APPLESTAR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/r2c_dp2_gloo.log 2>&1; rc=$?
echo "dp2 gloo exit $rc"; grep metric gpurun_out/r2c_dp2_gloo.log | cut -c1-300; [ $rc -eq 0 ] || { tail -30 gpurun_out/r2c_dp2_gloo.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2c_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r2c_pytest_gpu.log; fatal $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r2c_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r2c_bench.log | cut -c1-300; fatal $rc
