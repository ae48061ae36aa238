#!/bin/bash
# Whole-step HIP graphs: equivalence test, then eager vs graphed bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 200 --timeout-method thread -k "graphed_train_step or trainer_step or direct_master" > gpurun_out/r2d_test.log 2>&1; rc=$?
echo "test exit $rc"; tail -25 gpurun_out/r2d_test.log; fatal $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r2d_bench_graph.log 2>&1; rc=$?
echo "bench graph exit $rc"; tail -3 gpurun_out/r2d_bench_graph.log | cut -c1-1500; fatal $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-graph > gpurun_out/r2d_bench_eager.log 2>&1; rc=$?
echo "bench eager exit $rc"; tail -1 gpurun_out/r2d_bench_eager.log | cut -c1-300; fatal $rc
