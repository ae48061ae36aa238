#!/bin/bash
# Attribution pass + refreshed SL bench and inference latency on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
T=r2db
timeout -k 10 300 python tools/memcpy_sources.py --out gpurun_out/${T}_memcpy_sources.txt > gpurun_out/${T}_memcpy.log 2>&1 || { tail -20 gpurun_out/${T}_memcpy.log; exit 1; }
timeout -k 10 300 python tools/op_time_sources.py --out gpurun_out/${T}_op_time_sources.txt > gpurun_out/${T}_optime.log 2>&1 || { tail -20 gpurun_out/${T}_optime.log; exit 1; }
timeout -k 10 300 python bench.py --mode sl --steps 20 --warmup 4 > gpurun_out/${T}_bench_sl.log 2>&1 || { tail -20 gpurun_out/${T}_bench_sl.log; exit 1; }
tail -1 gpurun_out/${T}_bench_sl.log
timeout -k 10 400 python tools/bench_inference.py --batches 1,16,64 --iters 30 > gpurun_out/${T}_inference.log 2>&1 || { tail -20 gpurun_out/${T}_inference.log; exit 1; }
tail -8 gpurun_out/${T}_inference.log
