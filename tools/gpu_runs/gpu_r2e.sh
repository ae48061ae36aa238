#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r2e_bench_graph.log 2>&1; rc=$?
echo "bench graph exit $rc"; tail -1 gpurun_out/r2e_bench_graph.log | grep -o '"ms_per_step.*' | cut -c1-40; grep -o '"host_ms_per_step.*' gpurun_out/r2e_bench_graph.log; fatal $rc
APPLESTAR_GRAPH_SIDE_STREAMS=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r2e_bench_graph_side.log 2>&1; rc=$?
echo "bench graph+side exit $rc"; tail -1 gpurun_out/r2e_bench_graph_side.log | grep -o '"ms_per_step.*' | cut -c1-40; grep -o '"host_ms_per_step.*' gpurun_out/r2e_bench_graph_side.log; fatal $rc
