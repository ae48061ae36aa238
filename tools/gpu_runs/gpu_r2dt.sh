#!/bin/bash
# current-state attribution: rocprof kernel stats, small-op sources (elementwise / cast / launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
TAG=r2dt_prof bash tools/gpu_prof.sh > gpurun_out/r2dt_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2dt_prof_summary.log; exit 1; }
head -12 gpurun_out/r2dt_prof_summary.log
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python tools/elementwise_attrib.py --top 90 --out gpurun_out/r2dt_elementwise_attrib.txt > gpurun_out/r2dt_ea.log 2>&1 || { tail -20 gpurun_out/r2dt_ea.log; exit 1; }
timeout -k 10 300 python tools/cast_sources.py --out gpurun_out/r2dt_cast_sources.txt > gpurun_out/r2dt_cs.log 2>&1 || { tail -20 gpurun_out/r2dt_cs.log; exit 1; }
head -30 gpurun_out/r2dt_elementwise_attrib.txt
