#!/bin/bash
# host side of the step: cProfile + phase timing (pipelined) on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_profile.py --steps 10 --out gpurun_out/r2dg_host_profile.txt > gpurun_out/r2dg_host.log 2>&1 || { tail -20 gpurun_out/r2dg_host.log; exit 1; }
head -60 gpurun_out/r2dg_host_profile.txt
timeout -k 10 300 python tools/host_phases.py --batch 6 --unroll 64 --max-entities 512 --steps 10 --no-sync > gpurun_out/r2dg_host_phases.txt 2>&1 || { tail -20 gpurun_out/r2dg_host_phases.txt; exit 1; }
tail -30 gpurun_out/r2dg_host_phases.txt
