#!/bin/bash
# attribution of the small torch ops (casts, copies, adds) after the derived-weight change
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python tools/elementwise_attrib.py --steps 2 --top 80 --out gpurun_out/r2dl_elementwise_attrib.txt > gpurun_out/r2dl_ew.log 2>&1 || { tail -20 gpurun_out/r2dl_ew.log; exit 1; }
head -90 gpurun_out/r2dl_elementwise_attrib.txt
