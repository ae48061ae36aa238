#!/bin/bash
# stream concurrency: plain run, then under rocprofv3 kernel tracing (does the tracer serialise?)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/stream_overlap_check.py > $R/gpurun_out/r2de_overlap_plain.log 2>&1 || exit 1
tail -1 $R/gpurun_out/r2de_overlap_plain.log
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r2de_prof -o run --output-format csv -- python3 $R/tools/stream_overlap_check.py > $R/gpurun_out/r2de_overlap_traced.log 2>&1 || exit 1
tail -1 $R/gpurun_out/r2de_overlap_traced.log
rm -rf $R/gpurun_out/r2de_prof
