#!/bin/bash
# MI355X check: GPU tests, native bench, optional rocprofv3 kernel stats (PROFILE=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  echo "pytest exit $?" >> gpurun_out/${TAG}_pytest_gpu.log
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-8} --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
if [ "${PROFILE:-0}" = "1" ]; then
  ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 )
  echo "prof exit $?"
fi
if [ "${PHASES:-0}" = "1" ]; then
  timeout -k 10 600 python tools/phase_timing.py > gpurun_out/${TAG}_phases.log 2>&1; echo "phases exit $?"
  cat gpurun_out/${TAG}_phases.log | tail -15
fi
