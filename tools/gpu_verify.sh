#!/bin/bash
# Round-end shaped verification on the GPU box (each GPU step under its own time limit, chained so the first
# failure ends the call):
#   bench (BENCH_ARGS, default the driver's N=1 call) -> smoke() -> pytest -m gpu (TESTS = test paths / -k
#   expression, default the whole suite) -> optional rocprofv3 kernel trace of the fp32 step (PROF=1).
# NOBENCH=1 / NOSMOKE=1 / NOTESTS=1 skip a step.  Outputs under gpurun_out/${TAG:-v}_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
T=${TAG:-v}
if [ -z "$NOBENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -20 gpurun_out/${T}_bench.err; exit 1; }
  cat gpurun_out/${T}_bench.json
fi
if [ -z "$NOSMOKE" ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -1 gpurun_out/${T}_smoke.log
fi
if [ -z "$NOTESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_pytest.txt 2>&1; rc=$?
  tail -3 gpurun_out/${T}_pytest.txt
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${T}_pytest.txt | head -20; exit $rc; }
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run --output-format csv -- \
    python3 bench.py ${PROF_ARGS:---precision fp32 --steps 4 --warmup 2} > gpurun_out/${T}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${T}_prof.log; exit 1; }
  python3 tools/prof_steady.py $(find gpurun_out/${T}_prof -name '*kernel_trace.csv' | head -1) 3 70 > gpurun_out/${T}_steady.txt
  head -14 gpurun_out/${T}_steady.txt
fi
exit 0
