#!/bin/bash
# Round-end shaped verification: bench first on the fresh box, then smoke, then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
[ -n "$NOBENCH" ] || timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err || { echo bench failed; tail -20 gpurun_out/v_bench.err; exit 1; }
[ -n "$NOBENCH" ] || cat gpurun_out/v_bench.json
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/v_smoke.log; exit 1; }
tail -1 gpurun_out/v_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/v_pytest.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "$WGRAD32_AB" ]; then
  APPLESTAR_WGRAD32_PIPE=0 timeout -k 10 120 python -u tools/bench_wgrad32.py > gpurun_out/v_wgrad32_ab.jsonl 2>/dev/null &&
  APPLESTAR_WGRAD32_BK=256 timeout -k 10 120 python -u tools/bench_wgrad32.py >> gpurun_out/v_wgrad32_ab.jsonl 2>/dev/null; rc=$?
  cat gpurun_out/v_wgrad32_ab.jsonl
fi
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/v_prof -o run --output-format csv -- python3 bench.py --precision fp32 --steps 4 --warmup 2 > gpurun_out/v_prof.log 2>&1 || { echo prof failed; tail gpurun_out/v_prof.log; exit 1; }
  python3 tools/prof_steady.py $(find gpurun_out/v_prof -name '*kernel_trace.csv' | head -1) 3 70 > gpurun_out/v_fp32_steady.txt; rc=$?
  head -12 gpurun_out/v_fp32_steady.txt
fi
exit $rc
