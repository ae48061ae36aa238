set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/s30_pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/s30_pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s30_smoke.txt 2>&1 || { tail -5 gpurun_out/s30_smoke.txt; exit 1; }
tail -1 gpurun_out/s30_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/s30_bench_default.log 2>&1 || { tail -5 gpurun_out/s30_bench_default.log; exit 1; }
grep '"metric"' gpurun_out/s30_bench_default.log | cut -c1-300
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p30 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --precision fp32 --inference 0 > $R/gpurun_out/s30_prof.log 2>&1 || { tail -20 $R/gpurun_out/s30_prof.log; exit 1; }
cd $R
t=$(find /tmp/p30 -name '*kernel_trace.csv' | head -1)
python3 tools/prof_steady.py "$t" 3 70 > gpurun_out/s30_steady_fp32.txt
head -10 gpurun_out/s30_steady_fp32.txt
