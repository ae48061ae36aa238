set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/s41_pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/s41_pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s41_smoke.txt 2>&1 || { tail -5 gpurun_out/s41_smoke.txt; exit 1; }
tail -1 gpurun_out/s41_smoke.txt
timeout -k 10 500 python -u bench.py > gpurun_out/s41_bench_default.log 2>&1 || { tail -5 gpurun_out/s41_bench_default.log; exit 1; }
grep '"metric"' gpurun_out/s41_bench_default.log | cut -c1-400
grep -i "bf16\|inference\|B=1\|sl " gpurun_out/s41_bench_default.log | cut -c1-200 | tail -12
