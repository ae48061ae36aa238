set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r6f_pytest_gpu.txt 2>&1; rc=$?
tail -4 gpurun_out/r6f_pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6f_smoke.txt 2>&1 || { tail -5 gpurun_out/r6f_smoke.txt; exit 1; }
tail -1 gpurun_out/r6f_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r6f_bench_default.json 2> gpurun_out/r6f_bench_default.log || { tail -5 gpurun_out/r6f_bench_default.log; exit 1; }
cat gpurun_out/r6f_bench_default.json
