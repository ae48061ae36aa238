set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bo_encoder" > gpurun_out/r9b_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r9b_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9b_pytest.txt | head; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r9b_p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --precision fp32 --inference 0 --sl 0 > $GRAFT_REPO_ROOT/gpurun_out/r9b_prof.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 gpurun_out/r9b_prof.log; exit 1; }
f=$(find /tmp/r9b_p -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r9b_kernel_stats.csv; grep -E "bo_fwd|bo_bwd" gpurun_out/r9b_kernel_stats.csv | cut -c1-250
for i in 1 2; do timeout -k 10 300 python -u bench.py --precision fp32 --inference 0 --sl 0 > gpurun_out/r9b_bench_$i.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/r9b_bench_$i.json')); print(d['ms_per_step'], d['config']['step_ms_min'])"; done
