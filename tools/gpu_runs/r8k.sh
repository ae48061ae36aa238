set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_phased_backward_gpu.py -x -q --timeout 200 --timeout-method thread -k "deferred or phased" > gpurun_out/r8k_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8k_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8k_pytest.txt | head; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8k_bench_rewalk$i.json 2> gpurun_out/r8k_bench_rewalk$i.log || exit 1
APPLESTAR_DEFER_CHECK=1 timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8k_bench_walk$i.json 2> gpurun_out/r8k_bench_walk$i.log || exit 1
done
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 --graph > gpurun_out/r8k_bench_graph.json 2> gpurun_out/r8k_bench_graph.log || { tail -3 gpurun_out/r8k_bench_graph.log; exit 1; }
python -c "
import json
for f in ('rewalk1','walk1','rewalk2','walk2','graph'):
    d=json.load(open('gpurun_out/r8k_bench_'+f+'.json')); c=d['config']; print(f, d['ms_per_step'], c['host_ms_per_step'], c['step_ms_min'], c['step_ms_median'])
"
