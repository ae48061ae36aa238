set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_glue_fusions_gpu.py -x -q --timeout 200 --timeout-method thread -k "gated or gate" > gpurun_out/r8o_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8o_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8o_pytest.txt | head; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8o_bench_on$i.json 2> gpurun_out/r8o_bench_on$i.log || exit 1
APPLESTAR_GATE_PSB=0 timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8o_bench_off$i.json 2> gpurun_out/r8o_bench_off$i.log || exit 1
done
python -c "
import json
for f in ('on1','off1','on2','off2'):
    d=json.load(open('gpurun_out/r8o_bench_'+f+'.json')); c=d['config']; print(f, d['ms_per_step'], c['step_ms_min'], c['step_ms_median'])
"
