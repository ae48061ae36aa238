set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_model_parity_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "premask or gradlink or grad_link or linear or composition or parity or fp32" > gpurun_out/r9m_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r9m_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9m_pytest.txt | head; exit 1; }
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --precision fp32 --premask > gpurun_out/r9m_glue_premask.txt 2>&1 || { tail -5 gpurun_out/r9m_glue_premask.txt; exit 1; }
sed -n '/not folded/,$p' gpurun_out/r9m_glue_premask.txt | head -20
for i in 1 2; do
timeout -k 10 300 python -u bench.py --precision fp32 --inference 0 --sl 0 > gpurun_out/r9m_bench_on$i.json 2>/dev/null || exit 1
APPLESTAR_PREMASK_RES=0 timeout -k 10 300 python -u bench.py --precision fp32 --inference 0 --sl 0 > gpurun_out/r9m_bench_off$i.json 2>/dev/null || exit 1
done
python -c "
import json
for f in ('on1','off1','on2','off2'):
    d=json.load(open('gpurun_out/r9m_bench_'+f+'.json')); c=d['config']; print(f, d['ms_per_step'], c['step_ms_min'], c['step_ms_median'])"
