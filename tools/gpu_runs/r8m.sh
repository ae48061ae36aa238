set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "v2_variants or conv3x3_f32 or psb" > gpurun_out/r8m_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8m_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8m_pytest.txt | head; exit 1; }
timeout -k 10 300 python -u tools/bench_f32_kernels.py conv > gpurun_out/r8m_conv.jsonl 2>&1 || exit 1
APPLESTAR_CONV_V2=-1 timeout -k 10 300 python -u tools/bench_f32_kernels.py conv > gpurun_out/r8m_conv_psb.jsonl 2>&1 || exit 1
paste -d'\n' <(grep kernel gpurun_out/r8m_conv_psb.jsonl) <(grep kernel gpurun_out/r8m_conv.jsonl)
for i in 1 2; do
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8m_bench_v2$i.json 2> gpurun_out/r8m_bench_v2$i.log || exit 1
APPLESTAR_CONV_V2=-1 timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8m_bench_psb$i.json 2> gpurun_out/r8m_bench_psb$i.log || exit 1
done
python -c "
import json
for f in ('v21','psb1','v22','psb2'):
    d=json.load(open('gpurun_out/r8m_bench_'+f+'.json')); c=d['config']; print(f, d['ms_per_step'], c['step_ms_min'], c['step_ms_median'])
"
