set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py -x -q --timeout 120 --timeout-method thread -k "psb or v2_variants or epi2 or skip_link" > gpurun_out/r8f_pytest_conv.txt 2>&1; rc=$?
tail -2 gpurun_out/r8f_pytest_conv.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8f_pytest_conv.txt | head; exit 1; }
APPLESTAR_CONV_V2=-1 timeout -k 10 200 python -u tools/bench_conv_psb.py 30 psb > gpurun_out/r8f_conv.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_conv_psb.py 30 psb v4 v2 v4 >> gpurun_out/r8f_conv.jsonl 2>&1 || exit 1
grep shape gpurun_out/r8f_conv.jsonl
timeout -k 10 400 python -u -m pytest tests/test_phased_backward_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r8f_pytest_phased.txt 2>&1; rc=$?
tail -2 gpurun_out/r8f_pytest_phased.txt; [ $rc -eq 0 ] || grep -E "^E " gpurun_out/r8f_pytest_phased.txt | head -5
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8f_bench_v2.json 2> gpurun_out/r8f_bench_v2.log || exit 1
APPLESTAR_CONV_V2=-1 timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8f_bench_psb.json 2> gpurun_out/r8f_bench_psb.log || exit 1
python -c "import json;[print(f, json.load(open('gpurun_out/'+f))['ms_per_step']) for f in ('r8f_bench_v2.json','r8f_bench_psb.json')]"
