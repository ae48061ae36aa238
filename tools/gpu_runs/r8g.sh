set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_f32_psb" > gpurun_out/r8g_pytest_gemm.txt 2>&1; rc=$?
tail -2 gpurun_out/r8g_pytest_gemm.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8g_pytest_gemm.txt | head; exit 1; }
timeout -k 10 300 python -u tools/bench_gemm_psb.py 30 > gpurun_out/r8g_gemm_v2.jsonl 2>&1 || { tail gpurun_out/r8g_gemm_v2.jsonl; exit 1; }
cat gpurun_out/r8g_gemm_v2.jsonl | grep -v amdgpu.ids
for V in 12 10; do
APPLESTAR_GEMM_PSB_VARIANT=$V timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8g_bench_gemm$V.json 2> gpurun_out/r8g_bench_gemm$V.log || exit 1
done
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8g_bench_base.json 2> gpurun_out/r8g_bench_base.log || exit 1
python -c "import json;[print(f, json.load(open('gpurun_out/'+f))['ms_per_step']) for f in ('r8g_bench_gemm12.json','r8g_bench_gemm10.json','r8g_bench_base.json')]"
