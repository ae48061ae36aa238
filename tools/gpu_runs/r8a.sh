set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_flat_model.py tests/test_model_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r8a_pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/r8a_pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --inference 0 > gpurun_out/r8a_bench.json 2> gpurun_out/r8a_bench.log || { tail -5 gpurun_out/r8a_bench.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r8a_bench.json'));print('fp32', d['ms_per_step'], 'bf16', d['mixed_bf16']['ms_per_step'], 'sl', d['sl_fp32']['ms_per_step'])"
grep -i "warn" gpurun_out/r8a_bench.log | head -5 || true
