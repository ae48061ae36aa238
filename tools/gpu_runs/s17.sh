set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_glue_fusions_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or ln or affine or embed or spatial or bo_ or reduce or linear_f32" > gpurun_out/s17_pytest.txt 2>&1 || { tail -40 gpurun_out/s17_pytest.txt; exit 1; }
tail -1 gpurun_out/s17_pytest.txt
timeout -k 10 300 python -u tools/diag/poison_probe.py --precision fp32 --backward > gpurun_out/s17_poison_bwd_fp32.txt 2>&1 || { tail -20 gpurun_out/s17_poison_bwd_fp32.txt; exit 1; }
grep "^\[" gpurun_out/s17_poison_bwd_fp32.txt; grep -c "grad\." gpurun_out/s17_poison_bwd_fp32.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s17_fp32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/s17_fp32_$i.json'));print('fp32', $i, d['ms_per_step'])"
done
