set -o pipefail
mkdir -p gpurun_out
APPLESTAR_LSTM_KS=16 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lstm or trainer" > gpurun_out/s28_pytest.txt 2>&1 || { tail -40 gpurun_out/s28_pytest.txt; exit 1; }
tail -1 gpurun_out/s28_pytest.txt
for i in 1 2; do
  for v in 16 8; do
    APPLESTAR_LSTM_KS=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s28_fp32_ks${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s28_fp32_ks${v}_$i.json'));print('fp32 lstm_ks=$v', $i, d['ms_per_step'])"
    APPLESTAR_LSTM_KS=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s28_bf16_ks${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s28_bf16_ks${v}_$i.json'));print('bf16 lstm_ks=$v', $i, d['ms_per_step'])"
  done
done
