set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "varlen_attention" > gpurun_out/attn_pytest.txt 2>&1 || { tail -30 gpurun_out/attn_pytest.txt; exit 1; }
tail -2 gpurun_out/attn_pytest.txt
timeout -k 10 200 python -u tools/bench_f32_kernels.py attn > gpurun_out/attn_micro2.jsonl 2>&1 || { tail -20 gpurun_out/attn_micro2.jsonl; exit 1; }
cat gpurun_out/attn_micro2.jsonl
