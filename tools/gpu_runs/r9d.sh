set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_glue_fusions_gpu.py::test_deferred_head_wgrads_equal_inline" "tests/test_model_parity_gpu.py::test_fp32_benchmark_composition_matches_cpu" -v --timeout 200 --timeout-method thread > gpurun_out/r9d_a.txt 2>&1; echo "isolated rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r9d_a.txt | head -8 | cut -c1-200
timeout -k 10 600 python -u -m pytest tests/test_phased_backward_gpu.py tests/test_model_parity_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r9d_b.txt 2>&1; echo "ordered rc=$?"; grep -E "FAILED|^E " gpurun_out/r9d_b.txt | head -8 | cut -c1-200; tail -1 gpurun_out/r9d_b.txt
