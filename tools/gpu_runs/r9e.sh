set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_model_parity_gpu.py::test_fp32_benchmark_composition_matches_cpu" "tests/test_glue_fusions_gpu.py::test_deferred_head_wgrads_equal_inline" -v --timeout 200 --timeout-method thread > gpurun_out/r9e.txt 2>&1; rc=$?; grep -E "PASSED|FAILED|^E " gpurun_out/r9e.txt | head -8 | cut -c1-250; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision fp32 > gpurun_out/r9c_timeline_fp32.txt 2>&1 || { tail -20 gpurun_out/r9c_timeline_fp32.txt; exit 1; }
grep -v amdgpu gpurun_out/r9c_timeline_fp32.txt
