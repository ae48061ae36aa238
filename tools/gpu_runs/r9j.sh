set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in 2 3; do
APPLESTAR_WGRAD_STG=$M timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv3x3_f32_matches_fp64 or linear_f32_grads or wgrad or linear_f32_relu" > gpurun_out/r9j_pytest_$M.txt 2>&1; rc=$?
echo "mode $M"; tail -1 gpurun_out/r9j_pytest_$M.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9j_pytest_$M.txt | head; exit 1; }
done
for M in 1 2 3; do
APPLESTAR_WGRAD_STG=$M timeout -k 10 300 python -u tools/bench_f32_kernels.py wgrad > gpurun_out/r9j_wgrad_$M.jsonl 2>&1 || exit 1
done
paste -d'\n' <(grep kernel gpurun_out/r9j_wgrad_1.jsonl) <(grep kernel gpurun_out/r9j_wgrad_2.jsonl) <(grep kernel gpurun_out/r9j_wgrad_3.jsonl) | cut -c1-160
