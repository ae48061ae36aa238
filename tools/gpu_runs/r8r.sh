set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "su_sample" > gpurun_out/r8r_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8r_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8r_pytest.txt | head; exit 1; }
timeout -k 10 200 python -u tools/bench_su_sample.py > gpurun_out/r8r_su.jsonl 2>&1 || { tail -5 gpurun_out/r8r_su.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/r8r_su.jsonl
