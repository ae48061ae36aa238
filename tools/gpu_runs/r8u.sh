set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv3x3 or su_sample" > gpurun_out/r8u_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8u_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8u_pytest.txt | head; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --precision fp32 --sl 0 > gpurun_out/r8u_bench.json 2> gpurun_out/r8u_bench.log || { tail -5 gpurun_out/r8u_bench.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r8u_bench.json')); print(d.get('inference_p50_ms'))"
APPLESTAR_CONV_SPLITK=0 APPLESTAR_SU_WIDE=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --precision fp32 --sl 0 > gpurun_out/r8u_bench_off.json 2> gpurun_out/r8u_bench_off.log || { tail -5 gpurun_out/r8u_bench_off.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r8u_bench_off.json')); print(d.get('inference_p50_ms'))"
