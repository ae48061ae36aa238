set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bf16_gpu_vs_cpu or upstream_amplification" -s > gpurun_out/r5f_parity.txt 2>&1 || { tail -40 gpurun_out/r5f_parity.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r5f_parity.txt | tail -2
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --timed --top 45 > gpurun_out/r5f_glue_timed.txt 2>&1 || { tail -30 gpurun_out/r5f_glue_timed.txt; exit 1; }
grep -A 60 "event-timed" gpurun_out/r5f_glue_timed.txt | cut -c1-200
