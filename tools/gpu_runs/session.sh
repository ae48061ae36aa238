set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_gemm_k128.py > gpurun_out/probe_k128_staged.jsonl 2>&1 || { tail -20 gpurun_out/probe_k128_staged.jsonl; exit 1; }
APPLESTAR_GEMM_F32_STAGED=0 timeout -k 10 200 python -u tools/probe_gemm_k128.py > gpurun_out/probe_k128_direct.jsonl 2>&1 || { tail -20 gpurun_out/probe_k128_direct.jsonl; exit 1; }
grep M gpurun_out/probe_k128_staged.jsonl gpurun_out/probe_k128_direct.jsonl
