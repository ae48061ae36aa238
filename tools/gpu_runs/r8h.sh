set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
APPLESTAR_WGRAD_WIDE=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/r8h_pytest_wgrad.txt 2>&1; rc=$?
tail -2 gpurun_out/r8h_pytest_wgrad.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8h_pytest_wgrad.txt | head; exit 1; }
timeout -k 10 300 python -u tools/bench_f32_kernels.py wgrad > gpurun_out/r8h_wgrad_base.jsonl 2>&1 || exit 1
APPLESTAR_WGRAD_WIDE=1 timeout -k 10 300 python -u tools/bench_f32_kernels.py wgrad > gpurun_out/r8h_wgrad_wide.jsonl 2>&1 || exit 1
paste -d'\n' <(grep kernel gpurun_out/r8h_wgrad_base.jsonl) <(grep kernel gpurun_out/r8h_wgrad_wide.jsonl)
TAG=r8h_pmc_wgrad FILTER=wgrad_f32_pipe COUNTERS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh python3 tools/bench_f32_kernels.py wgrad || exit 1
APPLESTAR_WGRAD_WIDE=1 timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8h_bench_wide.json 2> gpurun_out/r8h_bench_wide.log || exit 1
timeout -k 10 300 python -u bench.py --inference 0 --sl 0 --precision fp32 > gpurun_out/r8h_bench_base.json 2> gpurun_out/r8h_bench_base.log || exit 1
python -c "import json;[print(f, json.load(open('gpurun_out/'+f))['ms_per_step']) for f in ('r8h_bench_wide.json','r8h_bench_base.json')]"
