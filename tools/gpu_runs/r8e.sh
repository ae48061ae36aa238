set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r8e_pmc_conv_a FILTER=conv3x3 COUNTERS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh python3 tools/bench_conv_psb.py 3 psb v2 || exit 1
TAG=r8e_pmc_conv_b FILTER=conv3x3 COUNTERS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh python3 tools/bench_conv_psb.py 3 psb v2 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_phased_backward_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r8e_pytest_phased.txt 2>&1; rc=$?
tail -4 gpurun_out/r8e_pytest_phased.txt; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r8e_pytest_phased.txt | head -5; exit 1; }
APPLESTAR_RUN_SLOW=1 timeout -k 20 500 python -u -m pytest tests/test_learning_pipeline_gpu.py -v -s --timeout 420 --timeout-method thread -k bf16 > gpurun_out/r8e_pytest_learn_bf16.txt 2>&1; rc=$?
grep -E '"progress"|PASSED|FAILED|passed|failed' gpurun_out/r8e_pytest_learn_bf16.txt | tail -8; exit $rc
