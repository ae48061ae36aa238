set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd $R && mkdir -p gpurun_out
TAG=r7c_pmc_inf_b1_a FILTER= bash tools/gpu_pmc.sh python3 tools/bench_inference.py --batches 1 --iters 3 --modes policy > /dev/null && \
cd $R && TAG=r7c_pmc_inf_b1_b FILTER= COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh python3 tools/bench_inference.py --batches 1 --iters 3 --modes policy > /dev/null && \
cd $R && grep -h -E "su_sample|conv3x3|bo_fwd|head_sample_kernel<float|gate_chain" gpurun_out/r7c_pmc_inf_b1_a_summary.txt gpurun_out/r7c_pmc_inf_b1_b_summary.txt | cut -c1-400
