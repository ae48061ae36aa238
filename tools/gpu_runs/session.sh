set -o pipefail
mkdir -p gpurun_out
TAG=ent_pmc1 FILTER=entity_embed_fwd bash tools/gpu_pmc.sh python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --precision fp32 --inference 0 || exit 1
TAG=ent_pmc2 FILTER=entity_embed_fwd COUNTERS="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS" bash tools/gpu_pmc.sh python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --precision fp32 --inference 0 || exit 1
