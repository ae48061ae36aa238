set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for WG in 3072 1024 2048 6144 3072; do
APPLESTAR_WGRAD_F32_WG=$WG timeout -k 10 300 python -u bench.py --precision fp32 --inference 0 --sl 0 > gpurun_out/r9q_bench_wg$WG.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r9q_bench_wg$WG.json')); print('wg $WG', d['ms_per_step'], d['config']['step_ms_min'], d['config']['step_ms_median'])"
done
