set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for WG in 1024 2048 3072 512 1024; do
APPLESTAR_WGRAD_WG=$WG timeout -k 10 300 python -u bench.py --precision bf16 --inference 0 --sl 0 > gpurun_out/r9n_bench_bf16_wg$WG.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r9n_bench_bf16_wg$WG.json')); print('wg $WG', d['ms_per_step'], d['config']['step_ms_min'])"
done
