set -o pipefail
mkdir -p gpurun_out
b() {  # name precision env...
  N=$1; P=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision $P --inference 0 $BARGS > gpurun_out/r6g_bench_$N.json 2> gpurun_out/r6g_bench_$N.log || { tail -5 gpurun_out/r6g_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6g_bench_$N.json'));print('$N', d['ms_per_step'], 'host', d['config'].get('host_ms_per_step'))"
}
BARGS="--graph" b bf16_graph_side bf16 APPLESTAR_GRAPH_SIDE_STREAMS=1 || exit 1
BARGS="--graph" b fp32_graph_side fp32 APPLESTAR_GRAPH_SIDE_STREAMS=1 || exit 1
timeout -k 10 300 python tools/host_profile.py --precision bf16 --steps 8 --top 45 > gpurun_out/r6g_host_profile_bf16.txt 2>&1 || { tail -5 gpurun_out/r6g_host_profile_bf16.txt; exit 1; }
head -70 gpurun_out/r6g_host_profile_bf16.txt | tail -60
timeout -k 10 300 python tools/actor_step_profile.py --steps 300 > gpurun_out/r6g_actor_step_profile.json 2>/dev/null || exit 1
tail -1 gpurun_out/r6g_actor_step_profile.json
timeout -k 10 400 python bench.py > gpurun_out/r6g_bench_default.json 2> gpurun_out/r6g_bench_default.log || { tail -5 gpurun_out/r6g_bench_default.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6g_bench_default.json'));print('default', d['ms_per_step'], d['mixed_bf16']['ms_per_step'], d['inference_p50_ms'])"
