set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s20_wg32_default.jsonl 2>/dev/null || exit 1
APPLESTAR_WGRAD32_PIPE=1 timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s20_wg32_pipe.jsonl 2>/dev/null || exit 1
APPLESTAR_WGRAD32_BK=256 timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s20_wg32_bk256.jsonl 2>/dev/null || exit 1
APPLESTAR_WGRAD_STG_NARROW=1 timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s20_wg32_stg.jsonl 2>/dev/null || exit 1
paste -d' ' <(python -c "import json;[print(d['shape'],d['us']) for d in map(json.loads,open('gpurun_out/s20_wg32_default.jsonl'))]") <(python -c "import json;[print(d['us']) for d in map(json.loads,open('gpurun_out/s20_wg32_pipe.jsonl'))]") <(python -c "import json;[print(d['us']) for d in map(json.loads,open('gpurun_out/s20_wg32_bk256.jsonl'))]") <(python -c "import json;[print(d['us']) for d in map(json.loads,open('gpurun_out/s20_wg32_stg.jsonl'))]")
