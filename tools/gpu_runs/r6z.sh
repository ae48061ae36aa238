set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r6z_pytest_gpu.txt 2>&1; rc=$?
tail -4 gpurun_out/r6z_pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6z_smoke.txt 2>&1 || { tail -5 gpurun_out/r6z_smoke.txt; exit 1; }
tail -1 gpurun_out/r6z_smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r6z_bench_default.json 2> gpurun_out/r6z_bench_default.log || { tail -5 gpurun_out/r6z_bench_default.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6z_bench_default.json'));print('default', d['ms_per_step'], d['value'], d['mixed_bf16']['ms_per_step'], d['inference_p50_ms'])"
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r6z_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r6z_bench_inference.jsonl | cut -c1-200
timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32 > gpurun_out/r6z_pipeline_envs32.json 2> gpurun_out/r6z_pipeline_envs32.log || { tail -20 gpurun_out/r6z_pipeline_envs32.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r6z_pipeline_envs32.json'));print({k: d[k] for k in ('learner_iters_per_s','learner_samples_per_s_fed','learner_train_ms_mean','fresh_samples_per_s')})"
