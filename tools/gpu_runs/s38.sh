set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in 32 64; do
  timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_$E > gpurun_out/s38_pipeline_envs$E.json 2> gpurun_out/s38_pipeline_envs$E.log || { tail -20 gpurun_out/s38_pipeline_envs$E.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s38_pipeline_envs$E.json'));print($E, d['actor_agent_steps_per_s'], d['learner_iters_per_s'], d['learner_train_ms_mean'])"
done
