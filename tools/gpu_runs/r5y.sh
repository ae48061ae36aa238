set -o pipefail
mkdir -p gpurun_out
run() {  # name, extra env...
  N=$1; shift
  env "$@" timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 30 --precision fp32 --workdir /tmp/pipe_$N $PIPE_ARGS > gpurun_out/r5y_pipeline_$N.json 2> gpurun_out/r5y_pipeline_$N.log || { tail -20 gpurun_out/r5y_pipeline_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5y_pipeline_$N.json'));print('$N', {k: d[k] for k in ('learner_iters_per_s','learner_train_ms_mean','learner_train_main_thread_cpu_ms_mean','fresh_samples_per_s')})"
}
PIPE_ARGS="--max-reuse 1000000000" run discard APPLESTAR_RING_DIAG=discard || exit 1
PIPE_ARGS="" run unpinned APPLESTAR_RING_DIAG=unpinned || exit 1
