set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in fp32 bf16; do
timeout -k 20 540 python -u tools/learn_pipeline.py --envs 24 --seconds 360 --precision $P --lr 1e-4 --report 30 --workdir /tmp/learn_$P --out gpurun_out/r8b_learn_$P.json > gpurun_out/r8b_learn_$P.log 2>&1 || { grep -v "HTTP/1.1" gpurun_out/r8b_learn_$P.log | tail -20; exit 1; }
grep '"progress"' gpurun_out/r8b_learn_$P.log | tail -14
python -c "import json;d=json.load(open('gpurun_out/r8b_learn_$P.json'));print('$P', d['first_bin'], d['last_bin'], d['learner_iterations'])"
done
