set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --precision fp32 --premask > gpurun_out/r9l_glue_premask.txt 2>&1 || { tail -5 gpurun_out/r9l_glue_premask.txt; exit 1; }
sed -n '/not folded/,$p' gpurun_out/r9l_glue_premask.txt | head -40
