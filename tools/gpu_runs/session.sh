set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/glue_sites.py --steps 1 --precision bf16 --shapes > gpurun_out/glue_sites_bf16.txt 2> gpurun_out/glue_sites_bf16.err || { tail -20 gpurun_out/glue_sites_bf16.err; exit 1; }
