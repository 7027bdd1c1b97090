# Full 2001-step plan of the 10k-agent warehouse (510x220, 30k tasks) on one GPU; CPU prefix 2 steps.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1080 python -u scripts/scale_bench.py wh10k --cpu-steps 2 > gpurun_out/wh10k_full.jsonl 2> gpurun_out/wh10k_full.log
