# wh10k CPU baseline on the GPU box's host: oracle prefix of 100 timesteps (window at 30), GPU full plan
# -> gpurun_out/wh_cpu100.jsonl
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/scale_bench.py wh10k --cpu-steps 100 --cpu-windows 30 > gpurun_out/wh_cpu100.jsonl 2> gpurun_out/wh_cpu100.log
