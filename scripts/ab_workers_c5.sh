#!/bin/bash
# C5 worker capacity A/B (diagnostic build): default (bitmap staged in LDS, 1 wave per CU) vs
# TSW_WORKER_FB=0 (no staged bitmap: heap-only LDS, several waves per CU, g-scores in global slots),
# each with TSW_WORKER_HCAP heap sizes.
set -o pipefail
mkdir -p gpurun_out
for cfg in "def:" "nofb:TSW_WORKER_FB=0" "nofb2k:TSW_WORKER_FB=0 TSW_ASTAR_WAVE_HCAP=2048"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  env $envs TSW_PLAN_DEBUG=1 timeout -k 10 150 python -u scripts/scale_bench.py c5 --cpu-steps 1 --diag \
    > gpurun_out/c5w_$tag.jsonl 2> gpurun_out/c5w_$tag.log || exit 1
done
