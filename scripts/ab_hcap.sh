#!/bin/bash
# A/B (diagnostic build): worker LDS heap entries (TSW_ASTAR_WAVE_HCAP) — more worker waves per CU —
# on wh10k and C5, with the tier hand-off counts from the plan-debug line.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_hcap.txt
for cfg in wh10k:0 wh10k:2048 wh10k:1024 c5:0 c5:1024; do
  inst=${cfg%%:*}; h=${cfg#*:}; e=""; [ $h != 0 ] && e="TSW_ASTAR_WAVE_HCAP=$h"
  env $e TSW_PLAN_DEBUG=1 timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1 --diag > gpurun_out/abh.jsonl 2> gpurun_out/abh.log || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abh.jsonl').read().strip().splitlines()[-1]); print('$inst hcap=$h', d['gpu_end_to_end_s'], d['coop_workers'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_hcap.txt
  grep "tier-2" gpurun_out/abh.log | tail -1 | sed 's/.*tier-2/  tier-2/' >> gpurun_out/ab_hcap.txt
done
cat gpurun_out/ab_hcap.txt
