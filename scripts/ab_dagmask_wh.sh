#!/bin/bash
# A/B (diagnostic build): DAG early-exit test period on wh10k (global g-score workers, default 63).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_dagmask_wh.txt
for m in 63 31 127 15; do
  TSW_DAG_MASK=$m timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 1 --diag > gpurun_out/abdw.jsonl 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abdw.jsonl').read().strip().splitlines()[-1]); print('wh10k mask=$m', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_dagmask_wh.txt
done
cat gpurun_out/ab_dagmask_wh.txt
