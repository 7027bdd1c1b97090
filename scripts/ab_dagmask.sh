#!/bin/bash
# A/B (diagnostic build): DAG early-exit test period (TSW_DAG_MASK + 1 pops) on C3, interleaved.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_dagmask.txt
for rep in 1 2; do
  for m in 15 7 3 31; do
    TSW_DAG_MASK=$m timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abd.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abd.json') if l.startswith('{')][-1]); print('c3 mask=$m', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_dagmask.txt
  done
done
cat gpurun_out/ab_dagmask.txt
