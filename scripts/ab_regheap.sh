#!/bin/bash
# A/B: register-resident A* heap (TSW_ASTAR_REGHEAP=63, default) vs the LDS array only (=0), interleaved.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_reg.txt
for rep in 1 2; do
  for r in 63 0; do
    TSW_ASTAR_REGHEAP=$r timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/ab_reg_c3_$r.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/ab_reg_c3_$r.json') if l.startswith('{')][-1]); k=b['kernel_stats']; print('c3 reg=$r', b['ms_per_step'], round(k['coop_wait_ms']/3,1))" >> gpurun_out/ab_reg.txt
    TSW_ASTAR_REGHEAP=$r timeout -k 10 150 python -u scripts/scale_bench.py wh10k --cpu-steps 1 > gpurun_out/ab_reg_wh_$r.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab_reg_wh_$r.jsonl').read().strip().splitlines()[-1]); print('wh10k reg=$r', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_reg.txt
  done
done
cat gpurun_out/ab_reg.txt
TSW_PLAN_DEBUG=1 timeout -k 10 100 python -u scripts/scale_bench.py c3 --cpu-steps 1 > gpurun_out/c3_dbg.jsonl 2> gpurun_out/c3_dbg.log
