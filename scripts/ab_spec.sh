#!/bin/bash
# A/B (diagnostic build): speculation depth with every worker on chains — walk-ahead hops
# (TSW_WIDE_PREFETCH, default 8) and DAG levels past the first unresolved cell (TSW_DAG_PREFETCH, 6),
# on wh10k, C5 and C3.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_spec.txt
CFGS="def: w16:TSW_WIDE_PREFETCH=16 w4:TSW_WIDE_PREFETCH=4 d9:TSW_DAG_PREFETCH=9 d3:TSW_DAG_PREFETCH=3"
for inst in wh10k c5; do
  for cfg in $CFGS; do
    tag=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1 --diag > gpurun_out/abs2.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abs2.jsonl').read().strip().splitlines()[-1]); print('$inst $tag', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_spec.txt
  done
done
for cfg in $CFGS; do
  tag=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abs2.json 2>/dev/null || exit 1
  python -c "import json; b=json.loads([l for l in open('gpurun_out/abs2.json') if l.startswith('{')][-1]); print('c3 $tag', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_spec.txt
done
cat gpurun_out/ab_spec.txt
