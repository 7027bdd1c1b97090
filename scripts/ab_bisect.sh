#!/bin/bash
# Same-box A/B against this round's earlier commits (worktrees _ab_<rev>/, each built in-tree), interleaved:
# wh10k full plans and C3 bench lines.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_bisect.txt
for rep in 1 2; do
  for d in _ab_base _ab_d01bafc .; do
    (cd $d && timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 1) > gpurun_out/abb.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abb.jsonl').read().strip().splitlines()[-1]); print('wh10k $d', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_bisect.txt
    (cd $d && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded) > gpurun_out/abb_c3.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abb_c3.json') if l.startswith('{')][-1]); print('c3 $d', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_bisect.txt
  done
done
cat gpurun_out/ab_bisect.txt
