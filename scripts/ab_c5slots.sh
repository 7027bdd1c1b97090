#!/bin/bash
# Same-box A/B on C5 (and C3 / wh10k once): K3 scratch slots 4 GB / 910 (worktree _ab_prev) vs 20 GB
# (working tree), with the default 4,096-entry worker heap and with TSW_ASTAR_WAVE_HCAP=2048 (diag build).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_c5slots.txt
for rep in 1 2; do
  for cfg in "_ab_prev:" ".:" ".:TSW_ASTAR_WAVE_HCAP=2048"; do
    d=${cfg%%:*}; e=${cfg#*:}
    (cd $d && env $e TSW_PLAN_DEBUG=1 timeout -k 10 200 python -u scripts/scale_bench.py c5 --cpu-steps 1 --diag) > gpurun_out/abs.jsonl 2> gpurun_out/abs.log || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abs.jsonl').read().strip().splitlines()[-1]); print('c5 $d $e', d['gpu_end_to_end_s'], d['coop_workers'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_c5slots.txt
    grep "tier-2" gpurun_out/abs.log | tail -1 | sed 's/.*tier-2/  tier-2/' >> gpurun_out/ab_c5slots.txt
  done
done
for d in _ab_prev .; do
  (cd $d && timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 1) > gpurun_out/abs.jsonl 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abs.jsonl').read().strip().splitlines()[-1]); print('wh10k $d', d['gpu_end_to_end_s'], d['coop_workers'], d['prefix_bit_exact'])" >> gpurun_out/ab_c5slots.txt
  (cd $d && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded) > gpurun_out/abs_c3.json 2>/dev/null || exit 1
  python -c "import json; b=json.loads([l for l in open('gpurun_out/abs_c3.json') if l.startswith('{')][-1]); print('c3 $d', b['ms_per_step'])" >> gpurun_out/ab_c5slots.txt
done
cat gpurun_out/ab_c5slots.txt
