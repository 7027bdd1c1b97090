#!/bin/bash
# Same-box A/B of this round's net effect: the product build at HEAD vs the round's starting commit
# (a worktree under _ab_base/, built in-tree there), interleaved, C3 bench line + wh10k / C5 full plans.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_round.txt
for rep in 1 2; do
  for side in head base; do
    d=.; [ $side = base ] && d=_ab_base
    (cd $d && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded) > gpurun_out/abr_c3_$side.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abr_c3_$side.json') if l.startswith('{')][-1]); print('c3 $side', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_round.txt
  done
done
for inst in wh10k c5; do
  for side in head base; do
    d=.; [ $side = base ] && d=_ab_base
    (cd $d && timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1) > gpurun_out/abr_${inst}_$side.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abr_${inst}_$side.jsonl').read().strip().splitlines()[-1]); print('$inst $side', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_round.txt
  done
done
cat gpurun_out/ab_round.txt
