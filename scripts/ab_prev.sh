#!/bin/bash
# Same-box A/B: working tree (.) vs the last commit (worktree _ab_prev/, built in-tree), interleaved:
# C3 bench lines, wh10k / C5 full plans, and the C3 plan-debug queue-delay line of each side.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_prev.txt
for rep in 1 2; do
  for d in _ab_prev .; do
    (cd $d && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded) > gpurun_out/abp_c3.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abp_c3.json') if l.startswith('{')][-1]); print('c3 $d', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_prev.txt
  done
done
for inst in wh10k c5; do
  for d in _ab_prev .; do
    (cd $d && timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1) > gpurun_out/abp.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abp.jsonl').read().strip().splitlines()[-1]); print('$inst $d', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_prev.txt
  done
done
for d in _ab_prev .; do
  (cd $d && TSW_PLAN_DEBUG=1 timeout -k 10 100 python -u scripts/scale_bench.py c3 --cpu-steps 1 --diag) > /dev/null 2> gpurun_out/abp_dbg.log || exit 1
  echo "$d $(grep 'queue delay' gpurun_out/abp_dbg.log | tail -1)" >> gpurun_out/ab_prev.txt
done
cat gpurun_out/ab_prev.txt
