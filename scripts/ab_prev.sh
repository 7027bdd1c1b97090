#!/bin/bash
# Same-box A/B: working tree (.) vs the last commit (worktree _ab_prev/, built in-tree), interleaved:
# a GPU parity subset of the working tree, C3 bench lines, wh10k / C5 full plans.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_prev.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "astar or get_path or mapd or wh10k or c5 or serpentine" > gpurun_out/ab_prev_tests.log 2>&1 || { tail -5 gpurun_out/ab_prev_tests.log; exit 1; }
tail -1 gpurun_out/ab_prev_tests.log >> gpurun_out/ab_prev.txt
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
cat gpurun_out/ab_prev.txt
