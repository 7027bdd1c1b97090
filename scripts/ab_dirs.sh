#!/bin/bash
# Same-box A/B of whole trees (each built in-tree): C3 bench lines and full-horizon wh10k / C5 plans,
# interleaved per repetition. Usage (from the repo root, through gpurun):
#   bash scripts/ab_dirs.sh OUT REPS INSTANCES DIR...     e.g.  bash scripts/ab_dirs.sh ab.txt 2 "wh10k c5" _ab_base .
# -> gpurun_out/OUT, one line per run: <instance> <dir> <seconds> <K3 wait ms> <bit-exact prefix>
set -o pipefail
out=gpurun_out/$1; reps=$2; inst=$3; shift 3
mkdir -p gpurun_out
: > "$out"
for rep in $(seq 1 "$reps"); do
  for d in "$@"; do
    (cd "$d" && timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded) \
      > gpurun_out/abd_c3.json 2>gpurun_out/abd_c3.err || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abd_c3.json') if l.startswith('{')][-1]); print('c3 $d', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1), [round(x/3,1) for x in b['kernel_stats']['plan_section_ms']])" >> "$out"
    for i in $inst; do
      (cd "$d" && timeout -k 10 200 python -u scripts/scale_bench.py "$i" --cpu-steps 1) > gpurun_out/abd.jsonl 2>/dev/null || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/abd.jsonl').read().strip().splitlines()[-1]); print('$i $d', d['gpu_end_to_end_s'], d.get('coop_wait_ms'), d['prefix_bit_exact'])" >> "$out"
    done
  done
done
cat "$out"
