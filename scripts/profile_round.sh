#!/bin/bash
# Profiles the default bench on one MI355X (run through gpurun from the repo root).
#   1. bench.py, the driver's default command                      -> $OUT/bench.json
#   2. per workload (plan = the C3 planning leg, plan_exit = the same plan in exit mode — the planner's
#      k_plan dispatches alone, K3 as host-launched passes, for the planner / worker traffic split —
#      bfs = K1 on den520d, 10k goals), each its own
#      process so no kernel's launches mix workloads:
#        rocprofv3 --kernel-trace --stats                           -> $OUT/<wl>_trace/
#        separate PMC passes FETCH_SIZE and WRITE_SIZE              -> $OUT/<wl>_pmc_fetch, _pmc_write
# Then: python scripts/summarize_profile.py $OUT profiles/<tag>
# Each GPU step has its own time limit; steps are chained with && so a failure stops the run.
set -o pipefail
TAG=${1:-r5}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PLAN="--steps 1 --warmup 0 --no-cpu --no-bfs"
PLANX="--steps 1 --warmup 0 --no-cpu --no-bfs --exit-mode"
BFS="--no-plan --no-cpu --bfs-reps 2"
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err &&
for WL in plan plan_exit bfs; do
  if [ $WL = plan ]; then A=$PLAN; elif [ $WL = plan_exit ]; then A=$PLANX; else A=$BFS; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${WL}_trace -o run -- python3 bench.py $A > $OUT/${WL}_trace.json 2> $OUT/${WL}_trace.err &&
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${WL}_pmc_fetch -o run -- python3 bench.py $A > $OUT/${WL}_pmc_fetch.json 2> $OUT/${WL}_pmc_fetch.err &&
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${WL}_pmc_write -o run -- python3 bench.py $A > $OUT/${WL}_pmc_write.json 2> $OUT/${WL}_pmc_write.err || exit 1
done
# planner / worker traffic split of the coop dispatch (scripts/warm_split.py): cold vs warm plan
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/warm_pmc_fetch -o run -- python3 scripts/warm_plan.py --reps 1 > $OUT/warm_pmc_fetch.json 2> $OUT/warm_pmc_fetch.err &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/warm_pmc_write -o run -- python3 scripts/warm_plan.py --reps 1 > $OUT/warm_pmc_write.json 2> $OUT/warm_pmc_write.err &&
# ... and without task chains (diagnostic library, TSW_TASK_CHAINS=0): the warm plan's bytes are then the planner's
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/warmnc_pmc_fetch -o run -- python3 scripts/warm_plan.py --reps 1 --no-chains > $OUT/warmnc_pmc_fetch.json 2> $OUT/warmnc_pmc_fetch.err &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/warmnc_pmc_write -o run -- python3 scripts/warm_plan.py --reps 1 --no-chains > $OUT/warmnc_pmc_write.json 2> $OUT/warmnc_pmc_write.err || exit 1
