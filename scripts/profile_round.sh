#!/bin/bash
# Profiles the default bench on one MI355X (run through gpurun from the repo root).
#   1. bench.py (HIP-event timings, CPU baseline)            -> $OUT/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command   -> $OUT/trace/
#   3. separate PMC passes: FETCH_SIZE, WRITE_SIZE            -> $OUT/pmc_fetch, $OUT/pmc_write
# Each GPU step has its own time limit; steps are chained with && so a failure stops the run.
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu --bfs-reps 1"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
