#!/bin/bash
# Round-end evidence (run through gpurun from the repo root): scripts/profile_round.sh TAG, then the K1
# instruction-count pass (scripts/k1_sq.py), smoke() and the driver's default bench line.
set -o pipefail
TAG=${1:-r6}
OUT=gpurun_out/prof_$TAG
export TMPDIR=/tmp
bash scripts/profile_round.sh $TAG &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/k1_sq -o run -- python3 bench.py --no-plan --no-cpu --bfs-reps 2 > $OUT/k1_sq.json 2> $OUT/k1_sq.err
