#!/bin/bash
# K1 residency probe (run through gpurun from the repo root): den520d-like cave, 10k goals, with the
# in-kernel cycle split (TSW_BFS_PROF=1) at 1, 2 and 3 waves per SIMD (TSW_BFS_WAVES = 4, 8, 16 per
# workgroup; 16 is capped to 12 by LDS). The BFS cycles per goal at 1 wave per SIMD are the level
# loop's own dependent latency; at 3 they include the issue contention of the co-resident waves.
# Then the two-goals-per-wave variant (TSW_BFS_PAIR=1) at its LDS-bound residency, with and
# without the split. -> gpurun_out/bfs_occ.log
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bfs_occ.log
for wv in 4 8 16; do
  echo "[bfs_occ] TSW_BFS_WAVES=$wv" >> gpurun_out/bfs_occ.log
  TSW_BFS_WAVES=$wv TSW_BFS_PROF=1 timeout -k 10 120 python scripts/bfs_bench.py 10000 2 cave \
    >> gpurun_out/bfs_occ.log 2>&1 || exit $?
done
for pr in 1 0; do
  echo "[bfs_occ] TSW_BFS_PAIR=1 prof=$pr" >> gpurun_out/bfs_occ.log
  if [ $pr = 1 ]; then export TSW_BFS_PROF=1; else unset TSW_BFS_PROF; fi
  TSW_BFS_PAIR=1 timeout -k 10 120 python scripts/bfs_bench.py 10000 3 cave >> gpurun_out/bfs_occ.log 2>&1 || exit $?
done
unset TSW_BFS_PROF
echo "[bfs_occ] default" >> gpurun_out/bfs_occ.log
timeout -k 10 120 python scripts/bfs_bench.py 10000 3 cave >> gpurun_out/bfs_occ.log 2>&1 || exit $?
