set -o pipefail
export TMPDIR=/tmp
for w in 2 4 6 7; do TSW_BFS_KERNEL=blk TSW_BFS_WAVES=$w timeout -k 10 120 python scripts/bfs_bench.py 10000 3 || exit 1; done > gpurun_out/bfs_waves.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_blk -o run -- python3 scripts/bfs_bench.py 10000 1 > gpurun_out/pmc_blk.log 2>&1
