set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_bfs.log 2>&1 &&
for w in 8 10 12; do TSW_BFS_KERNEL=blk TSW_BFS_WAVES=$w timeout -k 10 120 python scripts/bfs_bench.py 10000 3 || exit 1; done > gpurun_out/bfs_cmp.log 2>&1 &&
TSW_BFS_KERNEL=blk TSW_BFS_PROF=1 timeout -k 10 120 python scripts/bfs_bench.py 10000 1 >> gpurun_out/bfs_cmp.log 2>&1
