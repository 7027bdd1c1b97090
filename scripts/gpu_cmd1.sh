set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_bfs.log 2>&1 &&
TSW_BFS_KERNEL=blk timeout -k 10 120 python scripts/bfs_bench.py 10000 3 > gpurun_out/bfs_cmp.log 2>&1 &&
TSW_BFS_KERNEL=blk TSW_BFS_PROF=1 timeout -k 10 120 python scripts/bfs_bench.py 10000 1 >> gpurun_out/bfs_cmp.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 scripts/bfs_bench.py 10000 1 > gpurun_out/pmc_w.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 scripts/bfs_bench.py 10000 1 > gpurun_out/pmc_f.log 2>&1
