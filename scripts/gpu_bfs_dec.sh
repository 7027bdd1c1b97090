set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_bfs_tests.log 2>&1 &&
TSW_BFS_PROF=1 timeout -k 10 120 python scripts/bfs_bench.py 10000 3 > gpurun_out/bfs_prof.log 2>&1 &&
timeout -k 10 120 python scripts/bfs_bench.py 10000 5 > gpurun_out/bfs_lpt.log 2>&1
