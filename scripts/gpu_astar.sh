set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "astar or mapd or next_hop" > gpurun_out/gpu_astar_tests.log 2>&1 &&
timeout -k 10 300 python scripts/astar_bench.py --out gpurun_out/astar_bench.json > gpurun_out/astar_bench.log 2>&1
