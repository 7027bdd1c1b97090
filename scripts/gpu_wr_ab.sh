# rules relabel: targeted prefetch after misses; parity tests + scale instances
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -k "mapd or step or kat or block" > gpurun_out/gpu_wr_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/scale_bench.py c3 --cpu-steps 2 > gpurun_out/wr_c3.jsonl 2> gpurun_out/wr_c3.log &&
TSW_PLAN_DEBUG=1 timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 --cpu-steps 1 > gpurun_out/wr_wh10k.jsonl 2> gpurun_out/wr_wh10k.log
