set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_par.log 2>&1 &&
timeout -k 10 300 python -u scripts/scale_bench.py c3 --cpu-steps 2 > gpurun_out/scale.log 2>&1 &&
timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 --cpu-steps 2 >> gpurun_out/scale.log 2>&1
