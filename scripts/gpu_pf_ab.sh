# A/B of the prefetch depth (TSW_WIDE_PREFETCH hops) on the scale instances + lazy planner parity tests
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -k "mapd or step or kat" > gpurun_out/gpu_pf_tests.log 2>&1 &&
for h in 2 4 8; do
  TSW_WIDE_PREFETCH=$h timeout -k 10 300 python -u scripts/scale_bench.py c3 --cpu-steps 2 > gpurun_out/pf_c3_$h.jsonl 2> gpurun_out/pf_c3_$h.log || exit 1
  TSW_WIDE_PREFETCH=$h timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 --cpu-steps 1 > gpurun_out/pf_wh10k_$h.jsonl 2> gpurun_out/pf_wh10k_$h.log || exit 1
done
