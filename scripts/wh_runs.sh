# Repeated full-horizon wh10k plans (bimodal run time check) + C5 -> gpurun_out/whr_*.jsonl
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  TSW_PLAN_DEBUG=1 timeout -k 10 300 python -u scripts/scale_bench.py wh10k --cpu-steps 1 --diag > gpurun_out/whr_$i.jsonl 2> gpurun_out/whr_$i.log || exit $?
done
timeout -k 10 300 python -u scripts/scale_bench.py c5 --cpu-steps 1 > gpurun_out/whr_c5.jsonl 2> gpurun_out/whr_c5.log
