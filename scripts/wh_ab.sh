# wh10k A/B of planner knobs over a horizon (diag library, planner debug) -> gpurun_out/wab_<i>.jsonl/.log
# usage: bash scripts/wh_ab.sh INSTANCE MAX_T "ENV=.." ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
inst=$1; mt=$2; shift 2
i=0
for e in "$@"; do
  env $e TSW_PLAN_DEBUG=1 timeout -k 10 300 python -u scripts/scale_bench.py $inst --max-t $mt --cpu-steps 1 --diag > gpurun_out/wab_$i.jsonl 2> gpurun_out/wab_$i.log || exit $?
  i=$((i+1))
done
