#!/bin/bash
# One parameterised GPU launcher (run through gpurun from the repo root), replacing round 1's
# one-off scripts. Usage: bash scripts/gpu_run.sh STEP [STEP ...]; environment variables (A/B knobs,
# TSW_*) apply to every step. Each step has its own time limit and writes under gpurun_out/.
# The script stops at the first step that fails hard: a test run with failures (rc 1) still lets
# the next steps run, any other non-zero status (fault, abort, time limit) ends the call.
#   tests        pytest -m gpu (every GPU test, per-test limit)        -> gpurun_out/gpu_tests.log
#   tests:EXPR   pytest -m gpu -k EXPR
#   smoke        __graft_entry__.smoke()                               -> gpurun_out/smoke.log
#   bench        the driver's default bench.py line                    -> gpurun_out/bench.json
#   plan         bench.py planning leg only (3 plans)                  -> gpurun_out/plan.json
#   scale:NAME   scripts/scale_bench.py NAME (c3 | wh10k | c5), full horizon -> gpurun_out/scale_NAME.jsonl
#   scaleT:NAME:T  same, horizon capped at T timesteps
#   profile      scripts/profile_round.sh r3 (trace + PMC per workload)
#   astar        scripts/astar_bench.py                                -> gpurun_out/astar_bench.json
#   bfs          scripts/bfs_bench.py (K1 cells/s, den520d + 1024^2) -> gpurun_out/bfs_bench.log
#   rehearse2    bench.py at N=2 on one GPU over gloo                  -> gpurun_out/rehearse2.json
#   bfsocc       scripts/bfs_occ_probe.sh (K1 residency / PAIR probe)  -> gpurun_out/bfs_occ.log
#   abplan       scripts/ab_plan.sh with the defaults (planner section clocks) -> gpurun_out/ab_0.json/.err
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run LIMIT CMD... ; returns the command's status
  local lim=$1; shift
  timeout -k 10 "$lim" "$@"
}
for step in "$@"; do
  echo "[gpu_run] $step $(date +%T)"
  case $step in
    tests|tests:*)
      k=(); [ "$step" != tests ] && k=(-k "${step#tests:}")
      log=gpurun_out/gpu_tests.log; [ "$step" != tests ] && log=gpurun_out/gpu_tests_k.log
      run 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1
      rc=$?; tail -3 $log; [ $rc -le 1 ] || exit $rc ;;
    smoke) run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $? ;;
    bench) run 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $? ;;
    plan) run 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-bfs > gpurun_out/plan.json 2> gpurun_out/plan.err || exit $? ;;
    scale:*) n=${step#scale:}; run 1100 python -u scripts/scale_bench.py $n > gpurun_out/scale_$n.jsonl 2> gpurun_out/scale_$n.log || exit $? ;;
    scaleT:*) a=${step#scaleT:}; n=${a%%:*}; t=${a#*:}
      run 900 python -u scripts/scale_bench.py $n --max-t $t > gpurun_out/scale_${n}_t$t.jsonl 2> gpurun_out/scale_${n}_t$t.log || exit $? ;;
    profile) bash scripts/profile_round.sh r4 || exit $? ;;
    astar) run 300 python scripts/astar_bench.py --out gpurun_out/astar_bench.json > gpurun_out/astar_bench.log 2>&1 || exit $? ;;
    bfs) run 300 python scripts/bfs_bench.py 10000 5 cave > gpurun_out/bfs_bench.log 2>&1 &&
         run 300 python scripts/bfs_bench.py 2048 3 sort >> gpurun_out/bfs_bench.log 2>&1 || exit $? ;;
    rehearse2) run 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --dist-backend gloo \
        > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log || exit $? ;;
    bfsocc) bash scripts/bfs_occ_probe.sh || exit $? ;;
    abplan) bash scripts/ab_plan.sh "TSW_X=0" || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] done $(date +%T)"
