set -o pipefail
export TMPDIR=/tmp
B="python3 scripts/astar_bench.py --child gpurun_out/astar_pm"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/astar_pmc1 -o run -- $B > gpurun_out/astar_pmc1.log 2>&1 &&
TSW_ASTAR_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/astar_pmc2 -o run -- $B > gpurun_out/astar_pmc2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/astar_pmc3 -o run -- $B > gpurun_out/astar_pmc3.log 2>&1
