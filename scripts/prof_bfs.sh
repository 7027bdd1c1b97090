#!/bin/bash
# PMC passes over the K1 micro-bench (one rocprofv3 run per counter group, each under its own limit).
set -o pipefail
OUT=gpurun_out/prof_bfs
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 scripts/bfs_bench.py 10000 1"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- $B > $OUT/p4.log 2>&1
