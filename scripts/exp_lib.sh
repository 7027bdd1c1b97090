#!/bin/bash
# Diagnostic library variant for experiments: k_plan<1,1,1,0> (C3's instantiation, tsw_plan_v0.hip) compiled
# with extra hipcc flags, linked with the diag build's other objects ->
# p2p_distributed_tswap_amd/exp/libtswap_hip_diag_<name>.so.  Usage: bash scripts/exp_lib.sh NAME FLAGS...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result -Wno-unused-value -I include"
mkdir -p build/exp_$name p2p_distributed_tswap_amd/exp
/opt/rocm/bin/hipcc $F "$@" -c -o build/exp_$name/tsw_plan_v0.o p2p_distributed_tswap_amd/csrc/tsw_plan_v0.hip
objs="build/exp_$name/tsw_plan_v0.o build/common/*.o $(ls build/diag/*.o | grep -v tsw_plan_v0.o)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o p2p_distributed_tswap_amd/exp/libtswap_hip_diag_$name.so $objs
