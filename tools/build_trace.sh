#!/bin/bash
# Debug build of libgymsim with the GJK trace of one env (gs_pairs.h GS_GJK_TRACE):
#   tools/build_trace.sh <env>   -> isaacgymenv_amd/_lib/libgymsim_trace.so (select with GS_LIBGYMSIM=libgymsim_trace.so)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/isaacgymenv_amd/csrc
OUT=$ROOT/isaacgymenv_amd/_lib/trace_obj
mkdir -p $OUT
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -DGS_GJK_TRACE=$1 -I $ROOT/include -I $CS"
pids=()
for T in $(python3 -c "import sys; sys.path.insert(0, '$ROOT'); from isaacgymenv_amd.build import topologies; print(' '.join(topologies()))"); do
  for F in 0 1 2 3; do
    /opt/rocm/bin/hipcc $FL -DGS_INST_TOPO=$T -DGS_INST_FORM=$F -c $CS/gs_phys_inst.hip -o $OUT/inst_${T}_$F.o & pids+=($!)
  done
done
for f in gs_physics gs_team gs_kinematics gs_host gs_capi; do
  /opt/rocm/bin/hipcc $FL -c $CS/$f.hip -o $OUT/$f.o & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/isaacgymenv_amd/_lib/libgymsim_trace.so $OUT/*.o -lpthread
