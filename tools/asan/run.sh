#!/bin/bash
# ASan + UBSan build of libgymsim's host backend and a replay through the C ABI.
# The host-side sanitizers instrument gs_host.hip (the solver / narrowphase / kinematics headers it instantiates on
# the host: gs_solver.h, gs_pairs.h, gs_kinematics.h, gs_terrain.h) and gs_capi.hip; the device objects are the
# product build's (isaacgymenv_amd/_lib/obj/libgymsim, built by `python -m isaacgymenv_amd.build`), never run here.
#   tools/asan/run.sh [case] [n]        case: hound111 (default) | hound | anymal | ant
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
CS=$ROOT/isaacgymenv_amd/csrc
OBJ=$ROOT/isaacgymenv_amd/_lib/obj/libgymsim
OUT=${ASAN_OUT:-/tmp/gs_asan}
CASE=${1:-hound111}
N=${2:-64}
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
FL="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fno-slp-vectorize -I $ROOT/include -I $CS"
if [ ! -f $OUT/gs_host.o ] || [ $CS/gs_host.hip -nt $OUT/gs_host.o ] || [ $CS/gs_pairs.h -nt $OUT/gs_host.o ] || [ $CS/gs_solver.h -nt $OUT/gs_host.o ]; then
  /opt/rocm/bin/hipcc $FL $SAN -c $CS/gs_host.hip -o $OUT/gs_host.o &
  /opt/rocm/bin/hipcc $FL $SAN -c $CS/gs_capi.hip -o $OUT/gs_capi.o &
  wait
fi
/opt/rocm/bin/hipcc $FL $SAN -c $ROOT/tools/asan/host_replay.cpp -o $OUT/host_replay.o
OTHERS=$(ls $OBJ/*.o | grep -v "gs_host.o\|gs_capi.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address -fsanitize=undefined -fno-gpu-sanitize -o $OUT/host_replay \
  $OUT/host_replay.o $OUT/gs_host.o $OUT/gs_capi.o $OTHERS -lpthread
python3 $ROOT/tools/asan/dump_case.py $OUT/$CASE.bin --case $CASE --n $N
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 $OUT/host_replay $OUT/$CASE.bin
python3 $ROOT/tools/asan/dump_case.py $OUT/$CASE.bin --case $CASE --n $N --compare
