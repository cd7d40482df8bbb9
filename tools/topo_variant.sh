#!/bin/bash
# A/B build of libgymsim with extra compile definitions for ONE topology's plane kernels (forms 0 and 2; the
# other objects are the in-tree build's):  tools/topo_variant.sh <name> <topology, e.g. hound> -DFOO=1 ...
#   -> isaacgymenv_amd/_lib/libgymsim_<name>.so  (select with GS_LIBGYMSIM=libgymsim_<name>.so)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; TOPO=$2; shift 2
OBJ=$ROOT/isaacgymenv_amd/_lib/obj/libgymsim
TMP=$(mktemp -d)
CS=$ROOT/isaacgymenv_amd/csrc
for f in 0 2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -fno-slp-vectorize -I $ROOT/include -I $CS \
    "$@" -DGS_INST_TOPO=Topo_$TOPO -DGS_INST_FORM=$f -o $TMP/inst_$f.o $CS/gs_phys_inst.hip &
done
wait
OBJS=""
for o in $OBJ/*.o; do
  case $(basename $o) in
    gs_phys_inst_${TOPO}_0.o) OBJS="$OBJS $TMP/inst_0.o";;
    gs_phys_inst_${TOPO}_2.o) OBJS="$OBJS $TMP/inst_2.o";;
    *) OBJS="$OBJS $o";;
  esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/isaacgymenv_amd/_lib/libgymsim_$NAME.so $OBJS -lpthread
rm -rf $TMP
