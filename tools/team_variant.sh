#!/bin/bash
# A/B build of libgymsim with extra compile definitions for the lane-team kernels (gs_team.hip; the other
# objects are the in-tree build's):  tools/team_variant.sh <name> -DGS_TEAM_BLOCK=32 ...
#   -> isaacgymenv_amd/_lib/libgymsim_<name>.so  (select with GS_LIBGYMSIM=libgymsim_<name>.so; TEAM_SRC=<file>
#   compiles another gs_team.hip in its place)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OBJ=$ROOT/isaacgymenv_amd/_lib/obj/libgymsim
TMP=$(mktemp -d)
CS=$ROOT/isaacgymenv_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -fno-slp-vectorize -I $ROOT/include -I $CS \
  "$@" -o $TMP/gs_team.o ${TEAM_SRC:-$CS/gs_team.hip}
OBJS=""
for o in $OBJ/*.o; do
  case $(basename $o) in
    gs_team.o) OBJS="$OBJS $TMP/gs_team.o";;
    *) OBJS="$OBJS $o";;
  esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/isaacgymenv_amd/_lib/libgymsim_$NAME.so $OBJS -lpthread
rm -rf $TMP
