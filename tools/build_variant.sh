#!/bin/bash
# Build a profiling variant of libgymsim from an alternative gs_team.hip (A/B kernel experiments).
#   tools/build_variant.sh <path/to/gs_team_variant.hip> <name>   -> isaacgymenv_amd/_lib/libgymsim_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p $TMP/pkg/csrc $TMP/include
cp $ROOT/include/*.h $TMP/include/
cp $ROOT/isaacgymenv_amd/csrc/*.hip $ROOT/isaacgymenv_amd/csrc/*.h $TMP/pkg/csrc/
cp "$1" $TMP/pkg/csrc/gs_team.hip
CS=$TMP/pkg/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -DGS_PHASE_PROFILE \
  -I $TMP/include -I $CS -o $ROOT/isaacgymenv_amd/_lib/libgymsim_$2.so $CS/gs_physics.hip $CS/gs_team.hip $CS/gs_capi.hip
rm -rf $TMP
