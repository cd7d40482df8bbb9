#!/bin/bash
# SQ counter passes on the UsefulHound simulate kernel, self-collision on and off.
#   bash tools/probes/hound_sq.sh <tag>   -> gpurun_out/<tag>/sc<0|1>_<g>/run_counter_collection.csv
set -o pipefail
TAG=${1:-hound_sq}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for sc in ${SCS:-1 0}; do
  GS_SELF_COLLIDE=$sc timeout -k 10 200 python3 $ROOT/tools/probes/hound_sq.py > $OUT/time_sc$sc.log 2>&1 || exit 1
  g=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"; do
    g=$((g+1))
    GS_SELF_COLLIDE=$sc timeout -k 10 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/sc${sc}_$g -o run -- \
      python3 $ROOT/tools/probes/hound_sq.py > $OUT/sc${sc}_$g.log 2>&1 || exit 1
  done
done
echo done
