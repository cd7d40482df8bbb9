#!/bin/bash
# SQ counter passes for the physics kernel (one rocprofv3 --pmc pass per group; kernel-trace only).
#   bash tools/sq_counters.sh <tag>   -> gpurun_out/<tag>/sq_*/run_counter_collection.csv
set -o pipefail
TAG=${1:-sq}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS" \
           "SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/sq_$i -o run -- \
    python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/sq_$i.log 2>&1 || exit 1
done
