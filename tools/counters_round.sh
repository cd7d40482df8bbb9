#!/bin/bash
# Counter session on one GPU box (each rocprofv3 --pmc pass its own run, kernel trace only):
#   1. FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/hbm_calib, the physics kernel's
#      access shapes + a streaming control);
#   2. FETCH_SIZE / WRITE_SIZE of bench.py (the physics kernel's traffic);
#   3. SQ groups of bench.py (VALU / LDS / wait / instruction-fetch counters of every physics kernel).
# Usage: bash tools/counters_round.sh <tag>      (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-counters}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 10"
timeout -k 10 120 $ROOT/tools/hbm_calib > $OUT/calib_bytes.json || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/calib_$c -o run -- \
    $ROOT/tools/hbm_calib > $OUT/calib_$c.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/bench_$c -o run -- \
    $BENCH > $OUT/bench_$c.log 2>&1 || exit 1
done
echo "calibration + traffic ok"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS" \
           "SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM_NORM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/sq_$i -o run -- \
    $BENCH > $OUT/sq_$i.log 2>&1 || { echo "sq group $i failed: $grp"; exit 1; }
done
echo "sq ok"
cd $ROOT && python3 tools/counter_summary.py $OUT && du -sh $OUT
