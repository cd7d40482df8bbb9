#!/bin/bash
# Short GPU session for one kernel change: the named GPU tests, then the default bench under rocprofv3 --stats.
# Usage: bash tools/gpu_quick.sh <tag> "<pytest -k expression>" [bench args]   (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-quick}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
export PARITY_REPORT=$OUT/parity.txt
export PARITY_DUMP=$OUT/dump
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$2" > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 ${@:3} > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && rm -f $OUT/stats/*kernel_trace.csv && grep -h "k_pd_step_team\|k_simulate\|k_pair_records\|k_pd_step_wave" $OUT/stats/run_kernel_stats.csv | cut -c1-160 && tail -c 400 $OUT/bench.json
