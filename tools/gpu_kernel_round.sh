#!/bin/bash
# One GPU session for a physics-kernel change: every GPU test, the bench (headline + other configs) under
# rocprofv3 --stats, and the FETCH_SIZE / WRITE_SIZE passes of the headline kernel (each its own run).
# Usage: bash tools/gpu_kernel_round.sh <tag> [pytest -k expr]     (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-kernel}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
export PARITY_REPORT=$OUT/parity.txt
export PARITY_DUMP=$OUT/dump
KEXPR=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -1 $OUT/pytest_gpu.log &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --other-steps 50 > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && rm -f $OUT/stats/*kernel_trace.csv &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/pmc_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/pmc_write.log 2>&1 && echo "write ok" &&
grep -h "k_pd_step_team\|k_simulate\|k_pair_records" $OUT/stats/run_kernel_stats.csv | cut -c1-200 ; du -sh $OUT
