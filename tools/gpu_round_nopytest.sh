#!/bin/bash
# The GPU round without the test suite (tools/gpu_round.sh after pytest): smoke(), bench, torchrun bench, kernel-trace stats.
# Usage: bash tools/gpu_round_nopytest.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/stats.log 2>&1 && echo "stats ok" && rm -f $OUT/stats/*kernel_trace.csv
