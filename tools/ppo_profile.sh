#!/bin/bash
# PPO learner profile on the GPU box: bench.py's PPO leg under rocprofv3 --kernel-trace --stats.
#   bash tools/ppo_profile.sh <outdir>
set -e
OUT=$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 3 --other-steps 0 > $GRAFT_REPO_ROOT/$OUT/bench.json 2> $GRAFT_REPO_ROOT/$OUT/bench.err
# keep the summaries only (gpurun copies back at most 64 MiB)
find $GRAFT_REPO_ROOT/$OUT/prof -type f ! -name "*stats*" -delete
