#!/bin/bash
# One GPU-box session: GPU tests, smoke(), the default bench line, the bench under torch.distributed.run (1 rank), a kernel-trace profile and two PMC passes.
# Usage: bash tools/gpu_round.sh <tag>     (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-run}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
export PARITY_REPORT=$OUT/parity.txt
export PARITY_DUMP=$OUT/dump
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 200 --warmup 20 --other-steps 20 --no-cpu-baseline > $OUT/bench_torchrun1.json 2> $OUT/bench_torchrun1.err && echo "torchrun ok" &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/stats.log 2>&1 && echo "stats ok" && rm -f $OUT/stats/*kernel_trace.csv &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/pmc_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/pmc_write.log 2>&1 && echo "write ok" && du -sh $OUT
