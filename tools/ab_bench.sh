#!/bin/bash
# A/B helper for kernel experiments on the GPU box: physics parity tests, then N short benches.
#   bash tools/ab_bench.sh <outdir> [N]
set -e
OUT=$1; N=${2:-2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_physics_gpu.py > $OUT/pytest.log 2>&1
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/bench$i.json 2> $OUT/bench.err
  python -c "import json; d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1]); print('bench', round(d['value']/1e6,2), 'M env-steps/s kernel_ms', round(d['roofline']['kernel_ms'],5))" >> $OUT/summary.txt
done
tail -1 $OUT/pytest.log >> $OUT/summary.txt
