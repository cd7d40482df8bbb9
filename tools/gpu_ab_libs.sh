#!/bin/bash
# A/B of libgymsim variants on one box: for each name, N short benches with GS_LIBGYMSIM=libgymsim_<name>.so
# ("default" = libgymsim.so), alternating, then one line per run (env-steps/s, HIP-event kernel ms).
#   bash tools/gpu_ab_libs.sh <outdir> <N> name1 name2 ...
set -o pipefail
OUT=$1; N=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do
  for name in "$@"; do
    lib=libgymsim_$name.so; [ "$name" = default ] && lib=libgymsim.so
    GS_LIBGYMSIM=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/bench_${name}_$i.json 2> $OUT/bench_${name}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/bench_${name}_$i.json').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e6,3), 'M env-steps/s kernel_ms', round(d['roofline']['kernel_ms'],5))" | tee -a $OUT/summary.txt
  done
done
