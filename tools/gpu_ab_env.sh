#!/bin/bash
# A/B of an environment switch on the headline bench: N alternating short benches per setting, one line per run.
#   bash tools/gpu_ab_env.sh <outdir> <N> "NAME=VALUE" "NAME=VALUE" ...    (e.g. GS_FUSED_TAIL=0 GS_FUSED_TAIL=1)
set -o pipefail
OUT=$1; N=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do
  for kv in "$@"; do
    tag=$(echo "$kv" | tr "= " "__")
    env $kv timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $OUT/bench_${tag}_$i.json 2> $OUT/bench_${tag}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/bench_${tag}_$i.json').read().strip().splitlines()[-1]); print('$kv', round(d['value']/1e6,3), 'M env-steps/s ms_per_step', round(d['ms_per_step'],5), 'kernel_ms', round(d['roofline']['kernel_ms'],5))" | tee -a $OUT/summary.txt
  done
done
