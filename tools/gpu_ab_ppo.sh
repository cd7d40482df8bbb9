#!/bin/bash
# A/B of environment settings on the PPO leg: N alternating runs per setting, one line per run (samples/s,
# rollout / update ms per epoch).   bash tools/gpu_ab_ppo.sh <outdir> <N> "A=1 B=2" "A=3" ...
set -o pipefail
OUT=$1; N=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do
  for kv in "$@"; do
    tag=$(echo "$kv" | tr "= " "__")
    env $kv timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 6 --other-steps 0 > $OUT/ppo_${tag}_$i.json 2> $OUT/ppo_${tag}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/ppo_${tag}_$i.json').read().strip().splitlines()[-1])['ppo']; print('$kv', round(d['value']/1e6,3), 'M samples/s rollout', round(d['rollout_ms'],3), 'update', round(d['update_ms'],3))" | tee -a $OUT/summary.txt
  done
done
