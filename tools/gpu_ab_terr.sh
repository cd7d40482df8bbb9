#!/bin/bash
# A/B of libgymsim variants on the trimesh AnymalTerrain config (TASK=UsefulHound / Ant: that config instead): for each name, N short benches with
# GS_LIBGYMSIM=libgymsim_<name>.so ("default" = libgymsim.so), alternating; one line per run (trimesh env-steps/s,
# HIP-event simulate ms).     bash tools/gpu_ab_terr.sh <outdir> <N> name1 name2 ...
set -o pipefail
OUT=$1; N=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do
  for name in "$@"; do
    lib=libgymsim_$name.so; [ "$name" = default ] && lib=libgymsim.so
    GS_LIBGYMSIM=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-epochs 0 \
      --other-steps ${OTHER_STEPS:-200} --others ${TASK:-AnymalTerrain} > $OUT/bench_${name}_$i.json 2> $OUT/bench_${name}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/bench_${name}_$i.json').read().strip().splitlines()[-1]); o=d['other_configs'][0]; print('$name', round(o['value']/1e6,3), 'M env-steps/s simulate_ms', round(o['simulate_kernel_ms'],5))" | tee -a $OUT/summary.txt
  done
done
