#!/bin/bash
# A/B of the lane-team workgroup width on the plane (headline) and trimesh configs: the default libgymsim and the
# variants built by tools/team_variant.sh (GS_TEAM_BLOCK=32 / 16), each: bench.py with the trimesh config, the
# physics kernels' rocprofv3 averages.   bash tools/team_block_ab.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for V in default "$@"; do
  if [ "$V" = default ]; then export GS_LIBGYMSIM=libgymsim.so; else export GS_LIBGYMSIM=libgymsim_$V.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V -o run -- python3 $ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --ppo-epochs 0 --other-steps 100 > $OUT/$V.json 2> $OUT/$V.err || exit 1
  rm -f $OUT/$V/*kernel_trace.csv
  echo "== $V" >> $OUT/summary.txt
  grep -h "_team<" $OUT/$V/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,110-220 >> $OUT/summary.txt
  python3 -c "import json; d=json.loads(open('$OUT/$V.json').read().strip().splitlines()[-1]); print('headline', round(d['value']/1e6,2), 'M', 'trimesh', [round(o['value']/1e6,2) for o in d['other_configs'] if 'trimesh' in o['workload']])" >> $OUT/summary.txt
done
cat $OUT/summary.txt
