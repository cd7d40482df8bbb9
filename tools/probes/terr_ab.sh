set -o pipefail
mkdir -p gpurun_out/r05ad
for v in A C D A C D; do
  GS_LIBGYMSIM=libgymsim_ab_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --ppo-epochs 0 --steps 50 --warmup 10 --other-steps 100 > gpurun_out/r05ad/bench_$v.json 2>/dev/null || exit 1
  python - "$v" <<'PY'
import json, sys
b = json.loads(open(f"gpurun_out/r05ad/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], [round(o["value"] / 1e6, 3) for o in b["other_configs"]], flush=True)
PY
done
