set -o pipefail
TAG=${1:-team_ab}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
ROOT=$PWD
timeout -k 10 400 python -u -m pytest tests/test_physics_gpu.py tests/test_hound_gpu.py tests/test_tgs_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; echo "pytest rc $?"
for st in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --ppo-epochs 0 --other-steps 0 --steps 500 --warmup 50 --physx-solver-type $st > gpurun_out/$TAG/bench_$st.json 2>/dev/null || exit 1
  python -c "import json; b=json.loads(open('gpurun_out/$TAG/bench_$st.json').read().strip().splitlines()[-1]); print('$st', b['value'], b['roofline']['kernel_ms'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/$TAG/pmc_fetch -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $ROOT/gpurun_out/$TAG/pmc_fetch.log 2>&1 && echo fetch ok &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/gpurun_out/$TAG/pmc_write -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-epochs 0 --other-steps 0 > $ROOT/gpurun_out/$TAG/pmc_write.log 2>&1 && echo write ok
