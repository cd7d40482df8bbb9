#!/bin/bash
# One GPU session for the round-4 learner / trimesh work: the named GPU tests, the per-layer linear probe, a PPO
# A/B (library layers vs the MFMA layers) and the trimesh phase profile.
# Usage: bash tools/gpu_ab.sh <tag> "<pytest -k expression>"   (outputs under gpurun_out/<tag>/)
set -o pipefail
TAG=${1:-ab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export PARITY_REPORT=$OUT/parity.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 200 python -u tools/probes/linear_probe.py --out $OUT/linear_probe.json > $OUT/probe.log 2>&1 && echo "probe ok" &&
IGE_MFMA_LAYERS=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-steps 0 --ppo-epochs 5 > $OUT/bench_lib.json 2> $OUT/bench_lib.err && echo "bench lib ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-steps 30 --ppo-epochs 5 > $OUT/bench_mfma.json 2> $OUT/bench_mfma.err && echo "bench mfma ok" &&
timeout -k 10 240 python -u tools/phase_profile.py --trimesh --steps 30 --warmup 10 > $OUT/phase_trimesh.txt 2>&1 && echo "phase ok"
