#!/bin/bash
# GPU session for the trimesh work: terrain GPU tests (parity report), the bench with the other configs (trimesh
# AnymalTerrain among them) and the trimesh phase profile.   Usage: bash tools/gpu_terr.sh <tag>
set -o pipefail
TAG=${1:-terr}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export PARITY_REPORT=$OUT/parity.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "terrain or trimesh" > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 400 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --other-steps 30 --ppo-epochs 2 > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" &&
timeout -k 10 240 python -u tools/phase_profile.py --trimesh --steps 30 --warmup 10 > $OUT/phase_trimesh.txt 2>&1 && echo "phase ok"
