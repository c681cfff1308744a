#!/bin/bash
# GPU round trip (run via gpurun from the repo root): -m gpu tests, smoke, the default bench line, then the
# headline frame's kernel-trace stats.   tools/gpu_r03d.sh TAG
set -o pipefail
TAG=${1:-r03d}
mkdir -p gpurun_out
bash tools/gpu_round.sh "$TAG" || exit $?
KS_ARGS="--gi-steps 0 --no-render-multi" STEPS=3 WARMUP=1 bash tools/kstats.sh cornell_direct_1920x1080_8x8 || exit $?
