#!/bin/bash
# round 6: child slots as two halves (reflected, refracted) — parity (goldens incl. reflection / refraction and GI
# scenes, headline rows, lazy ambient, split invariance), the headline frame, then a PMC checkpoint of the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "reference_canvas or headline or benchmark_scene or lazy_ambient or gather" \
    tests/test_gpu_stochastic.py -k "cornell_gi_24 or cornell_shipped" \
    > gpurun_out/pytest_r06_k.log 2>&1 || { tail -30 gpurun_out/pytest_r06_k.log; exit 1; }
tail -2 gpurun_out/pytest_r06_k.log
bash tools/gpu_ab.sh cornell_direct_1920x1080_8x8 r06_child_halves "FRT_X=0" "FRT_X=1" || exit 1
bash tools/prof.sh r06k_headline cornell_direct_1920x1080_8x8 \
    "k_shade_lit k_prepare frt_jit_sub frt_jit_shadow frt_jit_trace frt_jit_subtile frt_jit_tile k_combine_resolve k_combine"
