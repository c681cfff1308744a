#!/bin/bash
# Build a variant of libfrt_device.so into exp/<name>.so with extra compile flags (variants/ travels to the GPU box, exp/ does not; A/B runs swap it in:
# tools/ab_gi.sh, tools/gi_round.sh).   tools/build_variant.sh NAME -DFOO=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/variants"
python3 -c "import sys; sys.path.insert(0, '$R'); from fast_ray_tracer_amd import build as b; b.write_jit_embed()"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I"$R/include" \
    -I"$R/fast_ray_tracer_amd/csrc" "$@" -o "$R/variants/$NAME.so" "$R/fast_ray_tracer_amd/csrc/frt_engine.hip" \
    "$R/fast_ray_tracer_amd/csrc/frt_jit.hip" -lhiprtc
echo "$R/variants/$NAME.so"
