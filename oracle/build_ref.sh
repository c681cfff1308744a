#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY — builds the *reference* renderer (the real
# gbordelon/fast_ray_tracer C sources, compiled where they lie under
# /root/reference; nothing is copied into this repo) into oracle/_ref/.
#
#   oracle/build_ref.sh <scene_main.c> <name>
#
# produces oracle/_ref/bin/<name>: the reference library objects + the given
# codegen output (yaml_parser.py scene.yml > main.c) + oracle/ref_harness.c,
# with main.c's render_multi / trace_photons calls routed through the harness so the
# raw canvas and the render_multi wall time can be captured
# (FRT_REF_CANVAS=<file>, FRT_REF_STATS=<file>), and pm_balance wrapped (--wrap) so the photon
# maps and pm_irradiance_estimate results can be dumped (FRT_REF_PM_*). Used to pin the CPU oracle
# (tests/golden/make_golden.py) and as bench.py's cpu_baseline ("reference").
#
# Container workarounds recorded in SURVEY.md section 8(c): the reference
# Makefile needs bash (<<<), src/libs/core_select is macOS-only and unused,
# png.h lives in /opt/conda. -march=native is dropped so the binaries also run
# on the GPU box's host CPU; the reference is ISO C11 (no FP contraction), so
# results do not depend on it.
set -euo pipefail

REF=${FRT_REFERENCE_DIR:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
MAIN=${1:?usage: build_ref.sh <main.c> <name>}
NAME=${2:?usage: build_ref.sh <main.c> <name>}

if [ ! -d "$REF/src" ]; then
    echo "build_ref.sh: reference sources not found at $REF" >&2
    exit 3
fi

CC=${CC:-gcc}
CFLAGS=(-std=c11 -O2 -w -D_DEFAULT_SOURCE -I/opt/conda/include)
LDFLAGS=(-L/opt/conda/lib -Wl,-rpath,/opt/conda/lib -Wl,--wrap=pm_balance -lpng16 -lz -lm -lpthread)

mkdir -p "$OUT/obj" "$OUT/bin"

objs=()
while IFS= read -r src; do
    rel=${src#"$REF"/}
    obj="$OUT/obj/$(echo "$rel" | tr '/' '_' | sed 's/\.c$/.o/')"
    if [ ! -f "$obj" ] || [ "$src" -nt "$obj" ]; then
        "$CC" "${CFLAGS[@]}" -c "$src" -o "$obj"
    fi
    objs+=("$obj")
done < <(find "$REF/src" -name '*.c' ! -path '*core_select*' | sort)

harness="$OUT/obj/frt_ref_harness.o"
if [ ! -f "$harness" ] || [ "$HERE/ref_harness.c" -nt "$harness" ]; then
    "$CC" "${CFLAGS[@]}" -I"$REF" -c "$HERE/ref_harness.c" -o "$harness"
fi

"$CC" "${CFLAGS[@]}" -I"$REF" -Drender_multi=frt_ref_render_multi -Dtrace_photons=frt_ref_trace_photons \
    -c "$MAIN" -o "$OUT/obj/main_$NAME.o"
"$CC" -o "$OUT/bin/$NAME" "$OUT/obj/main_$NAME.o" "$harness" "${objs[@]}" "${LDFLAGS[@]}"
echo "$OUT/bin/$NAME"
