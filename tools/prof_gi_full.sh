#!/bin/bash
# The GI frame at full size (cornell_gi_1920x1080_8x8; run via gpurun from the repo root):
#   1. the estimate's counters and phase cycles (variants/prof.so, -DFRT_WALK_PROF) on the same scene at
#      480x270 (the same camera and photon maps per pixel; the instrumented build is slow)
#   2. rocprofv3 --kernel-trace --stats of one frame (this workload alone)
#   3. PMC passes over k_gather_est (one counter block set per pass)
set -o pipefail
TAG=${1:-r03}
SC=cornell_gi_1920x1080_8x8
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gifull_$TAG
mkdir -p "$OUT"
B="--scene $SC --gi-steps 0 --no-cpu-baseline --no-render-multi --steps 1 --warmup 0"
cp "$R/fast_ray_tracer_amd/lib/libfrt_device.so" /tmp/frt_base.so
cp "$R/variants/prof.so" "$R/fast_ray_tracer_amd/lib/libfrt_device.so"
timeout -k 10 300 python3 "$R/bench.py" ${B/$SC/cornell_gi_480x270_8x8} > "$OUT/prof.json" 2> "$OUT/prof.err"
rc=$?
cp /tmp/frt_base.so "$R/fast_ray_tracer_amd/lib/libfrt_device.so"
[ $rc -ne 0 ] && exit $rc
grep "estimate prof" "$OUT/prof.err" | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $B > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
pmc() {
    local d=$1; shift
    timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-include-regex k_gather_est -f csv -d "$OUT/$d" -o run -- \
        python3 "$R/bench.py" $B > "$OUT/$d.json" 2> "$OUT/$d.err"
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
pmc tcc TCC_HIT_sum TCC_MISS_sum || exit $?
pmc clk GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
cd "$R"
python3 tools/pmc_summary.py "$OUT" k_gather_est "$SC" > "$OUT/pmc_k_gather_est.json" || exit $?
cat "$OUT/pmc_k_gather_est.json"
