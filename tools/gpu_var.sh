#!/bin/bash
# A/B of device-library builds (variants/<name>.so from tools/build_variant.sh; "base" = the tree's build) on
# one scene, each through tools/gpu_ab.sh:   tools/gpu_var.sh <scene> <label> base NAME ... [base]
set -o pipefail
sc=$1; label=$2; shift 2
cp fast_ray_tracer_amd/lib/libfrt_device.so /tmp/frt_base.so
: > gpurun_out/ab_${label}_all.txt
rc=0
for lib in "$@"; do
  if [ "$lib" = base ]; then cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so; else cp variants/$lib.so fast_ray_tracer_amd/lib/libfrt_device.so; fi
  bash tools/gpu_ab.sh $sc ${label}_$lib "FRT_LIB=$lib" || { rc=1; break; }
  cat gpurun_out/ab_${label}_$lib.txt >> gpurun_out/ab_${label}_all.txt
done
cp /tmp/frt_base.so fast_ray_tracer_amd/lib/libfrt_device.so
exit $rc
