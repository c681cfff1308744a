mkdir -p gpurun_out
for sc in cornell_direct_800_4x4 checkered_sphere_800; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --gi-steps 0 --no-cpu-baseline --no-render-multi --scene $sc > gpurun_out/r02_bench_$sc.json 2>/dev/null || exit 1
  tail -1 gpurun_out/r02_bench_$sc.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', d['ms_per_step'], d['value'], d['kernel_ms_per_frame'])"
done
for ps in 6 8 10 14; do
  FRT_JIT_PART=$ps timeout -k 10 300 python bench.py --steps 3 --warmup 1 --gi-steps 0 --no-cpu-baseline --no-render-multi 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('part $ps', d['ms_per_step'], d['shadow_pass']['kernels_ms_per_frame'])" || exit 1
done
