// VALU cost microbenchmark (tools only): cycles per wave64 instruction for the
// op kinds the traversal uses, measured at full occupancy with 8 independent
// chains per lane. Build: hipcc --offload-arch=gfx950 -O3 valu_cost.hip -o valu_cost
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 2048;

#define BODY(OP)                                                           \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) { OP; }

template <int KIND>
__global__ void __launch_bounds__(256) k_bench(double* out, float* outf, double seed) {
    double a[8], b[8];
    float f[8];
    unsigned u[8];
    const double x = seed + threadIdx.x * 1e-9;
    for (int k = 0; k < 8; ++k) {
        a[k] = x + k;
        b[k] = 1.0 + x * k;
        f[k] = (float)a[k];
        u[k] = threadIdx.x * 7 + k;
    }
    for (int it = 0; it < kIters; ++it) {
        if constexpr (KIND == 0) BODY(f[k] = __builtin_fmaf(f[k], 0.999f, 0.001f))
        if constexpr (KIND == 1) BODY(a[k] = __builtin_fma(a[k], 0.999, 0.001))
        if constexpr (KIND == 2) BODY(a[k] = a[k] + b[k])
        if constexpr (KIND == 3) BODY(a[k] = a[k] * 0.999)
        if constexpr (KIND == 4) BODY(a[k] = b[k] / a[k])
        if constexpr (KIND == 5) BODY(a[k] = __builtin_amdgcn_rcp(a[k]))
        if constexpr (KIND == 6) BODY(a[k] = __builtin_sqrt(a[k]))
        if constexpr (KIND == 7) BODY(u[k] = u[k] * 3u + 1u)
        if constexpr (KIND == 8) BODY(a[k] = a[k] > b[k] ? a[k] - 1.0 : b[k])
        if constexpr (KIND == 9) BODY(f[k] = __builtin_amdgcn_rcpf(f[k]))
    }
    double s = 0;
    float sf = 0;
    for (int k = 0; k < 8; ++k) {
        s += a[k] + (double)u[k];
        sf += f[k];
    }
    if (s == 12345.678) out[0] = s;
    if (sf == 12345.678f) outf[0] = sf;
}

int main() {
    const char* names[] = {"v_fma_f32", "v_fma_f64", "v_add_f64", "v_mul_f64", "f64 divide (IEEE)",
                           "v_rcp_f64", "f64 sqrt (IEEE)", "u32 mul+add", "f64 cmp+select+add", "v_rcp_f32"};
    double* out;
    float* outf;
    hipMalloc(&out, 8);
    hipMalloc(&outf, 8);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8 * 4;  // 8 blocks of 4 waves per CU = 32 waves / CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](int kind) {
        void (*fns[])(double*, float*, double) = {k_bench<0>, k_bench<1>, k_bench<2>, k_bench<3>, k_bench<4>,
                                                  k_bench<5>, k_bench<6>, k_bench<7>, k_bench<8>, k_bench<9>};
        hipLaunchKernelGGL(fns[kind], dim3(blocks), dim3(256), 0, 0, out, outf, 0.5);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(fns[kind], dim3(blocks), dim3(256), 0, 0, out, outf, 0.5);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double waves = 5.0 * blocks * 4;
        const double ops = waves * kIters * 8;  // wave-level "ops" (C-level operations)
        const double simd_cycles = ms * 1e-3 * p.clockRate * 1e3 * cus * 4;
        std::printf("%-22s %8.3f ms  %6.2f SIMD-cycles per wave-op (clock %d MHz)\n", names[kind], ms,
                    simd_cycles / ops, p.clockRate / 1000);
    };
    for (int k = 0; k < 10; ++k) run(k);
    return 0;
}
