// Accuracy of v_rcp_f64 (tools only): max relative error over random and edge inputs,
// raw and after one / two Newton steps. Build: hipcc --offload-arch=gfx950 -O3 rcp_accuracy.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__global__ void k_rcp(const double* in, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double d = in[i];
    double r0 = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r0, 1.0);
    double r1 = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-d, r1, 1.0);
    double r2 = __builtin_fma(r1, e, r1);
    out[3 * i] = r0;
    out[3 * i + 1] = r1;
    out[3 * i + 2] = r2;
}

int main() {
    const int n = 1 << 22;
    double* h = new double[n];
    double* o = new double[3 * (size_t)n];
    uint64_t s = 0x12345678abcdefULL;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        double m = 1.0 + (double)(s >> 11) * (1.0 / 9007199254740992.0);  // [1, 2)
        int ex = (int)((s >> 3) % 80) - 40;
        h[i] = std::ldexp(m, ex) * ((s & 1) ? -1.0 : 1.0);
        if (i < 64) h[i] = std::ldexp(1.0 + i * (1.0 / 64), 0);  // near powers of two
        if (i >= 64 && i < 128) h[i] = std::nextafter(std::ldexp(1.0, i - 96), 0.0);
    }
    double *din, *dout;
    (void)hipMalloc(&din, n * sizeof(double));
    (void)hipMalloc(&dout, 3 * (size_t)n * sizeof(double));
    (void)hipMemcpy(din, h, n * sizeof(double), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rcp, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
    (void)hipMemcpy(o, dout, 3 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    double worst[3] = {0, 0, 0};
    long not_cr[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        double exact = 1.0 / h[i];
        for (int k = 0; k < 3; ++k) {
            double rel = std::fabs((o[3 * i + k] - exact) / exact);
            if (rel > worst[k]) worst[k] = rel;
            if (o[3 * i + k] != exact) not_cr[k]++;
        }
    }
    for (int k = 0; k < 3; ++k)
        std::printf("newton steps %d: max rel err %.3e (= 2^%.1f), not correctly rounded %ld of %d\n", k, worst[k],
                    worst[k] > 0 ? std::log2(worst[k]) : -999.0, not_cr[k], n);
    return 0;
}
