// Store-pattern microbenchmark (MI355X): 27 doubles per lane written as
//   (a) 27 columns of `cap` records (column-major, the engine's Cols layout)
//   (b) one 216-byte record per lane (array of structs)
// for n = 2M lanes, plus (c) (a) with a dependent global load chain before the stores.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void cols(double* w, long cap, long n, const double* in) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = in ? in[i] : (double)i;
#pragma unroll
    for (int f = 0; f < 27; ++f) w[f * cap + i] = x + f;
}
__global__ void aos(double* w, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = (double)i;
#pragma unroll
    for (int f = 0; f < 27; ++f) w[i * 27 + f] = x + f;
}
__global__ void chain(const int* idx, long n, int hops, double* out) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int j = (int)(i & 1023);
    for (int h = 0; h < hops; ++h) j = idx[j];
    out[i] = j;
}
int main() {
    const long n = 2 << 20, cap = 4 << 20;
    double* w;
    hipMalloc(&w, 27 * cap * sizeof(double));
    int* idx;
    hipMalloc(&idx, 1024 * sizeof(int));
    int h_idx[1024];
    for (int k = 0; k < 1024; ++k) h_idx[k] = (k * 37 + 11) & 1023;
    hipMemcpy(idx, h_idx, sizeof(h_idx), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        cols<<<n / 256, 256>>>(w, cap, n, nullptr);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("cols  cap=4M  %.3f ms  %.0f GB/s\n", ms, 27 * 8.0 * n / ms / 1e6);
        hipEventRecord(a);
        cols<<<n / 256, 256>>>(w, n, n, nullptr);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("cols  cap=n   %.3f ms  %.0f GB/s\n", ms, 27 * 8.0 * n / ms / 1e6);
        hipEventRecord(a);
        aos<<<n / 256, 256>>>(w, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("aos           %.3f ms  %.0f GB/s\n", ms, 27 * 8.0 * n / ms / 1e6);
        for (int hops : {1, 4, 16}) {
            hipEventRecord(a);
            chain<<<n / 256, 256>>>(idx, n, hops, w);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            printf("chain hops=%2d %.3f ms\n", hops, ms);
        }
    }
    return 0;
}
