// Device-scope atomics microbenchmark (MI355X): one atomicAdd per wave (lane 0) for 2M lanes,
// (a) all waves on one counter, (b) spread over 16 counters on separate 256-byte lines,
// (c) returning vs non-returning, (d) one per 256-thread block.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool kRet>
__global__ void k(unsigned long long* c, int spread, unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        unsigned long long* p = c + 32 * ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % spread);
        if (kRet) {
            unsigned long long v = atomicAdd(p, 1ull);
            if (v == 0xffffffffffffull) sink[0] = v;
        } else {
            atomicAdd(p, 1ull);
        }
    }
}
__global__ void kblock(unsigned long long* c) {
    if (threadIdx.x == 0) atomicAdd(c, 1ull);
}
int main() {
    unsigned long long *c, *sink;
    hipMalloc(&c, 64 * 32 * sizeof(unsigned long long));
    hipMalloc(&sink, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    const int blocks = (2 << 20) / 256;
    for (int rep = 0; rep < 2; ++rep) {
        for (int spread : {1, 16, 64}) {
            hipEventRecord(a);
            k<true><<<blocks, 256>>>(c, spread, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            printf("returning     spread=%2d  %d atomics  %.3f ms\n", spread, blocks * 4, ms);
            hipEventRecord(a);
            k<false><<<blocks, 256>>>(c, spread, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            printf("non-returning spread=%2d  %d atomics  %.3f ms\n", spread, blocks * 4, ms);
        }
        hipEventRecord(a);
        kblock<<<blocks, 256>>>(c);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("per block (non-returning, one counter)  %d atomics  %.3f ms\n", blocks, ms);
    }
    return 0;
}
