// Host round-trip latency on one stream (round 5): a tiny kernel writing 64 counters, their copy to host memory and
// a stream synchronize, repeated; pageable vs pinned destination, and the device's default vs spin scheduling.
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/sync.hip -o /tmp/sync && /tmp/sync [spin]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_count(unsigned* c, int n) {
    if (threadIdx.x < 64) c[threadIdx.x * 64] = threadIdx.x + n;
}

int main(int argc, char** argv) {
    if (argc > 1 && !std::strcmp(argv[1], "spin")) hipSetDeviceFlags(hipDeviceScheduleSpin);
    if (argc > 1 && !std::strcmp(argv[1], "yield")) hipSetDeviceFlags(hipDeviceScheduleYield);
    hipSetDevice(0);
    unsigned* d = nullptr;
    hipMalloc(&d, 64 * 64 * sizeof(unsigned));
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<unsigned> pageable(64 * 64);
    unsigned* pinned = nullptr;
    hipHostMalloc(&pinned, 64 * 64 * sizeof(unsigned), hipHostMallocDefault);
    for (int mode = 0; mode < 3; ++mode) {
        const int reps = 2000;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            hipLaunchKernelGGL(k_count, dim3(1), dim3(64), 0, s, d, i);
            if (mode == 0) hipMemcpyAsync(pageable.data(), d, 64 * 64 * sizeof(unsigned), hipMemcpyDeviceToHost, s);
            if (mode == 1) hipMemcpyAsync(pinned, d, 64 * 64 * sizeof(unsigned), hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
        }
        auto t1 = std::chrono::steady_clock::now();
        std::printf("%s %s: %.2f us per kernel + copy + sync\n", argc > 1 ? argv[1] : "default",
                    mode == 0 ? "pageable" : mode == 1 ? "pinned" : "no copy",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
    }
    return 0;
}
