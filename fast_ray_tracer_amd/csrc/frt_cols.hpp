// frt-mi355x column-major record arrays for the per-path-node / per-sample
// buffers of the wavefront engine.
//
// A record of W 8-byte words is stored as W columns: word f of record i at
// w[f * cap + i]. The lanes of a wave handle consecutive records, so each
// word they load or store is one contiguous 512-byte run instead of 64
// scattered pieces of 64 different cache lines (the array-of-structs layout
// made every 216-byte NodeRec store 27 separate L2 requests per lane).
#pragma once

#include "frt_math.hpp"

namespace frt {

template <class T>
struct Cols {
    static_assert(sizeof(T) % 8 == 0, "records of whole 8-byte words");
    static constexpr int kWords = (int)(sizeof(T) / 8);
    uint64_t* w = nullptr;
    int64_t cap = 0;  // records per column

    __device__ __forceinline__ void store(int64_t i, const T& v) const {
        uint64_t t[kWords];
        __builtin_memcpy(t, &v, sizeof(T));
#pragma unroll
        for (int f = 0; f < kWords; ++f) w[f * cap + i] = t[f];
    }
    // loads every word; the ones a kernel does not use are dead and dropped
    __device__ __forceinline__ T load(int64_t i) const {
        uint64_t t[kWords];
#pragma unroll
        for (int f = 0; f < kWords; ++f) t[f] = w[f * cap + i];
        T v;
        __builtin_memcpy(&v, t, sizeof(T));
        return v;
    }
    static size_t bytes(int64_t cap) { return (size_t)cap * sizeof(T); }
};

// an (ambient, diffuse, specular) ColorTriple (color.h:5) without the unused
// fourth channel; kernels work on the 12-double form (channel 3 of each = 0)
struct Tri9 {
    double v[9];
};

__device__ __forceinline__ void tri_store(const Cols<Tri9>& c, int64_t i, const double* col12) {
    Tri9 t;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        t.v[k] = col12[k];
        t.v[3 + k] = col12[4 + k];
        t.v[6 + k] = col12[8 + k];
    }
    c.store(i, t);
}

__device__ __forceinline__ void tri_load(const Cols<Tri9>& c, int64_t i, double* col12) {
    const Tri9 t = c.load(i);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        col12[k] = t.v[k];
        col12[4 + k] = t.v[3 + k];
        col12[8 + k] = t.v[6 + k];
    }
    col12[3] = col12[7] = col12[11] = 0.0;
}

}  // namespace frt
