// frt-mi355x shadow pass pieces shared by the engine's k_shadow and the
// scene-specialised shadow kernels generated at upload (frt_jit.cpp): the
// per-(path node, light sample) lane setup of is_shadowed (renderer.c:74-93)
// and the segmented reduction of unshadowed counts.
#pragma once

#include "frt_traverse.hpp"

namespace frt {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

// area-light cache row for (path node, light, draw): the reference draws
// rand() % cache_len twice per (hit, light) (light.c:196, renderer.c:915);
// with a single-row cache both are row 0, as in the reference
__device__ __forceinline__ int light_row_n(int rows, uint64_t seed, uint64_t key, int light, int draw) {
    if (rows <= 1) return 0;
    uint64_t h = mix64(seed ^ mix64(key * 0x9e3779b97f4a7c15ULL + (uint64_t)(light * 2 + draw + 1)));
    return (int)(h % (uint64_t)rows);
}

__device__ __forceinline__ int light_row(const frt_light& L, uint64_t seed, uint64_t key, int light, int draw) {
    return light_row_n(L.rows, seed, key, light, draw);
}

// Ray queues of the levels are segmented: a block appends to segment
// blockIdx % kQueueSegs through that segment's own counter (one per 256-byte
// line), because device-scope atomics on one address serialise (~12 ns each:
// tools/microbench/atomics.hip). Segment j of a level's queue holds entries
// [qprefix[j], qprefix[j+1]) of the level at j * qsegcap + (i - qprefix[j]).
constexpr int kQueueSegs = 64;
constexpr int kCounterLine = 32;  // 8-byte words per counter line (256 bytes)

struct Batch {
    int64_t sample_begin;  // first global sample index of the batch
    int64_t pixel_begin;   // first pixel (in render order) of the batch
    int64_t num_samples;
    int64_t row_begin, row_stride;
    uint64_t seed;
    int32_t spp, level;
    int32_t remaining;     // path_length - level
    int32_t stats;         // the frame collects statistics (frt_frame_stats): the diagnostic counters are counted
    const int64_t* qprefix;  // this level's queue segments (kQueueSegs + 1 prefix counts); null: contiguous
    int64_t qsegcap;         // entries per segment of this level's queue
    int64_t next_segcap;     // entries per segment of the next level's queue
    const uint32_t* qperm;   // the level's entries in parent order: entry i at storage slot qperm[i]; null: the segments
};

// storage slot of entry i of the level's queue
__device__ __forceinline__ int64_t queue_slot(const Batch& B, int64_t i) {
    if (B.qperm != nullptr) return B.qperm[i];
    if (B.qprefix == nullptr) return i;
    int lo = 0, hi = kQueueSegs;  // the last segment j with qprefix[j] <= i
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (B.qprefix[mid] <= i) lo = mid;
        else hi = mid;
    }
    return (int64_t)lo * B.qsegcap + (i - B.qprefix[lo]);
}

// what the shadow pass reads of a path node, 40 bytes per node (the pass re-reads it from 100 lanes;
// keeping it apart from the path-node columns keeps its HBM traffic at about one line per node, and the
// unpadded record keeps k_prepare's writes of it at 40 bytes: a wave stores 20 whole lines)
struct alignas(8) ShadowHead {
    double over_point[3];
    uint64_t key;
    int32_t material;  // -1: the ray missed
    int32_t pad;
};
static_assert(sizeof(ShadowHead) == 40, "ShadowHead layout");

// one lane per (path node, light sample j); lanes of a node are consecutive
struct ShadowLane {
    Ray r;
    double distance;
    int64_t node;
    int light;
    bool valid;  // tid < n * samples_per_node
    bool live;   // the node has a hit to shade
};

__device__ __forceinline__ void shadow_lane(const DevScene& S, const Batch& B, const ShadowHead* __restrict__ shead,
                                            int64_t n, const int32_t* __restrict__ j_light,
                                            const int32_t* __restrict__ j_point, int32_t samples_per_node,
                                            int64_t tid, ShadowLane& L) {
    L.valid = tid >= 0 && tid < n * samples_per_node;
    L.node = 0;
    L.light = 0;
    L.live = false;
    L.r = Ray{{0, 0, 0}, {0, 0, 1}};
    L.distance = 0.0;
    if (L.valid) {
        L.node = tid / samples_per_node;
        const int j = (int)(tid % samples_per_node);
        L.light = j_light[j];
        const int pt = j_point[j];
        const ShadowHead* nr = shead + L.node;
        if (nr->material >= 0) {
            L.live = true;
            const frt_light& lt = S.lights[L.light];
            const int row = light_row(lt, B.seed, nr->key, L.light, 0);
            const double* lp = S.light_points + lt.points + 3 * ((int64_t)row * lt.num_samples + pt);
            // is_shadowed (renderer.c:74-93)
            double v[3] = {lp[0] - nr->over_point[0], lp[1] - nr->over_point[1], lp[2] - nr->over_point[2]};
            L.distance = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            L.r.o[0] = nr->over_point[0];
            L.r.o[1] = nr->over_point[1];
            L.r.o[2] = nr->over_point[2];
            normalize3(v, L.r.d);
        }
    }
}

// segmented wave reduction: lanes with the same (node, light) are contiguous;
// one integer atomic per segment
__device__ __forceinline__ void shadow_count(const DevScene& S, const ShadowLane& L, bool lit, int32_t* counts) {
    const int lane = threadIdx.x & 63;
    const int64_t key = L.valid ? L.node * S.num_lights + L.light : -1 - (int64_t)lane;
    const int64_t prev = __shfl_up(key, 1, 64);
    const bool head = lane == 0 || prev != key;
    const unsigned long long heads = __ballot(head);
    const unsigned long long lits = __ballot(lit);
    if (L.valid && head) {
        const unsigned long long above = lane == 63 ? 0ull : (heads >> (lane + 1)) << (lane + 1);
        const int next = above ? __ffsll((long long)above) - 1 : 64;
        const unsigned long long seg = (next >= 64 ? ~0ull : ((1ull << next) - 1)) & ~((1ull << lane) - 1);
        const int c = __popcll(lits & seg);
        if (c) atomicAdd(counts + key, c);
    }
}

}  // namespace frt
