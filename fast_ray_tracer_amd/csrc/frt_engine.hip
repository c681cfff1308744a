// frt-mi355x render engine: wavefront kernels + the C ABI of include/frt_device.h.
//
// The reference's per-sample recursion color_at -> shade_hit -> {lights,
// reflected_color, refracted_color} (renderer.c:348-827) is unrolled into
// depth levels. For one batch of camera samples:
//
//   k_trace    (level d)  camera ray (d = 0) or queued ray -> closest hit
//                         (ordered BVH/CSG walk, per-lane state in LDS)
//   k_prepare  (level d)  prepare_computations, spawn reflection /
//                         refraction rays into queue d+1
//   k_shadow   (level d)  one lane per (hit, light sample): ordered any-hit
//                         walk; unshadowed counts reduced per wave, one
//                         integer atomic per (hit, light) segment
//   k_shade    (level d)  lighting_microfacet over the light's point row
//   k_combine  (d = D..0) bottom-up: surface + reflected*refl + refracted*Tf*d
//                         with the reference's schlick / dissolve order,
//                         written into the parent's fixed child slot
//   k_resolve             per pixel: ordered sum over (v,u) samples, /total,
//                         (A+D+S)/3
//
// Children write into fixed parent slots and shadow counts are integers, so
// the image is independent of wave scheduling. Zero-weight secondary rays
// (refraction through opaque surfaces, Tf = 0: 94-100 % of the reference's
// secondary rays) are not traced; their contribution is an exact 0.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "frt_device.h"
#include "frt_jit.h"
#include "frt_shade.hpp"
#include "frt_shadow.hpp"
#include "frt_jit_rt.hpp"
#include "frt_camera.hpp"
#include "frt_cols.hpp"

namespace frt {

constexpr int kBlock = 256;
constexpr int kMaxPathLength = 11;  // 12-bit heap code of a path node in its key (k_prepare)

// path-node record of one level; node i of level d belongs to queued ray i
struct NodeRec {
    double over_point[3];
    uint64_t key;     // (global sample << 12) | heap code of the path node
    int32_t material; // -1: the ray missed
    int32_t parent;   // node index in level d-1 (-1 at level 0)
    int32_t slot;     // 0 = reflected child, 1 = refracted child
    int32_t flags;    // bit0 reflect applies, bit1 refract applies, bit2 schlick mix, bit3 dissolve
    double normalv[3];
    double eyev[3];
    double Ka[3], Kd[3], Ks[3];
    double refl[3];
    double Ns, over_d, rf;
};
static_assert(sizeof(NodeRec) == 216, "NodeRec layout");

// NodeRec in HBM: the fields every path node needs (10 column words), its over_point and key from the
// node's ShadowHead (which k_prepare writes for the shadow pass anyway: no second copy), and its material
// colours (13 words), which k_prepare stores only for materials with patterns on them (kOwnColors; every
// other reader takes them from the material table): the colours of pattern-free materials are never
// written or read per node, and a missed ray writes only its material / parent / slot words. Words that a
// node's flags or its level make constant are not written either: parent / slot at level 0 (-1, 0), over_d
// unless a pattern sets it (kOwnD; else the material's 1 - Tr, as prepare computes it), the Schlick factor
// unless kMix (else 0).
struct NodeCore {
    int32_t material, flags, parent, slot;
    double normalv[3], eyev[3];
    double over_d, rf;
};
struct NodeColors {
    double Ka[3], Kd[3], Ks[3], refl[3];
    double Ns;
};
static_assert(sizeof(NodeCore) == 80 && sizeof(NodeColors) == 104, "NodeCols layout");
// k*Spawned: the child ray was queued (its k_combine writes the parent's slot; otherwise the slot reads as 0)
enum NodeFlags : int32_t { kReflApplies = 1, kRefrApplies = 2, kMix = 4, kDissolve = 8, kReflSpawned = 16, kRefrSpawned = 32 };
enum : int32_t { kOwnColors = 64, kOwnD = 128 };  // (NodeFlags bits) the node's colours / over_d are in NodeCols

struct NodeCols {
    Cols<NodeCore> core;
    Cols<NodeColors> col;
    const ShadowHead* head = nullptr;  // over_point, key (the level's ShadowHead array)
    int32_t root = 0;                  // level 0: parent / slot are -1 / 0 and not stored
    // level 0 of a scene without GI: eyev is the camera ray's direction negated, which its one reader (shade_node,
    // through camera_eyev) recomputes from the node's sample; its 24 bytes per node are not stored
    int32_t eye_cam = 0;
    static size_t bytes(int64_t cap) { return Cols<NodeCore>::bytes(cap) + Cols<NodeColors>::bytes(cap); }
    void set(uint64_t* base, int64_t cap) {  // (host) one allocation of bytes(cap)
        core.w = base;
        core.cap = cap;
        col.w = base + (size_t)Cols<NodeCore>::kWords * cap;
        col.cap = cap;
    }
    __device__ __forceinline__ void store(int64_t i, const NodeRec& v, bool own_colors, bool own_d) const {
        NodeCore c;
        for (int k = 0; k < 3; ++k) {
            c.normalv[k] = v.normalv[k];
            c.eyev[k] = v.eyev[k];
        }
        c.material = v.material;
        c.parent = v.parent;
        c.slot = v.slot;
        c.flags = v.flags | (own_colors ? kOwnColors : 0) | (own_d ? kOwnD : 0);
        c.over_d = v.over_d;
        c.rf = v.rf;
        uint64_t t[10];
        __builtin_memcpy(t, &c, sizeof(c));
        const int64_t cap = core.cap;
        core.w[i] = t[0];
        if (!root) core.w[cap + i] = t[1];
#pragma unroll
        for (int f = 2; f < 5; ++f) core.w[f * cap + i] = t[f];
        if (!eye_cam) {
#pragma unroll
            for (int f = 5; f < 8; ++f) core.w[f * cap + i] = t[f];
        }
        if (own_d) core.w[8 * cap + i] = t[8];
        if (c.flags & kMix) core.w[9 * cap + i] = t[9];
        if (own_colors) {
            NodeColors o;
            for (int k = 0; k < 3; ++k) {
                o.Ka[k] = v.Ka[k];
                o.Kd[k] = v.Kd[k];
                o.Ks[k] = v.Ks[k];
                o.refl[k] = v.refl[k];
            }
            o.Ns = v.Ns;
            col.store(i, o);
        }
    }
    // a missed ray: material -1 with its parent and slot (the words k_combine reads)
    __device__ __forceinline__ void store_miss(int64_t i, int32_t parent, int32_t slot) const {
        core.w[i] = (uint64_t)(uint32_t)-1;  // (flags 0)
        if (!root) core.w[core.cap + i] = (uint64_t)(uint32_t)parent | ((uint64_t)(uint32_t)slot << 32);
    }
    __device__ __forceinline__ NodeRec load(int64_t i, const frt_material* __restrict__ mats) const {
        uint64_t t[10];
        const int64_t cap = core.cap;
        t[0] = core.w[i];
        t[1] = root ? (uint64_t)(uint32_t)-1 : core.w[cap + i];
#pragma unroll
        for (int f = 2; f < 5; ++f) t[f] = core.w[f * cap + i];
#pragma unroll
        for (int f = 5; f < 8; ++f) t[f] = eye_cam ? 0ull : core.w[f * cap + i];  // (eye_cam: camera_eyev)
        const int32_t mat = (int32_t)(uint32_t)t[0], fl = (int32_t)(t[0] >> 32);
        const double od = (fl & kOwnD) ? __longlong_as_double((long long)core.w[8 * cap + i])
                          : mat >= 0 ? 1.0 - mats[mat].Tr : 0.0;
        const double rf = (fl & kMix) ? __longlong_as_double((long long)core.w[9 * cap + i]) : 0.0;
        t[8] = (uint64_t)__double_as_longlong(od);
        t[9] = (uint64_t)__double_as_longlong(rf);
        NodeCore c;
        __builtin_memcpy(&c, t, sizeof(c));
        NodeRec v;
        const ShadowHead& hd = head[i];  // (dead, and not loaded, where a kernel uses neither field)
        for (int k = 0; k < 3; ++k) {
            v.over_point[k] = hd.over_point[k];
            v.normalv[k] = c.normalv[k];
            v.eyev[k] = c.eyev[k];
        }
        v.key = hd.key;
        v.material = c.material;
        v.parent = c.parent;
        v.slot = c.slot;
        v.flags = c.flags;
        v.over_d = c.over_d;
        v.rf = c.rf;
        if (c.material < 0) {
            for (int k = 0; k < 3; ++k) v.Ka[k] = v.Kd[k] = v.Ks[k] = v.refl[k] = 0.0;
            v.Ns = 0.0;
        } else if (c.flags & kOwnColors) {
            const NodeColors o = col.load(i);
            for (int k = 0; k < 3; ++k) {
                v.Ka[k] = o.Ka[k];
                v.Kd[k] = o.Kd[k];
                v.Ks[k] = o.Ks[k];
                v.refl[k] = o.refl[k];
            }
            v.Ns = o.Ns;
        } else {
            const frt_material& M = mats[c.material];
            for (int k = 0; k < 3; ++k) {
                v.Ka[k] = M.Ka[k];
                v.Kd[k] = M.Kd[k];
                v.Ks[k] = M.Ks[k];
                v.refl[k] = M.refl[k];
            }
            v.Ns = M.Ns;
        }
        return v;
    }
};










extern __shared__ __align__(16) char frt_walk_smem[];

// closest hit of every ray of one level (level 0: camera rays generated in place)
// (waves per SIMD asked of the compiler: 4 fit the walk without the torus's quartic in 128 VGPRs without
// spills, measured 10.1 -> 8.7 ms per headline frame over the compiler's own 3; the torus variants keep theirs)
#ifndef FRT_TRACE_WAVES
#define FRT_TRACE_WAVES 4
#endif
template <int kFeat>
__global__ void __launch_bounds__(kTraceBlock)
__attribute__((amdgpu_waves_per_eu((kFeat & kFeatTorus) ? 1 : FRT_TRACE_WAVES, 8))) k_trace(DevScene S, Batch B, const QueuedRay* __restrict__ q, int64_t n,
                                                       HitRec* __restrict__ hits, double* __restrict__ hn12, unsigned* err,
                                                       int filter_casts) {
    // every lane of the wave takes part in the (wave-coherent) walk; queued rays with
    // parent < -1 are placeholders (final-gather slots of nodes without a gather)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n && (q == nullptr || q[queue_slot(B, i)].parent >= -1);
    Ray r{{0, 0, 0}, {0, 0, 1}};
    unsigned e = 0;
    if (live) {
        if (q == nullptr) {
            uint64_t key;
            camera_ray(S, B, i, r, key, e);
        } else {
            const QueuedRay& qr = q[queue_slot(B, i)];
            for (int k = 0; k < 3; ++k) {
                r.o[k] = qr.o[k];
                r.d[k] = qr.d[k];
            }
        }
    }
    double t;
    double n12[2];
    const int node = walk<false, kFeat>(S, r, 0.0, live, t, frt_walk_smem, e, n12, filter_casts != 0);
    if (i < n) {
        hits[i] = live ? HitRec{t, node, 0} : HitRec{0.0, -1, 0};
        if (hn12 != nullptr) {
            hn12[2 * i] = live ? n12[0] : 1.0;
            hn12[2 * i + 1] = live ? n12[1] : 1.0;
        }
    }
    if (e) atomicOr(err, e);
}

// the rays frt_jit_trace (frt_jit.hip) could not settle in binary32: the generic walk, grid-stride over the list
// (whole waves per step, as k_shadow_redo)
template <int kFeat>
__global__ void __launch_bounds__(kTraceBlock) k_trace_redo(DevScene S, Batch B, const QueuedRay* __restrict__ q, int64_t n,
                                                            HitRec* __restrict__ hits, unsigned* err,
                                                            const int32_t* __restrict__ redo,
                                                            const unsigned* __restrict__ redo_count, unsigned redo_cap) {
    const unsigned cnt = min(*redo_count, redo_cap);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned e = 0;
    for (int64_t base = wave * 64; base < (int64_t)cnt; base += nwaves * 64) {
        const int64_t k = base + (threadIdx.x & 63);
        const int64_t i = k < (int64_t)cnt ? (int64_t)redo[k] : -1;
        const bool live = i >= 0 && i < n;
        Ray r{{0, 0, 0}, {0, 0, 1}};
        if (live) {
            if (q == nullptr) {
                uint64_t key;
                camera_ray(S, B, i, r, key, e);
            } else {
                const QueuedRay& qr = q[queue_slot(B, i)];
                for (int a = 0; a < 3; ++a) {
                    r.o[a] = qr.o[a];
                    r.d[a] = qr.d[a];
                }
            }
        }
        double t;
        double n12[2];
        const int node = walk<false, kFeat>(S, r, 0.0, live, t, frt_walk_smem, e, n12, false);
        if (live) hits[i] = HitRec{t, node, 0};  // (every refractive index is one where this runs: no n12)
    }
    if (e) atomicOr(err, e);
}

// prepare_computations + spawn of the reflection / refraction rays (renderer.c:369-605)
#ifndef FRT_PREPARE_WAVES
#define FRT_PREPARE_WAVES 1
#endif
// (one path node; returns whether it has a hit, its over_point in op)
template <bool kPat>
__device__ __forceinline__ bool prepare_node(const DevScene& S, const Batch& B, const QueuedRay* __restrict__ q,
                                             int64_t n, const HitRec* __restrict__ hits, const double* __restrict__ hn12,
                                             NodeCols& rec,
                                             ShadowHead* __restrict__ heads, QueuedRay* __restrict__ next_q,
                                             unsigned long long* counters, unsigned* err, int64_t node, double* op,
                                             int* spawned = nullptr) {
    // this block's counter line: next-level queue segment count (word level + 1), pruned (16), hits (17)
    unsigned long long* line = counters + kCounterLine * (blockIdx.x % kQueueSegs);
    const int64_t seg_base = (int64_t)(blockIdx.x % kQueueSegs) * B.next_segcap;
#ifdef FRT_WALK_PROF
    unsigned long long pt0 = prof_stamp();
    auto pstamp = [&](int k) {
        const unsigned long long t1 = prof_stamp();
        if ((threadIdx.x & 63) == 0) atomicAdd(S.dbg + kDbgProf + 8 + k, t1 - pt0);
        pt0 = t1;
    };
#define PSTAMP(k) pstamp(k)
#else
#define PSTAMP(k)
#endif
    Ray r;
    uint64_t key;
    int32_t parent = -1, slot = 0;
    if (q == nullptr) {
        unsigned ce = 0;
        camera_ray(S, B, node, r, key, ce);
    } else {
        const QueuedRay& qr = q[queue_slot(B, node)];
        for (int k = 0; k < 3; ++k) {
            r.o[k] = qr.o[k];
            r.d[k] = qr.d[k];
        }
        key = qr.key;
        parent = qr.parent;
        slot = qr.slot;
    }
    PSTAMP(0);
    const HitRec hr = hits[node];
    PSTAMP(1);
    if (hr.node < 0) {
        rec.store_miss(node, parent, slot);
        heads[node].material = -1;
        return false;
    }
    Hit h{hr.t, -1, -1, hr.node};
    Comps c;
    prepare<kPat>(S, r, h, c);
    c.n1 = hn12 != nullptr ? hn12[2 * node] : 1.0;
    c.n2 = hn12 != nullptr ? hn12[2 * node + 1] : 1.0;
    PSTAMP(2);
    if (B.stats) wave_count(line + 17, true);  // shaded path nodes (statistics frames only: an atomic per wave)
    const frt_material& M = S.materials[c.material];
    NodeRec nr;
    for (int k = 0; k < 3; ++k) {
        nr.over_point[k] = c.over_point[k];
        nr.normalv[k] = c.normalv[k];
        nr.eyev[k] = c.eyev[k];
        nr.Ka[k] = c.Ka[k];
        nr.Kd[k] = c.Kd[k];
        nr.Ks[k] = c.Ks[k];
        nr.refl[k] = c.refl[k];
    }
    nr.Ns = c.Ns;
    nr.over_d = c.over_d;
    nr.rf = 0.0;
    nr.key = key;
    nr.material = c.material;
    nr.parent = parent;
    nr.slot = slot;
    int32_t flags = 0;
    if (S.cfg.include_specular) {
        const bool reflect_applies = B.remaining > 0 && M.reflective;
        bool refract_applies = false;
        double refr_dir[3] = {0, 0, 0};
        if (B.remaining > 0 && c.over_d > 0.0) {  // refracted_color (renderer.c:535-573)
            double n_ratio = c.n1 / c.n2;
            double cos_i = dot3(c.eyev, c.normalv);
            double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
            if (!(sin2_t > 1.0)) {
                refract_applies = true;
                double cos_t = sqrt(1.0 - sin2_t);
                double s1 = n_ratio * cos_i - cos_t;
                for (int k = 0; k < 3; ++k) {
                    double t1 = c.normalv[k] * s1;
                    double t2 = c.eyev[k] * n_ratio;
                    refr_dir[k] = t1 - t2;
                }
            }
        }
        if (reflect_applies) flags |= kReflApplies;
        if (refract_applies) flags |= kRefrApplies;
        if (M.reflective && c.over_d < 1.0) {
            flags |= kMix;
            nr.rf = schlick(c.eyev, c.normalv, c.n1, c.n2);
        }
        if (M.Tr > 0.0 && c.over_d > 0.0) flags |= kDissolve;

        const uint64_t code = key & 0xFFFull;
        const uint64_t base = key & ~0xFFFull;
        // spawn only children whose weight can be non-zero (zero-weight subtrees add exactly 0)
        const bool want_refl = reflect_applies && (c.refl[0] != 0.0 || c.refl[1] != 0.0 || c.refl[2] != 0.0);
        const bool tf_zero = M.Tf[0] == 0.0 && M.Tf[1] == 0.0 && M.Tf[2] == 0.0;
        const bool want_refr = refract_applies && !tf_zero;
        if (want_refl) flags |= kReflSpawned;
        if (want_refr) flags |= kRefrSpawned;
        // slots in this block's segment of the next level's queue; dense (spawned != nullptr): the fixed slots
        // node (reflected) and n + node (refracted), no atomics, the caller records which are taken
        const bool dense = spawned != nullptr;
        const unsigned long long at_refl = dense ? 0ull : wave_append(line + B.level + 1, want_refl);
        const unsigned long long at_refr = dense ? 0ull : wave_append(line + B.level + 1, want_refr);
        if (dense) *spawned = (want_refl ? 1 : 0) | (want_refr ? 2 : 0);
        if (B.stats) {  // pruned zero-weight rays (statistics frames only)
            wave_count(line + 16, reflect_applies && !want_refl);
            wave_count(line + 16, refract_applies && !want_refr);
        }
        if (want_refl) {
            if (dense || (int64_t)at_refl < B.next_segcap) {
                QueuedRay qo;
                for (int k = 0; k < 3; ++k) {
                    qo.o[k] = c.over_point[k];
                    qo.d[k] = c.reflectv[k];
                }
                qo.key = base | ((code * 2) & 0xFFFull);
                qo.parent = (int32_t)node;
                qo.slot = 0;
                next_q[dense ? node : seg_base + (int64_t)at_refl] = qo;
            } else {
                atomicOr(err, kErrQueueOverflow);
            }
        }
        if (want_refr) {
            if (dense || (int64_t)at_refr < B.next_segcap) {
                QueuedRay qo;
                for (int k = 0; k < 3; ++k) {
                    qo.o[k] = c.under_point[k];
                    qo.d[k] = refr_dir[k];
                }
                qo.key = base | ((code * 2 + 1) & 0xFFFull);
                qo.parent = (int32_t)node;
                qo.slot = 1;
                next_q[dense ? n + node : seg_base + (int64_t)at_refr] = qo;
            } else {
                atomicOr(err, kErrQueueOverflow);
            }
        }
    }
    nr.flags = flags;
    PSTAMP(3);
    // the colours per node only where a pattern makes them vary (prepare: map_Ka / Kd / Ks / refl / Ns)
    const bool own = kPat && (M.map_Ka >= 0 || M.map_Kd >= 0 || M.map_Ks >= 0 || M.map_refl >= 0 || M.map_Ns >= 0);
    rec.store(node, nr, own, kPat && M.map_d >= 0);
    ShadowHead hd;
    for (int k = 0; k < 3; ++k) hd.over_point[k] = c.over_point[k];
    hd.key = key;
    hd.material = c.material;
    hd.pad = 0;
    heads[node] = hd;
    PSTAMP(4);
    for (int k = 0; k < 3; ++k) op[k] = c.over_point[k];
    return true;
}

// the box of the over_points of a tile's path nodes (tile_log2 of them, consecutive lanes of one wave), rounded
// outward to binary32, for frt_jit_tile (frt_jit_rt.hpp beam_box32); a tile without hits gets an empty box
// (stbox: the boxes of the tile's sub-tiles of 2^sub_log2 nodes as well, for frt_jit_subtile)
__device__ __forceinline__ void tile_box(int64_t node, int64_t n, bool hit, const double* op, float* __restrict__ tbox,
                                         int tile_log2, float* __restrict__ stbox, int sub_log2) {
    float lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = hit ? __double2float_rd(op[a]) : __builtin_huge_valf();
        hi[a] = hit ? __double2float_ru(op[a]) : -__builtin_huge_valf();
    }
    for (int off = 1; off < (1 << tile_log2); off <<= 1) {
        if (stbox != nullptr && off == (1 << sub_log2) && node < n && (node & (off - 1)) == 0) {
            float* b = stbox + 6 * (node >> sub_log2);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                b[a] = lo[a];
                b[a + 3] = hi[a];
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], off, 64));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off, 64));
        }
    }
    if (node < n && (node & ((1 << tile_log2) - 1)) == 0) {
        float* b = tbox + 6 * (node >> tile_log2);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            b[a] = lo[a];
            b[a + 3] = hi[a];
        }
    }
}

template <bool kPat>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kPat ? 1 : FRT_PREPARE_WAVES, 8)))
k_prepare(DevScene S, Batch B, const QueuedRay* __restrict__ q, int64_t n, const HitRec* __restrict__ hits,
          const double* __restrict__ hn12,
          NodeCols rec, ShadowHead* __restrict__ heads, QueuedRay* __restrict__ next_q, unsigned long long* counters,
          unsigned* err, float* __restrict__ tbox, int tile_log2, float* __restrict__ stbox, int sub_log2,
          int32_t* __restrict__ counts, unsigned long long* __restrict__ spawn_masks) {
    const int64_t node = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double op[3] = {0.0, 0.0, 0.0};
    bool hit = false;
    // (the level's unshadowed counts start at 0: zeroed here, in the node's own coalesced words, instead of a
    // memset launch per level)
    if (node < n && counts != nullptr)
        for (int l = 0; l < S.num_lights; ++l) counts[node * S.num_lights + l] = 0;
    // (spawn_masks: the next level's queue dense, slot node / n + node taken; per wave of 64 nodes g the lanes'
    // reflected / refracted bits as masks g / G + g, G = the level's waves; every wave writes both, no clearing)
    int spawned = 0;
    if (node < n)
        hit = prepare_node<kPat>(S, B, q, n, hits, hn12, rec, heads, next_q, counters, err, node, op,
                                 spawn_masks != nullptr ? &spawned : nullptr);
    if (spawn_masks != nullptr) {  // (every lane of the wave is here)
        const unsigned long long mr = __ballot(spawned & 1), mt = __ballot((spawned >> 1) & 1);
        const int64_t g = node >> 6, G = (n + 63) >> 6;
        if ((threadIdx.x & 63) == 0 && g < G) {
            spawn_masks[g] = mr;
            spawn_masks[G + g] = mt;
        }
    }
    if (tbox != nullptr) tile_box(node, n, hit, op, tbox, tile_log2, stbox, sub_log2);
}

// one lane per (node, light sample j); lanes of a node are consecutive
#ifdef FRT_SHADOW_WAVES
#define FRT_SHADOW_ATTR __attribute__((amdgpu_waves_per_eu(FRT_SHADOW_WAVES, 8)))
#else
#define FRT_SHADOW_ATTR
#endif
template <int kFeat>
__global__ void __launch_bounds__(kTraceBlock) FRT_SHADOW_ATTR k_shadow(DevScene S, Batch B, const ShadowHead* __restrict__ shead, int64_t n,
                                                        const int32_t* __restrict__ j_light,
                                                        const int32_t* __restrict__ j_point, int32_t samples_per_node,
                                                        int32_t* __restrict__ counts, unsigned* err) {
    ShadowLane L;
    shadow_lane(S, B, shead, n, j_light, j_point, samples_per_node, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, L);
    // every lane of the wave takes part in the (wave-coherent) walk
    unsigned e = 0;
    double unused;
#ifdef FRT_EXPERIMENT_NOWALK
    const bool lit = L.live && L.distance > 0.5;
#else
    const bool lit = walk<true, kFeat>(S, L.r, L.distance, L.live, unused, frt_walk_smem, e) == 0 && L.live;
#endif
    if (e) atomicOr(err, e);
    shadow_count(S, L, lit, counts);
}

// lanes the scene-specialised shadow kernel (frt_jit.cpp) handed back — rays
// with non-finite components, which its decisions do not cover — through the
// generic walk; grid-stride over the queue, whole waves per step, one atomic per lit lane
template <int kFeat>
__global__ void __launch_bounds__(kTraceBlock) k_shadow_redo(DevScene S, Batch B, const ShadowHead* __restrict__ shead, int64_t n,
                                                             const int32_t* __restrict__ j_light,
                                                             const int32_t* __restrict__ j_point, int32_t samples_per_node,
                                                             int32_t* __restrict__ counts, unsigned* err,
                                                             const int64_t* __restrict__ redo,
                                                             const unsigned* __restrict__ redo_count, unsigned redo_cap) {
    const unsigned cnt = min(*redo_count, redo_cap);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned e = 0;
    for (int64_t base = wave * 64; base < (int64_t)cnt; base += nwaves * 64) {
        const int64_t k = base + (threadIdx.x & 63);
        ShadowLane L;
        shadow_lane(S, B, shead, n, j_light, j_point, samples_per_node, k < (int64_t)cnt ? redo[k] : -1, L);
        double unused;
        const bool lit = walk<true, kFeat>(S, L.r, L.distance, L.live, unused, frt_walk_smem, e) == 0 && L.live;
        if (lit) atomicAdd(counts + L.node * S.num_lights + L.light, 1);
    }
    if (e) atomicOr(err, e);
}

#ifndef FRT_SHADE_FACTOR
#define FRT_SHADE_FACTOR 1
#endif
#ifndef FRT_SHADE_ALG
#define FRT_SHADE_ALG 1
#endif
#ifndef FRT_SHADE_SKIP
#define FRT_SHADE_SKIP 1
#endif
// FRT_SHADE_FMA (default 1): the light point's three dot products (|v|^2, v.n, v.e) as one product and two fused
// multiply-adds instead of three products and two sums (each within an ulp of the separately rounded sum, like the
// Newton-refined estimates beside them); 0: the reference's separately rounded operations (A/B builds)
#ifndef FRT_SHADE_FMA
#define FRT_SHADE_FMA 1
#endif
__device__ __forceinline__ double dot3_shade(const double* a, const double* b) {
    if (FRT_SHADE_FMA) return __builtin_fma(a[0], b[0], __builtin_fma(a[1], b[1], a[2] * b[2]));
    return dot3(a, b);
}
// a level-0 node's eyev where the level does not store it (NodeCols::eye_cam): prepare_computations' negated ray
// direction (frt_shade.hpp prepare) of the node's camera ray, the same camera_ray k_prepare traced, bit for bit
__device__ __forceinline__ void camera_eyev(const DevScene& S, const Batch& B, int64_t i, double* eyev) {
    Ray r;
    uint64_t key;
    unsigned ce = 0;
    camera_ray(S, B, i, r, key, ce);
    for (int k = 0; k < 3; ++k) eyev[k] = r.d[k] * -1.0;
}

// lighting_microfacet (renderer.c:895-979) per light, summed as shade_hit does (renderer.c:704-725): the
// A, D, S triples of path node i into out (out[4k + c]: term k, channel c)
// (lds_row: k_shade_lit's per-wave LDS staging of a multi-row light's row, kLdsPoints points; nullptr elsewhere)
constexpr int kLdsPoints = 128;
// (c0 >= 0: the unshadowed count of a scene's one light, staged by the caller; counts[i] is then not read)
__device__ __forceinline__ void shade_node(const DevScene& S, const Batch& B, const NodeRec& nr, int64_t i,
                                           const int32_t* __restrict__ counts, double* out, double* lds_row = nullptr,
                                           int32_t c0 = -1) {
    double sA[3] = {0, 0, 0}, sD[3] = {0, 0, 0}, sS[3] = {0, 0, 0};
    if (S.cfg.include_direct) {
        for (int li = 0; li < S.num_lights; ++li) {
            const frt_light& L = S.lights[li];
            const int32_t cnt = c0 >= 0 ? c0 : counts[i * S.num_lights + li];
            double inten;
            if (L.type == FRT_AREA_LIGHT || L.type == FRT_CIRCLE_LIGHT) {
                inten = (double)cnt / (double)L.num_samples;  // light.c:229-242
            } else {
                inten = cnt ? 1.0 : 0.0;  // light.c:245-251
            }
            double amb[3], cA[3] = {0, 0, 0}, cD[3] = {0, 0, 0}, cS[3] = {0, 0, 0};
            for (int k = 0; k < 3; ++k) amb[k] = nr.Ka[k] * L.intensity[k];
            if (!feq(inten, 0.0)) {
                if (S.cfg.include_diffuse || S.cfg.include_spec_highlight) {
                    double ned = 0.0;
                    if (S.cfg.include_spec_highlight) ned = dot3(nr.normalv, nr.eyev);
                    double dacc[3] = {0, 0, 0}, sacc[3] = {0, 0, 0};
                    // The per-channel sums factored out of the point loop (FRT_SHADE_FACTOR=0 builds: per point
                    // and channel as the reference writes it, A/B runs) — the diffuse term
                    // sum_p Kd I (l.n) = Kd I sum_p (l.n), the specular one sum_p (Ks + (1 - Ks) F) I b =
                    // Ks I sum_p b + (1 - Ks) I sum_p F b — and the distribution term's constant (Ns + 2) / 2pi
                    // folded: three running sums instead of nine, the same terms in another association
                    // (relative differences of a few ulps per point, far inside the 1e-4 canvas tolerance)
                    constexpr bool kFactored = FRT_SHADE_FACTOR != 0;
                    double sum_ldn = 0.0, sum_b = 0.0, sum_fb = 0.0;
                    const double cdist = (nr.Ns + 2) * 0.5 * k1Pi;
                    // The light vector and the half vector by their shared terms (FRT_SHADE_ALG, default 1): with
                    // v = p - over_point, m2 = v.v and r = 1/|v|, lightv = v r, so lightv.n = (v.n) r and
                    // lightv.e = (v.e) r; the half vector h = (lightv + e) / |lightv + e| has |lightv + e|^2 =
                    // lightv.lightv + 2 lightv.e + e.e, and n.h, e.h, lightv.h are (n.lightv + n.e) / |..|,
                    // (lightv.e + e.e) / |..|, (lightv.lightv + lightv.e) / |..|: two dot products and a few
                    // multiplies per point instead of the normalised vectors and five dot products (a few ulps
                    // from vector_normalize's path, like the reciprocal estimates; ned = n.e is the node's).
                    // FRT_SHADE_ALG=0 builds: the vectors as the reference forms them (A/B runs).
                    constexpr bool kAlg = FRT_SHADE_ALG != 0;
                    const double ee = dot3(nr.eyev, nr.eyev);
                    // pow_ns's exponent test once per node (the same Ns for every point: pow_plan / pow_apply)
                    const double nsd = nr.Ns;
                    const PowPlan pplan = pow_plan(nsd);
                    // The specular tail (FRT_SHADE_SKIP, default 1): with Ns = 200 the lobe (n.h)^Ns is below 2^-60 of
                    // the point's diffuse term for most (node, point) pairs, yet every lane paid the reciprocal, the
                    // power and the quotient. A point's specular terms are at most (|Ks| + |1 - Ks|) I brdf per channel
                    // (F <= 1: 0 <= 1 - l.h <= 1), brdf <= cdist (n.h)^Ns / (4 (l.n) (n.e)) (G <= 1), and its diffuse
                    // term is Kd I (l.n); when cdist (n.h)^Ns < 2^-62 rK (l.n)^2 (n.e), rK = min_k Kd_k / (|Ks_k| +
                    // |1 - Ks_k|), the point's specular terms lie below 2^-62 of its diffuse ones and are left out
                    // (the node's colour moves by less than 2^-60 of itself; the Newton-refined estimates above are
                    // within 2^-46). Tested in binary32 logarithms with 4 binades of margin (the conversions and
                    // v_log_f32 are within 1e-4 of a binade at Ns <= 4096). Per lane: a lane's result does not
                    // depend on its wave; the arithmetic is skipped where every lane of the wave skips.
                    float skip_c = __builtin_huge_valf();  // log2(cdist / (rK (n.e))) + 62 + 4; +inf: never skip
                    if (FRT_SHADE_SKIP && kFactored && kAlg && S.cfg.include_diffuse && S.cfg.include_spec_highlight &&
                        nsd >= 2.0 && nsd <= 4096.0 && ned > 0x1p-100) {
                        double rk = 1.0;
                        for (int k = 0; k < 3; ++k) rk = fmin(rk, nr.Kd[k] / (fabs(nr.Ks[k]) + fabs(1.0 - nr.Ks[k])));
                        if (rk > 0x1p-100) skip_c = __log2f((float)(cdist / (rk * ned))) + 66.0f;
                    }
                    const float nsf = (float)nsd;
                    // one light point's terms (lp: the point)
                    auto term = [&](const double* lp) {
                        double diff[3] = {lp[0] - nr.over_point[0], lp[1] - nr.over_point[1], lp[2] - nr.over_point[2]};
                        double lv[3] = {0.0, 0.0, 0.0}, ldn, m2 = 0.0, rl = 0.0;
                        if (kAlg) {
                            m2 = dot3_shade(diff, diff);
                            rl = rsqrt_shade(m2);
                            ldn = dot3_shade(diff, nr.normalv) * rl;
                        } else {
                            normalize3_shade(diff, lv);
                            ldn = dot3(lv, nr.normalv);
                        }
                        if (S.cfg.include_diffuse && ldn >= 0.0) {
                            if (kFactored) {
                                sum_ldn += ldn;
                            } else {
                                for (int k = 0; k < 3; ++k) {
                                    double cc = nr.Kd[k] * L.intensity[k];
                                    cc *= ldn;
                                    dacc[k] += cc;
                                }
                            }
                        }
                        if (S.cfg.include_spec_highlight && ldn >= 0.0) {
                            double ndl, ndh, edh, ldh;
                            if (kAlg) {
                                ndl = ldn;
                                const double el = dot3_shade(diff, nr.eyev) * rl, ll = (m2 * rl) * rl;
                                const double rh = rsqrt_shade(ll + 2.0 * el + ee);
                                ndh = fmax(0.0, (ldn + ned) * rh);
                                edh = fmax(0.0, (el + ee) * rh);
                                ldh = (ll + el) * rh;
                                // (the specular tail test; NaN compares false: not skipped)
                                const bool tail = ldn > 0x1p-100 &&
                                                  nsf * __log2f((float)ndh) - 2.0f * __log2f((float)ldn) + skip_c < 0.0f;
                                if (__ballot(!tail) == 0ull) return;
                                if (tail) return;
                            } else {
                                ndl = dot3(nr.normalv, lv);
                                double tmp[3] = {lv[0] + nr.eyev[0], lv[1] + nr.eyev[1], lv[2] + nr.eyev[2]}, hv[3];
                                normalize3_shade(tmp, hv);
                                ndh = fmax(0.0, dot3(nr.normalv, hv));
                                edh = fmax(0.0, dot3(nr.eyev, hv));
                                ldh = dot3(lv, hv);
                            }
                            double dist_term = kFactored ? pow_apply(ndh, nsd, pplan) * cdist
                                                         : (nr.Ns + 2) * pow_ns(ndh, nr.Ns) * 0.5 * k1Pi;
                            // pow(1 - ldh, 5.0) (renderer.c:969) by squaring: within an ulp or two of the
                            // reference's libm pow, like the device pow it replaces
                            const double om = 1.0 - ldh, om2 = om * om;
                            double factor = om2 * om2 * om;
                            double brdf = brdf_shade(dist_term, ndh, edh, ndl, ned);
                            if (kFactored) {
                                sum_b += brdf;
                                sum_fb += factor * brdf;
                            } else {
                                for (int k = 0; k < 3; ++k) {
                                    double f = nr.Ks[k] + (1.0 - nr.Ks[k]) * factor;
                                    sacc[k] += f * L.intensity[k] * brdf;
                                }
                            }
                        }
                    };
                    // Two light points at a time (FRT_SHADE_PAIR=1 builds, off by default: k_shade_lit 8.85 -> 9.0 ms
                    // per headline frame with it, profiles/r06_ab_shade_pair.txt; the factored sums with the shared-term
                    // vectors): each point's terms are one long dependent chain (two reciprocal square roots with their
                    // Newton steps, the tail test's logarithms), and the per-point branches of the slow-path checks and
                    // of the tail test kept the compiler from overlapping consecutive points. Here the two points'
                    // chains run side by side up to the tail test, the slow paths and the specular terms sit behind one
                    // ballot for both, and every lane computes the same values as term() and adds them to the sums in
                    // the same order (point p before p + 1): bit-identical.
#ifndef FRT_SHADE_PAIR
#define FRT_SHADE_PAIR 0
#endif
                    constexpr bool kPair = FRT_SHADE_PAIR && kAlg && kFactored && FRT_SHADE_FAST;
                    // the specular terms of one point past its tail test (term()'s arithmetic)
                    auto spec_rest = [&](double ndl, double ndh, double edh, double ldh) {
                        const double dist_term = pow_apply(ndh, nsd, pplan) * cdist;
                        const double om = 1.0 - ldh, om2 = om * om;
                        const double factor = om2 * om2 * om;
                        const double brdf = brdf_shade(dist_term, ndh, edh, ndl, ned);
                        sum_b += brdf;
                        sum_fb += factor * brdf;
                    };
                    auto term2 = [&](const double* lp0, const double* lp1) {
                        double d0[3], d1[3];
                        for (int k = 0; k < 3; ++k) {
                            d0[k] = lp0[k] - nr.over_point[k];
                            d1[k] = lp1[k] - nr.over_point[k];
                        }
                        const double m20 = dot3_shade(d0, d0), m21 = dot3_shade(d1, d1);
                        double rl0 = rsqrt_nr(m20), rl1 = rsqrt_nr(m21);
                        {
                            const bool s0 = !shade_in_range(m20), s1 = !shade_in_range(m21);
                            if (__builtin_expect(__ballot(s0 || s1) != 0ull, 0)) {
                                if (s0) rl0 = 1.0 / sqrt(m20);
                                if (s1) rl1 = 1.0 / sqrt(m21);
                            }
                        }
                        const double ldn0 = dot3_shade(d0, nr.normalv) * rl0, ldn1 = dot3_shade(d1, nr.normalv) * rl1;
                        if (S.cfg.include_diffuse && ldn0 >= 0.0) sum_ldn += ldn0;
                        if (S.cfg.include_diffuse && ldn1 >= 0.0) sum_ldn += ldn1;
                        if (!S.cfg.include_spec_highlight) return;
                        const bool n0 = ldn0 >= 0.0, n1 = ldn1 >= 0.0;
                        const double el0 = dot3_shade(d0, nr.eyev) * rl0, ll0 = (m20 * rl0) * rl0;
                        const double el1 = dot3_shade(d1, nr.eyev) * rl1, ll1 = (m21 * rl1) * rl1;
                        const double h20 = ll0 + 2.0 * el0 + ee, h21 = ll1 + 2.0 * el1 + ee;
                        double rh0 = rsqrt_nr(h20), rh1 = rsqrt_nr(h21);
                        {
                            const bool s0 = n0 && !shade_in_range(h20), s1 = n1 && !shade_in_range(h21);
                            if (__builtin_expect(__ballot(s0 || s1) != 0ull, 0)) {
                                if (s0) rh0 = 1.0 / sqrt(h20);
                                if (s1) rh1 = 1.0 / sqrt(h21);
                            }
                        }
                        const double ndh0 = fmax(0.0, (ldn0 + ned) * rh0), ndh1 = fmax(0.0, (ldn1 + ned) * rh1);
                        const bool t0 = ldn0 > 0x1p-100 &&
                                        nsf * __log2f((float)ndh0) - 2.0f * __log2f((float)ldn0) + skip_c < 0.0f;
                        const bool t1 = ldn1 > 0x1p-100 &&
                                        nsf * __log2f((float)ndh1) - 2.0f * __log2f((float)ldn1) + skip_c < 0.0f;
                        const bool g0 = n0 && !t0, g1 = n1 && !t1;
                        if (__ballot(g0 || g1) == 0ull) return;
                        if (g0) spec_rest(ldn0, ndh0, fmax(0.0, (el0 + ee) * rh0), (ll0 + el0) * rh0);
                        if (g1) spec_rest(ldn1, ndh1, fmax(0.0, (el1 + ee) * rh1), (ll1 + el1) * rh1);
                    };
                    const double* row0 = S.light_points + L.points;
                    const int ns = L.num_samples;
                    // a wave-uniform row: the same point in every lane, so its address is wave-uniform and the loads go
                    // through the scalar cache (the point's coordinates in SGPRs, no vector memory latency)
                    // (the constant address space: without it the compiler cannot prove that nothing the kernel stores
                    // aliases the points, and emits vector flat loads of the uniform address, waited on every point)
#ifndef FRT_SHADE_CONST_PTS
#define FRT_SHADE_CONST_PTS 1
#endif
#if FRT_SHADE_CONST_PTS
                    using const_pts = const __attribute__((address_space(4))) double*;
#else
                    using const_pts = const double*;
#endif
                    auto uniform_points = [&](const double* up) {
                        const const_pts sp = (const_pts)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(
                                                              (int)(uint32_t)(uint64_t)up)) |
                                                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(
                                                               (int)(uint32_t)((uint64_t)up >> 32))
                                                           << 32));
                        double a[3] = {sp[0], sp[1], sp[2]};
                        int p = 0;
                        if (kPair) {  // (pairs of points, the next pair's scalar loads ahead of this pair's arithmetic)
                            const const_pts q1 = sp + 3 * min(1, ns - 1);
                            double b[3] = {q1[0], q1[1], q1[2]};
                            for (; p + 1 < ns; p += 2) {
                                const double lp0[3] = {a[0], a[1], a[2]}, lp1[3] = {b[0], b[1], b[2]};
                                const const_pts qa = sp + 3 * min(p + 2, ns - 1), qb = sp + 3 * min(p + 3, ns - 1);
                                a[0] = qa[0];
                                a[1] = qa[1];
                                a[2] = qa[2];
                                b[0] = qb[0];
                                b[1] = qb[1];
                                b[2] = qb[2];
                                term2(lp0, lp1);
                            }
                        }
                        for (; p < ns; ++p) {  // (the next point's scalar loads ahead of this one's arithmetic)
                            const double lp[3] = {a[0], a[1], a[2]};
                            const const_pts q = sp + 3 * min(p + 1, ns - 1);
                            a[0] = q[0];
                            a[1] = q[1];
                            a[2] = q[2];
                            term(lp);
                        }
                    };
                    const int row = L.rows <= 1 ? 0 : light_row(L, B.seed, nr.key, li, 1);
                    const int ra = __builtin_amdgcn_readfirstlane(row);
                    if (L.rows <= 1) {
                        uniform_points(row0);  // one cache row
                    } else if (__ballot(row != ra) == 0ull && lds_row != nullptr) {
                        // the wave shares its row (the lit list in row order): the row into the wave's LDS in one
                        // coalesced round trip by the active lanes, then every lane reads the same point (a broadcast).
                        // (Measured slower than the scalar loads below once those were real scalar loads: the LDS
                        // reads' latency is paid on every point, the scalar loads run a point ahead.)
                        const double* rp = row0 + 3 * (int64_t)ra * ns;
                        const unsigned long long act = __ballot(true);
                        const int lane = (int)(threadIdx.x & 63);
                        const int rank = __popcll(act & ((1ull << lane) - 1)), nact = __popcll(act);
                        for (int c0 = 0; c0 < ns; c0 += kLdsPoints) {
                            const int cn = min(kLdsPoints, ns - c0);
                            __builtin_amdgcn_wave_barrier();
                            for (int w = rank; w < 3 * cn; w += nact) lds_row[w] = rp[3 * c0 + w];
                            __builtin_amdgcn_wave_barrier();
                            __builtin_amdgcn_s_waitcnt(0xc07f);  // (lgkmcnt(0): the stores are done before the reads)
                            for (int p = 0; p < cn; ++p) {
                                const double lp[3] = {lds_row[3 * p], lds_row[3 * p + 1], lds_row[3 * p + 2]};
                                term(lp);
                            }
                        }
                    } else if (__ballot(row != ra) == 0ull) {
                        uniform_points(row0 + 3 * (int64_t)ra * ns);  // (the wave shares its row)
                    } else {
                        // the node's own row (per lane): each point's loads issued two points ahead of its arithmetic
                        // (the rows are scattered over the 157 MB cache, so a load's latency is a trip to HBM or MALL)
                        const double* pts = row0 + 3 * (int64_t)row * ns;
                        double a[3] = {pts[0], pts[1], pts[2]};
                        const double* q1 = pts + 3 * min(1, ns - 1);
                        double b[3] = {q1[0], q1[1], q1[2]};
                        for (int p = 0; p < ns; ++p) {
                            const double lp[3] = {a[0], a[1], a[2]};
                            a[0] = b[0];
                            a[1] = b[1];
                            a[2] = b[2];
                            const double* q = pts + 3 * min(p + 2, ns - 1);
                            b[0] = q[0];
                            b[1] = q[1];
                            b[2] = q[2];
                            term(lp);
                        }
                    }
                    if (kFactored)
                        for (int k = 0; k < 3; ++k) {
                            dacc[k] = nr.Kd[k] * L.intensity[k] * sum_ldn;
                            sacc[k] = nr.Ks[k] * L.intensity[k] * sum_b + (1.0 - nr.Ks[k]) * L.intensity[k] * sum_fb;
                        }
                    double scaling = inten / (double)L.num_samples;
                    for (int k = 0; k < 3; ++k) {
                        cD[k] = (0.0 + dacc[k]) * scaling;
                        cS[k] = (0.0 + sacc[k]) * scaling;
                    }
                }
            }
            if (S.cfg.include_ambient)
                for (int k = 0; k < 3; ++k) cA[k] = 0.0 + amb[k];
            for (int k = 0; k < 3; ++k) {
                sA[k] += cA[k];
                sD[k] += cD[k];
                sS[k] += cS[k];
            }
        }
    }
    for (int k = 0; k < 3; ++k) {
        out[k] = sA[k];
        out[4 + k] = sD[k];
        out[8 + k] = sS[k];
    }
    out[3] = out[7] = out[11] = 0.0;
}

// the node's shading loops over light points: some light reaches it (a non-zero unshadowed count:
// lighting_microfacet's `if (!feq(intensity, 0))`, renderer.c:909) and diffuse or highlights are on
__device__ __forceinline__ bool shade_heavy(const DevScene& S, const int32_t* __restrict__ counts, int64_t i) {
    if (!S.cfg.include_direct || !(S.cfg.include_diffuse || S.cfg.include_spec_highlight)) return false;
    for (int li = 0; li < S.num_lights; ++li)
        if (counts[i * S.num_lights + li] != 0) return true;
    return false;
}

// shade_node of a node without light-point work (not shade_heavy): the ambient terms, the same additions
// (every diffuse / specular term an exact 0)
__device__ __forceinline__ void ambient_node(const DevScene& S, const NodeRec& nr, double* out) {
    double sA[3] = {0, 0, 0};
    if (S.cfg.include_direct && S.cfg.include_ambient)
        for (int li = 0; li < S.num_lights; ++li) {
            const frt_light& L = S.lights[li];
            for (int k = 0; k < 3; ++k) sA[k] += 0.0 + nr.Ka[k] * L.intensity[k];
        }
    for (int k = 0; k < 3; ++k) {
        out[k] = sA[k];
        out[4 + k] = 0.0;
        out[8 + k] = 0.0;
    }
    out[3] = out[7] = out[11] = 0.0;
}

// Shading in two kernels: most path nodes of a frame see no light sample at all (cornell 1920x1080: 83 % of
// the (node, light) pairs are wholly shadowed), and a wave runs its light-point loops whenever one lane
// needs them. k_shade writes the nodes without light-point work (ambient only) and appends the others to
// kShadeSegs segments of a list (one atomic per wave on its segment's line); k_shade_lit shades the
// listed nodes with every lane busy.
// kLazy (no GI on the surface triples): the nodes without light-point work are not written at all; k_combine
// computes their ambient terms where it would read them (ambient_node), so k_shade reads only the material
// and count words.
constexpr int kShadeSegs = 64;
static_assert(kShadeSegs == jit::kMixSegs, "k_shade_lit reads its slots with jit::mix_slot");
template <bool kLazy>
__global__ void __launch_bounds__(kBlock) k_shade(DevScene S, Batch B, NodeCols rec, int64_t n,
                                                  const int32_t* __restrict__ counts, Cols<Tri9> surface,
                                                  uint32_t* __restrict__ lit, unsigned* __restrict__ lcount,
                                                  uint32_t segcap) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool heavy = false, mine = false;
    NodeRec nr{};
    if (i < n) {
        nr = rec.load(i, S.materials);
        mine = nr.material >= 0;
        heavy = mine && lit != nullptr && shade_heavy(S, counts, i);
    }
    if (!kLazy && mine && !heavy) {
        double out[12];
        if (rec.eye_cam) camera_eyev(S, B, i, nr.eyev);
        shade_node(S, B, nr, i, counts, out);
        tri_store(surface, i, out);
    }
    if (lit != nullptr) {
        const unsigned long long m = __ballot(heavy);
        if (m) {
            const int lane = threadIdx.x & 63;
            const int seg = (int)(blockIdx.x % kShadeSegs);
            unsigned base = 0;
            if (lane == 0) base = atomicAdd(lcount + seg * jit::kMixLine, (unsigned)__popcll(m));
            base = __shfl(base, 0, 64);
            const unsigned at = base + (unsigned)__popcll(m & ((1ull << lane) - 1));
            if (heavy) lit[(size_t)seg * segcap + at] = (uint32_t)i;  // (segcap: a whole segment's blocks fit)
        }
    }
}

// A secondary level's queue entries with their parent-order keys (the reflected children first, then the
// refracted, each in parent order) and storage slots, for the radix sort behind Batch.qperm (FRT_QUEUE_SORT).
// B: the level's queue segments (qprefix, qsegcap).
// FRT_QUEUE_SORT=2: the taken slots of the dense queue in order, from k_prepare's masks (2G of them) and the
// exclusive scan of their popcounts (offs, 2G + 1 entries: offs[2G] the total, into counter word 20). One thread
// per mask: slot = (g < G ? 0 : n) + 64 (g mod G) + bit.
struct MaskPopc {
    const unsigned long long* m;
    int64_t count;
    __host__ __device__ uint32_t operator()(int64_t i) const { return i < count ? (uint32_t)__popcll(m[i]) : 0u; }
};
__global__ void __launch_bounds__(kBlock) k_spawn_expand(const unsigned long long* __restrict__ masks,
                                                         const uint32_t* __restrict__ offs, int64_t n, int64_t G,
                                                         uint32_t* __restrict__ qperm,
                                                         unsigned long long* __restrict__ counters) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) counters[20] = offs[2 * G];
    if (g >= 2 * G) return;
    unsigned long long m = masks[g];
    uint32_t at = offs[g];
    const uint32_t slot0 = (uint32_t)((g < G ? 0 : n) + ((g < G ? g : g - G) << 6));
    while (m != 0ull) {
        qperm[at++] = slot0 + (uint32_t)__builtin_ctzll(m);
        m &= m - 1ull;
    }
}

// (shift: the parents' low bits left out of the key, runs of 2^shift parents in the segments' order)
__global__ void __launch_bounds__(kBlock) k_queue_keys(Batch B, const QueuedRay* __restrict__ q, int64_t n, int pbits,
                                                       int shift, uint32_t* __restrict__ keys,
                                                       uint32_t* __restrict__ slots) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = queue_slot(B, i);
    const QueuedRay& qr = q[s];
    keys[i] = ((uint32_t)(qr.slot & 1) << (pbits - shift)) | ((uint32_t)qr.parent >> shift);
    slots[i] = (uint32_t)s;
}

// With a multi-row light (the shipped area-light cache: 65 535 rows of 100 points, 157 MB) every listed node reads
// the row its shading draw picks, 2.4 KB of the cache per node and a different row in every lane (22 GB fetched per
// headline-size launch, memory-bound). The list is put in row order first (k_lit_rows lists the nodes densely with
// their rows, a device radix sort over the rows' 16 bits orders them), so k_shade_lit's waves mostly share one row
// and read it through the scalar cache. Each lane's result is its own node's (the order changes which nodes share a wave, not what a lane
// computes).
__device__ __forceinline__ unsigned lit_total(const unsigned* __restrict__ lcount) {  // (uniform per wave)
    const int lane = threadIdx.x & 63;
    unsigned incl = lcount[lane * jit::kMixLine];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    return __shfl(incl, 63, 64);
}

// the listed nodes densely with their rows of light sort_light (the sort's keys and values)
__global__ void __launch_bounds__(kBlock) k_lit_rows(DevScene S, Batch B, const ShadowHead* __restrict__ head,
                                                     const uint32_t* __restrict__ lit, const unsigned* __restrict__ lcount,
                                                     uint32_t segcap, int sort_light, uint32_t* __restrict__ rows,
                                                     uint32_t* __restrict__ nodes) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned total = lit_total(lcount);
    if (blockIdx.x * blockDim.x + (threadIdx.x & ~63u) >= total) return;  // (whole waves)
    const size_t slot = jit::mix_slot(m < total ? m : 0u, lcount, segcap);
    if (m >= total) return;
    const uint32_t i = lit[slot];
    rows[m] = (uint32_t)light_row(S.lights[sort_light], B.seed, head[i].key, sort_light, 1);
    nodes[m] = i;
}

// The multi-row light's shading in row order without scattered record traffic (FRT_SHADE_STAGE=1; scenes without
// GI; the default, 2, keeps only the triples' part): in row order every lane's node is a random one, so its ~10 record words (NodeCols columns, ShadowHead,
// counts) were ~10 scattered lines per node and its 9 colour-column stores 9 partial lines (profiles/
// r05_pmc_k_shade_lit_shipped.json: 7.5 GB fetched, 5.1 GB written per launch for 0.8 GB of triples). k_lit_stage
// reads the records in list order (the list is in node order within each wave: near-coalesced) and writes what the
// shading reads as one 96-byte record per listed node (LitStage), indexed by the list position m0 the sort carries as
// its value; k_shade_lit<true> then reads one record per lane and writes its triple as 72 contiguous bytes at its
// sorted position m (the wave's 64 triples one 4.6 KB run), with the node's spos[i] = m; k_combine finds the triple
// through spos. Each lane still computes its own node's result (bit-identical to list order).
struct LitStage {
    double over_point[3], normalv[3], eyev[3];
    uint64_t key;
    int32_t material, flags;
    uint32_t node;
    int32_t c0;  // the one light's unshadowed count (-1: several lights, read from counts)
};
static_assert(sizeof(LitStage) == 96, "LitStage layout");

__global__ void __launch_bounds__(kBlock) k_lit_stage(DevScene S, Batch B, NodeCols rec, const int32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ lit, const unsigned* __restrict__ lcount,
                                                      uint32_t segcap, int sort_light, uint32_t* __restrict__ rows,
                                                      uint32_t* __restrict__ vals, LitStage* __restrict__ stage) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned total = lit_total(lcount);
    if (blockIdx.x * blockDim.x + (threadIdx.x & ~63u) >= total) return;  // (whole waves)
    const size_t slot = jit::mix_slot(m < total ? m : 0u, lcount, segcap);
    if (m >= total) return;
    const uint32_t i = lit[slot];
    NodeRec nr = rec.load(i, S.materials);
    if (rec.eye_cam) camera_eyev(S, B, i, nr.eyev);
    LitStage r;
    for (int k = 0; k < 3; ++k) {
        r.over_point[k] = nr.over_point[k];
        r.normalv[k] = nr.normalv[k];
        r.eyev[k] = nr.eyev[k];
    }
    r.key = nr.key;
    r.material = nr.material;
    r.flags = nr.flags;
    r.node = i;
    r.c0 = S.num_lights == 1 ? counts[i] : -1;
    uint64_t w[12];
    __builtin_memcpy(w, &r, sizeof(r));
    uint64_t* dst = (uint64_t*)(stage + m);
#pragma unroll
    for (int k = 0; k < 12; ++k) dst[k] = w[k];
    rows[m] = (uint32_t)light_row(S.lights[sort_light], B.seed, nr.key, sort_light, 1);
    vals[m] = m;
}

// the listed nodes (k_shade); one lane each, the grid sized for every node of the level (4 waves per SIMD asked
// of the compiler: 128 VGPRs with a few spilled outside the light-point loop, 16.5 -> 15.9 ms per headline
// frame over its own 3)
#ifndef FRT_SHADE_WAVES
#define FRT_SHADE_WAVES 4
#endif
// (kRows: the list in light-row order, a multi-row light's row staged per wave in LDS)
template <bool kRows>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FRT_SHADE_WAVES, 8))) k_shade_lit(DevScene S, Batch B, NodeCols rec,
                                                      const int32_t* __restrict__ counts, Cols<Tri9> surface,
                                                      const uint32_t* __restrict__ lit,
                                                      const unsigned* __restrict__ lcount, uint32_t segcap,
                                                      const uint32_t* __restrict__ flat,
                                                      const LitStage* __restrict__ stage, uint32_t* __restrict__ spos) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    // the listed total: every lane reads one segment's count (uniform per wave)
    const int lane = threadIdx.x & 63;
    const unsigned c = lcount[lane * jit::kMixLine];
    unsigned incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    const unsigned total = __shfl(incl, 63, 64);
    if (blockIdx.x * blockDim.x + (threadIdx.x & ~63u) >= total) return;  // (whole waves)
    int64_t i = 0;
    NodeRec nr{};
    int32_t c0 = -1;
    const bool staged = kRows && stage != nullptr;  // (the staged records in row order, k_lit_stage)
    const bool sorted_out = kRows && spos != nullptr;  // (the triples in row order, found through spos)
    if (staged) {
        if (m >= total) return;
        const uint64_t* src = (const uint64_t*)(stage + flat[m]);
        uint64_t w[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) w[k] = src[k];
        LitStage r;
        __builtin_memcpy(&r, w, sizeof(r));
        for (int k = 0; k < 3; ++k) {
            nr.over_point[k] = r.over_point[k];
            nr.normalv[k] = r.normalv[k];
            nr.eyev[k] = r.eyev[k];
        }
        nr.key = r.key;
        nr.material = r.material;
        nr.flags = r.flags;
        c0 = r.c0;
        i = (int64_t)r.node;
    } else {
        if (flat != nullptr) {  // (the list in row order)
            if (m >= total) return;
            i = (int64_t)flat[m];
        } else {
            const size_t slot = jit::mix_slot(m < total ? m : 0u, lcount, segcap);
            if (m >= total) return;
            i = (int64_t)lit[slot];
        }
        nr = rec.load(i, S.materials);
        if (rec.eye_cam) camera_eyev(S, B, i, nr.eyev);
    }
    if (staged) {  // (the colours: a pattern node's own, or its material's)
        if (nr.flags & kOwnColors) {
            const NodeColors o = rec.col.load(i);
            for (int k = 0; k < 3; ++k) {
                nr.Ka[k] = o.Ka[k];
                nr.Kd[k] = o.Kd[k];
                nr.Ks[k] = o.Ks[k];
            }
            nr.Ns = o.Ns;
        } else {
            const frt_material& M = S.materials[nr.material];
            for (int k = 0; k < 3; ++k) {
                nr.Ka[k] = M.Ka[k];
                nr.Kd[k] = M.Kd[k];
                nr.Ks[k] = M.Ks[k];
            }
            nr.Ns = M.Ns;
        }
    }
    double out[12];
// FRT_SHADE_LDS_ROWS=1: a wave's shared row staged through LDS (A/B runs). 0 (default): read through the scalar
// cache like the single-row light's points, 14.2 -> 13.1 ms per shipped frame (profiles/r05_ab_shade_scalar_rows.txt)
#ifndef FRT_SHADE_LDS_ROWS
#define FRT_SHADE_LDS_ROWS 0
#endif
    if (kRows && FRT_SHADE_LDS_ROWS) {
        __shared__ double lds_rows[kBlock / 64][3 * kLdsPoints];  // (a multi-row light's row per wave, 3 KB)
        shade_node(S, B, nr, i, counts, out, lds_rows[threadIdx.x >> 6], c0);
    } else {
        shade_node(S, B, nr, i, counts, out, nullptr, c0);
    }
    if (sorted_out) {
        uint64_t* dst = surface.w + (size_t)9 * m;  // (the level's surface memory as 9-word records, sorted order)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            dst[k] = (uint64_t)__double_as_longlong(out[k]);
            dst[3 + k] = (uint64_t)__double_as_longlong(out[4 + k]);
            dst[6 + k] = (uint64_t)__double_as_longlong(out[8 + k]);
        }
        spos[i] = m;
        return;
    }
    tri_store(surface, i, out);
}

// bottom-up combine of one node (shade_hit's specular block, renderer.c:773-822): its A, D, S triples into col
// (counts != nullptr: the surface triples of nodes without light-point work were not written, k_shade<true>)
// (spos != nullptr: the level's lit nodes were shaded in row order from staged records, k_lit_stage; a lit node's
// triple is the 9-word record spos[i] of the surface memory)
__device__ __forceinline__ void combine_node(const DevScene& S, const int32_t* __restrict__ counts,
                                             const NodeRec& nr, int64_t i, Cols<Tri9> surface, Cols<Tri9> child,
                                             const frt_material* __restrict__ mats, int32_t include_specular,
                                             double* col, const uint32_t* __restrict__ spos = nullptr) {
    if (nr.material < 0) {
        for (int k = 0; k < 12; ++k) col[k] = 0.0;
        return;
    }
    if (counts != nullptr && !shade_heavy(S, counts, i)) {
        ambient_node(S, nr, col);
    } else if (spos != nullptr) {
        const uint64_t* src = surface.w + (size_t)9 * spos[i];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            col[k] = __longlong_as_double((long long)src[k]);
            col[4 + k] = __longlong_as_double((long long)src[3 + k]);
            col[8 + k] = __longlong_as_double((long long)src[6 + k]);
        }
        col[3] = col[7] = col[11] = 0.0;
    } else {
        tri_load(surface, i, col);
    }
    if (include_specular) {
        const frt_material& M = mats[nr.material];
        // reflected / refracted_color from the children's slots; a child that was not traced
        // (zero weight, or nothing to spawn) contributes an exact 0
        double R[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, T[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        // (a level's child slots as two halves of its child columns, reflected then refracted: slot s of node i at
        // s * cap / 2 + i, so the child level's stores and this level's loads run along consecutive nodes)
        const int64_t half = child.cap >> 1;
        if (nr.flags & kReflSpawned) tri_load(child, i, R);
        if (nr.flags & kRefrSpawned) tri_load(child, half + i, T);
        double rl[12], rr[12];
        for (int t = 0; t < 12; t += 4) {
            for (int k = 0; k < 3; ++k) {
                rl[t + k] = (nr.flags & kReflApplies) ? 0.0 + R[t + k] * nr.refl[k] : 0.0;
                double tt = T[t + k] * M.Tf[k];
                tt *= nr.over_d;
                rr[t + k] = (nr.flags & kRefrApplies) ? 0.0 + tt : 0.0;
            }
        }
        if (nr.flags & kMix) {
            for (int t = 0; t < 12; t += 4) {
                for (int k = 0; k < 3; ++k) {
                    rl[t + k] *= nr.rf;
                    rr[t + k] *= 1.0 - nr.rf;
                }
            }
        }
        for (int t = 0; t < 12; t += 4)
            for (int k = 0; k < 3; ++k) col[t + k] += rl[t + k];
        if (nr.flags & kDissolve)
            for (int t = 0; t < 12; t += 4)
                for (int k = 0; k < 3; ++k) col[t + k] *= 1.0 - nr.over_d;
        for (int t = 0; t < 12; t += 4)
            for (int k = 0; k < 3; ++k) col[t + k] += rr[t + k];
    }
}

// bottom-up combine of one level
// (level 0 without k_combine_resolve: samples land in sample_out in sample order, coalesced stores; k_resolve
// reads each pixel's run)
__global__ void __launch_bounds__(kBlock) k_combine(DevScene S, const int32_t* __restrict__ counts, NodeCols rec,
                                                    int64_t n, Cols<Tri9> surface, Cols<Tri9> child,
                                                    Cols<Tri9> parent_child, Cols<Tri9> sample_out, int32_t spp,
                                                    const frt_material* __restrict__ mats, int32_t include_specular,
                                                    const uint32_t* __restrict__ spos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NodeRec nr = rec.load(i, mats);
    double col[12];
    combine_node(S, counts, nr, i, surface, child, mats, include_specular, col, spos);
    if (nr.parent >= 0) {
        // (a missed child writes its zeros; slot halves as combine_node reads them)
        tri_store(parent_child, (int64_t)nr.slot * (parent_child.cap >> 1) + nr.parent, col);
    } else {
        tri_store(sample_out, i, col);  // sample order (pixel-major): one coalesced run per column
    }
}

// Level 0 combined and resolved in one pass (spp <= kFuseBlock): the level's nodes are the batch's samples
// in sample order, so a block takes ppb = kFuseBlock / spp whole pixels, one thread per sample, stages the
// nine A / D / S columns of its samples in LDS and sums each pixel's run in sub-sample order (k_resolve's
// arithmetic, the same additions in the same order), without the samples' round trip through HBM.
constexpr int kFuseBlock = 256;
__global__ void __launch_bounds__(kFuseBlock) k_combine_resolve(DevScene S, const int32_t* __restrict__ counts,
                                                                NodeCols rec, int64_t n, Cols<Tri9> surface,
                                                                Cols<Tri9> child, int32_t spp, int32_t ppb,
                                                                int64_t npix, const frt_material* __restrict__ mats,
                                                                int32_t include_specular, double* __restrict__ out,
                                                                const uint32_t* __restrict__ spos) {
    // (each pixel's column sum goes back into the first slot of the run it was summed from: only the thread that
    // summed a run reads it, and the block's LDS stays at 18.5 KB, so six blocks fit a CU instead of four)
#ifndef FRT_RESOLVE_INPLACE
#define FRT_RESOLVE_INPLACE 1
#endif
    __shared__ double stage[9][kFuseBlock + 1];
#if !FRT_RESOLVE_INPLACE
    __shared__ double sum_sep[9][kFuseBlock];
#endif
    const int t = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * ppb;
    const int64_t i = p0 * spp + t;
    if (t < ppb * spp && i < n) {
        const NodeRec nr = rec.load(i, mats);
        double col[12];
        combine_node(S, counts, nr, i, surface, child, mats, include_specular, col, spos);
#pragma unroll
        for (int f = 0; f < 9; ++f) stage[f][t] = col[(f / 3) * 4 + f % 3];
    }
    __syncthreads();
    for (int q = t; q < ppb * 9; q += kFuseBlock) {
        const int lp = q / 9, f = q - lp * 9;
        if (p0 + lp >= npix) continue;
        const double* st = stage[f] + lp * spp;
        double acc = 0.0;
        for (int kk = 0; kk < spp; ++kk) acc += st[kk];
#if FRT_RESOLVE_INPLACE
        stage[f][lp * spp] = acc * (1.0 / (double)spp);
#else
        sum_sep[f][lp] = acc * (1.0 / (double)spp);
#endif
    }
    __syncthreads();
#if FRT_RESOLVE_INPLACE
    auto sum = [&](int f, int lp) { return stage[f][lp * spp]; };
#else
    auto sum = [&](int f, int lp) { return sum_sep[f][lp]; };
#endif
    for (int q = t; q < ppb * 4; q += kFuseBlock) {
        const int lp = q >> 2, f = q & 3;
        const int64_t p = p0 + lp;
        if (p >= npix) continue;
        double* o = out + 4 * p;
        if (f == 3) {
            o[3] = 0.0;
            continue;
        }
        double v = 0.0 + sum(f, lp);  // (A + D + S) / 3 of channel f
        v += sum(3 + f, lp);
        v += sum(6 + f, lp);
        v *= 1.0 / 3.0;
        o[f] = v;
    }
}

// pixel_multi_sample + render_multi_helper's (A+D+S)/3 (renderer.c:132-181, 216-233)
// A block handles 64 pixels with nine waves, wave f summing column f (one of the nine A/D/S channels) of its
// pixels, one lane per pixel, in sub-sample order. A pixel's samples are one contiguous run per column (k_combine
// stores in sample order), so each wave stages kResolveChunk samples of its 64 pixels through LDS: every wave load
// instruction reads 8 whole 64-byte runs instead of touching 64 lines for 8 bytes each. Nine waves per 64 pixels
// keep enough loads in flight for a batch of only 32 768 pixels (the headline batch) to fill the chip.
constexpr int kResolveChunk = 8;
constexpr int kResolveBlock = 64 * 9;
__global__ void __launch_bounds__(kResolveBlock) k_resolve(Cols<Tri9> sample_col, int64_t npix, int32_t spp,
                                                           double* __restrict__ out) {
    __shared__ double stage[9][64 * (kResolveChunk + 1)];
    __shared__ double sum[9][64];
    const int lane = threadIdx.x & 63, f = threadIdx.x >> 6;
    double* st = stage[f];
    const int64_t p0 = (int64_t)blockIdx.x * 64;  // the block's first pixel
    const int64_t nsamp = npix * spp;
    const uint64_t* col = sample_col.w + (int64_t)f * sample_col.cap;
    double acc = 0.0;
    for (int kb = 0; kb < spp; kb += kResolveChunk) {
        const int kc = min(kResolveChunk, spp - kb);
#pragma unroll
        for (int m = 0; m < kResolveChunk; ++m) {  // element e: pixel e / kResolveChunk, sample kb + e % kResolveChunk
            const int e = lane + 64 * m, lp = e / kResolveChunk, kk = e % kResolveChunk;
            const int64_t si = (p0 + lp) * spp + kb + kk;
            if (kk < kc && si < nsamp) st[lp * (kResolveChunk + 1) + kk] = __longlong_as_double(col[si]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int kk = 0; kk < kc; ++kk) acc += st[lane * (kResolveChunk + 1) + kk];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    sum[f][lane] = acc * (1.0 / (double)spp);
    __syncthreads();
    const int64_t p = p0 + lane;
    if (f >= 4 || p >= npix) return;
    double* o = out + 4 * p;
    if (f == 3) {
        o[3] = 0.0;
        return;
    }
    double v = 0.0 + sum[f][lane];  // (A + D + S) / 3 of channel f
    v += sum[3 + f][lane];
    v += sum[6 + f][lane];
    v *= 1.0 / 3.0;
    o[f] = v;
}


}  // namespace frt

#include "frt_gi.hpp"

namespace frt {

// =====================================================================
// global illumination: photon tracing (photon_tracer.c) and the GI terms
// of shade_hit (renderer.c:727-770)
// =====================================================================

constexpr uint64_t kTagPhoton = 0x9a0be7f1d3c2b5a1ULL;
constexpr uint64_t kTagGather = 0x51f15e0ddeadc0deULL;

struct StoredPhoton {
    double pos[3], power[3], dir[3];
    uint64_t key;  // emission index << 8 | bounce (the reference's storage order)
};

__device__ __forceinline__ bool any_positive(const double* c) { return c[0] > 0 || c[1] > 0 || c[2] > 0; }

// emit_photon (light.c:14-99): one photon of light L, emission index e
__device__ inline void emit_photon(const DevScene& S, const frt_light& L, uint64_t seed, uint64_t e, Ray& r) {
    if (L.type == FRT_POINT_LIGHT) {
        double d[3];
        for (int a = 0; a < 4096; ++a) {  // rejection in the unit ball (light.c:80-92)
            for (int k = 0; k < 3; ++k) d[k] = 2 * rng_uniform(seed, e, 8 + 3 * a + k) - 1;
            if (!(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] > 1)) break;
        }
        for (int k = 0; k < 3; ++k) {
            r.o[k] = L.position[k];
            r.d[k] = d[k];
        }
        return;
    }
    if (L.type == FRT_HEMISPHERE_LIGHT) {
        for (int k = 0; k < 3; ++k) r.o[k] = L.position[k];
    } else {  // area / circle: a random point of a random cache row (light_surface_points + rand())
        const uint64_t h1 = mix64(seed ^ mix64(e * 0x9e3779b97f4a7c15ULL + 1));
        const uint64_t h2 = mix64(seed ^ mix64(e * 0x9e3779b97f4a7c15ULL + 2));
        const int64_t row = (int64_t)(h1 % (uint64_t)(L.rows > 0 ? L.rows : 1));
        const int64_t pt = (int64_t)(h2 % (uint64_t)(L.num_samples > 0 ? L.num_samples : 1));
        const double* p = S.light_points + L.points + 3 * (row * L.num_samples + pt);
        for (int k = 0; k < 3; ++k) r.o[k] = p[k];
    }
    double nt[3], nb[3];
    coordinate_system(L.normal, nt, nb);
    hemisphere_dir(L.normal, nt, nb, rng_uniform(seed, e, 3), rng_uniform(seed, e, 4), r.d);
}

// photons of light `light` with emission indices e0 .. e0+n-1 -> the first photon queue
__global__ void __launch_bounds__(kBlock) k_photon_emit(DevScene S, uint64_t seed, int light, uint64_t e0, int64_t n,
                                                        QueuedRay* __restrict__ q, double* __restrict__ power) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const frt_light& L = S.lights[light];
    const uint64_t e = e0 + (uint64_t)i;
    Ray r;
    emit_photon(S, L, seed, e, r);
    QueuedRay qr;
    for (int k = 0; k < 3; ++k) {
        qr.o[k] = r.o[k];
        qr.d[k] = r.d[k];
        power[3 * i + k] = L.intensity[k];
    }
    qr.key = e;
    qr.parent = -1;
    qr.slot = 0;  // bit0 had_diffuse, bit1 had_specular
    q[i] = qr;
}

// power_at's hit half + photon_hit (photon_tracer.c:114-182) for one bounce
template <bool kPat>
__global__ void __launch_bounds__(kBlock) k_photon_hit(DevScene S, uint64_t seed, int map, int depth,
                                                       const QueuedRay* __restrict__ q, const double* __restrict__ power,
                                                       int64_t n, const HitRec* __restrict__ hits,
                                                       const double* __restrict__ hn12,
                                                       QueuedRay* __restrict__ next_q, double* __restrict__ next_power,
                                                       unsigned long long* next_count, int64_t next_cap,
                                                       StoredPhoton* __restrict__ store, unsigned long long* store_count,
                                                       int64_t store_cap, unsigned* err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const HitRec hr = hits[i];
    if (hr.node < 0) return;
    const QueuedRay qr = q[i];
    Ray r;
    for (int k = 0; k < 3; ++k) {
        r.o[k] = qr.o[k];
        r.d[k] = qr.d[k];
    }
    double pp[3] = {power[3 * i], power[3 * i + 1], power[3 * i + 2]};
    if (pp[0] <= 0 && pp[1] <= 0 && pp[2] <= 0) return;  // shadow / dead photons
    Hit h{hr.t, -1, -1, hr.node};
    Comps c;
    prepare<kPat>(S, r, h, c);
    c.n1 = hn12 != nullptr ? hn12[2 * i] : 1.0;
    c.n2 = hn12 != nullptr ? hn12[2 * i + 1] : 1.0;
    const frt_material& M = S.materials[c.material];
    const bool had_diffuse = (qr.slot & 1) != 0, had_specular = (qr.slot & 2) != 0;
    const uint64_t e = qr.key;
    const double avg_d = (c.Kd[0] + c.Kd[1] + c.Kd[2]) / 3.0;
    const bool store_it = any_positive(c.Kd) && (map == 0 ? had_specular : had_diffuse);
    const unsigned long long at_store = wave_append(store_count, store_it);
    {
        if (store_it) {
            const unsigned long long at = at_store;
            if ((int64_t)at < store_cap) {
                StoredPhoton sp;
                for (int k = 0; k < 3; ++k) {
                    sp.pos[k] = c.p[k];
                    sp.power[k] = c.Kd[k] * pp[k];
                    sp.dir[k] = r.d[k];  // the photon ray's direction (pm_store's dir)
                }
                sp.key = (e << 8) | (uint64_t)depth;
                store[at] = sp;
            } else {
                atomicOr(err, kErrQueueOverflow);
            }
            if (map == 0) return;  // a caustic photon ends at its first diffuse store
        }
    }
    // russian roulette (photon_tracer.c:154-179)
    const double rr = rng_uniform(seed ^ 0x7u, e, 64 + (uint64_t)depth);
    const double avg_s = (c.refl[0] + c.refl[1] + c.refl[2]) / 3.0;
    const double avg_t = (M.Tf[0] + M.Tf[1] + M.Tf[2]) / 3.0;
    int choice = -1;  // 0 diffuse, 1 specular, 2 refract
    if (map == 1) {
        const double total = avg_d + avg_s + avg_t;
        if (rr * total < avg_d) choice = 0;
        else if (rr * total < avg_d + avg_s) choice = 1;
        else if (rr * total < avg_d + avg_s + avg_t) choice = 2;
    } else {
        const double total = avg_s + avg_t;
        if (rr * total < avg_s) choice = 1;
        else if (rr * total < avg_s + avg_t) choice = 2;
    }
    bool emit = choice >= 0;  // every lane reaches the queue append below (wave_append)
    QueuedRay nq;
    double np[3];
    int flags = qr.slot;
    if (!emit) {
    } else if (choice == 0) {  // reflect_photon_diffuse (photon_tracer.c:31-62)
        for (int k = 0; k < 3; ++k) np[k] = c.Kd[k] * pp[k];
        double nt[3], nb[3], d[3];
        coordinate_system(c.normalv, nt, nb);
        hemisphere_dir(c.normalv, nt, nb, rng_uniform(seed ^ 0x9u, e, 2 * (uint64_t)depth),
                       rng_uniform(seed ^ 0x9u, e, 2 * (uint64_t)depth + 1), d);
        for (int k = 0; k < 3; ++k) {
            nq.o[k] = c.over_point[k];
            nq.d[k] = d[k];
        }
        flags |= 1;
    } else if (choice == 1) {  // reflect_photon_specular (photon_tracer.c:64-77)
        emit = M.reflective != 0;
        const double sc = 1.0 / avg_s;
        for (int k = 0; k < 3; ++k) {
            np[k] = pp[k] * sc;
            nq.o[k] = c.over_point[k];
            nq.d[k] = c.reflectv[k];
        }
        flags |= 2;
    } else {  // refract_photon (photon_tracer.c:81-112)
        emit = !feq(M.Tr, 0.0);
        const double n_ratio = c.n1 / c.n2;
        const double cos_i = dot3(c.eyev, c.normalv);
        const double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
        emit = emit && !(sin2_t > 1.0);
        const double cos_t = sqrt(1.0 - sin2_t);
        const double s1 = n_ratio * cos_i - cos_t;
        const double sc = 1.0 / avg_t;
        for (int k = 0; k < 3; ++k) {
            const double t1 = c.normalv[k] * s1;
            const double t2 = c.eyev[k] * n_ratio;
            nq.o[k] = c.under_point[k];
            nq.d[k] = t1 - t2;
            np[k] = pp[k] * sc;
        }
        flags |= 2;
    }
    const unsigned long long at = wave_append(next_count, emit);
    if (!emit) return;
    if ((int64_t)at >= next_cap) {
        atomicOr(err, kErrQueueOverflow);
        return;
    }
    nq.key = e;
    nq.parent = -1;
    nq.slot = flags;
    next_q[at] = nq;
    for (int k = 0; k < 3; ++k) next_power[3 * at + k] = np[k];
}

// the wave's LDS for wave_irradiance_estimate (frt_gi.hpp); blocks of kBlock threads
#define FRT_EST_LDS_W(name, cap, waves)                                                                   \
    __shared__ uint2 name##_ent[waves][cap];                                                              \
    __shared__ unsigned name##_hist[waves][256];                                                          \
    __shared__ unsigned name##_sel[waves][kEstSel];                                                       \
    const EstLds name{name##_ent[threadIdx.x >> 6], name##_hist[threadIdx.x >> 6], name##_sel[threadIdx.x >> 6], \
                      (unsigned)(cap)}
#define FRT_EST_LDS(name, cap) FRT_EST_LDS_W(name, cap, kBlock / 64)

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the lanes' estimate requests one after another, each by the whole wave; every lane of the
// wave must call this at the same point. est: this lane's scaled estimate (photon_estimate)
__device__ inline void wave_photon_estimates(const PhotonMapDev& M, const DevScene& S, bool want, const double* point,
                                             const double* eyev, double scale_num, double* est, const EstLds& L) {
    est[0] = est[1] = est[2] = 0.0;
    unsigned long long reqs = __ballot(want);
    while (reqs) {
        const int j = __builtin_ctzll(reqs);
        reqs &= reqs - 1;
        double x[3], nrm[3], e[3];
        for (int k = 0; k < 3; ++k) {  // wave-uniform: scalar registers
            x[k] = readlane_d(point[k], j);
            nrm[k] = readlane_d(eyev[k], j);
        }
        // the reference passes eyev as the estimate's normal (renderer.c:875)
        const int64_t used = wave_irradiance_estimate(M, x, nrm, S.cfg.irradiance_radius, S.cfg.irradiance_num,
                                                      S.cfg.cone_filter_k, e, L,
                                                      S.dbg ? S.dbg + kDbgProf + 13 : nullptr);
        if (est_lane() == j && used > 0) {
            const double f = scale_num / (double)used;
            for (int k = 0; k < 3; ++k) est[k] = e[k] * f;
        }
    }
}

// per shaded node: the visualisation term (lighting_gi) and the caustics term (renderer.c:740-761)
__global__ void __launch_bounds__(kBlock) k_gi_node(DevScene S, NodeCols rec, int64_t n,
                                                    double* __restrict__ gi_extra) {
    FRT_EST_LDS(lds, kEstCap);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    NodeRec nr{};
    bool want = false;
    if (i < n) {
        nr = rec.load(i, S.materials);
        want = nr.material >= 0 && any_positive(nr.Kd);
    }
    double vis[3] = {0, 0, 0}, cau[3] = {0, 0, 0};
    if (S.cfg.visualize_photon_map)  // lighting_gi, visualize branch: the raw estimate
        wave_photon_estimates(S.pmaps[1], S, want, nr.over_point, nr.eyev, 10.0 * (double)S.cfg.irradiance_num, vis,
                              lds);
    if (S.cfg.include_caustics) wave_photon_estimates(S.pmaps[0], S, want, nr.over_point, nr.eyev, 100.0, cau, lds);
    if (i >= n) return;
    double* out = gi_extra + 6 * i;
    for (int k = 0; k < 6; ++k) out[k] = 0.0;
    if (!want) return;
    const double edn = dot3(nr.eyev, nr.normalv);
    if (S.cfg.visualize_photon_map)
        for (int k = 0; k < 3; ++k) out[k] = vis[k];
    if (S.cfg.include_caustics) {
        if (S.cfg.visualize_photon_map) {
            for (int k = 0; k < 3; ++k) out[3 + k] = cau[k];
        } else {
            for (int k = 0; k < 3; ++k) {
                double ck = nr.Kd[k] * cau[k];
                out[3 + k] = 0.0 + ck * edn;
            }
        }
    }
}

// final_gather's rays (renderer.c:648-687): gu x gv cosine-weighted hemisphere
// directions (a jittered CMJ pattern per gather) from over_point
__global__ void __launch_bounds__(kBlock) k_gather_gen(DevScene S, uint64_t seed, NodeCols rec,
                                                       int64_t node0, int64_t nodes, QueuedRay* __restrict__ gq) {
    const int G = S.cfg.gi_usteps * S.cfg.gi_vsteps;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nodes * G) return;
    const int64_t node = node0 + t / G;
    const int slot = (int)(t % G);
    const NodeRec nr = rec.load(node, S.materials);
    QueuedRay qr;
    qr.key = nr.key;
    qr.slot = slot;
    if (nr.material < 0 || !any_positive(nr.Kd)) {
        qr.parent = -2;  // placeholder
        for (int k = 0; k < 3; ++k) qr.o[k] = qr.d[k] = 0.0;
        gq[t] = qr;
        return;
    }
    double jit[2], nt[3], nb[3], d[3];
    cmj_point(seed ^ kTagGather, nr.key, S.cfg.gi_usteps, S.cfg.gi_vsteps, slot % S.cfg.gi_usteps,
              slot / S.cfg.gi_usteps, jit);
    coordinate_system(nr.normalv, nt, nb);
    hemisphere_dir(nr.normalv, nt, nb, jit[0], jit[1], d);
    for (int k = 0; k < 3; ++k) {
        qr.o[k] = nr.over_point[k];
        qr.d[k] = d[k];
    }
    qr.parent = (int32_t)node;
    gq[t] = qr;
}

// what the final gather's estimate needs of one gather ray's hit (k_gather_hit -> k_gather_est)
struct GatherReq {
    double pt[3], ev[3];  // lighting_gi's estimate point (over_point) and "normal" (eyev)
    double kd[3], edn;    // over_Kd, eyev . normalv
    double jit0;          // the sample's first coordinate (final_gather: "scale by theta")
    int32_t want, pad;
};

// the sort key of a gather request (k_gather_est's spatial order, below): a 21-bit Morton code of its point in the
// photon grid's box, 128 cells per axis, and bit 21 set for requests without an estimate (last); the radix sort
// then takes 3 passes of 8 bits
constexpr int kGatherKeyBits = 22;
__device__ __forceinline__ uint32_t spread7(uint32_t v) {  // 7 bits to every third of 21
    v &= 0x7Fu;
    v = (v | (v << 8)) & 0x0000F00Fu;
    v = (v | (v << 4)) & 0x000C30C3u;
    v = (v | (v << 2)) & 0x00249249u;
    return v;
}

__device__ __forceinline__ uint32_t gather_key(const PhotonMapDev& M, bool want, const double* pt) {
    if (!want) return 1u << 21;
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
        const double ext = (double)max(M.dims[k], 1) * M.cell;
        const double f = (pt[k] - M.origin[k]) / ext * 128.0;
        q[k] = f >= 127.0 ? 127u : f > 0.0 ? (uint32_t)f : 0u;  // (NaN: 0)
    }
    return spread7(q[0]) | (spread7(q[1]) << 1) | (spread7(q[2]) << 2);
}

// color_at_gi + shade_hit_gi (renderer.c:320-345, 627-645) per gather ray up to the estimate: the
// hit's prepare_computations and material, written as a GatherReq
template <bool kPat>
__global__ void __launch_bounds__(kBlock) k_gather_hit(DevScene S, uint64_t seed, const QueuedRay* __restrict__ gq,
                                                       const HitRec* __restrict__ hits, int64_t n,
                                                       GatherReq* __restrict__ req, uint32_t* __restrict__ keys,
                                                       uint32_t* __restrict__ idx) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    bool want = false;
    double pt[3] = {0, 0, 0}, ev[3] = {0, 0, 0}, kd[3] = {0, 0, 0}, edn = 0.0;
    QueuedRay qr{};
    {
        qr = gq[t];
        const HitRec hr = hits[t];
        if (qr.parent >= 0 && hr.node >= 0) {
            Ray r;
            for (int k = 0; k < 3; ++k) {
                r.o[k] = qr.o[k];
                r.d[k] = qr.d[k];
            }
            const int leaf = hr.node;
            const frt_material& M = S.materials[S.nodes[leaf].material];
            double p[3], diffuse[3];
            for (int k = 0; k < 3; ++k) p[k] = r.o[k] + r.d[k] * hr.t;
            if (kPat && M.map_Kd >= 0) pattern_at_shape<kPatternDepth>(S, M.map_Kd, leaf, p, diffuse);
            else copy3(M.Kd, diffuse);
            if (any_positive(diffuse)) {
                Hit h{hr.t, -1, -1, leaf};
                Comps cp;
                prepare<kPat>(S, r, h, cp);
                if (any_positive(cp.Kd)) {  // lighting_gi (renderer.c:863-892)
                    want = true;
                    edn = dot3(cp.eyev, cp.normalv);
                    for (int k = 0; k < 3; ++k) {
                        pt[k] = cp.over_point[k];
                        ev[k] = cp.eyev[k];
                        kd[k] = cp.Kd[k];
                    }
                }
            }
        }
    }
    double jit[2];
    cmj_point(seed ^ kTagGather, qr.key, S.cfg.gi_usteps, S.cfg.gi_vsteps, qr.slot % S.cfg.gi_usteps,
              qr.slot / S.cfg.gi_usteps, jit);
    GatherReq r;
    for (int k = 0; k < 3; ++k) {
        r.pt[k] = pt[k];
        r.ev[k] = ev[k];
        r.kd[k] = kd[k];
    }
    r.edn = edn;
    r.jit0 = jit[0];
    r.want = want ? 1 : 0;
    r.pad = 0;
    req[t] = r;
    if (keys) {  // (the estimate's spatial order)
        keys[t] = gather_key(S.pmaps[1], want, pt);
        idx[t] = (uint32_t)t;
    }
}

// the gather hits' photon estimates (lighting_gi, renderer.c:863-892) in a kernel that holds only
// the estimate's state: kGatherReqPerWave consecutive requests per wave, one after another, each read
// through the scalar cache (wave-uniform address) and estimated by the whole wave; lane 0 stores the
// result. Measured on cornell_gi_480x270_8x8 (tools/ab_gi.sh): 8 or 64 requests per wave with 1 or 4
// waves per block land within 3 %; one request per wave (no scratch at all) is 20-70 % slower (a wave
// launch and LDS setup per request); 3 waves per SIMD (no spills) is 8 % slower than 4 (a few spilled
// VGPRs).
#ifndef FRT_GATHER_CAP
#define FRT_GATHER_CAP 768
#endif
constexpr int kGatherEstCap = FRT_GATHER_CAP;
#ifndef FRT_EST_WAVES
#define FRT_EST_WAVES 4
#endif
// (one wave per block since round 5: with the requests in spatial order, 4 / 2 / 8 waves per block measured 20.76 s
// of estimate per 1920x1080 GI frame against 20.28 s with 1, profiles/r05_ab_gi_sort.txt)
#ifndef FRT_GATHER_WAVES_PER_BLOCK
#define FRT_GATHER_WAVES_PER_BLOCK 1
#endif
constexpr int kGatherWavesPerBlock = FRT_GATHER_WAVES_PER_BLOCK;
#ifndef FRT_GATHER_REQ_PER_WAVE
#define FRT_GATHER_REQ_PER_WAVE 64
#endif
constexpr int kGatherReqPerWave = FRT_GATHER_REQ_PER_WAVE;
// (Round 3 sorted the requests by a Morton key with one shared counter, 1793 -> 1855 ms, and dealt contiguous
// block runs to the XCDs, 2600 ms: the dense regions then crowd onto one XCD. Round 5's per-XCD queues that steal
// the other groups' leftovers keep the balance: below.)
// work: nullptr — wave w takes requests [w kGatherReqPerWave, (w + 1) kGatherReqPerWave); else a queue
// counter: resident waves take kGatherBatch requests at a time until none are left (the dense queries'
// waves no longer set the launch's tail)
#ifndef FRT_GATHER_BATCH
#define FRT_GATHER_BATCH 16
#endif
constexpr int kGatherBatch = FRT_GATHER_BATCH;
constexpr int kGatherGroups = 8;  // (the XCDs: blocks blockIdx % 8 share one)
// The estimate reads ~20 KB of the photon map per query and its queries, in gather order, scatter over the room:
// every byte came from beyond the XCD's L2 (FETCH_SIZE x 2 per query = the byte model, 6.4 TB/s of fabric reads,
// profiles/r03_pmc_k_gather_est_*.json), and 3 waves per SIMD estimate as fast as 4 (profiles/r05_ab_gi_order.txt):
// the fabric, not the latency chain, bounds it. k_gather_hit gives each request a Morton key of its point in the
// photon grid's box (gather_key; requests without an estimate last), a radix sort orders the requests' indices by it (perm),
// and k_gather_est deals the sorted order to the 8 groups of blocks that share an XCD (blockIdx % 8: its own
// contiguous eighth, taken kGatherBatch at a time, then the other groups' leftovers), so the queries in flight on
// one XCD are neighbours and share the photons in its L2. Results go to each request's own slot: the order changes
// nothing in a query's arithmetic (test_gather_order_equals_request_order).
__global__ void __launch_bounds__(64 * kGatherWavesPerBlock) __attribute__((amdgpu_waves_per_eu(FRT_EST_WAVES, 8)))
k_gather_est(DevScene S, const GatherReq* __restrict__ req, int64_t n, double* __restrict__ gather_col,
             unsigned* __restrict__ work, const uint32_t* __restrict__ perm) {
    FRT_EST_LDS_W(lds, kGatherEstCap, kGatherWavesPerBlock);
    auto query = [&](int64_t t) {
        const GatherReq& r = req[t];
        double out3[3] = {0.0, 0.0, 0.0};
        if (r.want) {
            double x[3], nrm[3], e[3], est[3] = {0.0, 0.0, 0.0};
            for (int k = 0; k < 3; ++k) {
                x[k] = r.pt[k];
                nrm[k] = r.ev[k];  // the reference passes eyev as the estimate's normal (renderer.c:875)
            }
            const int64_t used = wave_irradiance_estimate(S.pmaps[1], x, nrm, S.cfg.irradiance_radius,
                                                          S.cfg.irradiance_num, S.cfg.cone_filter_k, e, lds,
                                                          S.dbg ? S.dbg + kDbgProf + 13 : nullptr);
            if (used > 0) {
                const double f = 10.0 * (double)S.cfg.irradiance_num / (double)used;
                for (int k = 0; k < 3; ++k) est[k] = e[k] * f;
            }
            if (S.cfg.visualize_photon_map) {  // lighting_gi returns the raw estimate here too
                for (int k = 0; k < 3; ++k) out3[k] = est[k] * kPi;  // shade_hit_gi: x pi
            } else {
                for (int k = 0; k < 3; ++k) {
                    double dk = r.kd[k] * est[k];
                    dk = dk * r.edn;
                    out3[k] = dk * kPi;  // shade_hit_gi: x pi
                }
            }
        }
        if (est_lane() == 0)
            for (int k = 0; k < 3; ++k) gather_col[3 * t + k] = out3[k] * r.jit0;
    };
    // one call site of the estimate (a second one doubles its register pressure: spills)
    const bool queue = work != nullptr;
    const int per = queue ? kGatherBatch : kGatherReqPerWave;
    int64_t t0 = ((int64_t)blockIdx.x * kGatherWavesPerBlock + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))) *
                 kGatherReqPerWave;
    // (perm: the sorted order, dealt in kGatherGroups contiguous ranges, one counter each on its own line; a wave starts
    // at its block's group and moves on to the next group when that range is done)
    int g = perm != nullptr ? (int)(blockIdx.x % kGatherGroups) : 0;
    int tried = 0;
    int64_t lo = 0, len = n;
    auto group_range = [&](int gg) {
        lo = n * gg / kGatherGroups;
        len = n * (gg + 1) / kGatherGroups - lo;
    };
    if (perm != nullptr) group_range(g);
    for (bool first = true;; first = false) {  // (every wave leaves once every counter passes its range)
        if (queue) {
            unsigned base = 0;
            if (est_lane() == 0) base = atomicAdd(work + (perm != nullptr ? g * 64 : 0), (unsigned)kGatherBatch);
            t0 = (int64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)__shfl(base, 0, 64));
            if (perm != nullptr && t0 >= len) {  // (this group's range is done: the next group's)
                if (++tried >= kGatherGroups) break;
                g = (g + 1) % kGatherGroups;
                group_range(g);
                continue;
            }
        } else if (!first) {
            break;
        }
        if (t0 >= (perm != nullptr ? len : n)) break;
        for (int j = 0; j < per; ++j) {
            const int64_t ts = t0 + j;
            if (ts >= (perm != nullptr ? len : n)) break;
            query(perm != nullptr ? (int64_t)perm[lo + ts] : ts);
        }
    }
}

// frt_pm_estimate's kernel: one wave per query (pos[3], normal[3]), the estimate as lighting_gi
// calls it before its scaling
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FRT_EST_WAVES, 8))) k_pm_estimate(
    PhotonMapDev M, const double* __restrict__ q, int64_t nq, double radius, int k, double cone_k,
    double* __restrict__ irrad, int64_t* __restrict__ found) {
    FRT_EST_LDS(lds, kGatherEstCap);
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x) / 64 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= nq) return;  // (whole waves)
    double x[3], nrm[3], e[3];
    for (int j = 0; j < 3; ++j) {
        x[j] = q[6 * w + j];
        nrm[j] = q[6 * w + 3 + j];
    }
    const int64_t used = wave_irradiance_estimate(M, x, nrm, radius, k, cone_k, e, lds);
    if (est_lane() == 0) {
        for (int j = 0; j < 3; ++j) irrad[3 * w + j] = e[j];
        found[w] = used;
    }
}

// final_gather's sum (slot order = the reference's v-outer, u-inner loop), x 2 pi / rays, x over_Kd
__global__ void __launch_bounds__(kBlock) k_gather_reduce(DevScene S, NodeCols rec, int64_t node0,
                                                          int64_t nodes, const double* __restrict__ gather_col,
                                                          double* __restrict__ fgather) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nodes) return;
    const int64_t node = node0 + t;
    const int G = S.cfg.gi_usteps * S.cfg.gi_vsteps;
    const NodeRec nr = rec.load(node, S.materials);
    double* out = fgather + 3 * node;
    out[0] = out[1] = out[2] = 0.0;
    if (nr.material < 0 || !any_positive(nr.Kd)) return;
    double total[3] = {0, 0, 0};
    for (int sl = 0; sl < G; ++sl)
        for (int k = 0; k < 3; ++k) total[k] += gather_col[3 * (t * G + sl) + k];
    const double sc = 2 * kPi / (double)G;
    for (int k = 0; k < 3; ++k) out[k] = (total[k] * sc) * nr.Kd[k];
}

// shade_hit's GI block (renderer.c:727-770): ambient += indirect, final gather, caustics; clamp to sqrt(3)
__global__ void __launch_bounds__(kBlock) k_gi_apply(DevScene S, NodeCols rec, int64_t n,
                                                     const double* __restrict__ gi_extra,
                                                     const double* __restrict__ fgather, Cols<Tri9> surface) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NodeRec nr = rec.load(i, S.materials);
    if (nr.material < 0 || !any_positive(nr.Kd)) return;
    double a[12];
    tri_load(surface, i, a);
    for (int k = 0; k < 3; ++k) a[k] += gi_extra[6 * i + k];
    if (fgather != nullptr)
        for (int k = 0; k < 3; ++k) a[k] += fgather[3 * i + k];
    for (int k = 0; k < 3; ++k) a[k] += gi_extra[6 * i + 3 + k];
    const double len = a[0] + a[1] + a[2];
    if (len > 1.7320508075688772) {
        for (int k = 0; k < 3; ++k) a[k] *= 1.0 / len;
        for (int k = 0; k < 3; ++k) a[k] *= 1.7320508075688772;
    }
    tri_store(surface, i, a);
}

}  // namespace frt

// ======================================================================
// host side: scene upload, buffer management, frame driver, C ABI
// ======================================================================

// per-launch lines, node sites, beam sites; the tile kernel's beam sites at 1024 + 6144 + 2048
constexpr size_t kJitStatWords = 16384;

// Page-locked host memory for the counts the host reads back to size its next launch (a pageable destination
// costs ~16 us more per read-back: tools/microbench/sync.hip, profiles/r05_sync_latency.txt)
template <typename T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    bool resize(size_t m) {  // (contents zeroed)
        if (m > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            n = 0;
            if (hipHostMalloc((void**)&p, m * sizeof(T), hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                return false;
            }
            n = m;
        }
        std::memset(p, 0, n * sizeof(T));
        return true;
    }
    T* data() { return p; }
    const T* data() const { return p; }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
};

struct frt_scene_handle {
    int device = 0;
    frt::DevScene S{};
    std::vector<void*> owned;
    hipStream_t stream = nullptr;
    // light-sample lookup for k_shadow
    int32_t* j_light = nullptr;
    int32_t* j_point = nullptr;
    int32_t samples_per_node = 0;
    size_t lds_bytes = 0;  // dynamic LDS of the traversal kernels
    // scene-specialised shadow kernel (frt_jit.hip); nullptr: the generic k_shadow runs
    void* jit_shadow = nullptr;
    void* jit_beam = nullptr;          // its pair kernel (frt_jit_beam)
    void* jit_tile = nullptr;          // tile pair kernel (frt_jit_tile) and its listed tiles' node pairs
    void* jit_list = nullptr;          //   (frt_jit_beam_list); null: frt_jit_beam decides every pair
    int tile = 0;                      // path nodes per tile (frt_jit_tile_size), 0 without the tile kernels
    uint64_t scene_key = 0;            // hash of the flattened scene's content (shared photon maps)
    void* jit_sub = nullptr;           // sub-part pair kernel (frt_jit_sub); null: the node pairs' rays are walked
    int sub = 0;                       // sub-parts per part (frt_jit_sub_count) with jit_sub, else 0
    int sub_ps = 0;                    // samples per sub-part slot (frt_jit_sub_ps)
    const int32_t* light_psamp2 = nullptr;  // the sub-parts' samples (frt_jit_light_subparts), -1 padded
    const float* light_sbox = nullptr;      // the sub-parts' boxes over every cache row, binary32 outward
    uint32_t* slist = nullptr;         // the tile sub-pairs left mixed (frt_jit_sub's list), kMixSegs segments
    int64_t slist_cap = 0;
    uint64_t sub_pairs = 0, sub_mixed = 0;
    void* jit_subtile = nullptr;       // sub-tile pair kernel (frt_jit_subtile); null: whole tiles to frt_jit_beam_list
    void* jit_trace = nullptr;         // closest-hit kernel (frt_jit_trace); null: k_trace for every ray
    int32_t* tredo = nullptr;          // rays frt_jit_trace hands to the generic walk (k_trace_redo), + counter
    int64_t tredo_cap = 0;
    int subtile = 0;                   // path nodes per sub-tile (frt_jit_subtile_size) with jit_subtile, else 0
    // the (node, sample) pairs the sub-part / sub-tile stages leave: decided by frt_jit_beam_list one node beam per
    // lane (FRT_JIT_NODE_BEAM=1), or walked by frt_jit_shadow directly (the default: a node's beam to one sample is
    // one ray, and the per-ray walk costs a third of the beam walk's instructions; round 5, profiles/r05_ab_nodebeam.txt:
    // headline 41.5 -> 36.4 ms, shipped light 90.5 -> 76.4 ms)
    bool node_beam = false;
    float* stbox = nullptr;            // the level's sub-tile boxes (k_prepare): 6 floats per sub-tile
    int64_t stbox_cap = 0;
    uint32_t* s2list = nullptr;        // the sub-tile pairs left mixed (frt_jit_subtile's list)
    int64_t s2list_cap = 0;
    uint64_t subtile_pairs = 0, subtile_mixed = 0;
    float* tbox = nullptr;             // the level's tile boxes (k_prepare): 6 floats per tile
    int64_t tbox_cap = 0;
    uint32_t* tlist = nullptr;         // undecided (tile, light part) pairs, kMixSegs segments
    int64_t tlist_cap = 0;
    uint64_t tile_pairs = 0, tile_mixed = 0, node_pairs = 0, node_mixed = 0;  // this frame's pair-kernel counts
    bool jit_beam_on = true;           // FRT_JIT_BEAM=0: every pair is walked ray by ray (A/B)
    const int32_t* light_psamp = nullptr;  // the parts' samples (frt_jit_light_parts), -1 padded
    const float* light_aabb = nullptr; // per light, per cache row: the points' box (binary32, outward)
    uint32_t* mixed = nullptr;         // mixed (node, light) pairs, kMixSegs segments
    int64_t mixed_cap = 0;
    unsigned* mcount = nullptr;        // the segments' counters (kMixSegs lines of kMixLine words): four regions, one per
                                       // stage of a shadow pass (tile, sub-part, sub-tile, node pairs), zeroed together
    uint64_t sync_epoch = 0;           // stream_sync calls (the level loop's early counter read-back)
    PinnedBuf<unsigned> host_mcount;
    PinnedBuf<unsigned long long> host_counters;  // (the level's queue counters, read back per level)
    PinnedBuf<unsigned> host_lcount;  // (k_shade's list counts: the row sort's size, the lit-node statistic)
    int64_t* redo = nullptr;           // lanes handed back to the generic walk
    unsigned* redo_count = nullptr;
    unsigned redo_cap = 0;
    frt_frame_stats* cur_st = nullptr;  // the instrumented frame's stats (sub-kernel timers), else null
    uint64_t rays_walked = 0;           // shadow rays walked one by one in this frame
    uint64_t pairs_walked = 0;          // (node, light part) pairs they belong to (list entries walked)
    uint64_t heads_walked = 0;          // ShadowHeads the per-ray kernel read (a node per lane group of an entry)
    unsigned long long uniform_stats[3] = {0, 0, 0};  // FRT_JIT_STATS: (node, light) pairs all lit / all shadowed / mixed
    // k_shade's list of nodes with light-point work (kShadeSegs segments) and its segment counters
    uint32_t* shade_lit = nullptr;
    int64_t shade_lit_cap = 0;
    // the lit list in row order (k_shade -> k_lit_rows -> radix sort) for a multi-row light: the listed nodes' rows
    // (keys, and the sort's alternate buffer), the ordered list (and the unsorted values)
    int sort_light = -1;               // the first light with more than one cache row (FRT_SHADE_SORT=0: none)
    int shade_stage = 0;               // its shading from staged records / into row order (FRT_SHADE_STAGE)
    uint32_t* lit_row = nullptr;
    int64_t lit_row_cap = 0;
    uint32_t* lit_flat = nullptr;
    int64_t lit_flat_cap = 0;
    frt::LitStage* lit_stage = nullptr;  // (k_lit_stage's records, FRT_SHADE_STAGE)
    int64_t lit_stage_cap = 0;
    int queue_sort = 2;                 // a level's queue in parent order (FRT_QUEUE_SORT: 2 dense, 1 sorted, 0 off)
    int queue_sort_shift = 0;           // (FRT_QUEUE_SORT_SHIFT)
    uint32_t* qsort = nullptr;          // (its keys, their alternate buffer and the storage slots, 3 words per entry)
    int64_t qsort_cap = 0;
    unsigned long long* spawn_masks = nullptr;  // (FRT_QUEUE_SORT=2: the next level's taken slots, k_prepare)
    int64_t spawn_masks_cap = 0;
    uint32_t* spawn_offs = nullptr;              // (their popcounts' exclusive scan)
    int64_t spawn_offs_cap = 0;
    unsigned char* scan_tmp = nullptr;  // (the device sort's temporary storage)
    int64_t scan_tmp_cap = 0;
    unsigned* shade_lcount = nullptr;
    int64_t shade_lcount_cap = 0;
    unsigned long long* jit_stats = nullptr;  // FRT_JIT_STATS=1: 64 lines x 32 words, [0] live lanes, [1] binary64 re-walks;
                                              // then {waves, lanes} per node (frt_jit_rt.hpp node_stat)
    // work buffers (grow on demand)
    struct Level {
        frt::NodeCols rec;
        frt::ShadowHead* head = nullptr;
        frt::QueuedRay* q = nullptr;
        frt::Cols<frt::Tri9> surface;
        frt::Cols<frt::Tri9> child;  // two slots per node: i (reflected), cap + i (refracted), cap = the level's
        int64_t* qprefix = nullptr;                     // queue segments of this level (frt_shadow.hpp)
        std::vector<int64_t> hprefix = std::vector<int64_t>(frt::kQueueSegs + 1, 0);
        int32_t* counts = nullptr;
        uint32_t* spos = nullptr;  // (lit nodes shaded from staged records: a node's sorted position, k_shade_lit)
        bool staged = false;       // this batch's shading of the level went through k_lit_stage
        uint32_t* qperm = nullptr;  // (the queue in parent order, k_queue_keys + radix sort; qperm_cap entries)
        int64_t qperm_cap = 0;
        bool sorted = false;        // this batch's queue of the level is read through qperm
        int64_t cap = 0;
    };
    std::vector<Level> levels;
    frt::HitRec* hits = nullptr;  // closest hits of the level being traced
    int64_t hits_cap = 0;
    double* hn12 = nullptr;  // the refractive indices of the level's hits (scenes with indices other than one)
    int64_t hn12_cap = 0;
    frt::Cols<frt::Tri9> sample_col;
    int64_t sample_cap = 0;
    double* out_dev = nullptr;
    int64_t out_cap = 0;
    // kQueueSegs lines of kCounterLine words: [d] queue segment count of level d, [16] pruned,
    // [17] shaded path nodes (per segment); line 0 [24] / [25]: photon store / photon queue
    unsigned long long* counters = nullptr;
    unsigned* err = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct Mark {
        int slot;
        size_t a, b;
    };
    std::vector<hipEvent_t> ev_pool;
    std::vector<Mark> ev_marks;
    size_t ev_used = 0;
    // global illumination: photon maps (traced per render seed) and work buffers
    std::vector<frt_light> host_lights;
    struct Gi {
        bool built = false;
        uint64_t seed = 0;
        void* map_mem[2] = {nullptr, nullptr};  // one allocation per map: pos | power | dir | start
        uint64_t photons[2] = {0, 0};
        frt::QueuedRay* pq[2] = {nullptr, nullptr};
        double* ppow[2] = {nullptr, nullptr};
        int64_t pq_cap[2] = {0, 0}, ppow_cap[2] = {0, 0};
        frt::HitRec* phits = nullptr;
        int64_t phits_cap = 0;
        double* pn12 = nullptr;  // (as hn12, for the photons' hits)
        int64_t pn12_cap = 0;
        frt::StoredPhoton* store = nullptr;
        int64_t store_cap = 0;
        frt::QueuedRay* gq = nullptr;
        frt::HitRec* ghits = nullptr;
        double* gcol = nullptr;
        frt::GatherReq* greq = nullptr;
        int64_t gq_cap = 0, ghits_cap = 0, gcol_cap = 0, greq_cap = 0;
        unsigned* gwork = nullptr;  // k_gather_est's queue counters (one 256-byte line per XCD group)
        uint32_t* gkeys = nullptr;  // the requests' sort keys and indices (and the sort's alternate buffers)
        int64_t gkeys_cap = 0;
        double* extra = nullptr;
        double* fgather = nullptr;
        int64_t extra_cap = 0, fgather_cap = 0;
    } gi;
};

static thread_local std::string g_last_error;

static inline void hip_ignore(hipError_t) {}

static int fail(const std::string& msg) {
    g_last_error = msg;
    return -1;
}

#define FRT_HIP(call)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) return fail(std::string(#call) + ": " + hipGetErrorString(e_));          \
    } while (0)

template <typename T>
static const T* upload(frt_scene_handle* h, const T* src, size_t count, int& rc) {
    if (count == 0 || src == nullptr) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e != hipSuccess) {
        rc |= fail(std::string("hipMalloc: ") + hipGetErrorString(e));
        return nullptr;
    }
    h->owned.push_back(p);
    e = hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        rc |= fail(std::string("hipMemcpy: ") + hipGetErrorString(e));
        return nullptr;
    }
    return (const T*)p;
}

template <typename T>
static int grow(T** p, int64_t& cap, int64_t need) {
    if (need <= cap) return 0;
    int64_t nc = std::max<int64_t>(need, cap * 2);
    if (*p) FRT_HIP(hipFree(*p));
    *p = nullptr;
    FRT_HIP(hipMalloc((void**)p, (size_t)nc * sizeof(T)));
    cap = nc;
    return 0;
}

__global__ void k_warm(unsigned* p) { p[threadIdx.x] += 1u; }

extern "C" {

int frt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ---- meshes (frt_traverse.hpp MeshDesc): group subtrees of groups and triangles only ----
// A mesh root: a group whose children are all groups without transforms or triangles without transforms,
// recursively (the group itself may carry a transform: the walk applies it before the search), outside
// any CSG, with at least kMeshMinTris triangles, and not inside a larger one. Scenes the scene-specialised
// shadow kernel takes (<= 512 nodes) keep the plain walk.
constexpr int kMeshMinTris = 64;

struct MeshBuild {
    struct Tri {
        double lo[3], hi[3], c[3];
        int32_t node, prim;
    };
    std::vector<Tri> tris;
    std::vector<frt::MeshNode> nodes;
    std::vector<int2> refs;
    int depth = 0;

    static float down(double v) {
        float f = (float)v;
        if ((double)f > v) f = std::nextafter(f, -INFINITY);
        return f;
    }
    static float up(double v) {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, INFINITY);
        return f;
    }
    struct Sub {
        double lo[3], hi[3];
        int32_t ref, mindfs;
    };
    // binned SAH over tris[b, e); returns the subtree's box, reference and smallest pre-order index
    Sub build(int b, int e, int d) {
        depth = std::max(depth, d);
        Sub out;
        for (int a = 0; a < 3; ++a) {
            out.lo[a] = INFINITY;
            out.hi[a] = -INFINITY;
        }
        out.mindfs = 0x7fffffff;
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                out.lo[a] = std::min(out.lo[a], tris[(size_t)i].lo[a]);
                out.hi[a] = std::max(out.hi[a], tris[(size_t)i].hi[a]);
                clo[a] = std::min(clo[a], tris[(size_t)i].c[a]);
                chi[a] = std::max(chi[a], tris[(size_t)i].c[a]);
            }
        for (int i = b; i < e; ++i) out.mindfs = std::min(out.mindfs, tris[(size_t)i].node);
        const int n = e - b;
        if (n <= 4) {  // leaf: triangles in pre-order
            std::sort(tris.begin() + b, tris.begin() + e, [](const Tri& x, const Tri& y) { return x.node < y.node; });
            const int first = (int)refs.size();
            for (int i = b; i < e; ++i) refs.push_back(make_int2(tris[(size_t)i].node, tris[(size_t)i].prim));
            out.ref = ~((first << 3) | (n - 1));
            return out;
        }
        constexpr int kBins = 16;
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        int mid = b + n / 2;
        const double ext = chi[axis] - clo[axis];
        if (ext > 0.0) {
            struct Bin {
                double lo[3], hi[3];
                int n = 0;
            } bins[kBins];
            for (auto& bn : bins)
                for (int a = 0; a < 3; ++a) {
                    bn.lo[a] = INFINITY;
                    bn.hi[a] = -INFINITY;
                }
            auto bin_of = [&](const Tri& t) {
                return std::min(kBins - 1, (int)((t.c[axis] - clo[axis]) / ext * kBins));
            };
            for (int i = b; i < e; ++i) {
                Bin& bn = bins[bin_of(tris[(size_t)i])];
                bn.n++;
                for (int a = 0; a < 3; ++a) {
                    bn.lo[a] = std::min(bn.lo[a], tris[(size_t)i].lo[a]);
                    bn.hi[a] = std::max(bn.hi[a], tris[(size_t)i].hi[a]);
                }
            }
            auto area = [](const double* lo, const double* hi) {
                const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
                return x < 0 ? 0.0 : 2.0 * (x * y + y * z + z * x);
            };
            double best = INFINITY;
            int split = -1;
            for (int k = 1; k < kBins; ++k) {
                double l0[3] = {INFINITY, INFINITY, INFINITY}, h0[3] = {-INFINITY, -INFINITY, -INFINITY};
                double l1[3] = {INFINITY, INFINITY, INFINITY}, h1[3] = {-INFINITY, -INFINITY, -INFINITY};
                int n0 = 0, n1 = 0;
                for (int j = 0; j < kBins; ++j) {
                    double* lo = j < k ? l0 : l1;
                    double* hi = j < k ? h0 : h1;
                    (j < k ? n0 : n1) += bins[j].n;
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = std::min(lo[a], bins[j].lo[a]);
                        hi[a] = std::max(hi[a], bins[j].hi[a]);
                    }
                }
                if (n0 == 0 || n1 == 0) continue;
                const double cost = area(l0, h0) * n0 + area(l1, h1) * n1;
                if (cost < best) {
                    best = cost;
                    split = k;
                }
            }
            if (split > 0) {
                auto it = std::partition(tris.begin() + b, tris.begin() + e,
                                         [&](const Tri& t) { return bin_of(t) < split; });
                mid = (int)(it - tris.begin());
            }
        }
        if (mid <= b || mid >= e) {  // (degenerate centroids) halves in pre-order
            std::sort(tris.begin() + b, tris.begin() + e, [](const Tri& x, const Tri& y) { return x.node < y.node; });
            mid = b + n / 2;
        }
        const int self = (int)nodes.size();
        nodes.emplace_back();
        const Sub l = build(b, mid, d + 1), r = build(mid, e, d + 1);
        frt::MeshNode& N = nodes[(size_t)self];
        const Sub* c[2] = {&l, &r};
        for (int k = 0; k < 2; ++k) {
            for (int a = 0; a < 3; ++a) {
                N.b[6 * k + a] = down(c[k]->lo[a]);
                N.b[6 * k + 3 + a] = up(c[k]->hi[a]);
            }
            N.child[k] = c[k]->ref;
            N.mindfs[k] = c[k]->mindfs;
        }
        out.ref = self;
        return out;
    }
};

// the scene's mesh roots (host): see kMeshMinTris above
static std::vector<int> mesh_roots(const frt_scene* sc) {
    const int nn = sc->num_nodes;
    std::vector<int> roots;
    const char* env = std::getenv("FRT_MESH");  // FRT_MESH=0: the plain walk everywhere (A/B runs)
    if (nn <= 512 || (env && std::strcmp(env, "0") == 0)) return roots;
    auto is_tri = [&](int i) { return sc->nodes[i].type == FRT_TRIANGLE || sc->nodes[i].type == FRT_SMOOTH_TRIANGLE; };
    // inner[i]: node i may sit inside a mesh (a triangle or a group without transform of such nodes)
    std::vector<char> inner((size_t)nn, 0), in_csg((size_t)nn, 0);
    std::vector<int> ntri((size_t)nn, 0);
    for (int i = 0; i < nn; ++i) {
        const int par = sc->nodes[i].parent;
        in_csg[(size_t)i] = par >= 0 && (in_csg[(size_t)par] || sc->nodes[par].type == FRT_CSG);
    }
    auto children_inner = [&](int i) {
        for (int j = i + 1; j < sc->nodes[i].skip; j = sc->nodes[j].skip)
            if (!inner[(size_t)j]) return false;
        return true;
    };
    for (int i = nn - 1; i >= 0; --i) {
        const frt_node& nd = sc->nodes[i];
        if (is_tri(i)) {
            inner[(size_t)i] = nd.xform < 0;
            ntri[(size_t)i] = 1;
        } else if (nd.type == FRT_GROUP) {
            for (int j = i + 1; j < nd.skip; j = sc->nodes[j].skip) ntri[(size_t)i] += ntri[(size_t)j];
            inner[(size_t)i] = nd.xform < 0 && nd.skip > i + 1 && children_inner(i);
        }
    }
    for (int i = 0; i < nn; ++i) {
        const frt_node& nd = sc->nodes[i];
        if (nd.type != FRT_GROUP || in_csg[(size_t)i] || nd.skip <= i + 1 || !children_inner(i) ||
            ntri[(size_t)i] < kMeshMinTris)
            continue;
        const int par = nd.parent;
        if (par >= 0 && inner[(size_t)i] && sc->nodes[par].type == FRT_GROUP && children_inner(par) &&
            !in_csg[(size_t)par])
            continue;  // inside a larger mesh (a root's ancestors are never all inner, so roots do not nest)
        roots.push_back(i);
    }
    return roots;
}

// the BVHs of the mesh roots (host; a pool of at most 16 threads takes the meshes one by one)
static std::vector<MeshBuild> mesh_build(const frt_scene* sc, const std::vector<int>& roots) {
    std::vector<MeshBuild> mb(roots.size());
    std::vector<std::thread> pool;
    std::atomic<size_t> next{0};
    const size_t nthreads = std::min<size_t>(roots.size(), 16);
    for (size_t t = 0; t < nthreads; ++t)
        pool.emplace_back([&]() {
          for (size_t m; (m = next.fetch_add(1)) < roots.size();) {
            const int g = roots[m];
            MeshBuild& B = mb[m];
            for (int j = g + 1; j < sc->nodes[g].skip; ++j) {
                if (sc->nodes[j].type != FRT_TRIANGLE && sc->nodes[j].type != FRT_SMOOTH_TRIANGLE) continue;
                MeshBuild::Tri t;
                const double* p = sc->prim_data + sc->nodes[j].prim;
                for (int a = 0; a < 3; ++a) {
                    const double v0 = p[FRT_TRI_P1 + a], v1 = v0 + p[FRT_TRI_E1 + a], v2 = v0 + p[FRT_TRI_E2 + a];
                    t.lo[a] = std::min(v0, std::min(v1, v2));
                    t.hi[a] = std::max(v0, std::max(v1, v2));
                    t.c[a] = 0.5 * (t.lo[a] + t.hi[a]);
                }
                t.node = j;
                t.prim = sc->nodes[j].prim;
                B.tris.push_back(t);
            }
            B.build(0, (int)B.tris.size(), 1);
          }
        });
    for (auto& t : pool) t.join();
    return mb;
}

constexpr int kMeshStackMax = 32;

// the scene's meshes: marks each root in wn (op = mesh index + 1), builds and uploads their BVHs;
// S.meshes / num_meshes / mesh_stack
static int build_meshes(frt_scene_handle* h, const frt_scene* sc, std::vector<frt::WalkNode>& wn) {
    frt::DevScene& S = h->S;
    S.meshes = nullptr;
    S.num_meshes = 0;
    S.mesh_stack = 0;
    const std::vector<int> roots = mesh_roots(sc);
    if (roots.empty()) return 0;
    std::vector<MeshBuild> mb = mesh_build(sc, roots);
    std::vector<frt::MeshDesc> desc(roots.size());
    int depth = 0;
    const int last_root = sc->num_roots > 0 ? sc->roots[sc->num_roots - 1] : -1;
    for (size_t m = 0; m < roots.size(); ++m) {
        int rc = 0;
        desc[m].nodes = upload(h, mb[m].nodes.data(), mb[m].nodes.size(), rc);
        desc[m].tris = upload(h, mb[m].refs.data(), mb[m].refs.size(), rc);
        if (rc) return -1;
        desc[m].root = roots[m];
        int top = roots[m];
        while (sc->nodes[top].parent >= 0) top = sc->nodes[top].parent;
        desc[m].last_root = top == last_root ? 1 : 0;
        depth = std::max(depth, mb[m].depth);
        wn[(size_t)roots[m]].op = (int32_t)m + 1;
    }
    int rc = 0;
    S.meshes = upload(h, desc.data(), desc.size(), rc);
    if (rc) return -1;
    S.num_meshes = (int32_t)roots.size();
    // the per-lane LDS stack of the mesh searches (4 * kTraceBlock bytes per entry in every traversal block):
    // capped, a search whose stack would overflow falls back to the group walk for its lane (mesh_closest /
    // mesh_first), so a degenerate BVH costs speed, never the upload
    S.mesh_stack = std::min(depth + 1, kMeshStackMax);
    return 0;
}

// walk visit records (frt_traverse.hpp WalkNode) of the flattened tree
static void build_walk_nodes(const frt_scene* sc, std::vector<frt::WalkNode>& wn) {
    auto invert4 = [](const double* m, double* out) -> bool {  // Gauss-Jordan, partial pivoting
        double a[4][8];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 8; ++c) a[r][c] = c < 4 ? m[4 * r + c] : (c - 4 == r ? 1.0 : 0.0);
        for (int c = 0; c < 4; ++c) {
            int p = c;
            for (int r = c + 1; r < 4; ++r)
                if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
            if (a[p][c] == 0.0) return false;
            for (int k = 0; k < 8; ++k) std::swap(a[c][k], a[p][k]);
            const double inv = 1.0 / a[c][c];
            for (int k = 0; k < 8; ++k) a[c][k] *= inv;
            for (int r = 0; r < 4; ++r)
                if (r != c) {
                    const double f = a[r][c];
                    for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
                }
        }
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) out[4 * r + c] = a[r][4 + c];
        return true;
    };
    wn.assign((size_t)std::max(1, sc->num_nodes), frt::WalkNode{});
    std::vector<std::array<double, 12>> comp((size_t)std::max(1, sc->num_nodes));
    for (int i = 0; i < sc->num_nodes; ++i) {
        const frt_node& nd = sc->nodes[i];
        frt::WalkNode& w = wn[(size_t)i];
        std::memset(&w, 0, sizeof(w));
        w.type = nd.type;
        w.skip = nd.skip;
        w.right = nd.right;
        w.op = nd.type == FRT_CSG ? nd.prim : 0;
        w.prim = nd.type == FRT_CSG || nd.type == FRT_GROUP ? 0 : nd.prim;
        w.has_xf = nd.xform >= 0 ? 1 : 0;
        const int m = nd.material;
        w.casts = (m >= 0 && m < sc->num_materials && sc->materials[m].casts_shadow) ? 1 : 0;
        for (int k = 0; k < 6; ++k) {
            w.bbox[k] = nd.bbox[k];
            w.bb32[k] = (float)nd.bbox[k];
        }
        for (int a = 0; a < 3; ++a)  // rounded up: box32's error bound must not shrink
            w.bmag[a] = std::nextafter((float)std::max(std::fabs(nd.bbox[a]), std::fabs(nd.bbox[a + 3])), INFINITY);
        const double* mi = nd.xform >= 0 ? sc->xforms + 16 * (size_t)nd.xform : nullptr;
        if (mi)
            for (int k = 0; k < 12; ++k) w.m[k] = mi[k];
        // composed world -> node map: C = M_node * C_parent (pre-order: the parent is done)
        w.parent = nd.parent;
        {
            double cp[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
            if (nd.parent >= 0) std::memcpy(cp, comp[(size_t)nd.parent].data(), sizeof(cp));
            double c[12];
            if (mi) {
                for (int r = 0; r < 3; ++r) {
                    for (int q = 0; q < 4; ++q) {
                        double v = 0.0;
                        for (int j = 0; j < 3; ++j) v += mi[4 * r + j] * cp[4 * j + q];
                        c[4 * r + q] = q == 3 ? v + mi[4 * r + 3] : v;
                    }
                }
            } else {
                std::memcpy(c, cp, sizeof(c));
            }
            std::memcpy(comp[(size_t)i].data(), c, sizeof(c));
            double n1 = 0.0, tt = 0.0;
            for (int r = 0; r < 3; ++r) {
                n1 = std::max(n1, std::fabs(c[4 * r]) + std::fabs(c[4 * r + 1]) + std::fabs(c[4 * r + 2]));
                tt = std::max(tt, std::fabs(c[4 * r + 3]));
                for (int q = 0; q < 4; ++q) w.cm[4 * r + q] = (float)c[4 * r + q];
            }
            w.cN = std::nextafter((float)(n1 * (1.0 + 1e-9)), INFINITY);
            w.cT = std::nextafter((float)(tt * (1.0 + 1e-9)), INFINITY);
            // axis-aligned frame (a signed permutation of the axes, up to entries below 2^-30 of a row's
            // largest, such as the remnants of cos(pi/2) in a 90-degree rotation): world-space slab planes
            // of cubes and finite composite boxes; local axis r tests world axis col[r]
            const bool slab_node = nd.type == FRT_CUBE || nd.type == FRT_GROUP || nd.type == FRT_CSG;
            bool aa = slab_node;
            int col[3] = {0, 1, 2};
            double small[3] = {0.0, 0.0, 0.0};
            for (int r = 0; r < 3 && aa; ++r) {
                int big = 0;
                for (int q = 1; q < 3; ++q)
                    if (std::fabs(c[4 * r + q]) > std::fabs(c[4 * r + big])) big = q;
                const double cb = std::fabs(c[4 * r + big]);
                if (!(cb > 0.0 && std::isfinite(cb))) aa = false;
                for (int q = 0; q < 3; ++q)
                    if (q != big) {
                        if (!(std::fabs(c[4 * r + q]) <= 0x1p-30 * cb)) aa = false;
                        small[r] += std::fabs(c[4 * r + q]);
                    }
                col[r] = big;
            }
            if (aa && (col[0] == col[1] || col[0] == col[2] || col[1] == col[2])) aa = false;
            double bmax = 0.0, sig = 0.0;
            for (int r = 0; r < 3 && aa; ++r) {
                const int wa = col[r];
                sig = std::max(sig, small[r] / std::fabs(c[4 * r + wa]));
                const double crw = c[4 * r + wa], cr3 = c[4 * r + 3];
                const double b0 = nd.type == FRT_CUBE ? -1.0 : nd.bbox[r], b1 = nd.type == FRT_CUBE ? 1.0 : nd.bbox[r + 3];
                const double B0 = (b0 - cr3) / crw, B1 = (b1 - cr3) / crw;
                if (!(std::isfinite(B0) && std::isfinite(B1) && std::isfinite(cr3))) {
                    aa = false;
                    break;
                }
                w.aab[wa] = (float)B0;
                w.aab[wa + 3] = (float)B1;
                if (!(std::isfinite(w.aab[wa]) && std::isfinite(w.aab[wa + 3]))) aa = false;
                bmax = std::max({bmax, std::fabs((double)w.aab[wa]), std::fabs((double)w.aab[wa + 3])});
                // |f32(d_w)| >= thr  =>  |local d_r| >= |c_rw d_w| - small_r >= EPSILON for the reference's
                // direction (relative error of f32(d) <= 6.6u, of the composed map and the chain ~1e-15)
                w.aathr[wa] = std::nextafter((float)((1e-5 + small[r]) / std::fabs(crw) * (1.0 + 1e-6)), INFINITY);
            }
            w.aa = aa ? 1 : 0;
            // a round sphere in the world: exact signed permutation (no remnants) with one |scale|
            w.sph_ok = 0;
            if (nd.type == FRT_SPHERE) {
                bool ok = true;
                int cl[3] = {-1, -1, -1};
                for (int r = 0; r < 3 && ok; ++r) {
                    int nz = 0;
                    for (int q = 0; q < 3; ++q)
                        if (c[4 * r + q] != 0.0) {
                            ++nz;
                            cl[r] = q;
                        }
                    ok = nz == 1 && std::isfinite(c[4 * r + cl[r]]) && std::isfinite(c[4 * r + 3]);
                }
                ok = ok && cl[0] != cl[1] && cl[0] != cl[2] && cl[1] != cl[2];
                if (ok) {
                    const double s0 = std::fabs(c[cl[0]]);
                    ok = s0 > 0.0 && std::fabs(c[4 + cl[1]]) == s0 && std::fabs(c[8 + cl[2]]) == s0;
                    for (int r = 0; r < 3 && ok; ++r) {
                        const double cen = -c[4 * r + 3] / c[4 * r + cl[r]];
                        w.sph[cl[r]] = (float)cen;
                        ok = std::isfinite(w.sph[cl[r]]);
                    }
                    const double rad = 1.0 / s0;
                    w.sph[3] = std::nextafter((float)(rad * (1.0 + 1e-6)), INFINITY);
                    ok = ok && std::isfinite(w.sph[3]) && rad > 1e-30;
                }
                w.sph_ok = ok ? 1 : 0;
            }
            w.aasig = aa && sig > 0.0 ? std::nextafter((float)(1.02 * sig), INFINITY) : 0.0f;
            w.aabmax = aa ? std::nextafter((float)(bmax * (1.0 + 1e-7)), INFINITY) : 0.0f;
        }
        for (int r = 0; r < 3; ++r) {
            w.mrow_l1[r] = 0.f;
            for (int c = 0; c < 3; ++c) {
                const double v = mi ? mi[4 * r + c] : (r == c ? 1.0 : 0.0);
                w.mrow[3 * r + c] = (float)v;
                w.mrow_l1[r] += (float)std::fabs(v);
            }
            w.mrow_l1[r] *= 1.0001f;
        }
        // prefilter bound in the parent frame (frt_traverse.hpp): cubes, spheres and transformed composites
        const bool composite = nd.type == FRT_GROUP || nd.type == FRT_CSG;
        const bool want = nd.type == FRT_CUBE || nd.type == FRT_SPHERE || (composite && mi);
        double fwd[16];
        bool ok = want && (!mi || invert4(mi, fwd));
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        if (ok && nd.type == FRT_SPHERE) {
            for (int a = 0; a < 3; ++a) {
                const double c = mi ? fwd[4 * a + 3] : 0.0;
                const double e = mi ? std::sqrt(fwd[4 * a] * fwd[4 * a] + fwd[4 * a + 1] * fwd[4 * a + 1] +
                                                fwd[4 * a + 2] * fwd[4 * a + 2])
                                    : 1.0;
                lo[a] = c - e;
                hi[a] = c + e;
            }
        } else if (ok) {
            const double bl[3] = {composite ? nd.bbox[0] : -1.0, composite ? nd.bbox[1] : -1.0,
                                  composite ? nd.bbox[2] : -1.0};
            const double bh[3] = {composite ? nd.bbox[3] : 1.0, composite ? nd.bbox[4] : 1.0,
                                  composite ? nd.bbox[5] : 1.0};
            for (int a = 0; a < 3; ++a) ok = ok && std::isfinite(bl[a]) && std::isfinite(bh[a]);
            for (int c = 0; ok && c < 8; ++c) {
                const double p[3] = {(c & 1) ? bh[0] : bl[0], (c & 2) ? bh[1] : bl[1], (c & 4) ? bh[2] : bl[2]};
                for (int a = 0; a < 3; ++a) {
                    const double v = mi ? fwd[4 * a] * p[0] + fwd[4 * a + 1] * p[1] + fwd[4 * a + 2] * p[2] +
                                              fwd[4 * a + 3]
                                        : p[a];
                    lo[a] = std::min(lo[a], v);
                    hi[a] = std::max(hi[a], v);
                }
            }
        }
        for (int a = 0; a < 3; ++a) ok = ok && std::isfinite(lo[a]) && std::isfinite(hi[a]);
        if (ok) {
            for (int a = 0; a < 3; ++a) {
                const double pad = 1e-7 * ((hi[a] - lo[a]) + std::max(std::fabs(lo[a]), std::fabs(hi[a]))) + 1e-12;
                w.pbox[a] = lo[a] - pad;
                w.pbox[a + 3] = hi[a] + pad;
            }
            w.pre = 1 | (nd.type == FRT_SPHERE ? 0 : 2);
        } else {
            w.pre = 0;
        }
    }
}

// TEST INFRASTRUCTURE / diagnostics (include/frt_device.h): generate and compile the scene-specialised
// shadow kernel of a flattened scene without a device. Returns 0 compiled, 1 not eligible, -1 compile error;
// `log` receives the reason / compiler log, `src` (if non-null) the generated source.
int frt_jit_check(const frt_scene* sc, char* log, size_t log_cap, char* src, size_t src_cap) {
    std::vector<frt::WalkNode> wn;
    build_walk_nodes(sc, wn);
    std::string why, clog;
    const std::string code = frt_jit_shadow_source(wn.data(), sc->num_nodes, sc->roots, sc->num_roots, sc->lights, sc->num_lights, why);
    auto put = [](char* dst, size_t cap, const std::string& v) {
        if (dst && cap) {
            std::snprintf(dst, cap, "%s", v.c_str());
        }
    };
    put(src, src_cap, code);
    if (code.empty()) {
        put(log, log_cap, why);
        return 1;
    }
    const int rc = frt_jit_compile_only(code, "gfx950", clog);
    put(log, log_cap, clog);
    return rc == 0 ? 0 : -1;
}

// Diagnostics: sqrt_core / recip_core and normalize3 (frt_math.hpp) against the compiler's sqrt, division
// and normalize3_ref, bit for bit. Lane i of wave w: components (2u - 1) 2^k, k uniform in [-K, K] with
// K = 250 on even waves (every squared magnitude in the core range: the fast path) and 320 on odd ones
// (some out of range: the fallback); the core functions alone on x = m2 and y = sqrt(m2) of in-range lanes.
__global__ void k_math_selftest(int64_t n, uint64_t seed, unsigned long long* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;  // (whole waves: n is a multiple of 64)
    const int K = ((i >> 6) & 1) ? 320 : 250;
    double v[3];
    for (int a = 0; a < 3; ++a) {
        const uint64_t h = frt::mix64(seed ^ frt::mix64((uint64_t)i * 3 + (uint64_t)a + 0x9e3779b97f4a7c15ULL));
        const double u = (double)(h >> 11) * 0x1.0p-53;
        const int k = (int)((h & 0x3ff) % (uint64_t)(2 * K + 1)) - K;
        v[a] = __builtin_ldexp(2.0 * u - 1.0, k);
    }
    double r[3], q[3];
    frt::normalize3(v, r);
    frt::normalize3_ref(v, q);
    unsigned long long b = 0;
    for (int a = 0; a < 3; ++a) b += __double_as_longlong(r[a]) != __double_as_longlong(q[a]);
    const double m2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    if (m2 >= 0x1p-600 && m2 <= 0x1p600) {
        const double s = sqrt(m2);
        b += __double_as_longlong(frt::sqrt_core(m2)) != __double_as_longlong(s);
        b += __double_as_longlong(frt::recip_core(s)) != __double_as_longlong(1.0 / s);
        // the shading's approximations (FRT_SHADE_NEWTON steps): reciprocal magnitude, reciprocal and
        // quotient within 2^-46 relative of 1.0 / sqrt(), 1.0 / y and a / y
        const double inv = 1.0 / s;
        b += !(fabs(frt::rsqrt_nr(m2) - inv) <= 0x1p-46 * inv);
        b += !(fabs(frt::recip_shade(s) - inv) <= 0x1p-46 * inv);
        const double a = fabs(v[0]) >= 0x1p-600 ? fabs(v[0]) : 0.0;
        b += !(fabs(frt::div_shade(a, s) - a / s) <= 0x1p-46 * (a / s));
        // the BRDF factor with one reciprocal (brdf_shade) within 2^-44 relative of the reference's two quotients
        // (renderer.c:952-963), dot products from the unit vector's components
        const double nh = fabs(r[0]), eh = fabs(r[1]), nl = fabs(r[2]), ne = fmax(fabs(r[0] * r[1]), 0x1p-20);
        const double gc = 2.0 * nh * (1.0 / eh);
        const double ref = (a * fmin(1.0, fmin(gc * ne, gc * nl))) / (4.0 * nl * ne);
        const double got = frt::brdf_shade(a, nh, eh, nl, ne);
        if (__builtin_isfinite(ref)) b += !(got == ref || fabs(got - ref) <= 0x1p-44 * fabs(ref));
    }
    if (b) atomicAdd(bad, b);
}

// Diagnostics (host only): the scene's meshes and their BVHs, checked. out[0] meshes, out[1] triangles in
// them, out[2] BVH nodes, out[3] deepest BVH level. Returns 0 when every BVH is sound (each of the mesh's
// triangles in exactly one leaf; every child box contains its triangles' vertices and its children's
// boxes; every child's smallest pre-order index right), else the number of violations.
int frt_mesh_check(const frt_scene* sc, int64_t* out, int n) {
    const std::vector<int> roots = mesh_roots(sc);
    const std::vector<MeshBuild> mb = mesh_build(sc, roots);
    int64_t stats[4] = {(int64_t)roots.size(), 0, 0, 0};
    int64_t bad = 0;
    for (size_t m = 0; m < roots.size(); ++m) {
        const MeshBuild& B = mb[m];
        stats[1] += (int64_t)B.tris.size();
        stats[2] += (int64_t)B.nodes.size();
        stats[3] = std::max<int64_t>(stats[3], B.depth);
        std::vector<int> seen((size_t)sc->num_nodes, 0);
        // (box lo/hi, smallest pre-order index) of a child reference, recursively checked
        std::function<void(int32_t, const float*, int32_t)> check = [&](int32_t ref, const float* box, int32_t mindfs) {
            int32_t mn = 0x7fffffff;
            auto inside = [&](double v, int a) { return (double)box[a] <= v && v <= (double)box[3 + a]; };
            if (ref < 0) {
                const int code = ~ref, first = code >> 3, cnt = (code & 7) + 1;
                for (int k = 0; k < cnt; ++k) {
                    const int2 t = B.refs[(size_t)(first + k)];
                    seen[(size_t)t.x]++;
                    mn = std::min(mn, t.x);
                    const double* p = sc->prim_data + t.y;
                    for (int a = 0; a < 3; ++a) {
                        const double v0 = p[FRT_TRI_P1 + a];
                        if (!inside(v0, a) || !inside(v0 + p[FRT_TRI_E1 + a], a) || !inside(v0 + p[FRT_TRI_E2 + a], a))
                            bad++;
                    }
                }
            } else {
                const frt::MeshNode& N = B.nodes[(size_t)ref];
                for (int c = 0; c < 2; ++c) {
                    for (int a = 0; a < 3; ++a)
                        if (N.b[6 * c + a] < box[a] || N.b[6 * c + 3 + a] > box[3 + a]) bad++;
                    check(N.child[c], N.b + 6 * c, N.mindfs[c]);
                    mn = std::min(mn, N.mindfs[c]);
                }
            }
            if (mn != mindfs) bad++;
        };
        const float all[6] = {-INFINITY, -INFINITY, -INFINITY, INFINITY, INFINITY, INFINITY};
        const frt::MeshNode& R = B.nodes[0];
        check(0, all, std::min(R.mindfs[0], R.mindfs[1]));
        for (int j = roots[m] + 1; j < sc->nodes[roots[m]].skip; ++j) {
            const bool tri = sc->nodes[j].type == FRT_TRIANGLE || sc->nodes[j].type == FRT_SMOOTH_TRIANGLE;
            if (seen[(size_t)j] != (tri ? 1 : 0)) bad++;
        }
    }
    for (int i = 0; i < n && i < 4; ++i) out[i] = stats[i];
    return (int)std::min<int64_t>(bad, 1 << 30);
}

// Diagnostics (current device): k_math_selftest over n lanes (rounded up to whole waves); the number of
// mismatching values, or -1 on a HIP error.
int64_t frt_math_selftest(int64_t n, uint64_t seed) {
    n = (std::max<int64_t>(n, 64) + 63) / 64 * 64;
    unsigned long long* bad = nullptr;
    if (hipMalloc((void**)&bad, sizeof(unsigned long long)) != hipSuccess) return -1;
    unsigned long long h = 0;
    bool ok = hipMemset(bad, 0, sizeof(h)) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_math_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, seed, bad);
        ok = hipGetLastError() == hipSuccess && hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
    }
    hip_ignore(hipFree(bad));
    return ok ? (int64_t)h : -1;
}

const char* frt_last_error(void) { return g_last_error.c_str(); }

static std::atomic<long long> g_maps_stat[2];  // photon passes traced, photon passes shared (build_photon_maps)

// this thread's last frt_scene_upload, in ms (frt_upload_phases)
static thread_local double t_upload_phases[8];

// process-wide photon passes: out[0] traced, out[1] taken from another device's trace (build_photon_maps)
int frt_photon_pass_stats(int64_t* out, int n) {
    for (int i = 0; i < n && i < 2; ++i) out[i] = g_maps_stat[i].load();
    return 2;
}

size_t frt_frame_stats_size(void) { return sizeof(frt_frame_stats); }

// a stream frt_device_warmup created, handed to the device's next frt_scene_upload (a process's first streams cost
// 10-160 ms each: tools/warmup_probe.py, profiles/r05_warmup_probe.txt)
static std::mutex g_warm_mu;
static hipStream_t g_warm_stream[64] = {};

void* frt_host_pinned_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void frt_host_pinned_free(void* p) {
    if (p) hip_ignore(hipHostFree(p));
}

int frt_device_warmup(int device) {
    // (FRT_WARMUP_TRACE: each step's time to stderr)
    static const bool trace = std::getenv("FRT_WARMUP_TRACE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!trace) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "frt warmup: %s %.2f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    };
    if (hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    mark("hipSetDevice");
    hip_ignore(hipFree(nullptr));  // (creates the context)
    mark("context");
    // the first allocation, copies both ways and kernel launch of a process set up the runtime's memory pools,
    // staging buffers and this library's code object on the device: paid here, beside the caller's work
    void* p = nullptr;
    if (hipMalloc(&p, 1 << 20) == hipSuccess) {
        mark("hipMalloc");
        hipStream_t s = nullptr;
        // (FRT_WARMUP_MODE=1: the null stream instead of a stream of its own, probes only)
        static const int wmode = std::getenv("FRT_WARMUP_MODE") ? std::atoi(std::getenv("FRT_WARMUP_MODE")) : 0;
        if (wmode == 1 || hipStreamCreate(&s) == hipSuccess) {  // (the handle's kind of stream: it may take it)
            mark("stream");
            unsigned host[64] = {0};
            hip_ignore(hipMemcpyAsync(p, host, sizeof(host), hipMemcpyHostToDevice, s));
            hip_ignore(hipStreamSynchronize(s));
            mark("H2D copy");
            hipLaunchKernelGGL(k_warm, dim3(1), dim3(64), 0, s, (unsigned*)p);
            hip_ignore(hipStreamSynchronize(s));
            mark("first kernel (code object load)");
            hip_ignore(hipMemcpyAsync(host, p, sizeof(host), hipMemcpyDeviceToHost, s));
            hip_ignore(hipStreamSynchronize(s));
            mark("D2H copy");
            if (s) {
                std::lock_guard<std::mutex> lk(g_warm_mu);
                if (device >= 0 && device < 64 && g_warm_stream[device] == nullptr) g_warm_stream[device] = s;
                else hip_ignore(hipStreamDestroy(s));
            }
        }
        hip_ignore(hipFree(p));
    }
    (void)hipGetLastError();
    return 0;
}

int frt_upload_phases(double* out, int n) {
    for (int i = 0; i < n && i < 8; ++i) out[i] = t_upload_phases[i];
    return 8;
}

int frt_scene_upload(const frt_scene* sc, int device, frt_scene_handle** out) {
    const auto up0 = std::chrono::steady_clock::now();
    auto up_last = up0;
    auto phase = [&](int i) {  // the time since the previous mark into phase i
        const auto t = std::chrono::steady_clock::now();
        t_upload_phases[i] += std::chrono::duration<double, std::milli>(t - up_last).count();
        up_last = t;
    };
    for (double& x : t_upload_phases) x = 0.0;
    if (sc == nullptr || out == nullptr) return fail("frt_scene_upload: null argument");
    if (sc->abi_version != FRT_ABI_VERSION) return fail("frt_scene_upload: ABI version mismatch");
    int ndev = frt_device_count();
    if (ndev <= 0) return fail("frt_scene_upload: no HIP device visible");
    if (device < 0 || device >= ndev) return fail("frt_scene_upload: device index out of range");
    FRT_HIP(hipSetDevice(device));
    frt_scene_handle* h = new frt_scene_handle();
    h->device = device;
    frt::DevScene& S = h->S;
    int rc = 0;
    if (sc->config.trace_caustic_map || sc->config.trace_global_map) {
        // the scene's identity for the process-wide photon-map sharing (build_photon_maps), only for scenes that
        // trace photons: FNV-1a over 8-byte words (the shipped light cache alone is 157 MB)
        uint64_t k = 0xcbf29ce484222325ull;
        auto mix = [&](const void* p, size_t n) {
            const unsigned char* c = (const unsigned char*)p;
            size_t i = 0;
            for (; i + 8 <= n; i += 8) {
                uint64_t w;
                std::memcpy(&w, c + i, 8);
                k ^= w;
                k *= 0x100000001b3ull;
            }
            for (; i < n; ++i) {
                k ^= c[i];
                k *= 0x100000001b3ull;
            }
        };
        mix(sc->nodes, sizeof(frt_node) * (size_t)sc->num_nodes);
        mix(sc->roots, sizeof(int32_t) * (size_t)sc->num_roots);
        mix(sc->xforms, sizeof(double) * 16 * (size_t)sc->num_xforms);
        mix(sc->prim_data, sizeof(double) * (size_t)sc->prim_len);
        mix(sc->materials, sizeof(frt_material) * (size_t)sc->num_materials);
        mix(sc->patterns, sizeof(frt_pattern) * (size_t)sc->num_patterns);
        mix(sc->textures, sizeof(frt_texture) * (size_t)sc->num_textures);
        mix(sc->texels, sizeof(double) * (size_t)sc->texel_len);
        mix(sc->lights, sizeof(frt_light) * (size_t)sc->num_lights);
        mix(sc->light_points, sizeof(double) * (size_t)sc->light_point_len);
        mix(&sc->config, sizeof(frt_config));
        h->scene_key = k;
    }
    phase(0);
    S.nodes = upload(h, sc->nodes, (size_t)sc->num_nodes, rc);
    S.roots = upload(h, sc->roots, (size_t)sc->num_roots, rc);
    S.xforms = upload(h, sc->xforms, (size_t)sc->num_xforms * 16, rc);
    S.prim = upload(h, sc->prim_data, (size_t)sc->prim_len, rc);
    S.materials = upload(h, sc->materials, (size_t)sc->num_materials, rc);
    S.patterns = upload(h, sc->patterns, (size_t)sc->num_patterns, rc);
    S.textures = upload(h, sc->textures, (size_t)sc->num_textures, rc);
    S.texels = upload(h, sc->texels, (size_t)sc->texel_len, rc);
    S.lights = upload(h, sc->lights, (size_t)sc->num_lights, rc);
    S.light_points = upload(h, sc->light_points, (size_t)sc->light_point_len, rc);
    S.sample_table = upload(h, sc->sample_table, (size_t)(2 * sc->camera.usteps * sc->camera.vsteps), rc);
    {
        // per node: does the leaf's material cast shadows (read by the shadow walk)
        std::vector<uint8_t> casts((size_t)std::max(1, sc->num_nodes), 0);
        for (int i = 0; i < sc->num_nodes; ++i) {
            const int m = sc->nodes[i].material;
            casts[(size_t)i] = (m >= 0 && m < sc->num_materials && sc->materials[m].casts_shadow) ? 1 : 0;
        }
        S.casts = upload(h, casts.data(), casts.size(), rc);
        // per node: its transform chain root-most first (frt_traverse.hpp xf_chain), n = -1 past three
        std::vector<int4> xchain((size_t)std::max(1, sc->num_nodes), make_int4(0, 0, 0, 0));
        for (int i = 0; i < sc->num_nodes; ++i) {
            int ids[64], n = 0;
            for (int x = sc->nodes[i].xform >= 0 ? i : sc->nodes[i].tparent; x >= 0 && n < 64; x = sc->nodes[x].tparent)
                ids[n++] = sc->nodes[x].xform;
            if (n <= 3) xchain[(size_t)i] = make_int4(n, n > 0 ? ids[n - 1] : 0, n > 1 ? ids[n - 2] : 0, n > 2 ? ids[n - 3] : 0);
            else xchain[(size_t)i] = make_int4(-1, 0, 0, 0);
        }
        S.xchain = upload(h, xchain.data(), xchain.size(), rc);
    }
    if (rc) {
        frt_scene_release(h);
        return -1;
    }
    phase(1);
    {
        std::vector<frt::WalkNode> wn;
        build_walk_nodes(sc, wn);
        if (rc == 0 && build_meshes(h, sc, wn)) {
            frt_scene_release(h);
            return -1;
        }
        S.wn = upload(h, wn.data(), wn.size(), rc);
        const char* jit_env = std::getenv("FRT_JIT");
        if (rc == 0 && sc->config.include_direct && !(jit_env && std::strcmp(jit_env, "0") == 0)) {
            std::string why, log;
            phase(2);
            const std::string src = frt_jit_shadow_source(wn.data(), sc->num_nodes, sc->roots, sc->num_roots, sc->lights, sc->num_lights, why);
            phase(3);
            FrtJitFns fns;
            if (!src.empty() && frt_jit_compile(src, h->device, fns, log) != 0) {
                why = "hiprtc: " + log.substr(0, 2000);
                fns = FrtJitFns{};
            }
            if (!src.empty()) {
                double ob = 0.0, ld = 0.0;
                frt_jit_last_phases(&ob, &ld);
                t_upload_phases[4] += ob;
                t_upload_phases[5] += ld;
                up_last = std::chrono::steady_clock::now();
            }
            h->jit_shadow = fns.shadow;
            h->jit_beam = fns.beam;
            h->jit_tile = fns.tile;
            h->jit_list = fns.list;
            h->tile = fns.tile && fns.list ? frt_jit_tile_size() : 0;
            h->jit_sub = fns.sub;
            h->sub = fns.sub ? frt_jit_sub_count() : 0;
            h->jit_subtile = fns.subtile;
            // (the closest-hit kernel writes n1 = n2 = 1: scenes with refractive indices other than one keep k_trace)
            h->jit_trace = sc->config.all_ni_one ? fns.trace : nullptr;
            h->subtile = fns.subtile ? frt_jit_subtile_size() : 0;
            // (multi-row lights get no sub-tile kernel unless FRT_JIT_SUBTILE asks for one, frt_jit_shadow_source: the
            // stage cut the shipped frame's per-ray lanes by 11 % for 6.5 ms; without it 76.4 -> 72.1 ms,
            // profiles/r05_ab_nodebeam.txt)
            if (h->jit_shadow) {
                h->redo_cap = 1u << 20;
                void* p = nullptr;
                if (hipMalloc(&p, h->redo_cap * sizeof(int64_t) + 64) != hipSuccess) {
                    frt_scene_release(h);
                    return fail("frt_scene_upload: redo queue allocation failed");
                }
                h->owned.push_back(p);
                h->redo = (int64_t*)p;
                h->redo_count = (unsigned*)(h->redo + h->redo_cap);
                const char* beam_env = std::getenv("FRT_JIT_BEAM");
                h->jit_beam_on = !(beam_env && std::strcmp(beam_env, "0") == 0);
                // each light's parts (frt_jit_light_parts) and, per cache row, the box of each part's points,
                // rounded outward to binary32; with a multi-row light (the shipped area-light cache) also, after
                // every light's row boxes, each part's box over all rows (the tile kernel's: a tile's nodes draw
                // different rows). The reference's CMJ keeps sample (u, v) of every row in light cell (u, v)
                // (sampler.c:423-460: the x shuffle swaps within a column, the y shuffle within a row), so the
                // union stays the size of the part's cells.
                std::vector<float> box;
                std::vector<int32_t> psamp;
                const int PS = frt_jit_part_size();
                auto push_box = [](std::vector<float>& v, const double* pl, const double* ph) {
                    for (int a = 0; a < 3; ++a) {
                        float f = (float)pl[a];
                        if ((double)f > pl[a]) f = std::nextafter(f, -INFINITY);
                        v.push_back(f);
                    }
                    for (int a = 0; a < 3; ++a) {
                        float f = (float)ph[a];
                        if ((double)f < ph[a]) f = std::nextafter(f, INFINITY);
                        v.push_back(f);
                    }
                };
                // the box of samples idx[0..cnt) (-1 entries skipped) over rows [r0, r1)
                auto sample_box = [&](const frt_light& lt, const int32_t* idx, int cnt, int r0, int r1, double* pl, double* ph) {
                    for (int a = 0; a < 3; ++a) {
                        pl[a] = INFINITY;
                        ph[a] = -INFINITY;
                    }
                    for (int r = r0; r < r1; ++r)
                        for (int k = 0; k < cnt; ++k) {
                            const int q = idx[k];
                            if (q < 0) continue;
                            const double* pt = sc->light_points + lt.points + 3 * ((int64_t)r * lt.num_samples + q);
                            for (int a = 0; a < 3; ++a) {
                                pl[a] = std::min(pl[a], pt[a]);
                                ph[a] = std::max(ph[a], pt[a]);
                            }
                        }
                };
                bool multi_row = false;
                std::vector<std::vector<int32_t>> orders((size_t)sc->num_lights);
                for (int l = 0; l < sc->num_lights; ++l) {
                    const frt_light& lt = sc->lights[l];
                    multi_row = multi_row || lt.rows > 1;
                    std::vector<int32_t>& order = orders[(size_t)l];
                    const int np = frt_jit_light_parts(lt, sc->light_points, PS, order);
                    psamp.insert(psamp.end(), order.begin(), order.end());
                    for (int r = 0; r < std::max(1, lt.rows); ++r)
                        for (int p = 0; p < np; ++p) {
                            double pl[3], ph[3];
                            sample_box(lt, order.data() + (size_t)p * PS, PS, r, r + 1, pl, ph);
                            push_box(box, pl, ph);
                        }
                }
                for (int l = 0; multi_row && l < sc->num_lights; ++l) {
                    const frt_light& lt = sc->lights[l];
                    const int np = (int)(orders[(size_t)l].size() / (size_t)PS);
                    for (int p = 0; p < np; ++p) {
                        double pl[3], ph[3];
                        sample_box(lt, orders[(size_t)l].data() + (size_t)p * PS, PS, 0, std::max(1, lt.rows), pl, ph);
                        push_box(box, pl, ph);
                    }
                }
                h->light_psamp = upload(h, psamp.data(), psamp.size(), rc);
                h->light_aabb = upload(h, box.data(), box.size(), rc);
                {
                    const char* nb = std::getenv("FRT_JIT_NODE_BEAM");
                    h->node_beam = nb && std::atoi(nb) != 0;
                }
                if (h->sub > 0) {  // the sub-parts: samples and boxes (over every cache row) by (global part, sub-part)
                    std::vector<int32_t> ps2;
                    std::vector<float> sbox;
                    const int Q = h->sub;
                    for (int l = 0; l < sc->num_lights; ++l) {
                        const frt_light& lt = sc->lights[l];
                        const int np = std::max(1, (lt.num_samples + PS - 1) / PS);
                        std::vector<int32_t> order2;
                        h->sub_ps = frt_jit_light_subparts(lt, sc->light_points, orders[(size_t)l], PS, Q, order2);
                        ps2.insert(ps2.end(), order2.begin(), order2.end());
                        for (int p = 0; p < np * Q; ++p) {
                            double pl[3], ph[3];
                            sample_box(lt, order2.data() + (size_t)p * h->sub_ps, h->sub_ps, 0, std::max(1, lt.rows), pl, ph);
                            push_box(sbox, pl, ph);
                        }
                    }
                    h->light_psamp2 = upload(h, ps2.data(), ps2.size(), rc);
                    h->light_sbox = upload(h, sbox.data(), sbox.size(), rc);
                }
                if (rc || hipMalloc((void**)&h->mcount, 4 * frt::jit::kMixSegs * frt::jit::kMixLine * sizeof(unsigned)) != hipSuccess) {
                    frt_scene_release(h);
                    return fail("frt_scene_upload: light box / pair list allocation failed");
                }
                h->owned.push_back(h->mcount);
                if (!h->host_mcount.resize((size_t)frt::jit::kMixSegs * frt::jit::kMixLine)) {
                    frt_scene_release(h);
                    return fail("frt_scene_upload: pinned host buffer allocation failed");
                }
                if (std::getenv("FRT_JIT_STATS")) {
                    if (hipMalloc((void**)&h->jit_stats, kJitStatWords * sizeof(unsigned long long)) != hipSuccess) {
                        frt_scene_release(h);
                        return fail("frt_scene_upload: jit stats allocation failed");
                    }
                    h->owned.push_back(h->jit_stats);
                    hip_ignore(hipMemset(h->jit_stats, 0, kJitStatWords * sizeof(unsigned long long)));
                }
            } else if (std::getenv("FRT_JIT_VERBOSE")) {
                std::fprintf(stderr, "frt: generic shadow walk (%s)\n", why.c_str());
            }
            if (std::getenv("FRT_JIT_DUMP") && !src.empty()) std::fprintf(stderr, "%s\n", src.c_str());
        }
    }
    {
        // per-lane walk capacities (see frt_traverse.hpp): exact bounds from the tree
        static const int kMaxHits[10] = {4, 2, 4, 1, 1, 2, 4, 1, 0, 0};  // by frt_node_type
        const int nn = sc->num_nodes;
        std::vector<int> xf_cnt(nn, 0), comp_cnt(nn, 0), csg_top(nn, -1), list_need(nn, 0);
        int xf_depth = 0, comp_depth = 0, list_cap = 0, features = 0;
        for (int i = 0; i < nn; ++i) {
            const frt_node& nd = sc->nodes[i];
            const int par = nd.parent;
            const bool composite = nd.type == FRT_GROUP || nd.type == FRT_CSG;
            if (nd.type == FRT_CSG) features |= frt::kFeatCsg;
            if (nd.type == FRT_TOROID) features |= frt::kFeatTorus;
            csg_top[i] = par >= 0 && csg_top[par] >= 0 ? csg_top[par] : (nd.type == FRT_CSG ? i : -1);
            xf_cnt[i] = (par >= 0 ? xf_cnt[par] : 0) + (composite && nd.xform >= 0 ? 1 : 0);
            comp_cnt[i] = (par >= 0 && csg_top[par] >= 0 ? comp_cnt[par] : 0) + (composite && csg_top[i] >= 0 ? 1 : 0);
            xf_depth = std::max(xf_depth, xf_cnt[i]);
            comp_depth = std::max(comp_depth, comp_cnt[i]);
            if (!composite && csg_top[i] >= 0 && nd.type >= 0 && nd.type < 10) {
                list_need[csg_top[i]] += kMaxHits[nd.type];
                list_cap = std::max(list_cap, list_need[csg_top[i]]);
            }
        }
        S.list_cap = list_cap;
        S.comp_depth = comp_depth;
        S.xf_depth = xf_depth;
        S.features = features;
        h->lds_bytes = (size_t)frt::walk_lds_bytes(list_cap, comp_depth, xf_depth, S.mesh_stack);
        if (h->lds_bytes > 64 * 1024) {
            frt_scene_release(h);
            return fail("frt_scene_upload: scene needs " + std::to_string(h->lds_bytes) +
                        " B of LDS per traversal block (CSG lists / nesting too large)");
        }
    }
    {
        const char* wf = std::getenv("FRT_WALK_FLAGS");  // A/B experiments only
        S.walk_flags = wf ? std::atoi(wf) : 0;
    }
    S.num_nodes = sc->num_nodes;
    S.num_roots = sc->num_roots;
    S.num_lights = sc->num_lights;
    S.num_patterns = sc->num_patterns;
    S.cam = sc->camera;
    S.cfg = sc->config;
    h->host_lights.assign(sc->lights, sc->lights + sc->num_lights);
    {  // the lit list in row order for the first multi-row area / circle light (FRT_SHADE_SORT=0: never)
        const char* e = std::getenv("FRT_SHADE_SORT");
        h->sort_light = -1;
        for (int l = 0; l < sc->num_lights && h->sort_light < 0 && !(e && std::atoi(e) == 0); ++l)
            if (sc->lights[l].rows > 1 && sc->lights[l].num_samples > 0) h->sort_light = l;
        // the row-ordered shading (FRT_SHADE_STAGE): 2 (default) the node records read in row order, the triples
        // written in row order (spos); 1 also the records staged in list order first (k_lit_stage); 0 both by node, as
        // round 5 did. Shipped frame: shade 14.2 / 13.1 / 12.9 ms for 0 / 1 / 2 (profiles/r06_ab_shipped_modes.txt)
        const char* se = std::getenv("FRT_SHADE_STAGE");
        h->shade_stage = h->sort_light >= 0 ? (se ? std::atoi(se) : 2) : 0;
        // the secondary levels' queues read in parent order (reflected children, then refracted): appended to
        // segment blockIdx % kQueueSegs, the segments' order put children of pixels 256 apart side by side, and the
        // shadow pass's tiles of consecutive nodes spread over the scene. FRT_QUEUE_SORT: 2 (default) the children
        // at fixed slots (no queue atomics) compacted in order; 1 the segments' entries radix-sorted by parent;
        // 0 the segments' order (A/B runs, profiles/r06_ab_queue_sort.txt)
        const char* qs = std::getenv("FRT_QUEUE_SORT");
        h->queue_sort = qs ? std::atoi(qs) : 2;
        const char* qsh = std::getenv("FRT_QUEUE_SORT_SHIFT");  // (A/B runs: parents' low bits out of the key)
        h->queue_sort_shift = qsh ? std::max(0, std::min(16, std::atoi(qsh))) : 0;
    }
    // path-node keys carry a 12-bit heap code (k_prepare: children 2c, 2c + 1 of code c, root 1) and
    // the per-segment counter lines hold the level queue counts in words 0..15: a path of length L
    // has codes up to 2^(L+1) - 1, so L <= 11. The reference accepts any length; deeper recursion
    // is refused here with the reason rather than rendered with colliding keys.
    if (S.cfg.path_length < 0 || S.cfg.path_length > frt::kMaxPathLength) {
        frt_scene_release(h);
        return fail("frt_scene_upload: path-length " + std::to_string(S.cfg.path_length) +
                    " is not supported (0.." + std::to_string(frt::kMaxPathLength) + ")");
    }
    if (S.cfg.use_gi && (S.cfg.gi_path_length >= 255 || S.cfg.photon_count <= 0)) {
        frt_scene_release(h);
        return fail("frt_scene_upload: global illumination needs photon maps (photon_count > 0) and path_length < 255");
    }

    std::vector<int32_t> jl, jp;
    for (int l = 0; l < sc->num_lights; ++l)
        for (int p = 0; p < sc->lights[l].num_samples; ++p) {
            jl.push_back(l);
            jp.push_back(p);
        }
    h->samples_per_node = (int32_t)jl.size();
    if (!jl.empty()) {
        h->j_light = (int32_t*)upload(h, jl.data(), jl.size(), rc);
        h->j_point = (int32_t*)upload(h, jp.data(), jp.size(), rc);
        if (rc) {
            frt_scene_release(h);
            return -1;
        }
    }
#if defined(FRT_WALK_STATS) || defined(FRT_WALK_PROF)
    if (hipMalloc((void**)&h->S.dbg, frt::kDbgSlots * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(h->S.dbg, 0, frt::kDbgSlots * sizeof(unsigned long long)) != hipSuccess) {
        frt_scene_release(h);
        return fail("frt_scene_upload: debug counters");
    }
#endif
    static const bool wtrace = std::getenv("FRT_WARMUP_TRACE") != nullptr;
    const auto ts0 = std::chrono::steady_clock::now();
    {
        std::lock_guard<std::mutex> lk(g_warm_mu);
        if (device >= 0 && device < 64 && g_warm_stream[device] != nullptr) {
            h->stream = g_warm_stream[device];  // (frt_device_warmup's)
            g_warm_stream[device] = nullptr;
        }
    }
    const bool stream_ok = h->stream != nullptr || hipStreamCreate(&h->stream) == hipSuccess;
    if (wtrace)
        std::fprintf(stderr, "frt upload: hipStreamCreate %.2f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count());
    if (!stream_ok || hipMalloc((void**)&h->counters, frt::kQueueSegs * frt::kCounterLine * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void**)&h->err, sizeof(unsigned)) != hipSuccess || hipEventCreate(&h->ev[0]) != hipSuccess ||
        hipEventCreate(&h->ev[1]) != hipSuccess) {
        frt_scene_release(h);
        return fail("frt_scene_upload: stream / counter allocation failed");
    }
    h->levels.resize((size_t)std::max(1, sc->config.path_length + 2));
    *out = h;
    phase(6);
    t_upload_phases[7] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - up0).count();
    return 0;
}

void frt_scene_release(frt_scene_handle* h) {
    if (!h) return;
    hip_ignore(hipSetDevice(h->device));
    if (h->jit_stats) {
        std::vector<unsigned long long> c(kJitStatWords);
        if (hipMemcpy(c.data(), h->jit_stats, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
            unsigned long long live = 0, amb = 0, pairs = 0, mixed = 0, tpairs = 0, tmixed = 0, spairs = 0, smixed = 0,
                               upairs = 0, umixed = 0;
            for (int j = 0; j < 64; ++j) {
                live += c[32 * j];
                amb += c[32 * j + 1];
                pairs += c[32 * j + 2];
                mixed += c[32 * j + 3];
                tpairs += c[32 * j + 4];
                tmixed += c[32 * j + 5];
                spairs += c[32 * j + 6];
                smixed += c[32 * j + 7];
                upairs += c[32 * j + 8];
                umixed += c[32 * j + 9];
            }
            if (tpairs)
                std::fprintf(stderr, "frt jit stats: tile pair kernel (%d nodes per tile): live tile pairs %llu, mixed %llu (%.2f%%)\n",
                             h->tile, tpairs, tmixed, 100.0 * (double)tmixed / (double)tpairs);
            std::fprintf(stderr, "frt jit stats: pair kernel: live pairs %llu, mixed %llu (%.2f%%)\n", pairs, mixed,
                         pairs ? 100.0 * (double)mixed / (double)pairs : 0.0);
            if (spairs)
                std::fprintf(stderr, "frt jit stats: sub-part pair kernel (%d sub-parts): live sub-pairs %llu, mixed %llu (%.2f%%)\n",
                             h->sub, spairs, smixed, 100.0 * (double)smixed / (double)spairs);
            if (upairs)
                std::fprintf(stderr, "frt jit stats: sub-tile pair kernel (%d nodes per sub-tile): live sub-tile pairs %llu, mixed %llu (%.2f%%)\n",
                             h->subtile, upairs, umixed, 100.0 * (double)umixed / (double)upairs);
            std::fprintf(stderr, "frt jit stats: live shadow lanes %llu, re-walked in binary64 %llu (%.4f%%)\n", live, amb,
                         live ? 100.0 * (double)amb / (double)live : 0.0);
            std::fprintf(stderr, "frt jit stats: (node, light) pairs: all lit %llu, all shadowed %llu, mixed %llu\n",
                         h->uniform_stats[0], h->uniform_stats[1], h->uniform_stats[2]);
            for (int k = 0; k < std::min(h->S.num_nodes, 512); ++k)
                if (c[2048 + 2 * k])
                    std::fprintf(stderr, "frt jit stats: node %d: %llu waves, %llu lanes tested; composites: %llu waves, %llu lanes entered\n",
                                 k, c[2048 + 2 * k], c[2048 + 2 * k + 1], c[3072 + 2 * k], c[3072 + 2 * k + 1]);
            for (int k = std::max(h->S.num_nodes, 100); k < 2048; ++k)  // the pair kernel's decision sites (frt_jit.hip)
                if (c[3072 + 2 * k + 1])
                    std::fprintf(stderr, "frt jit stats: beam site %d: %llu waves, %llu lanes\n", k, c[3072 + 2 * k],
                                 c[3072 + 2 * k + 1]);
            for (int k = 0; k < 2048; ++k)  // the tile kernel's
                if (c[9216 + 2 * k + 1])
                    std::fprintf(stderr, "frt jit stats: tile beam site %d: %llu waves, %llu lanes\n", k, c[9216 + 2 * k],
                                 c[9216 + 2 * k + 1]);
        }
    }
    for (void* p : h->owned) hip_ignore(hipFree(p));
    for (auto& L : h->levels) {
        hip_ignore(hipFree(L.rec.core.w));
        hip_ignore(hipFree(L.head));
        hip_ignore(hipFree(L.q));
        hip_ignore(hipFree(L.surface.w));
        hip_ignore(hipFree(L.child.w));
        hip_ignore(hipFree(L.counts));
        hip_ignore(hipFree(L.spos));
        hip_ignore(hipFree(L.qprefix));
        hip_ignore(hipFree(L.qperm));
    }
    hip_ignore(hipFree(h->hits));
    hip_ignore(hipFree(h->hn12));
    {
        auto& G = h->gi;
        for (int m = 0; m < 2; ++m) {
            hip_ignore(hipFree(G.map_mem[m]));
            hip_ignore(hipFree(G.pq[m]));
            hip_ignore(hipFree(G.ppow[m]));
        }
        hip_ignore(hipFree(G.phits));
        hip_ignore(hipFree(G.pn12));
        hip_ignore(hipFree(G.store));
        hip_ignore(hipFree(G.gq));
        hip_ignore(hipFree(G.ghits));
        hip_ignore(hipFree(G.gcol));
        hip_ignore(hipFree(G.greq));
        hip_ignore(hipFree(G.gwork));
        hip_ignore(hipFree(G.gkeys));
        hip_ignore(hipFree(G.extra));
        hip_ignore(hipFree(G.fgather));
    }
    hip_ignore(hipFree(h->sample_col.w));
    hip_ignore(hipFree(h->out_dev));
    hip_ignore(hipFree(h->counters));
    hip_ignore(hipFree(h->shade_lit));
    hip_ignore(hipFree(h->shade_lcount));
    hip_ignore(hipFree(h->lit_row));
    hip_ignore(hipFree(h->lit_flat));
    hip_ignore(hipFree(h->qsort));
    hip_ignore(hipFree(h->spawn_masks));
    hip_ignore(hipFree(h->spawn_offs));
    hip_ignore(hipFree(h->lit_stage));
    hip_ignore(hipFree(h->scan_tmp));
    hip_ignore(hipFree(h->mixed));
    hip_ignore(hipFree(h->tlist));
    hip_ignore(hipFree(h->slist));
    hip_ignore(hipFree(h->stbox));
    hip_ignore(hipFree(h->s2list));
    hip_ignore(hipFree(h->tredo));
    hip_ignore(hipFree(h->tbox));
    hip_ignore(hipFree(h->err));
    for (hipEvent_t e : h->ev_pool) hip_ignore(hipEventDestroy(e));
    if (h->ev[0]) hip_ignore(hipEventDestroy(h->ev[0]));
    if (h->ev[1]) hip_ignore(hipEventDestroy(h->ev[1]));
    if (h->stream) hip_ignore(hipStreamDestroy(h->stream));
    delete h;
}

static int ensure_level(frt_scene_handle* h, size_t d, int64_t need) {
    auto& L = h->levels[d];
    if (need <= L.cap) return 0;
    int64_t nc = std::max<int64_t>(need, L.cap * 2);
    hip_ignore(hipFree(L.rec.core.w));
    hip_ignore(hipFree(L.head));
    L.head = nullptr;
    hip_ignore(hipFree(L.q));
    hip_ignore(hipFree(L.surface.w));
    hip_ignore(hipFree(L.child.w));
    hip_ignore(hipFree(L.counts));
    hip_ignore(hipFree(L.spos));
    L.spos = nullptr;
    L.rec = {};
    L.q = nullptr;
    L.surface = {};
    L.child = {};
    L.counts = nullptr;
    {
        void* p = nullptr;
        FRT_HIP(hipMalloc(&p, frt::NodeCols::bytes(nc)));
        L.rec.set((uint64_t*)p, nc);
        L.rec.root = d == 0 ? 1 : 0;
        // (FRT_EYE_CAM=0: level 0 stores eyev too, A/B runs)
        static const bool eye_cam_env = !(std::getenv("FRT_EYE_CAM") && std::atoi(std::getenv("FRT_EYE_CAM")) == 0);
        L.rec.eye_cam = d == 0 && !h->S.cfg.use_gi && eye_cam_env ? 1 : 0;
    }
    FRT_HIP(hipMalloc((void**)&L.head, nc * sizeof(frt::ShadowHead)));
    L.rec.head = L.head;
    FRT_HIP(hipMalloc((void**)&L.q, nc * sizeof(frt::QueuedRay)));
    FRT_HIP(hipMalloc((void**)&L.surface.w, frt::Cols<frt::Tri9>::bytes(nc)));
    L.surface.cap = nc;
    FRT_HIP(hipMalloc((void**)&L.child.w, frt::Cols<frt::Tri9>::bytes(2 * nc)));
    L.child.cap = 2 * nc;
    if (!L.qprefix) FRT_HIP(hipMalloc((void**)&L.qprefix, (frt::kQueueSegs + 1) * sizeof(int64_t)));
    FRT_HIP(hipMalloc((void**)&L.counts, nc * std::max(1, h->S.num_lights) * sizeof(int32_t)));
    if (h->shade_stage) FRT_HIP(hipMalloc((void**)&L.spos, nc * sizeof(uint32_t)));
    L.cap = nc;
    return 0;
}

static inline unsigned grid_for(int64_t n, int block = frt::kBlock) { return (unsigned)((n + block - 1) / block); }

// a stream synchronize the level loop counts: the level's queue counters, copied to the host right after k_prepare,
// are complete once any later synchronize returned (the level's own end-of-level synchronize is then skipped)
static hipError_t stream_sync(frt_scene_handle* h) {
    const hipError_t e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) h->sync_epoch++;
    return e;
}

// shading in two kernels (k_shade lists the nodes with light-point work, k_shade_lit shades them);
// FRT_SHADE_SPLIT=0: one kernel for every node (A/B runs)
static bool shade_split() {
    const char* e = std::getenv("FRT_SHADE_SPLIT");
    return !(e && std::strcmp(e, "0") == 0);
}
// the ambient-only nodes' terms computed by k_combine instead of stored by k_shade: with the split and
// without GI (whose kernels add to the stored surface triples); FRT_SHADE_LAZY=0 stores them (A/B runs)
static bool shade_lazy(const frt_scene_handle* h) {
    const char* e = std::getenv("FRT_SHADE_LAZY");
    return shade_split() && !h->S.cfg.use_gi && !(e && std::strcmp(e, "0") == 0);
}

// Kernel timing without host synchronisation: events are recorded around each
// launch on the engine stream and read back once the frame has completed.
struct KTimer {
    frt_scene_handle* h;
    frt_frame_stats* st;
    int slot;
    size_t a = 0;
    static hipEvent_t event(frt_scene_handle* h, size_t i) {
        while (h->ev_pool.size() <= i) {
            hipEvent_t e;
            hip_ignore(hipEventCreate(&e));
            h->ev_pool.push_back(e);
        }
        return h->ev_pool[i];
    }
    KTimer(frt_scene_handle* h_, frt_frame_stats* st_, int slot_) : h(h_), st(st_), slot(slot_) {
        if (st) {
            a = h->ev_used++;
            hip_ignore(hipEventRecord(event(h, a), h->stream));
        }
    }
    ~KTimer() {
        if (st) {
            size_t b = h->ev_used++;
            hip_ignore(hipEventRecord(event(h, b), h->stream));
            h->ev_marks.push_back({slot, a, b});
        }
    }
};

static void collect_timings(frt_scene_handle* h, frt_frame_stats* st) {
    for (const auto& m : h->ev_marks) {
        float ms = 0.f;
        hip_ignore(hipEventElapsedTime(&ms, h->ev_pool[m.a], h->ev_pool[m.b]));
        if (m.slot < 8) {
            st->kernel_ms[m.slot] += ms;
            st->kernel_launches[m.slot] += 1;
        } else if (m.slot < 24) {
            st->sub_ms[m.slot - 8] += ms;
            st->sub_launches[m.slot - 8] += 1;
        }
    }
    h->ev_marks.clear();
    h->ev_used = 0;
}

}  // extern "C"

// scene-specialised traversal kernels: the template instance without CSG
// frames / the quartic keeps register pressure down for scenes that lack them
template <int F>
static void launch_trace_f(frt_scene_handle* h, const frt::Batch& B, const frt::QueuedRay* q, int64_t n,
                           frt::HitRec* hits, int filter_casts, double* hn12) {
    hipLaunchKernelGGL(frt::k_trace<F>, dim3(grid_for(n, frt::kTraceBlock)), dim3(frt::kTraceBlock), h->lds_bytes,
                       h->stream, h->S, B, q, n, hits, hn12, h->err, filter_casts);
}

template <int F>
static void launch_trace_redo_f(frt_scene_handle* h, const frt::Batch& B, const frt::QueuedRay* q, int64_t n,
                                frt::HitRec* hits) {
    const unsigned cap = (unsigned)(h->tredo_cap - 2);  // (the list, then its counter)
    hipLaunchKernelGGL(frt::k_trace_redo<F>, dim3(1024), dim3(frt::kTraceBlock), h->lds_bytes, h->stream, h->S, B, q, n,
                       hits, h->err, h->tredo, (const unsigned*)(h->tredo + cap), cap);
}

// hn12: where the hits' refractive indices go (null: every index is one, or nobody reads them); jit: the
// scene-specialised closest hit where the scene has one (the path's own rays, and since round 6 the final gather's
// hemisphere rays: profiles/r06_ab_gather_jit.txt)
static void launch_trace(frt_scene_handle* h, const frt::Batch& B, const frt::QueuedRay* q, int64_t n,
                         frt::HitRec* hits = nullptr, int filter_casts = 0, double* hn12 = nullptr, bool jit = false) {
    if (hits == nullptr) hits = h->hits;
    // the scene-specialised closest hit (frt_jit_trace), its undecided rays to the generic walk (k_trace_redo)
    static const bool jit_trace_env = !(std::getenv("FRT_JIT_TRACE") && std::atoi(std::getenv("FRT_JIT_TRACE")) == 0);
    if (jit && h->jit_trace && jit_trace_env && !filter_casts && hn12 == nullptr && n > 0 && n < ((int64_t)1 << 31)) {
        if (!grow(&h->tredo, h->tredo_cap, n + 2)) {  // (a list of every ray at worst, then its counter)
            unsigned cap = (unsigned)(h->tredo_cap - 2);
            unsigned* cnt = (unsigned*)(h->tredo + cap);
            hip_ignore(hipMemsetAsync(cnt, 0, sizeof(unsigned), h->stream));
            void* args[] = {&h->S, (void*)&B, (void*)&q, &n, &hits, &h->err, &h->tredo, &cnt, &cap};
            if (hipModuleLaunchKernel((hipFunction_t)h->jit_trace, (unsigned)grid_for(n, frt::kTraceBlock), 1, 1,
                                      frt::kTraceBlock, 1, 1, 0, h->stream, args, nullptr) == hipSuccess) {
                switch (h->S.features & 3) {
                case 0: launch_trace_redo_f<0>(h, B, q, n, hits); break;
                case 1: launch_trace_redo_f<1>(h, B, q, n, hits); break;
                case 2: launch_trace_redo_f<2>(h, B, q, n, hits); break;
                default: launch_trace_redo_f<3>(h, B, q, n, hits); break;
                }
                static const bool trace_stats = std::getenv("FRT_JIT_TRACE_STATS") != nullptr;
                if (trace_stats) {  // (debug: the undecided share per launch; synchronises)
                    unsigned c = 0;
                    hip_ignore(hipMemcpyAsync(&c, cnt, sizeof(c), hipMemcpyDeviceToHost, h->stream));
                    hip_ignore(hipStreamSynchronize(h->stream));
                    std::fprintf(stderr, "frt: frt_jit_trace level %d: %lld rays, %u to the generic walk\n", B.level,
                                 (long long)n, c);
                    // (FRT_JIT_TRACE_DUMP=<path>: the level-0 list of undecided rays, int32 ray indices, for analysis)
                    const char* dump = std::getenv("FRT_JIT_TRACE_DUMP");
                    if (dump && B.level == 0 && c > 0) {
                        std::vector<int32_t> v(std::min<size_t>(c, cap));
                        hip_ignore(hipMemcpy(v.data(), h->tredo, v.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
                        if (FILE* f = std::fopen(dump, "wb")) {
                            std::fwrite(v.data(), sizeof(int32_t), v.size(), f);
                            std::fclose(f);
                        }
                    }
                }
                return;
            }
            std::fprintf(stderr, "frt: scene-specialised closest-hit kernel launch failed; k_trace\n");
            (void)hipGetLastError();
            h->jit_trace = nullptr;
        } else {
            (void)hipGetLastError();
        }
    }
    switch (h->S.features & 3) {
    case 0: launch_trace_f<0>(h, B, q, n, hits, filter_casts, hn12); break;
    case 1: launch_trace_f<1>(h, B, q, n, hits, filter_casts, hn12); break;
    case 2: launch_trace_f<2>(h, B, q, n, hits, filter_casts, hn12); break;
    default: launch_trace_f<3>(h, B, q, n, hits, filter_casts, hn12); break;
    }
}

template <int F>
static void launch_shadow_f(frt_scene_handle* h, const frt::Batch& B, const frt::ShadowHead* rec, int64_t n, int32_t* counts) {
    const int64_t work = n * h->samples_per_node;
    hipLaunchKernelGGL(frt::k_shadow<F>, dim3(grid_for(work, frt::kTraceBlock)), dim3(frt::kTraceBlock), h->lds_bytes,
                       h->stream, h->S, B, rec, n, h->j_light, h->j_point, h->samples_per_node, counts, h->err);
}

template <int F>
static void launch_shadow_redo_f(frt_scene_handle* h, const frt::Batch& B, const frt::ShadowHead* rec, int64_t n,
                                 int32_t* counts) {
    hipLaunchKernelGGL(frt::k_shadow_redo<F>, dim3(64), dim3(frt::kTraceBlock), h->lds_bytes, h->stream, h->S, B, rec, n,
                       h->j_light, h->j_point, h->samples_per_node, counts, h->err, h->redo, h->redo_count, h->redo_cap);
}

// the block table of a segmented list (jit::SegTable) whose entries take lpe lanes each: returns the blocks,
// `total` the entries (a segment past its capacity keeps its capacity: the error flag is set)
static uint64_t seg_table(const PinnedBuf<unsigned>& host_mcount, uint32_t segcap, uint64_t lpe,
                          frt::jit::SegTable& seg, uint64_t& total) {
    uint64_t nblk = 0;
    total = 0;
    for (int j = 0; j < frt::jit::kMixSegs; ++j) {
        const uint64_t c = std::min<uint64_t>(host_mcount[(size_t)j * frt::jit::kMixLine], segcap);
        seg.bstart[j] = (uint32_t)nblk;
        seg.count[j] = (uint32_t)c;
        total += c;
        nblk += (c * lpe + frt::kTraceBlock - 1) / frt::kTraceBlock;
    }
    seg.bstart[frt::jit::kMixSegs] = (uint32_t)nblk;
    return nblk;
}

// (node0: the first node's index in the level, for its tile box)
static void launch_shadow(frt_scene_handle* h, const frt::Batch& B, const frt::ShadowHead* rec, int64_t n, int32_t* counts,
                          int64_t node0 = 0) {
    if (h->jit_shadow) {
        // scene-specialised kernels: the pair kernels decide whole (node, light part) pairs — frt_jit_tile
        // first for runs of tile consecutive nodes at once, frt_jit_beam_list for the nodes of the tile pairs
        // it cannot decide (or frt_jit_beam for every pair) — and frt_jit_shadow walks the rays of the pairs
        // left (32-bit lane index: at most 2^31 lanes per launch), then the generic walk takes the lanes
        // handed back (non-finite rays, usually none)
        using frt::jit::kMixLine;
        using frt::jit::kMixSegs;
        int64_t NP = 0;  // parts of frt_jit_part_size() samples per path node (frt_jit_beam)
        for (const auto& L : h->host_lights) NP += std::max(1, (L.num_samples + frt_jit_part_size() - 1) / frt_jit_part_size());
        // the pair kernel's lane index is 32-bit: batches of more than 2^31 - 1 (node, part) pairs run
        // as node ranges (the shadow kernels read a node's ShadowHead and write its counts only, so a
        // range is the same pass over rec + off and counts + off * lights; ranges start at tile boundaries)
        // (FRT_JIT_MAX_PAIRS lowers the limit: the tests split small batches this way)
        const char* mp_env = std::getenv("FRT_JIT_MAX_PAIRS");
        const long long mp = mp_env ? std::atoll(mp_env) : 0;
        int64_t kMaxPairs = mp >= 1 && mp < (1ll << 31) ? (int64_t)mp : (int64_t)((1ll << 31) - 1);
        // (the sub-part pass after the tile kernel: the per-ray kernel's list holds (node pair) * sub + q in 32 bits)
        // Small levels (the deep bounces: a few thousand nodes) skip the beam stages: each stage's launch is sized
        // on the host from the previous one's counts, a round trip (~15 us plus the idle GPU) that costs more than
        // walking their rays one by one; the per-ray walk of every pair gives the same counts (FRT_JIT_MIN_PAIRS,
        // default 2^18 (node, part) pairs)
        static const int64_t min_pairs = [] {
            const char* e = std::getenv("FRT_JIT_MIN_PAIRS");
            return e ? (int64_t)std::atoll(e) : (int64_t)1 << 18;
        }();
        const bool beam_on = h->jit_beam_on && n * NP >= min_pairs;
        const bool tiled = beam_on && h->tile > 0 && h->jit_tile && h->jit_list && h->tbox;
        const bool subbed = tiled && h->jit_sub && h->sub > 0 && h->light_psamp2 && h->light_sbox;
        if (subbed && h->node_beam) {
            kMaxPairs = std::min<int64_t>(kMaxPairs, (int64_t)(0xFFFFFFFFull / (uint64_t)h->sub));
        } else if (subbed) {
            // (the stages' lists hold tile-level entries, ((tile * NP + part) * sub + q) << log2(tile / subtile) +
            // sub-tile, and node pairs node * NP + part where a level's list goes to the node pair kernel: a level
            // runs in one range while both fit 32 bits — the headline's level 0, 132.7 M nodes, in one range instead
            // of four, a quarter of the stage launches and host round trips)
            int stl = 0;
            while (h->subtile > 0 && (1 << stl) < h->tile / h->subtile) ++stl;
            const uint64_t per_tile = ((uint64_t)NP * (uint64_t)h->sub) << stl;
            const int64_t tiled_max = (int64_t)(0xFFFFFFFFull / per_tile) * h->tile * NP;
            kMaxPairs = std::min<int64_t>(std::min<int64_t>(tiled_max, (int64_t)0xFFFFFFFFll),
                                          mp >= 1 && mp < (1ll << 31) ? (int64_t)mp : INT64_MAX);
        }
        if (n * NP > kMaxPairs) {
            int64_t per = std::max<int64_t>(1, kMaxPairs / NP);
            if (h->tile > 0) per = std::max<int64_t>(h->tile, per / h->tile * h->tile);
            for (int64_t off = 0; off < n; off += per)
                launch_shadow(h, B, rec + off, std::min(per, n - off), counts + off * h->S.num_lights, node0 + off);
            return;
        }
        const int64_t npairs = n * NP;
        uint32_t nn = (uint32_t)n;
        uint32_t segcap = 0;
        // the stages' list counters, one region each, zeroed by one memset for the pass
        unsigned* mc_tile = h->mcount;
        unsigned* mc_sub = h->mcount + kMixSegs * kMixLine;
        unsigned* mc_subtile = h->mcount + 2 * kMixSegs * kMixLine;
        unsigned* mc_node = h->mcount + 3 * kMixSegs * kMixLine;
        if (beam_on) hip_ignore(hipMemsetAsync(h->mcount, 0, 4 * kMixSegs * kMixLine * sizeof(unsigned), h->stream));
        uint64_t total_mixed = 0;
        const uint32_t* direct_in = nullptr;  // (the sub / sub-tile list walked by the per-ray kernel directly)
        uint32_t direct_subq = 0, direct_nodes = 0;
        if (beam_on) {
            frt::jit::SegTable tseg{};
            uint32_t tsegcap = 0;
            uint64_t list_blocks = 0, listed = 0;
            // the node pair kernel's input (tiled): the tile pairs left mixed, or the tile sub-pairs left mixed
            const uint32_t* list_in = h->tlist;
            uint32_t list_segcap = 0;
            const float* list_boxes = h->light_aabb;
            int tl = 0;
            while ((1 << tl) < h->tile) ++tl;
            if (tiled) {
                const int64_t ntiles = (n + h->tile - 1) >> tl;
                uint32_t ntp = (uint32_t)(ntiles * NP);
                const int64_t tblocks = (ntiles * NP + frt::kTraceBlock - 1) / frt::kTraceBlock;
                tsegcap = (uint32_t)std::max<int64_t>(frt::kTraceBlock, ((tblocks + kMixSegs - 1) / kMixSegs) * frt::kTraceBlock);
                if (grow(&h->tlist, h->tlist_cap, 2 * (int64_t)tsegcap * kMixSegs)) {  // (out of memory): the generic walk
                    (void)hipGetLastError();
                    h->jit_shadow = nullptr;
                    launch_shadow(h, B, rec, n, counts, node0);
                    return;
                }
                const float* tb = h->tbox + 6 * (node0 >> tl);
                const uint32_t* no_list = nullptr;
                uint32_t zero = 0;
                void* targs[] = {&h->S, (void*)&B, (void*)&rec, &ntp, &nn, (void*)&tb, (void*)&no_list, &tseg, &zero, &zero,
                                 &h->light_aabb, &counts, &h->tlist, &mc_tile, &tsegcap, &h->err, &h->jit_stats,
                                 &h->light_psamp2};
                hipError_t le;
                {
                    KTimer tt(h, h->cur_st, 12);
                    le = hipModuleLaunchKernel((hipFunction_t)h->jit_tile, grid_for(ntiles * NP, frt::kTraceBlock), 1, 1,
                                               frt::kTraceBlock, 1, 1, 0, h->stream, targs, nullptr);
                }
                if (le != hipSuccess) {
                    std::fprintf(stderr, "frt: scene-specialised tile kernel launch failed (%s); pairs per node\n",
                                 hipGetErrorString(le));
                    (void)hipGetLastError();
                    h->tile = 0;
                    launch_shadow(h, B, rec, n, counts, node0);
                    return;
                }
                if (hipMemcpyAsync(h->host_mcount.data(), mc_tile, h->host_mcount.size() * sizeof(unsigned),
                                   hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                    stream_sync(h) != hipSuccess)
                    return;
                list_blocks = seg_table(h->host_mcount, tsegcap, subbed ? (uint64_t)h->sub : (uint64_t)h->tile, tseg, listed);
                h->tile_pairs += ntp;
                h->tile_mixed += listed;
                list_in = h->tlist;
                list_segcap = tsegcap;
                if (subbed && listed > 0) {
                    // the sub-part pass: sub lanes per tile pair left mixed, the tile's beam to each sub-part's box
                    // resumed from the tile pair's point; the sub-pairs it leaves go to the node pair kernel
                    const uint64_t sblocks = list_blocks;
                    const frt::jit::SegTable sseg = tseg;
                    const uint32_t ssegcap = (uint32_t)std::max<uint64_t>(frt::kTraceBlock,
                                                                          ((sblocks + kMixSegs - 1) / kMixSegs) * frt::kTraceBlock);
                    if (grow(&h->slist, h->slist_cap, 2 * (int64_t)ssegcap * kMixSegs)) {  // (out of memory): the generic walk
                        (void)hipGetLastError();
                        h->jit_shadow = nullptr;
                        hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                        launch_shadow(h, B, rec, n, counts, node0);
                        return;
                    }
                    hipError_t se = hipSuccess;
                    {
                        KTimer ts(h, h->cur_st, 13);
                        const uint64_t max_blocks = ((1ull << 31) - 1) / frt::kTraceBlock;
                        uint32_t zero = 0;
                        for (uint64_t b0 = 0; b0 < sblocks && se == hipSuccess; b0 += max_blocks) {
                            uint32_t b0u = (uint32_t)b0;
                            void* sargs[] = {&h->S, (void*)&B, (void*)&rec, &zero, &nn, (void*)&tb, &h->tlist, (void*)&sseg, &b0u,
                                             &tsegcap, &h->light_sbox, &counts, &h->slist, &mc_sub, (void*)&ssegcap, &h->err,
                                             &h->jit_stats, &h->light_psamp2};
                            se = hipModuleLaunchKernel((hipFunction_t)h->jit_sub, (unsigned)std::min(max_blocks, sblocks - b0), 1, 1,
                                                       frt::kTraceBlock, 1, 1, 0, h->stream, sargs, nullptr);
                        }
                    }
                    if (se != hipSuccess) {
                        std::fprintf(stderr, "frt: scene-specialised sub-part kernel launch failed (%s); no sub-parts\n",
                                     hipGetErrorString(se));
                        (void)hipGetLastError();
                        h->jit_sub = nullptr;
                        h->sub = 0;
                        hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                        launch_shadow(h, B, rec, n, counts, node0);
                        return;
                    }
                    if (hipMemcpyAsync(h->host_mcount.data(), mc_sub, h->host_mcount.size() * sizeof(unsigned),
                                       hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                        stream_sync(h) != hipSuccess)
                        return;
                    uint64_t listed_s = 0;
                    // (FRT_JIT_SUBTILE_DEEP=0: levels past the camera's walk the sub-part list ray by ray, A/B runs)
                    static const bool subtile_deep =
                        !(std::getenv("FRT_JIT_SUBTILE_DEEP") && std::atoi(std::getenv("FRT_JIT_SUBTILE_DEEP")) == 0);
                    const bool subtiled = h->jit_subtile && h->subtile > 0 && h->subtile < h->tile && h->stbox &&
                                          (B.level == 0 || subtile_deep);
                    const uint64_t nst = subtiled ? (uint64_t)(h->tile / h->subtile) : 0;
                    list_blocks = seg_table(h->host_mcount, ssegcap, subtiled ? nst : (uint64_t)h->tile, tseg, listed_s);
                    h->sub_pairs += listed * (uint64_t)h->sub;
                    h->sub_mixed += listed_s;
                    listed = listed_s;
                    list_in = h->slist;
                    list_segcap = ssegcap;
                    list_boxes = h->light_sbox;
                    if (subtiled && listed_s > 0) {
                        // the sub-tile pass: the tile sub-pairs left, per sub-tile of the tile, from its own origin box
                        const uint64_t tblocks = list_blocks;
                        const frt::jit::SegTable s1seg = tseg;
                        const uint32_t s2segcap = (uint32_t)std::max<uint64_t>(
                            frt::kTraceBlock, ((tblocks + kMixSegs - 1) / kMixSegs) * frt::kTraceBlock);
                        if (grow(&h->s2list, h->s2list_cap, 2 * (int64_t)s2segcap * kMixSegs)) {  // (out of memory)
                            (void)hipGetLastError();
                            h->jit_shadow = nullptr;
                            hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                            launch_shadow(h, B, rec, n, counts, node0);
                            return;
                        }
                        int stl = 0;
                        while ((1 << stl) < h->subtile) ++stl;
                        const float* stb = h->stbox + 6 * (node0 >> stl);
                        hipError_t ue = hipSuccess;
                        {
                            KTimer tu(h, h->cur_st, 14);
                            const uint64_t max_blocks = ((1ull << 31) - 1) / frt::kTraceBlock;
                            uint32_t zero = 0;
                            for (uint64_t b0 = 0; b0 < tblocks && ue == hipSuccess; b0 += max_blocks) {
                                uint32_t b0u = (uint32_t)b0;
                                void* uargs[] = {&h->S, (void*)&B, (void*)&rec, &zero, &nn, (void*)&stb, &h->slist, (void*)&s1seg,
                                                 &b0u, (void*)&ssegcap, &h->light_sbox, &counts, &h->s2list, &mc_subtile,
                                                 (void*)&s2segcap, &h->err, &h->jit_stats, &h->light_psamp2};
                                ue = hipModuleLaunchKernel((hipFunction_t)h->jit_subtile, (unsigned)std::min(max_blocks, tblocks - b0),
                                                           1, 1, frt::kTraceBlock, 1, 1, 0, h->stream, uargs, nullptr);
                            }
                        }
                        if (ue != hipSuccess) {
                            std::fprintf(stderr, "frt: scene-specialised sub-tile kernel launch failed (%s); no sub-tiles\n",
                                         hipGetErrorString(ue));
                            (void)hipGetLastError();
                            h->jit_subtile = nullptr;
                            h->subtile = 0;
                            hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                            launch_shadow(h, B, rec, n, counts, node0);
                            return;
                        }
                        if (hipMemcpyAsync(h->host_mcount.data(), mc_subtile, h->host_mcount.size() * sizeof(unsigned),
                                           hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                            stream_sync(h) != hipSuccess)
                            return;
                        uint64_t listed_u = 0;
                        list_blocks = seg_table(h->host_mcount, s2segcap, (uint64_t)h->subtile, tseg, listed_u);
                        h->subtile_pairs += listed_s * nst;
                        h->subtile_mixed += listed_u;
                        listed = listed_u;
                        list_in = h->s2list;
                        list_segcap = s2segcap;
                    } else if (subtiled) {
                        list_blocks = 0;
                        listed = 0;
                    }
                } else if (subbed) {
                    list_blocks = 0;  // (no tile pair left)
                    listed = 0;
                }
            }
            if (subbed && !h->node_beam && list_in != h->tlist) {
                // the sub-part (sub-tile) stage's list goes to the per-ray kernel as it is (host_mcount holds its
                // counts): each entry's nodes times its sub-part's samples, one lane per (node, sample)
                direct_in = list_in;
                direct_subq = list_in == h->s2list ? 3u : 2u;
                direct_nodes = (uint32_t)(list_in == h->s2list ? h->subtile : h->tile);
                segcap = list_segcap;
                for (int j = 0; j < kMixSegs; ++j) total_mixed += std::min<uint64_t>(h->host_mcount[(size_t)j * kMixLine], segcap);
                h->node_pairs += total_mixed * direct_nodes;
                h->node_mixed += total_mixed * direct_nodes;
            } else {
            // the mixed list of the node pairs (the per-ray kernel's): per segment, every lane of the blocks that
            // append to it
            const int64_t pblocks = tiled ? (int64_t)list_blocks : (npairs + frt::kTraceBlock - 1) / frt::kTraceBlock;
            segcap = (uint32_t)std::max<int64_t>(frt::kTraceBlock, ((pblocks + kMixSegs - 1) / kMixSegs) * frt::kTraceBlock);
            uint32_t** nout = &h->mixed;
            int64_t& nout_cap = h->mixed_cap;
            // pairs, then their resume values (frt_jit_rt.hpp mix_append)
            if (grow(nout, nout_cap, 2 * (int64_t)segcap * kMixSegs)) {  // (out of memory): the generic walk
                (void)hipGetLastError();
                h->jit_shadow = nullptr;
                hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                launch_shadow(h, B, rec, n, counts, node0);
                return;
            }
            hipError_t le = hipSuccess;
            {
                KTimer tb(h, h->cur_st, 8);
                if (tiled) {
                    const uint64_t max_blocks = ((1ull << 31) - 1) / frt::kTraceBlock;
                    const float* no_box = nullptr;
                    uint32_t zero = 0;
                    for (uint64_t b0 = 0; b0 < list_blocks && le == hipSuccess; b0 += max_blocks) {
                        uint32_t b0u = (uint32_t)b0;
                        void* largs[] = {&h->S, (void*)&B, (void*)&rec, &zero, &nn, (void*)&no_box, (void*)&list_in, &tseg, &b0u,
                                         &list_segcap, (void*)&list_boxes, &counts, nout, &mc_node, &segcap, &h->err,
                                         &h->jit_stats, &h->light_psamp2};
                        le = hipModuleLaunchKernel((hipFunction_t)h->jit_list, (unsigned)std::min(max_blocks, list_blocks - b0), 1, 1,
                                                   frt::kTraceBlock, 1, 1, 0, h->stream, largs, nullptr);
                    }
                    h->node_pairs += listed * (uint64_t)(list_in == h->s2list ? h->subtile : h->tile);
                } else {
                    uint32_t np = (uint32_t)npairs;
                    const float* no_box = nullptr;
                    const uint32_t* no_list = nullptr;
                    frt::jit::SegTable no_seg{};
                    uint32_t zero = 0;
                    void* bargs[] = {&h->S, (void*)&B, (void*)&rec, &np, &nn, (void*)&no_box, (void*)&no_list, &no_seg, &zero, &zero,
                                     &h->light_aabb, &counts, nout, &mc_node, &segcap, &h->err, &h->jit_stats,
                                     &h->light_psamp2};
                    le = hipModuleLaunchKernel((hipFunction_t)h->jit_beam, grid_for(npairs, frt::kTraceBlock), 1, 1,
                                               frt::kTraceBlock, 1, 1, 0, h->stream, bargs, nullptr);
                    h->node_pairs += (uint64_t)npairs;
                }
            }
            if (le != hipSuccess) {
                std::fprintf(stderr, "frt: scene-specialised pair kernel launch failed (%s); every pair per ray\n",
                             hipGetErrorString(le));
                (void)hipGetLastError();
                h->jit_beam_on = false;
                hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                launch_shadow(h, B, rec, n, counts, node0);
                return;
            }
            if (hipMemcpyAsync(h->host_mcount.data(), mc_node, h->host_mcount.size() * sizeof(unsigned),
                               hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                stream_sync(h) != hipSuccess)
                return;
            for (int j = 0; j < kMixSegs; ++j) total_mixed += std::min<uint64_t>(h->host_mcount[(size_t)j * kMixLine], segcap);
            h->node_mixed += total_mixed;
            }
        } else {
            segcap = (uint32_t)std::max<int64_t>(1, npairs);
            if (grow(&h->mixed, h->mixed_cap, 2 * (int64_t)segcap * kMixSegs)) {  // (out of memory): the generic walk
                (void)hipGetLastError();
                h->jit_shadow = nullptr;
                launch_shadow(h, B, rec, n, counts, node0);
                return;
            }
            total_mixed = (uint64_t)npairs;  // every pair, in order (frt_jit_shadow's all_pairs)
        }
        uint32_t all_pairs = beam_on ? 0u : 1u;
        // lanes per pair (a part of frt_jit_part_size() samples, or a sub-part's slot after frt_jit_sub);
        // tid / lpp by multiply-shift
        uint32_t subq = direct_in ? direct_subq : subbed ? 1u : 0u;
        uint32_t lpp = direct_in ? direct_nodes * (uint32_t)h->sub_ps : subbed ? (uint32_t)h->sub_ps : (uint32_t)frt_jit_part_size();
        const uint32_t* mixed_in = direct_in ? direct_in : h->mixed;
        uint32_t shift = 32;
        while ((1u << (shift - 32)) < lpp) ++shift;  // 32 + ceil(log2 lpp)
        const uint64_t magic = (uint64_t)((((unsigned __int128)1 << shift) + lpp - 1) / lpp);
        uint32_t spn = (uint32_t)h->samples_per_node;
        const uint64_t max_pairs = std::max<uint64_t>(1, ((1ull << 31) - 1) / lpp);
        hip_ignore(hipMemsetAsync(h->redo_count, 0, sizeof(unsigned), h->stream));
        h->rays_walked += total_mixed * lpp;  // (parts of fewer samples count their padding lanes too)
        h->pairs_walked += total_mixed;
        // (ShadowHeads read: a node per lane group, each of the level's n nodes at most once per launch — the entries of
        // one tile re-read its nodes' records from L2)
        h->heads_walked += std::min<uint64_t>(direct_in ? total_mixed * direct_nodes : total_mixed, (uint64_t)n);
        KTimer tr(h, h->cur_st, 9);
        // the mixed pairs' blocks by segment (jit::SegTable); every pair in order without the pair kernel
        frt::jit::SegTable seg{};
        uint64_t nblk = 0;
        for (int j = 0; j < kMixSegs; ++j) {
            const uint64_t c = all_pairs ? 0 : std::min<uint64_t>(h->host_mcount[(size_t)j * kMixLine], segcap);
            seg.bstart[j] = (uint32_t)nblk;
            seg.count[j] = (uint32_t)c;
            nblk += (c * lpp + frt::kTraceBlock - 1) / frt::kTraceBlock;
        }
        seg.bstart[kMixSegs] = (uint32_t)nblk;
        const uint64_t max_blocks = ((1ull << 31) - 1) / frt::kTraceBlock;
        const uint64_t launches = all_pairs ? (total_mixed + max_pairs - 1) / max_pairs : (nblk + max_blocks - 1) / max_blocks;
        for (uint64_t li = 0; li < launches; ++li) {
            uint32_t total = 0, m0 = 0, b0 = 0;
            uint64_t grid = 0;
            if (all_pairs) {
                const uint64_t p0 = li * max_pairs, pc = std::min<uint64_t>(max_pairs, total_mixed - p0);
                total = (uint32_t)(pc * lpp);
                m0 = (uint32_t)p0;
                grid = (total + frt::kTraceBlock - 1) / frt::kTraceBlock;
            } else {
                b0 = (uint32_t)(li * max_blocks);
                grid = std::min<uint64_t>(max_blocks, nblk - b0);
            }
            void* args[] = {&h->S, (void*)&B, (void*)&rec, &total, &m0, (void*)&mixed_in, &seg, &b0, &segcap, &all_pairs,
                            &h->light_psamp, &subq, &h->light_psamp2, &lpp, (void*)&magic,
                            &shift, &spn, &counts, &h->redo, &h->redo_count, &h->redo_cap, &h->err, &h->jit_stats, &nn};
            const hipError_t le = hipModuleLaunchKernel((hipFunction_t)h->jit_shadow, (unsigned)grid,
                                                        1, 1, frt::kTraceBlock, 1, 1, 0, h->stream, args, nullptr);
            if (le != hipSuccess) {
                // the pair kernel may have written counts already: clear them and take the generic walk for
                // this launch and the rest of the handle's life instead of rendering everything shadowed
                std::fprintf(stderr, "frt: scene-specialised shadow kernel launch failed (%s); generic walk\n",
                             hipGetErrorString(le));
                (void)hipGetLastError();
                hip_ignore(hipMemsetAsync(counts, 0, (size_t)n * h->S.num_lights * sizeof(int32_t), h->stream));
                h->jit_shadow = nullptr;
                launch_shadow(h, B, rec, n, counts);
                return;
            }
        }
        switch (h->S.features & 3) {
        case 0: launch_shadow_redo_f<0>(h, B, rec, n, counts); break;
        case 1: launch_shadow_redo_f<1>(h, B, rec, n, counts); break;
        case 2: launch_shadow_redo_f<2>(h, B, rec, n, counts); break;
        default: launch_shadow_redo_f<3>(h, B, rec, n, counts); break;
        }
        return;
    }
    switch (h->S.features & 3) {
    case 0: launch_shadow_f<0>(h, B, rec, n, counts); break;
    case 1: launch_shadow_f<1>(h, B, rec, n, counts); break;
    case 2: launch_shadow_f<2>(h, B, rec, n, counts); break;
    default: launch_shadow_f<3>(h, B, rec, n, counts); break;
    }
}


// ---------------------------------------------------------------------
// photon maps (reference photon_tracer.c:203-257, pm.c)
// ---------------------------------------------------------------------

static uint64_t host_mix64(uint64_t x) {  // frt::mix64 on the host
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

// Photons of one light into one map, in the reference's storage order: emission
// by emission (each emission's stores in bounce order) until the stored count
// reaches the light's share, the last emission kept whole (trace_photons'
// "j += hit" loop). Emissions run in batches on the device; the batch size
// follows the measured store rate. The reference loops forever when a light
// can store nothing (no diffuse surface reachable); here the emission count is
// bounded and the map keeps what was found.
// the order of the stored photons by key (emission index << 8 | bounce, unique): LSD radix sort
// over 16-bit digits of (key, index) pairs, instead of sorting the 80-byte records
static std::vector<uint32_t> key_order(const std::vector<frt::StoredPhoton>& a) {
    const size_t n = a.size();
    std::vector<uint64_t> k(n), k2(n);
    std::vector<uint32_t> idx(n), idx2(n), cnt((size_t)65536 + 1);
    uint64_t mx = 0;
    for (size_t i = 0; i < n; ++i) {
        k[i] = a[i].key;
        idx[i] = (uint32_t)i;
        mx = std::max(mx, k[i]);
    }
    for (int shift = 0; shift < 64 && (mx >> shift) != 0; shift += 16) {
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (size_t i = 0; i < n; ++i) cnt[((k[i] >> shift) & 0xffff) + 1]++;
        for (size_t d = 0; d < 65536; ++d) cnt[d + 1] += cnt[d];
        for (size_t i = 0; i < n; ++i) {
            const uint32_t at = cnt[(k[i] >> shift) & 0xffff]++;
            k2[at] = k[i];
            idx2[at] = idx[i];
        }
        k.swap(k2);
        idx.swap(idx2);
    }
    return idx;
}

static int trace_light_photons(frt_scene_handle* h, int map, int light, uint64_t seed,
                               std::vector<frt::StoredPhoton>& out) {
    using namespace frt;
    auto& G = h->gi;
    const int64_t want = h->host_lights[(size_t)light].num_photons;
    const int path = h->S.cfg.gi_path_length;
    if (want <= 0 || path <= 0) return 0;
    const int64_t kMaxBatch = (int64_t)1 << 22;
    const uint64_t emit_limit = (uint64_t)want * 4096ull + ((uint64_t)1 << 26);
    const uint64_t lseed = host_mix64(seed ^ host_mix64(0x70686f746f6e0000ULL + (uint64_t)(map * 4096 + light)));
    std::vector<StoredPhoton> acc;
    uint64_t e0 = 0;
    int64_t batch = std::min<int64_t>(std::max<int64_t>(want, 4096), kMaxBatch);
    Batch B{};
    B.seed = seed;
    for (;;) {
        const int64_t store_cap = batch * (int64_t)std::min(path, 16);
        if (grow(&G.pq[0], G.pq_cap[0], batch) || grow(&G.pq[1], G.pq_cap[1], batch) ||
            grow(&G.ppow[0], G.ppow_cap[0], 3 * batch) || grow(&G.ppow[1], G.ppow_cap[1], 3 * batch) ||
            grow(&G.phits, G.phits_cap, batch) || grow(&G.store, G.store_cap, store_cap) ||
            (!h->S.cfg.all_ni_one && grow(&G.pn12, G.pn12_cap, 2 * batch)))
            return -1;
        double* pn12 = h->S.cfg.all_ni_one ? nullptr : G.pn12;
        unsigned long long* store_count = h->counters + 24;
        unsigned long long* next_count = h->counters + 25;
        FRT_HIP(hipMemsetAsync(h->counters + 24, 0, 2 * sizeof(unsigned long long), h->stream));
        hipLaunchKernelGGL(k_photon_emit, dim3(grid_for(batch)), dim3(kBlock), 0, h->stream, h->S, lseed, light, e0,
                           batch, G.pq[0], G.ppow[0]);
        FRT_HIP(hipGetLastError());
        int64_t n = batch;
        int cur = 0;
        for (int depth = 0; depth < path && n > 0; ++depth) {
            FRT_HIP(hipMemsetAsync(next_count, 0, sizeof(unsigned long long), h->stream));
            launch_trace(h, B, G.pq[cur], n, G.phits, 1, pn12);
            FRT_HIP(hipGetLastError());
            hipLaunchKernelGGL(h->S.num_patterns > 0 ? k_photon_hit<true> : k_photon_hit<false>, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, lseed, map, depth,
                               G.pq[cur], G.ppow[cur], n, G.phits, pn12, G.pq[cur ^ 1], G.ppow[cur ^ 1], next_count,
                               batch, G.store, store_count, store_cap, h->err);
            FRT_HIP(hipGetLastError());
            unsigned long long nn = 0;
            FRT_HIP(hipMemcpyAsync(&nn, next_count, sizeof(nn), hipMemcpyDeviceToHost, h->stream));
            FRT_HIP(hipStreamSynchronize(h->stream));
            n = (int64_t)std::min<unsigned long long>(nn, (unsigned long long)batch);
            cur ^= 1;
        }
        unsigned long long ns = 0;
        FRT_HIP(hipMemcpyAsync(&ns, store_count, sizeof(ns), hipMemcpyDeviceToHost, h->stream));
        FRT_HIP(hipStreamSynchronize(h->stream));
        ns = std::min<unsigned long long>(ns, (unsigned long long)store_cap);
        const size_t base = acc.size();
        acc.resize(base + (size_t)ns);
        if (ns) FRT_HIP(hipMemcpy(acc.data() + base, G.store, (size_t)ns * sizeof(StoredPhoton), hipMemcpyDeviceToHost));
        e0 += (uint64_t)batch;
        if ((int64_t)acc.size() >= want || e0 >= emit_limit) break;
        const double rate = (double)acc.size() / (double)e0;
        const double need = (double)(want - (int64_t)acc.size());
        batch = rate > 0 ? (int64_t)std::min<double>((double)kMaxBatch, need / rate * 1.25 + 1024.0)
                         : std::min<int64_t>(batch * 4, kMaxBatch);
    }
    // the reference's storage order: by emission, then bounce
    const std::vector<uint32_t> ord = key_order(acc);
    // keep the emissions up to the first one at which the count reaches `want`
    size_t keep = acc.size();
    if ((int64_t)acc.size() >= want) {
        const uint64_t last = acc[ord[(size_t)want - 1]].key >> 8;
        keep = (size_t)want;
        while (keep < acc.size() && (acc[ord[keep]].key >> 8) == last) ++keep;
    }
    out.reserve(out.size() + keep);
    for (size_t i = 0; i < keep; ++i) out.push_back(acc[ord[i]]);
    return 0;
}

// pm_store's direction bytes (pm.c:288-300): theta, phi of a unit direction
static void dir_bytes(const double* d, uint8_t* tp) {
    double at = std::acos(d[2]) * (256.0 / M_PI);
    int theta = std::isfinite(at) ? (int)at : 0;
    theta = theta > 255 ? 255 : theta;
    double ap = std::atan2(d[1], d[0]) * (256.0 / (2.0 * M_PI));
    int phi = std::isfinite(ap) ? (int)ap : 0;
    phi = phi > 255 ? 255 : (phi < 0 ? phi + 256 : phi);
    tp[0] = (uint8_t)(theta & 255);
    tp[1] = (uint8_t)(phi & 255);
}

// pm_photon_dir's tables (pm.c:60-66), the same expressions per byte value: {sin theta, cos theta} and
// {cos 2 phi, sin 2 phi} per byte
static const std::vector<double>& dir_tables() {
    static const std::vector<double> t = [] {
        std::vector<double> v(1024);
        for (int b = 0; b < 256; ++b) {
            const double angle = (double)b * (1.0 / 256.0) * M_PI;
            v[(size_t)(2 * b)] = std::sin(angle);
            v[(size_t)(2 * b + 1)] = std::cos(angle);
            v[(size_t)(512 + 2 * b)] = std::cos(2.0 * angle);
            v[(size_t)(512 + 2 * b + 1)] = std::sin(2.0 * angle);
        }
        return v;
    }();
    return t;
}

// ---- the reference's kd-tree (pm_balance, pm.c:329-494), restated ----
// The estimate's exact selection (frt_gi.hpp) needs each photon's place in Jensen's balanced heap:
// the photons the reference's search never reaches (pm.c:172 with half_stored_photons = n/2 - 1,
// pm.c:372) and, for the first heap overflow of pm_locate_photons, the near-first traversal order
// (split planes and positions of the internal nodes). Same median split (Sedgewick's partition),
// same median choice and split axis from the shrinking bounding box; the two halves of a segment are
// independent, so the first levels run on host threads. Checked against the reference's own
// balanced maps (tests/test_photon_map.py, fixture tests/golden/pm_cornell_10k.npz).
struct PmBalance {
    const double* pos;  // 3 per stored photon, stored index 1..n at pos + 3 * (i - 1)
    std::vector<int32_t> porg, pbal;
    std::vector<int8_t> plane;
    double at(int32_t i, int a) const { return pos[3 * (size_t)(i - 1) + a]; }
    void median_split(int start, int end, int median, int axis) {
        int left = start, right = end;
        while (right > left) {
            const double v = at(porg[(size_t)right], axis);
            int i = left - 1, j = right;
            for (;;) {
                while (at(porg[(size_t)++i], axis) < v) {
                }
                while (at(porg[(size_t)--j], axis) > v && j > left) {
                }
                if (i >= j) break;
                std::swap(porg[(size_t)i], porg[(size_t)j]);
            }
            std::swap(porg[(size_t)i], porg[(size_t)right]);
            if (i >= median) right = i - 1;
            if (i <= median) left = i + 1;
        }
    }
    void segment(int64_t index, int start, int end, std::array<double, 3> bmin, std::array<double, 3> bmax, int spawn) {
        int median = 1;
        while (4 * median <= end - start + 1) median += median;
        if (3 * median <= end - start + 1) {
            median += median;
            median += start - 1;
        } else {
            median = end - median + 1;
        }
        int axis = 2;
        if (bmax[0] - bmin[0] > bmax[1] - bmin[1] && bmax[0] - bmin[0] > bmax[2] - bmin[2]) axis = 0;
        else if (bmax[1] - bmin[1] > bmax[2] - bmin[2]) axis = 1;
        median_split(start, end, median, axis);
        pbal[(size_t)index] = porg[(size_t)median];
        plane[(size_t)index] = (int8_t)axis;
        const double split = at(porg[(size_t)median], axis);
        std::thread left_thread;
        if (median > start) {
            if (start < median - 1) {
                auto bmax2 = bmax;
                bmax2[axis] = split;
                if (spawn > 0)
                    left_thread = std::thread([=]() { segment(2 * index, start, median - 1, bmin, bmax2, spawn - 1); });
                else
                    segment(2 * index, start, median - 1, bmin, bmax2, 0);
            } else {
                pbal[(size_t)(2 * index)] = porg[(size_t)start];
            }
        }
        if (median < end) {
            if (median + 1 < end) {
                auto bmin2 = bmin;
                bmin2[axis] = split;
                segment(2 * index + 1, median + 1, end, bmin2, bmax, spawn > 0 ? spawn - 1 : 0);
            } else {
                pbal[(size_t)(2 * index + 1)] = porg[(size_t)end];
            }
        }
        if (left_thread.joinable()) left_thread.join();
    }
};

// heap_of[i] = heap index (1..n) of stored photon i (0-based), plane[h] = split axis of heap node h
static void pm_balance_heap(const double* pos, int64_t n, std::vector<int32_t>& heap_of, std::vector<int8_t>& plane) {
    heap_of.assign((size_t)n, 1);
    plane.assign((size_t)n + 1, 0);
    if (n <= 1) return;
    PmBalance B;
    B.pos = pos;
    B.porg.resize((size_t)n + 1);
    B.pbal.assign((size_t)n + 1, 0);
    B.plane.assign((size_t)n + 1, 0);
    for (int64_t i = 0; i <= n; ++i) B.porg[(size_t)i] = (int32_t)i;
    std::array<double, 3> bmin{INFINITY, INFINITY, INFINITY}, bmax{-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {  // pm_store's bounding box (pm.c:277-284)
            bmin[(size_t)a] = std::min(bmin[(size_t)a], pos[3 * i + a]);
            bmax[(size_t)a] = std::max(bmax[(size_t)a], pos[3 * i + a]);
        }
    const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    int spawn = 0;
    while ((1 << spawn) < threads && n > 65536) ++spawn;
    B.segment(1, 1, (int)n, bmin, bmax, spawn);
    for (int64_t h = 1; h <= n; ++h) heap_of[(size_t)(B.pbal[(size_t)h] - 1)] = (int32_t)h;
    plane.swap(B.plane);
}

// dense uniform grid over the photons (frt_gi.hpp wave_scan_cells): cell edge
// radius / 3, doubled while the grid would exceed kMaxGridCells; photons sorted
// by cell, x fastest (a row of cells is one contiguous range); one allocation
// per map: binary32 positions | power + direction records | cell starts
constexpr double kMaxGridCells = (double)(1 << 24);

// One photon map on the device from photons in the reference's storage order (positions, scaled powers,
// the stored theta / phi direction bytes): balanced as pm_balance would (heap index per photon, split
// planes), the photons the reference's search reaches binned into the dense grid (frt_gi.hpp
// wave_scan_cells; cell edge radius / 3, doubled while the grid would exceed kMaxGridCells; sorted by
// cell, x fastest, so a row of cells is one contiguous range). One allocation per map: binary32
// positions | 80-byte records (binary64 position, power, pm_photon_dir of the direction bytes, heap
// index) | cell starts | the kd-tree (binary64 position and split plane per heap index: the traversal
// order of the estimate's selection).
// a photon map's device arrays, prepared on the host (make_photon_map): what every device of a process
// uploads for the same scene and seed (shared_photon_maps)
struct HostPhotonMap {
    frt::PhotonMapDev M{};  // (counts, grid; the pointers are set at upload)
    std::vector<float> pos4;
    std::vector<double> rec, kd;
    std::vector<int32_t> start;
};

static int upload_host_map(const HostPhotonMap& H, void** out_mem, frt::PhotonMapDev& M) {
    *out_mem = nullptr;
    M = H.M;
    const size_t b_pos4 = H.pos4.size() * sizeof(float), b_pw = H.rec.size() * sizeof(double);
    const size_t b_start = H.start.size() * sizeof(int32_t), b_kd = H.kd.size() * sizeof(double);
    const size_t o_kd = (b_pos4 + b_pw + b_start + 63) & ~(size_t)63;
    FRT_HIP(hipMalloc(out_mem, o_kd + b_kd));
    char* mem = (char*)*out_mem;
    FRT_HIP(hipMemcpy(mem, H.pos4.data(), b_pos4, hipMemcpyHostToDevice));
    FRT_HIP(hipMemcpy(mem + b_pos4, H.rec.data(), b_pw, hipMemcpyHostToDevice));
    FRT_HIP(hipMemcpy(mem + b_pos4 + b_pw, H.start.data(), b_start, hipMemcpyHostToDevice));
    FRT_HIP(hipMemcpy(mem + o_kd, H.kd.data(), b_kd, hipMemcpyHostToDevice));
    M.pos4 = (const float*)mem;
    M.rec = (const double*)(mem + b_pos4);
    M.start = (const int32_t*)(mem + b_pos4 + b_pw);
    M.kd = (const double*)(mem + o_kd);
    return 0;
}

static int prepare_photon_map(int64_t n, const double* pos, const double* power, const uint8_t* tp,
                              double irradiance_radius, HostPhotonMap& H) {
    frt::PhotonMapDev& M = H.M;
    M = frt::PhotonMapDev{};
    if (n > ((int64_t)1 << 30)) return fail("photon map too large");
    std::vector<int32_t> heap_of;
    std::vector<int8_t> plane;
    pm_balance_heap(pos, n, heap_of, plane);
    const int64_t half = n / 2 - 1;  // pm_balance's half_stored_photons (pm.c:372)
    auto reachable = [&](int64_t hx) { return hx == 1 || (hx >> 1) < half; };
    double lo[3] = {0.0, 0.0, 0.0}, hi[3] = {0.0, 0.0, 0.0};
    bool first = true;
    int64_t nr = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!reachable(heap_of[(size_t)i])) continue;
        ++nr;
        const double* p = pos + 3 * i;
        if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))) continue;
        for (int k = 0; k < 3; ++k) {
            lo[k] = first ? p[k] : std::min(lo[k], p[k]);
            hi[k] = first ? p[k] : std::max(hi[k], p[k]);
        }
        first = false;
    }
    M.count = nr;
    static const double cell_div = [] {  // FRT_PM_CELL_DIV: cells per radius (A/B experiments only)
        const char* e = std::getenv("FRT_PM_CELL_DIV");
        const double v = e ? std::atof(e) : 3.0;
        return v >= 1.0 && v <= 16.0 ? v : 3.0;
    }();
    static const double max_cells = [] {  // FRT_PM_MAX_CELLS_LOG2: the grid's cell budget (A/B experiments only)
        const char* e = std::getenv("FRT_PM_MAX_CELLS_LOG2");
        const int v = e ? std::atoi(e) : 0;
        return v >= 10 && v <= 30 ? std::ldexp(1.0, v) : kMaxGridCells;
    }();
    double cell = (irradiance_radius > 0 ? irradiance_radius : 1.0) / cell_div;
    int64_t dims[3];
    for (;;) {
        double cells = 1.0;
        for (int k = 0; k < 3; ++k) {
            const double d = std::floor((hi[k] - lo[k]) / cell) + 1.0;
            dims[k] = d < 1e9 ? (int64_t)d : (int64_t)1e9;
            cells *= (double)dims[k];
        }
        if (cells <= max_cells) break;
        cell *= 2.0;
    }
    for (int k = 0; k < 3; ++k) {
        M.origin[k] = lo[k];
        M.dims[k] = (int32_t)dims[k];
    }
    M.cell = cell;
    M.inv_cell = 1.0 / cell;
    const int64_t ncells = dims[0] * dims[1] * dims[2];
    // the cell of each reachable photon, as the device computes it (floor((x - origin) * inv_cell)), clamped
    std::vector<int32_t> cell_of((size_t)n, -1), start((size_t)ncells + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (!reachable(heap_of[(size_t)i])) continue;
        int64_t c[3];
        for (int k = 0; k < 3; ++k) {
            const double f = std::floor((pos[3 * i + k] - M.origin[k]) * M.inv_cell);
            c[k] = std::isfinite(f) ? (int64_t)std::min(std::max(f, 0.0), (double)(dims[k] - 1)) : 0;
        }
        cell_of[(size_t)i] = (int32_t)((c[2] * dims[1] + c[1]) * dims[0] + c[0]);
        start[(size_t)cell_of[(size_t)i] + 1]++;
    }
    for (int64_t b = 0; b < ncells; ++b) start[(size_t)b + 1] += start[(size_t)b];
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    const size_t np = (size_t)std::max<int64_t>(nr, 1);
    const std::vector<double>& T = dir_tables();
    std::vector<float>& pos4 = H.pos4;
    std::vector<double>& rec = H.rec;
    std::vector<double>& kd = H.kd;
    pos4.assign(np * 4, 0.0f);
    rec.assign(np * 10, 0.0);
    kd.assign((size_t)(n + 1) * 4, 0.0);
    for (int64_t i = 0; i < n; ++i) {
        const int32_t hx = heap_of[(size_t)i];
        for (int k = 0; k < 3; ++k) kd[(size_t)(4 * hx + k)] = pos[3 * i + k];
        kd[(size_t)(4 * hx + 3)] = (double)plane[(size_t)hx];
        if (cell_of[(size_t)i] < 0) continue;
        const int64_t j = fill[(size_t)cell_of[(size_t)i]]++;
        for (int k = 0; k < 3; ++k) {
            pos4[(size_t)(4 * j + k)] = (float)pos[3 * i + k];
            rec[(size_t)(10 * j + k)] = pos[3 * i + k];
            rec[(size_t)(10 * j + 3 + k)] = power[3 * i + k];
        }
        // pm_photon_dir (pm.c:80-88): d = (sin theta cos 2 phi, sin theta sin 2 phi, cos theta)
        const int th = tp[2 * i], ph = tp[2 * i + 1];
        rec[(size_t)(10 * j + 6)] = T[(size_t)(2 * th)] * T[(size_t)(512 + 2 * ph)];
        rec[(size_t)(10 * j + 7)] = T[(size_t)(2 * th)] * T[(size_t)(512 + 2 * ph + 1)];
        rec[(size_t)(10 * j + 8)] = T[(size_t)(2 * th + 1)];
        const int64_t hb = hx;
        std::memcpy(&rec[(size_t)(10 * j + 9)], &hb, sizeof(hb));
    }
    H.start.swap(start);
    return 0;
}

static int make_photon_map(int64_t n, const double* pos, const double* power, const uint8_t* tp,
                           double irradiance_radius, void** out_mem, frt::PhotonMapDev& M) {
    *out_mem = nullptr;
    HostPhotonMap H;
    if (prepare_photon_map(n, pos, power, tp, irradiance_radius, H)) return -1;
    return upload_host_map(H, out_mem, M);
}

static int upload_photon_map(frt_scene_handle* h, int m, const HostPhotonMap& HM) {
    auto& G = h->gi;
    hip_ignore(hipFree(G.map_mem[m]));
    G.map_mem[m] = nullptr;
    frt::PhotonMapDev M{};
    if (upload_host_map(HM, &G.map_mem[m], M)) return -1;
    h->S.pmaps[m] = M;
    return 0;
}

static int build_photon_map(frt_scene_handle* h, const std::vector<frt::StoredPhoton>& ph, double scale,
                            HostPhotonMap& HM) {
    const int64_t n = (int64_t)ph.size();
    std::vector<double> pos((size_t)n * 3), power((size_t)n * 3);
    std::vector<uint8_t> tp((size_t)n * 2);
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            pos[(size_t)(3 * i + k)] = ph[(size_t)i].pos[k];
            power[(size_t)(3 * i + k)] = ph[(size_t)i].power[k] * scale;  // pm_scale_photon_power
        }
    // pm_store's direction bytes of every photon, on the host's cores (acos / atan2 per photon)
    {
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::thread::hardware_concurrency(), 16,
                                                                       n / 65536 + 1}));
        std::vector<std::thread> pool;
        for (int w = 0; w < nt; ++w)
            pool.emplace_back([&, w]() {
                const int64_t i0 = n * w / nt, i1 = n * (w + 1) / nt;
                for (int64_t i = i0; i < i1; ++i) dir_bytes(ph[(size_t)i].dir, tp.data() + 2 * i);
            });
        for (auto& th : pool) th.join();
    }
    return prepare_photon_map(n, pos.data(), power.data(), tp.data(), h->S.cfg.irradiance_radius, HM);
}

// The photon maps of one (scene, seed) are the same on every device (the counter RNG), so the devices of one
// process share them: the first handle to ask traces them on its device and prepares the host arrays (the
// balance, the grid, the records: host work on the process's CPUs), the others wait for that and upload the
// same arrays (render_multi over N devices: one photon pass, not N on the same CPUs). Entries are keyed by
// the scene content's hash and the seed and held weakly: the maps' host arrays (~130 MB per 1M-photon map) live
// while some handle of that (scene, seed) still uploads them, and are freed after the last one.
struct SharedMaps {
    std::mutex mu;
    std::condition_variable cv;
    int state = 0;  // 0 being produced, 1 ready, -1 failed
    HostPhotonMap maps[2];
    uint64_t photons[2] = {0, 0};
};
static std::mutex g_maps_mu;
static std::vector<std::pair<std::pair<uint64_t, uint64_t>, std::weak_ptr<SharedMaps>>> g_maps;


// trace_photons for one render seed: caustic map 0, global map 1
static int build_photon_maps(frt_scene_handle* h, uint64_t seed) {
    const auto& cfg = h->S.cfg;
    const int want[2] = {cfg.trace_caustic_map, cfg.trace_global_map};
    const bool timing = std::getenv("FRT_GI_TIMING") != nullptr;  // diagnostics: host-side phase times
    // FRT_SHARE_PHOTONS=0: every handle traces its own maps (A/B runs)
    const bool share = !(std::getenv("FRT_SHARE_PHOTONS") && std::atoi(std::getenv("FRT_SHARE_PHOTONS")) == 0);
    std::shared_ptr<SharedMaps> sm;
    bool producer = true;
    if (share) {
        const std::pair<uint64_t, uint64_t> key(h->scene_key, seed);
        std::lock_guard<std::mutex> lk(g_maps_mu);
        for (size_t i = 0; i < g_maps.size();) {  // (expired entries out)
            if (g_maps[i].second.expired()) {
                g_maps.erase(g_maps.begin() + (ptrdiff_t)i);
                continue;
            }
            if (g_maps[i].first == key) sm = g_maps[i].second.lock();
            ++i;
        }
        if (sm) {
            producer = false;
        } else {
            sm = std::make_shared<SharedMaps>();
            g_maps.emplace_back(key, sm);
        }
    } else {
        sm = std::make_shared<SharedMaps>();
    }
    if (producer) {
        // every exit from the producer (an exception included) leaves a final state, so no consumer waits forever
        struct Settle {
            SharedMaps* m;
            ~Settle() {
                bool notify = false;
                {
                    std::lock_guard<std::mutex> lk(m->mu);
                    if (m->state == 0) {
                        m->state = -1;
                        notify = true;
                    }
                }
                if (notify) m->cv.notify_all();
            }
        } settle{sm.get()};
        int rc = 0;
        for (int m = 0; m < 2 && rc == 0; ++m) {
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<frt::StoredPhoton> ph;
            if (want[m])
                for (int l = 0; l < h->S.num_lights && rc == 0; ++l) rc = trace_light_photons(h, m, l, seed, ph);
            if (rc) break;
            // pm_store keeps at most max_photons + 1 photons (pm.c:271)
            if ((int64_t)ph.size() > cfg.photon_count + 1) ph.resize((size_t)cfg.photon_count + 1);
            const auto t1 = std::chrono::steady_clock::now();
            rc = build_photon_map(h, ph, 1.0 / (double)cfg.photon_count, sm->maps[m]);
            sm->photons[m] = ph.size();
            if (timing) {
                const auto t2 = std::chrono::steady_clock::now();
                std::fprintf(stderr, "photon map %d: %zu photons, trace %.1f ms, build %.1f ms\n", m, ph.size(),
                             std::chrono::duration<double, std::milli>(t1 - t0).count(),
                             std::chrono::duration<double, std::milli>(t2 - t1).count());
            }
        }
        g_maps_stat[0]++;
        {
            std::lock_guard<std::mutex> lk(sm->mu);
            sm->state = rc ? -1 : 1;
        }
        sm->cv.notify_all();
        if (rc) {  // (a later frame may try again)
            std::lock_guard<std::mutex> lk(g_maps_mu);
            for (size_t i = 0; i < g_maps.size(); ++i)
                if (g_maps[i].second.lock() == sm) {
                    g_maps.erase(g_maps.begin() + (ptrdiff_t)i);
                    break;
                }
            return -1;
        }
    } else {
        std::unique_lock<std::mutex> lk(sm->mu);
        sm->cv.wait(lk, [&] { return sm->state != 0; });
        if (sm->state < 0) return fail("photon maps: the producing device failed");
        g_maps_stat[1]++;
    }
    for (int m = 0; m < 2; ++m) {
        if (upload_photon_map(h, m, sm->maps[m])) return -1;
        h->gi.photons[m] = sm->photons[m];
    }
    h->gi.built = true;
    h->gi.seed = seed;
    return 0;
}

// shade_hit's GI terms for the nodes of one level (renderer.c:727-770); chunks of
// nodes keep the final-gather queue bounded
static int shade_gi(frt_scene_handle* h, const frt::Batch& B, frt_scene_handle::Level& L, int64_t n, frt_frame_stats* st) {
    using namespace frt;
    auto& G = h->gi;
    const auto& cfg = h->S.cfg;
    if (grow(&G.extra, G.extra_cap, 6 * n) || grow(&G.fgather, G.fgather_cap, 3 * n)) return -1;
    hipLaunchKernelGGL(k_gi_node, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, L.rec, n, G.extra);
    FRT_HIP(hipGetLastError());
    const int64_t rays_per = (int64_t)cfg.gi_usteps * (int64_t)cfg.gi_vsteps;
    const bool gather = cfg.include_final_gather && rays_per > 0;
    if (gather) {
        // gather rays per chunk (FRT_GATHER_CHUNK): each chunk's estimate launch ends in a tail of its slowest queries;
        // 2^22 / 2^24 / 2^25 rays gave 29.33 / 28.97 / 28.92 s GI frames (profiles/r05_ab_gi_chunk.txt); 2^24 keeps
        // the chunk's buffers at 3.2 GB
        static const int64_t kChunkRays = [] {
            const char* e = std::getenv("FRT_GATHER_CHUNK");
            const long long v = e ? std::atoll(e) : 0;
            return v >= 1024 ? (int64_t)v : (int64_t)1 << 24;
        }();
        const int64_t chunk = std::max<int64_t>(1, kChunkRays / rays_per);
        for (int64_t n0 = 0; n0 < n; n0 += chunk) {
            const int64_t m = std::min(chunk, n - n0);
            const int64_t rays = m * rays_per;
            if (grow(&G.gq, G.gq_cap, rays) || grow(&G.ghits, G.ghits_cap, rays) || grow(&G.gcol, G.gcol_cap, 3 * rays) ||
                grow(&G.greq, G.greq_cap, rays))
                return -1;
            hipLaunchKernelGGL(k_gather_gen, dim3(grid_for(rays)), dim3(kBlock), 0, h->stream, h->S, B.seed, L.rec, n0, m,
                               G.gq);
            frt::Batch Bg = B;  // the gather rays form one contiguous queue
            Bg.qprefix = nullptr;
            Bg.qperm = nullptr;
            // the hemisphere rays through the scene-specialised closest hit where the scene has one (1387 -> 1363 ms per
            // cornell_gi_480x270_8x8 frame, profiles/r06_ab_gather_jit.txt; round 4's slower kernel lost there,
            // profiles/r04_ab_gi_trace.txt); FRT_GATHER_JIT=0: the generic walk (A/B runs)
            // (read per chunk, like the knobs below: a test switches them between frames of one process)
            const bool gather_jit = !(std::getenv("FRT_GATHER_JIT") && std::atoi(std::getenv("FRT_GATHER_JIT")) == 0);
            launch_trace(h, Bg, G.gq, rays, G.ghits, 0, nullptr, gather_jit);
            // FRT_GATHER_QUEUE=0: the static request ranges (A/B runs)
            const char* qenv = std::getenv("FRT_GATHER_QUEUE");
            const bool queue = !(qenv && std::strcmp(qenv, "0") == 0) && rays < (int64_t)0xF0000000u;
            // the requests in the spatial order of their points from 4096 of them (FRT_GATHER_SORT=0: gather order,
            // =1: sorted at any count)
            const int sort_mode = std::getenv("FRT_GATHER_SORT") ? std::atoi(std::getenv("FRT_GATHER_SORT")) : -1;
            const bool sorted = queue && sort_mode != 0 && (rays >= 4096 || sort_mode == 1) && rays < (int64_t)0x7FFFFFFF;
            if (sorted && grow(&G.gkeys, G.gkeys_cap, 4 * rays)) return -1;
            uint32_t *k0 = G.gkeys, *k1 = G.gkeys + rays, *i0 = G.gkeys + 2 * rays, *i1 = G.gkeys + 3 * rays;
            {
                KTimer th(h, st, 11);
                hipLaunchKernelGGL(h->S.num_patterns > 0 ? k_gather_hit<true> : k_gather_hit<false>, dim3(grid_for(rays)),
                                   dim3(kBlock), 0, h->stream, h->S, B.seed, G.gq, G.ghits, rays, G.greq,
                                   sorted ? k0 : nullptr, sorted ? i0 : nullptr);
            }
            {
                KTimer te(h, st, 10);
                if (queue) {
                    if (!G.gwork) FRT_HIP(hipMalloc((void**)&G.gwork, kGatherGroups * 64 * sizeof(unsigned)));
                    FRT_HIP(hipMemsetAsync(G.gwork, 0, kGatherGroups * 64 * sizeof(unsigned), h->stream));
                    const uint32_t* perm = nullptr;
                    if (sorted) {
                        size_t tmp_bytes = 0;
                        FRT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, i0, i1, (int)rays, 0,
                                                                   kGatherKeyBits, h->stream));
                        if (grow(&h->scan_tmp, h->scan_tmp_cap, (int64_t)tmp_bytes + 16)) return -1;
                        FRT_HIP(hipcub::DeviceRadixSort::SortPairs((void*)h->scan_tmp, tmp_bytes, k0, k1, i0, i1, (int)rays, 0,
                                                                   kGatherKeyBits, h->stream));
                        perm = i1;
                    }
                    int cus = 0;
                    FRT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
                    // every wave resident at once: FRT_EST_WAVES per SIMD, 4 SIMDs per CU
                    const int64_t blocks = std::max<int64_t>(1, (int64_t)cus * 4 * FRT_EST_WAVES / kGatherWavesPerBlock);
                    hipLaunchKernelGGL(k_gather_est, dim3((unsigned)blocks), dim3(64 * kGatherWavesPerBlock), 0, h->stream,
                                       h->S, G.greq, rays, G.gcol, G.gwork, perm);
                } else {
                    const int64_t gwaves = (rays + kGatherReqPerWave - 1) / kGatherReqPerWave;
                    hipLaunchKernelGGL(k_gather_est, dim3((unsigned)((gwaves + kGatherWavesPerBlock - 1) / kGatherWavesPerBlock)),
                                       dim3(64 * kGatherWavesPerBlock), 0, h->stream, h->S, G.greq, rays, G.gcol,
                                       (unsigned*)nullptr, (const uint32_t*)nullptr);
                }
            }
            hipLaunchKernelGGL(k_gather_reduce, dim3(grid_for(m)), dim3(kBlock), 0, h->stream, h->S, L.rec, n0, m, G.gcol,
                               G.fgather);
            FRT_HIP(hipGetLastError());
            if (st) st->gather_rays += (uint64_t)rays;
        }
    }
    hipLaunchKernelGGL(k_gi_apply, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, L.rec, n, G.extra,
                       gather ? G.fgather : nullptr, L.surface);
    FRT_HIP(hipGetLastError());
    return 0;
}

extern "C" {

#if defined(FRT_WALK_STATS) || defined(FRT_WALK_PROF)
// debug builds: dump the walk counters accumulated so far to stderr
static void dump_walk_stats(frt_scene_handle* h) {
    unsigned long long c[frt::kDbgSlots];
    if (hipMemcpy(c, h->S.dbg, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return;
    const char* names[8] = {"composite_visits", "leaf_visits", "active_lane_visits", "jumps", "walks", "live_lanes",
                            "prefilter_rejects", "lanes_tested"};
    for (int k = 0; k < 2; ++k) {
        std::fprintf(stderr, "walk stats (%s):", k == 0 ? "shadow" : "closest");
        for (int j = 0; j < 8; ++j) std::fprintf(stderr, " %s=%llu", names[j], c[8 * k + j]);
        std::fprintf(stderr, "\n");
    }
    // per node: wave visits / active lanes (shadow, then closest hit)
    for (int k = 0; k < 2; ++k) {
        std::fprintf(stderr, "node visits (%s):", k == 0 ? "shadow" : "closest");
        for (int i = 0; i < std::min(h->S.num_nodes, frt::kDbgNodes); ++i) {
            const unsigned long long* v = c + 16 + (k * frt::kDbgNodes + i) * 2;
            if (v[0]) std::fprintf(stderr, " %d:%llu/%llu", i, v[0], v[1]);
        }
        std::fprintf(stderr, "\n");
    }
    std::fprintf(stderr, "walk prof (shadow, cycles):");
    const char* pn[8] = {"setup", "close", "xf_pop", "composite", "leaf_xf", "leaf_test", "leaf_post", "loop"};
    for (int k = 0; k < 8; ++k) std::fprintf(stderr, " %s=%llu", pn[k], c[frt::kDbgProf + k]);
    std::fprintf(stderr, "\nestimate prof (cycles): scan=%llu select=%llu sum=%llu band=%llu; queries over k=%llu "
                 "unlisted=%llu slow_band=%llu order_check=%llu in_range_total=%llu order_check_cycles=%llu",
                 c[frt::kDbgProf + 13], c[frt::kDbgProf + 14], c[frt::kDbgProf + 15], c[frt::kDbgProf + 16],
                 c[frt::kDbgProf + 17], c[frt::kDbgProf + 18], c[frt::kDbgProf + 19], c[frt::kDbgProf + 20],
                 c[frt::kDbgProf + 21], c[frt::kDbgProf + 22]);
    std::fprintf(stderr, " reduce_tried=%llu reduce_fallback=%llu queries=%llu candidates_read=%llu records_read=%llu",
                 c[frt::kDbgProf + 23], c[frt::kDbgProf + 24], c[frt::kDbgProf + 25], c[frt::kDbgProf + 27],
                 c[frt::kDbgProf + 28]);
    std::fprintf(stderr, "\nprepare prof (cycles):");
    const char* qn[5] = {"ray", "hits_load", "prepare", "spawn", "stores"};
    for (int k = 0; k < 5; ++k) std::fprintf(stderr, " %s=%llu", qn[k], c[frt::kDbgProf + 8 + k]);
    std::fprintf(stderr, "\n");
}
#endif

static int render_frame(frt_scene_handle* h, const frt_frame_params* P, double* dev_out, frt_frame_stats* st);

// a failed frame leaves no half-built state behind: photon maps traced by it (maybe truncated by a
// store overflow) are not reused by the next frame with the same seed
static int render_impl(frt_scene_handle* h, const frt_frame_params* P, double* dev_out, frt_frame_stats* st) {
    h->cur_st = st;
    h->rays_walked = 0;
    h->pairs_walked = 0;
    h->heads_walked = 0;
    h->tile_pairs = h->tile_mixed = h->node_pairs = h->node_mixed = h->sub_pairs = h->sub_mixed = 0;
    h->subtile_pairs = h->subtile_mixed = 0;
    const int rc = render_frame(h, P, dev_out, st);
    if (rc) h->gi.built = false;
    return rc;
}

static int render_frame(frt_scene_handle* h, const frt_frame_params* P, double* dev_out, frt_frame_stats* st) {
    using namespace frt;
    FRT_HIP(hipSetDevice(h->device));
    const int64_t hs = h->S.cam.hsize;
    const int64_t stride = P->row_stride > 0 ? P->row_stride : 1;
    int64_t nrows = 0;
    for (int64_t r = P->row_begin; r < P->row_end; r += stride) nrows++;
    const int64_t npix = nrows * hs;
    const int32_t spp = (int32_t)(h->S.cam.usteps * h->S.cam.vsteps);
    if (spp <= 0) return fail("render: usteps*vsteps must be positive");
    // 8 M samples unless the caller asks for more. Each batch pays the shadow pass's host round trips (the list
    // counts that size its next launch) and every level's, so a handle that renders frame after frame takes the
    // whole frame in one batch (frt_render_params.batch_samples; bench.py: 2^27 = the headline frame, about
    // 70 GB of level state, 8 M / 32 M / 128 M samples per batch gave 54.3 / 49.1 / 48.0 ms headline frames,
    // tools/ab_batch.sh). The default suits one-shot calls (render_multi): a handle's first frame allocates its
    // level state, and the driver clears fresh device memory at ~11 GB/s, 6 s for 128 M samples
    // (tools/rm_batch.py, profiles/r04_ab_batch.txt). FRT_BATCH_SAMPLES overrides the default (A/B runs).
    const char* benv = std::getenv("FRT_BATCH_SAMPLES");
    const int64_t bdef = benv && std::atoll(benv) > 0 ? (int64_t)std::atoll(benv) : (int64_t)1 << 23;
    int64_t batch = P->batch_samples > 0 ? P->batch_samples : bdef;
    int64_t pix_per_batch = std::max<int64_t>(1, batch / spp);
    const int path = h->S.cfg.path_length;
    if (st) {
        std::memset(st, 0, sizeof(*st));
        (void)hipEventRecord(h->ev[0], h->stream);
    }
    FRT_HIP(hipMemsetAsync(h->err, 0, sizeof(unsigned), h->stream));
    FRT_HIP(hipMemsetAsync(h->counters, 0, frt::kQueueSegs * frt::kCounterLine * sizeof(unsigned long long), h->stream));
    if (h->S.cfg.use_gi && (!h->gi.built || h->gi.seed != P->seed)) {
        // the photon maps belong to the render seed: same seed, same image (also across row splits)
        hipEvent_t p0 = nullptr, p1 = nullptr;
        if (st) {
            hip_ignore(hipEventCreate(&p0));
            hip_ignore(hipEventCreate(&p1));
            hip_ignore(hipEventRecord(p0, h->stream));
        }
        const int rc = build_photon_maps(h, P->seed);
        if (st) {
            hip_ignore(hipEventRecord(p1, h->stream));
            hip_ignore(hipEventSynchronize(p1));
            float ms = 0.f;
            hip_ignore(hipEventElapsedTime(&ms, p0, p1));
            st->photon_ms = ms;
            st->photon_pass = 1;
            hip_ignore(hipEventDestroy(p0));
            hip_ignore(hipEventDestroy(p1));
        }
        if (rc) return rc;
    }
    if (st) {
        st->photons[0] = h->gi.photons[0];
        st->photons[1] = h->gi.photons[1];
    }
    if (!h->host_counters.resize((size_t)kQueueSegs * kCounterLine) ||
        !h->host_lcount.resize((size_t)kShadeSegs * jit::kMixLine))
        return fail("render: pinned host buffer allocation failed");
    auto& host_counters = h->host_counters;
    for (int64_t p0 = 0; p0 < npix; p0 += pix_per_batch) {
        const int64_t bp = std::min<int64_t>(pix_per_batch, npix - p0);
        const int64_t ns = bp * spp;
        if (ns > h->sample_cap) {
            hip_ignore(hipFree(h->sample_col.w));
            h->sample_col = {};
            h->sample_cap = 0;
            FRT_HIP(hipMalloc((void**)&h->sample_col.w, frt::Cols<frt::Tri9>::bytes(ns)));
            h->sample_col.cap = h->sample_cap = ns;
        }
        if (ensure_level(h, 0, ns)) return -1;
        Batch B{};
        B.sample_begin = 0;
        // global sample index of the first sample: pixel (row, col) in frame coordinates
        const int64_t first_row = P->row_begin + (p0 / hs) * stride;
        B.sample_begin = (first_row * hs + p0 % hs) * spp;
        B.pixel_begin = p0;
        B.num_samples = ns;
        B.row_begin = P->row_begin;
        B.row_stride = stride;
        B.seed = P->seed;
        B.spp = spp;
        B.stats = st != nullptr ? 1 : 0;
        std::vector<int64_t> count(path + 2, 0);
        count[0] = ns;
        // the queue counts (words 0..15) of every counter line
        FRT_HIP(hipMemset2DAsync(h->counters, kCounterLine * sizeof(unsigned long long), 0, 16 * sizeof(unsigned long long),
                                 kQueueSegs, h->stream));
        for (int d = 0; d <= path; ++d) {
            const int64_t n = count[d];
            if (n == 0) break;
            B.level = d;
            B.remaining = path - d;
            auto& L = h->levels[d];
            // a block appends up to 2 * kBlock rays to its segment: 2n plus one block's worth per segment
            if (ensure_level(h, d + 1, 2 * n + (int64_t)kQueueSegs * 2 * kBlock)) return -1;
            auto& N = h->levels[d + 1];
            B.qprefix = d > 0 ? L.qprefix : nullptr;
            B.qperm = d > 0 && L.sorted ? L.qperm : nullptr;
            B.qsegcap = L.cap / kQueueSegs;
            B.next_segcap = N.cap / kQueueSegs;
            if (h->S.num_lights < 1)  // (k_prepare zeroes the level's counts of its nodes' lights)
                FRT_HIP(hipMemsetAsync(L.counts, 0, (size_t)n * sizeof(int32_t), h->stream));
            if (grow(&h->hits, h->hits_cap, n)) return -1;
            if (!h->S.cfg.all_ni_one && grow(&h->hn12, h->hn12_cap, 2 * n)) return -1;
            double* hn12 = h->S.cfg.all_ni_one ? nullptr : h->hn12;
            const QueuedRay* q = d == 0 ? nullptr : L.q;
            bool dense = false;
            {
                KTimer t(h, st, d == 0 ? 5 : 0);
                launch_trace(h, B, q, n, h->hits, 0, hn12, true);
                FRT_HIP(hipGetLastError());
            }
            {
                KTimer t(h, st, 6);
                // tile boxes for frt_jit_tile (scene-specialised shadow kernels)
                const bool tiles = h->tile > 0 && h->jit_shadow && h->jit_beam_on && h->S.cfg.include_direct &&
                                   h->samples_per_node > 0;
                int tl = 0;
                while (tiles && (1 << tl) < h->tile) ++tl;
                if (tiles && grow(&h->tbox, h->tbox_cap, 6 * ((n >> tl) + 1))) return -1;
                const bool subtiles = tiles && h->subtile > 0 && h->subtile < h->tile;
                int stl = 0;
                while (subtiles && (1 << stl) < h->subtile) ++stl;
                if (subtiles && grow(&h->stbox, h->stbox_cap, 6 * ((n >> stl) + 1))) return -1;
                // the next level dense (FRT_QUEUE_SORT=2, default): child (node, slot) at slot n + node of its queue,
                // the taken slots compacted in order (reflected children in parent order, then the refracted) into
                // the next level's qperm, their count into counter word 20 (read back with the queue counts)
                dense = h->queue_sort == 2 && d < path && 2 * n <= (int64_t)UINT32_MAX && N.cap >= 2 * n;
                const int64_t G = (n + 63) >> 6;
                if (dense && (grow(&h->spawn_masks, h->spawn_masks_cap, 2 * G) ||
                              grow(&h->spawn_offs, h->spawn_offs_cap, 2 * G + 1) || grow(&N.qperm, N.qperm_cap, 2 * n)))
                    return -1;
                hipLaunchKernelGGL(h->S.num_patterns > 0 ? k_prepare<true> : k_prepare<false>, dim3(grid_for(n)),
                                   dim3(kBlock), 0, h->stream, h->S, B, q, n, h->hits, hn12,
                                   L.rec, L.head, N.q, h->counters, h->err, tiles ? h->tbox : nullptr, tl,
                                   subtiles ? h->stbox : nullptr, stl, L.counts, dense ? h->spawn_masks : nullptr);
                FRT_HIP(hipGetLastError());
                if (dense) {
                    hipcub::CountingInputIterator<int64_t> idx(0);
                    hipcub::TransformInputIterator<uint32_t, MaskPopc, hipcub::CountingInputIterator<int64_t>> popc(
                        idx, MaskPopc{h->spawn_masks, 2 * G});
                    size_t tmp_bytes = 0;
                    FRT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, popc, h->spawn_offs, (int)(2 * G + 1),
                                                             h->stream));
                    if (grow(&h->scan_tmp, h->scan_tmp_cap, (int64_t)tmp_bytes + 16)) return -1;
                    FRT_HIP(hipcub::DeviceScan::ExclusiveSum((void*)h->scan_tmp, tmp_bytes, popc, h->spawn_offs,
                                                             (int)(2 * G + 1), h->stream));
                    hipLaunchKernelGGL(k_spawn_expand, dim3(grid_for(2 * G)), dim3(kBlock), 0, h->stream, h->spawn_masks,
                                       h->spawn_offs, n, G, N.qperm, h->counters);
                    FRT_HIP(hipGetLastError());
                }
            }
            // the next level's queue counts are final here (k_prepare appends the level's rays): their copy rides on
            // the shadow pass's first synchronize, and the level ends without one of its own
            FRT_HIP(hipMemcpyAsync(host_counters.data(), h->counters, host_counters.size() * sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, h->stream));
            const uint64_t counters_epoch = h->sync_epoch;
            if (h->S.cfg.include_direct && h->samples_per_node > 0) {
                KTimer t(h, st, 1);
                launch_shadow(h, B, L.head, n, L.counts);
                FRT_HIP(hipGetLastError());
            }
            if (h->jit_stats && h->S.num_lights > 0) {  // FRT_JIT_STATS: (node, light) counts all-lit / all-shadowed / mixed
                std::vector<int32_t> hc((size_t)n * h->S.num_lights);
                std::vector<frt::ShadowHead> hh((size_t)n);
                FRT_HIP(hipMemcpyAsync(hc.data(), L.counts, hc.size() * sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
                FRT_HIP(hipMemcpyAsync(hh.data(), L.head, hh.size() * sizeof(frt::ShadowHead), hipMemcpyDeviceToHost, h->stream));
                FRT_HIP(hipStreamSynchronize(h->stream));
                for (int64_t i = 0; i < n; ++i) {
                    if (hh[(size_t)i].material < 0) continue;
                    for (int l = 0; l < h->S.num_lights; ++l) {
                        const int32_t c = hc[(size_t)(i * h->S.num_lights + l)];
                        h->uniform_stats[c == 0 ? 1 : (c == h->host_lights[(size_t)l].num_samples ? 0 : 2)]++;
                    }
                }
            }
            {
                KTimer t(h, st, 2);
                const bool split = shade_split();
                const int64_t nblocks = grid_for(n);
                const uint32_t segcap = (uint32_t)(((nblocks + kShadeSegs - 1) / kShadeSegs) * kBlock);
                if (split && (grow(&h->shade_lit, h->shade_lit_cap, (int64_t)segcap * kShadeSegs) ||
                              grow(&h->shade_lcount, h->shade_lcount_cap, (int64_t)kShadeSegs * jit::kMixLine)))
                    return -1;
                if (split)
                    FRT_HIP(hipMemsetAsync(h->shade_lcount, 0, (size_t)kShadeSegs * jit::kMixLine * sizeof(unsigned),
                                           h->stream));
                // the row sort (multi-row light): row counts beside the list, then the list in row order
                const bool sorted = split && h->sort_light >= 0;
                const int nrows = sorted ? std::max(1, h->host_lights[(size_t)h->sort_light].rows) : 0;
                int row_bits = 1;
                while (row_bits < 32 && (1ll << row_bits) < nrows) ++row_bits;
                // (the staged records: without GI, whose kernels read and write the surface columns by node)
                const bool sorted_out = sorted && shade_lazy(h) && L.spos != nullptr && h->shade_stage > 0;
                const bool staged = sorted_out && h->shade_stage == 1;
                L.staged = sorted_out;
                if (sorted) {
                    const int64_t lcap = (int64_t)segcap * kShadeSegs;
                    if (grow(&h->lit_row, h->lit_row_cap, 2 * lcap) || grow(&h->lit_flat, h->lit_flat_cap, 2 * lcap))
                        return -1;
                    if (staged && grow(&h->lit_stage, h->lit_stage_cap, lcap)) return -1;
                }
                if (shade_lazy(h))
                    hipLaunchKernelGGL(k_shade<true>, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, L.rec, n,
                                       L.counts, L.surface, h->shade_lit, h->shade_lcount, segcap);
                else
                    hipLaunchKernelGGL(k_shade<false>, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, L.rec, n,
                                       L.counts, L.surface, split ? h->shade_lit : nullptr, h->shade_lcount, segcap);
                if (sorted) {
                    KTimer ts(h, st, 16);  // (k_lit_rows + the radix sort, sub_ms["k_lit_sort"])
                    const int64_t lcap = (int64_t)segcap * kShadeSegs;
                    uint32_t *keys = h->lit_row, *keys2 = h->lit_row + lcap, *vals = h->lit_flat + lcap;
                    if (staged)
                        hipLaunchKernelGGL(k_lit_stage, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, L.rec,
                                           L.counts, h->shade_lit, h->shade_lcount, segcap, h->sort_light, keys, vals,
                                           h->lit_stage);
                    else
                        hipLaunchKernelGGL(k_lit_rows, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, L.head,
                                           h->shade_lit, h->shade_lcount, segcap, h->sort_light, keys, vals);
                    // (the listed count on the host: the sort's size)
                    auto& lc = h->host_lcount;
                    FRT_HIP(hipMemcpyAsync(lc.data(), h->shade_lcount, lc.size() * sizeof(unsigned), hipMemcpyDeviceToHost,
                                           h->stream));
                    FRT_HIP(stream_sync(h));
                    int64_t listed = 0;
                    for (int sgi = 0; sgi < kShadeSegs; ++sgi) listed += lc[(size_t)sgi * jit::kMixLine];
                    if (st != nullptr) st->lit_nodes += (uint64_t)listed;
                    if (listed > 0) {
                        size_t tmp_bytes = 0;
                        FRT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, vals, h->lit_flat,
                                                                   (int)listed, 0, row_bits, h->stream));
                        if (grow(&h->scan_tmp, h->scan_tmp_cap, (int64_t)tmp_bytes + 16)) return -1;
                        FRT_HIP(hipcub::DeviceRadixSort::SortPairs((void*)h->scan_tmp, tmp_bytes, keys, keys2, vals,
                                                                   h->lit_flat, (int)listed, 0, row_bits, h->stream));
                    }
                }
                if (split && st != nullptr && !sorted) {  // (the stats frame: the listed count, frt_frame_stats.lit_nodes)
                    auto& lc = h->host_lcount;
                    FRT_HIP(hipMemcpyAsync(lc.data(), h->shade_lcount, lc.size() * sizeof(unsigned), hipMemcpyDeviceToHost,
                                           h->stream));
                    FRT_HIP(hipStreamSynchronize(h->stream));
                    for (int sgi = 0; sgi < kShadeSegs; ++sgi) st->lit_nodes += lc[(size_t)sgi * jit::kMixLine];
                }
                if (split) {
                    KTimer tl(h, st, 15);  // (inside the shade slot: k_shade_lit alone, sub_ms[7])
#ifndef FRT_SHADE_LIT_BLOCK
#define FRT_SHADE_LIT_BLOCK 64  // (one wave per block: 9.15 -> 8.83 ms per headline frame, profiles/r05_ab_shade_block.txt; <= kBlock)
#endif
                    hipLaunchKernelGGL(sorted ? k_shade_lit<true> : k_shade_lit<false>, dim3(grid_for(n, FRT_SHADE_LIT_BLOCK)),
                                       dim3(FRT_SHADE_LIT_BLOCK), 0,
                                       h->stream, h->S, B, L.rec, L.counts, L.surface, h->shade_lit, h->shade_lcount, segcap,
                                       sorted ? (const uint32_t*)h->lit_flat : nullptr,
                                       staged ? (const frt::LitStage*)h->lit_stage : nullptr,
                                       sorted_out ? L.spos : nullptr);
                }
                FRT_HIP(hipGetLastError());
            }
            if (h->S.cfg.use_gi) {
                KTimer t(h, st, 7);
                if (shade_gi(h, B, L, n, st)) return -1;
            }
            if (h->sync_epoch == counters_epoch) FRT_HIP(stream_sync(h));  // (no synchronize since the counters' copy)
            // the next level's queue segments: prefix counts (a segment past its capacity is an error)
            int64_t next = 0;
            bool overflow = false;
            for (int j = 0; j < kQueueSegs && !dense; ++j) {
                N.hprefix[j] = next;
                int64_t c = (int64_t)host_counters[(size_t)j * kCounterLine + d + 1];
                if (c > B.next_segcap) {
                    overflow = true;
                    c = B.next_segcap;
                }
                next += c;
            }
            if (dense) next = (int64_t)host_counters[20];  // (the compaction's count)
            N.hprefix[kQueueSegs] = next;
            if (overflow) {
                unsigned e = kErrQueueOverflow;
                FRT_HIP(hipMemcpyAsync(h->err, &e, sizeof(unsigned), hipMemcpyHostToDevice, h->stream));
            }
            if (next > 0 && d < path && !dense)
                FRT_HIP(hipMemcpyAsync(N.qprefix, N.hprefix.data(), (kQueueSegs + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                                       h->stream));
            count[d + 1] = d < path ? next : 0;
            // the next level in parent order (FRT_QUEUE_SORT): its nodes, tiles and shading then follow the
            // parents' pixels; keys: refracted bit above the parent index
            int pbits = 1;
            while (pbits < 32 && (1ll << pbits) < n) ++pbits;
            N.sorted = dense || (h->queue_sort == 1 && d < path && next >= 4096 && !overflow && pbits < 32 &&
                                 N.cap <= (int64_t)UINT32_MAX);
            if (N.sorted && !dense) {
                KTimer t(h, st, 6);
                if (grow(&h->qsort, h->qsort_cap, 3 * next) || grow(&N.qperm, N.qperm_cap, next)) return -1;
                uint32_t *keys = h->qsort, *keys2 = h->qsort + next, *slots = h->qsort + 2 * next;
                Batch Bn = B;
                Bn.qprefix = N.qprefix;
                Bn.qsegcap = N.cap / kQueueSegs;
                Bn.qperm = nullptr;
                const int shift = std::min(h->queue_sort_shift, pbits - 1);
                hipLaunchKernelGGL(k_queue_keys, dim3(grid_for(next)), dim3(kBlock), 0, h->stream, Bn, N.q, next, pbits,
                                   shift, keys, slots);
                FRT_HIP(hipGetLastError());
                size_t tmp_bytes = 0;
                FRT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, slots, N.qperm, (int)next, 0,
                                                           pbits - shift + 1, h->stream));
                if (grow(&h->scan_tmp, h->scan_tmp_cap, (int64_t)tmp_bytes + 16)) return -1;
                FRT_HIP(hipcub::DeviceRadixSort::SortPairs((void*)h->scan_tmp, tmp_bytes, keys, keys2, slots, N.qperm,
                                                           (int)next, 0, pbits - shift + 1, h->stream));
            }
            if (st) {
                if (d > 0) st->secondary_rays += (uint64_t)n;
                else st->primary_rays += (uint64_t)n;
            }
        }
        // level 0 combined and resolved in one pass when a block holds whole pixels (FRT_FUSE_RESOLVE=0: the
        // two kernels, A/B runs)
        const char* fuse_env = std::getenv("FRT_FUSE_RESOLVE");
        const bool fuse = spp <= kFuseBlock && !(fuse_env && std::strcmp(fuse_env, "0") == 0);
        const bool lazy = shade_lazy(h);
        for (int d = path; d >= 0; --d) {
            const int64_t n = count[d];
            if (n == 0) continue;
            if (d == 0 && fuse) {
                KTimer t(h, st, 4);
                const int32_t ppb = kFuseBlock / spp;
                hipLaunchKernelGGL(k_combine_resolve, dim3((unsigned)((bp + ppb - 1) / ppb)), dim3(kFuseBlock), 0, h->stream,
                                   h->S, lazy ? h->levels[0].counts : nullptr, h->levels[0].rec, n, h->levels[0].surface, h->levels[0].child, spp, ppb, bp,
                                   h->S.materials, h->S.cfg.include_specular, dev_out + 4 * p0,
                                   h->levels[0].staged ? (const uint32_t*)h->levels[0].spos : nullptr);
                FRT_HIP(hipGetLastError());
                continue;
            }
            KTimer t(h, st, 3);
            const Cols<Tri9> parent_child = d > 0 ? h->levels[d - 1].child : Cols<Tri9>{};
            hipLaunchKernelGGL(k_combine, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S,
                               lazy ? h->levels[d].counts : nullptr, h->levels[d].rec, n,
                               h->levels[d].surface, h->levels[d].child, parent_child, h->sample_col, spp,
                               h->S.materials, h->S.cfg.include_specular,
                               h->levels[d].staged ? (const uint32_t*)h->levels[d].spos : nullptr);
            FRT_HIP(hipGetLastError());
        }
        if (!fuse) {
            KTimer t(h, st, 4);
            hipLaunchKernelGGL(k_resolve, dim3((unsigned)((bp + 63) / 64)), dim3(kResolveBlock), 0, h->stream, h->sample_col, bp, spp,
                               dev_out + 4 * p0);
            FRT_HIP(hipGetLastError());
        }
    }
    FRT_HIP(hipMemcpyAsync(host_counters.data(), h->counters, host_counters.size() * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, h->stream));
    unsigned err = 0;
    FRT_HIP(hipMemcpyAsync(&err, h->err, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    if (st) (void)hipEventRecord(h->ev[1], h->stream);
    FRT_HIP(hipStreamSynchronize(h->stream));
    if (st) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
        st->render_ms = ms;
        uint64_t pruned = 0, hits = 0;
        for (int j = 0; j < kQueueSegs; ++j) {
            pruned += host_counters[(size_t)j * kCounterLine + 16];
            hits += host_counters[(size_t)j * kCounterLine + 17];
        }
        st->pruned_secondary = pruned;
        st->hits = hits;
        st->shadow_rays = h->S.cfg.include_direct ? hits * (uint64_t)h->samples_per_node : 0;
        // DESIGN.md byte model of the per-ray shadow kernel: per list entry its 4-byte entry and 4-byte resume word;
        // per node of an entry its ShadowHead, read once for the entry's rays and at most once per launch for the node
        // (heads_walked: an entry of the sub-part list holds a tile's 64 nodes, of the node-pair list one), and one
        // 4-byte count added; with a multi-row light
        // each ray's 24-byte point from its node's row (a single-row light's points stay in cache); the generic walk:
        // per shaded node the ShadowHead + one 4-byte count per light
        constexpr double kHead = (double)sizeof(frt::ShadowHead);
        bool multi = false;
        for (const auto& L : h->host_lights) multi = multi || L.rows > 1;
        st->shadow_kernel_bytes = !(h->S.cfg.include_direct && h->samples_per_node > 0) ? 0.0
                                  : h->jit_shadow != nullptr ? (double)h->pairs_walked * 8.0 + (double)h->heads_walked * (kHead + 4.0) +
                                                                   (multi ? 24.0 * (double)h->rays_walked : 0.0)
                                                             : (double)hits * (kHead + 4.0 * h->S.num_lights);
        st->errors = err;
        st->shadow_jit = h->jit_shadow != nullptr ? 1 : 0;
        st->shadow_rays_walked = h->jit_shadow != nullptr ? h->rays_walked : st->shadow_rays;
        st->shadow_tile_pairs = h->tile_pairs;
        st->shadow_tile_mixed = h->tile_mixed;
        st->shadow_pairs = h->node_pairs;
        st->shadow_pairs_mixed = h->node_mixed;
        st->shadow_sub_pairs = h->sub_pairs;
        st->shadow_sub_mixed = h->sub_mixed;
        st->shadow_subtile_pairs = h->subtile_pairs;
        st->shadow_subtile_mixed = h->subtile_mixed;
        collect_timings(h, st);
    }
#if defined(FRT_WALK_STATS) || defined(FRT_WALK_PROF)
    dump_walk_stats(h);
#endif
    if (err) {
        char buf[128];
        std::snprintf(buf, sizeof(buf), "render: device error bits 0x%x", err);
        return fail(buf);
    }
    return 0;
}

int frt_render_rows_device(frt_scene_handle* h, const frt_frame_params* P, double* device_rgba, frt_frame_stats* st) {
    if (!h || !P || !device_rgba) return fail("frt_render_rows_device: null argument");
    return render_impl(h, P, device_rgba, st);
}

int frt_render_rows(frt_scene_handle* h, const frt_frame_params* P, double* host_rgba, frt_frame_stats* st) {
    if (!h || !P || !host_rgba) return fail("frt_render_rows: null argument");
    FRT_HIP(hipSetDevice(h->device));
    const int64_t stride = P->row_stride > 0 ? P->row_stride : 1;
    int64_t nrows = 0;
    for (int64_t r = P->row_begin; r < P->row_end; r += stride) nrows++;
    const int64_t n = nrows * h->S.cam.hsize * 4;
    if (grow(&h->out_dev, h->out_cap, std::max<int64_t>(n, 4))) return -1;
    int rc = render_impl(h, P, h->out_dev, st);
    if (rc) return rc;
    FRT_HIP(hipMemcpy(host_rgba, h->out_dev, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

// photon map test entry points (include/frt_device.h)
int frt_pm_balance(const double* pos, int64_t n, int32_t* heap_of, int8_t* plane) {
    if (n < 0 || n > ((int64_t)1 << 30) || (n > 0 && (!pos || !heap_of || !plane))) return fail("frt_pm_balance: bad arguments");
    std::vector<int32_t> ho;
    std::vector<int8_t> pl;
    pm_balance_heap(pos, n, ho, pl);
    std::memcpy(heap_of, ho.data(), (size_t)n * sizeof(int32_t));
    std::memcpy(plane, pl.data(), (size_t)(n + 1) * sizeof(int8_t));
    return 0;
}

int frt_pm_estimate(int device, const double* pos, const double* power, const uint8_t* theta_phi, int64_t n,
                    const double* queries, int64_t nq, double radius, int32_t k, double cone_k, double* irrad,
                    int64_t* found) {
    if (n < 0 || nq < 0 || k < 1 || !(radius > 0.0) || (nq > 0 && (!queries || !irrad || !found)) ||
        (n > 0 && (!pos || !power || !theta_phi)))
        return fail("frt_pm_estimate: bad arguments");
    if (nq == 0) return 0;
    FRT_HIP(hipSetDevice(device));
    void* mem = nullptr;
    frt::PhotonMapDev M{};
    double *dq = nullptr, *dirr = nullptr;
    int64_t* dfound = nullptr;
    int rc = make_photon_map(n, pos, power, theta_phi, radius, &mem, M);
    auto run = [&]() -> int {
        FRT_HIP(hipMalloc(&dq, (size_t)nq * 6 * sizeof(double)));
        FRT_HIP(hipMalloc(&dirr, (size_t)nq * 3 * sizeof(double)));
        FRT_HIP(hipMalloc(&dfound, (size_t)nq * sizeof(int64_t)));
        FRT_HIP(hipMemcpy(dq, queries, (size_t)nq * 6 * sizeof(double), hipMemcpyHostToDevice));
        const int64_t waves_per_block = frt::kBlock / 64;
        const int64_t blocks = (nq + waves_per_block - 1) / waves_per_block;
        hipLaunchKernelGGL(frt::k_pm_estimate, dim3((unsigned)blocks), dim3(frt::kBlock), 0, 0, M, dq, nq, radius, (int)k,
                           cone_k, dirr, dfound);
        FRT_HIP(hipGetLastError());
        FRT_HIP(hipMemcpy(irrad, dirr, (size_t)nq * 3 * sizeof(double), hipMemcpyDeviceToHost));
        FRT_HIP(hipMemcpy(found, dfound, (size_t)nq * sizeof(int64_t), hipMemcpyDeviceToHost));
        return 0;
    };
    if (rc == 0) rc = run();
    hip_ignore(hipFree(dq));
    hip_ignore(hipFree(dirr));
    hip_ignore(hipFree(dfound));
    hip_ignore(hipFree(mem));
    return rc;
}

}  // extern "C"
