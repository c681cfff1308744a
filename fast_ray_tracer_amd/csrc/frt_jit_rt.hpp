// frt-mi355x device helpers of the scene-specialised shadow kernels that
// frt_jit.cpp generates at upload (one straight-line walk per scene tree,
// compiled with hiprtc). Every helper makes exactly the decision the generic
// walk (frt_traverse.hpp, walk<true, F>) makes for the same node, so the
// generated kernel's unshadowed counts equal the generic kernel's.
#pragma once

#include "frt_shadow.hpp"

namespace frt {
namespace jit {

// composite box decision of the walk: binary32 with an error bound, binary64
// where it cannot decide; skip_behind: the subtree lies wholly behind the ray
// (only at the top level of the last world shape, see walk())
__device__ __forceinline__ bool box_enter(const WalkNode& nd, const Ray& lr, bool skip_behind) {
    Frame32 lf;
    frame32(lr, lf);
    float tmin32 = -1.0f, tmax32 = 1.0f, err32 = 0.0f;
    const int dec = lf.exact ? -1 : box32(nd.bb32, nd.bmag, lf, tmin32, tmax32, err32);
    double tmin = -1.0, tmax = 1.0;
    bool enter;
    if (dec >= 0) {
        enter = dec != 0;
        tmax = (double)tmax32 + (double)err32;
    } else if (origin_inside(nd.bbox, lr)) {
        enter = true;
    } else {
        double lrc[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) lrc[a] = recip<1>(lr.d[a]);
        enter = box_decide(nd.bbox, lr, lrc, tmin, tmax);
    }
    if (skip_behind && behind(tmax)) enter = false;
    return enter;
}

// a leaf outside CSG units (group.c:114-121 stop rule, intersection.c:42-55):
// its entries end the lane's walk when one of them is not <= 0; the lane is
// shadowed iff that leaf casts shadows and holds a t in (0, distance)
template <int kType, bool kXf>
__device__ __forceinline__ void leaf_top(const DevScene& S, const WalkNode& nd, const Ray& R, double dist, bool act,
                                         bool& alive, int& result, bool& any_entry) {
    const Ray lr = kXf ? xf_ray_walk(nd.m, R) : R;
    LeafHits H;
    if (kType == FRT_CUBE) cube_hits_for_decisions(lr, dist, H);
    else leaf_hits<true>(kType, S.prim + nd.prim, lr, H);
    if (act && H.t.n > 0) {
        any_entry = true;
        bool stop_here = false, blocked = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double t = H.t.at(j);
            if (j < H.t.n) {
                stop_here = stop_here || !(t <= 0);
                blocked = blocked || (t > 0 && t < dist);
            }
        }
        if (stop_here) {
            result = blocked && nd.casts ? 1 : 0;
            alive = false;
        }
    }
}

// a leaf inside a CSG unit: its (sorted) entries become the unit's slots
template <int kType, bool kXf>
__device__ __forceinline__ void leaf_slots(const DevScene& S, const WalkNode& nd, const Ray& R, bool act, double& t0,
                                           double& t1, bool& v0, bool& v1) {
    const Ray lr = kXf ? xf_ray_walk(nd.m, R) : R;
    LeafHits H;
    leaf_hits<true>(kType, S.prim + nd.prim, lr, H);
    t0 = H.t.v0;
    t1 = H.t.v1;
    v0 = act && H.t.n > 0;
    v1 = act && H.t.n > 1;
}

// intersection_allowed (csg.c:27-40); op: 0 union, 1 intersect, 2 difference
template <int kOp>
__device__ __forceinline__ bool allowed(bool lhit, bool inl, bool inr) {
    if (kOp == 0) return lhit ? !inr : !inl;
    if (kOp == 1) return lhit ? inr : inl;
    return lhit ? !inr : inl;
}

__device__ __forceinline__ bool finite_ray(const Ray& r, double dist) {
    bool f = __builtin_isfinite(dist);
#pragma unroll
    for (int a = 0; a < 3; ++a) f = f && __builtin_isfinite(r.o[a]) && __builtin_isfinite(r.d[a]);
    return f;
}

// ---- binary32 interval walk ----
// The walk above takes the reference's binary64 arithmetic step for step. Its
// decisions (box hit, entries, t <= 0, t < distance, the order of two entries)
// can mostly be proven from binary32 values with an error bound: every t is
// carried as an interval [lo, hi] that contains the reference's binary64 value,
// and a decision is taken only when the intervals settle it. A lane meeting an
// undecidable comparison (or a direction component near the reference's
// EPSILON slab branch) is marked `amb` and re-walked with the binary64 code.
//
// Error model (u = 2^-24, round to nearest; v_rcp_f32 / v_rsq_f32 within 1 ulp = 2u):
//  * world ray (ray32): v = light point - over_point in binary64 (the reference's own subtraction),
//    f32(v) (u), n2 = |f32(v)|^2 (<= 5u relative to |v|^2), rs = rsq(n2) (<= 2u + 2.5u),
//    d~ = f32(v) rs: every component within 6.6u (relative) of the reference's v_a / |v|; the
//    distance n2 rs within 5.6u of sqrt(v.v): DIST = dist~ (1 -+ 8u) (the product's rounding
//    included); o~ = f32(over_point) (u).
//  * frame: node k's ray = C_k (world ray), C_k = M_k ... M_1 composed in binary64 at upload,
//    evaluated as a 3-term fma chain on binary32 operands. Against the reference's sequential
//    binary64 transforms: |o - o_ref|_inf <= eo = 6u (cN |o_w|_inf + cT) — 3u for the chain, u for
//    each of the world-ray and matrix roundings, the reference's own rounding (~1e-16) and the
//    bound's rounding in the rest; |d - d_ref|_inf <= ed = 12u cN (|d_w|_inf <= 1: the world
//    direction's 6.6u in place of u).
//  * slab value t = (b - o_a) / d_a: |t~ - t_ref| <= 4.2u |t~| + (eo + u |b|) / |d_ref| + |t~| ed / |d_ref|
//    with 1 / |d_ref| <= 1 / (|d~_a| - ed); taken as 7u |t~| + ... and x1.01 on the
//    rest, covering the roundings of the bound arithmetic and of the interval ends.
//  * axis-aligned frame (C_k's 3x3 part diagonal, WalkNode::aa): the reference's local slab value
//    (b - o'_a) / d'_a with o'_a = c_aa o_a + c_a3, d'_a = c_aa d_a equals t* = (B - o_a) / d_a,
//    B = (b - c_a3) / c_aa, exactly in real arithmetic (its binary64 roundings are ~2^-50
//    relative). On the world ray: r~ = rcp(d~) = (1 + eta) / d_a with |eta| <= 8.7u, o r~ rounded
//    (u), B rounded to binary32 (u), t~ = fma(B~, r~, -o~ r~) rounded once (u):
//    |t~ - t*| <= 1.01u |t~| + (9.7u |B| + 10.7u |o|) / |d_a|, |1 / d_a| <= |r~| (1 + 8.8u); taken
//    as 2.5u |t~| + 12u (max|B| + max|o|) |r~|, the slack covering the roundings of the bound and
//    of the interval ends and the reference's binary64 roundings. A signed permutation of the axes
//    (90-degree rotations) is the same test on world axis col(a); its other entries (sigma <= 2^-29
//    of the row's largest: remnants of cos(pi/2)) move t by <= 1.0001 sigma (|o| + |t|) |1 / d_a|:
//    the |o| part lies inside K0's slack, the |t| part is added to K1 as aasig |r~|, and the
//    EPSILON threshold includes them.
//  * tmin = max of the axes' low values, tmax = min of the high ones: intervals of a max / min
//    are the max / min of the intervals.
constexpr float kU = 0x1p-24f;
constexpr float kXfErr = 6.0f * kU;
constexpr float kXfErrD = 12.0f * kU;
constexpr float kSlabRel = 7.0f * kU;
constexpr float kSlack = 1.01f;
constexpr float kAaK1 = 2.5f * kU;
constexpr float kAaK0 = 12.0f * kU;

struct Iv {
    float lo, hi;
};

// tri-state comparisons on intervals: 1 true, 0 false, -1 undecided
__device__ __forceinline__ int iv_le(const Iv& a, const Iv& b) { return a.hi <= b.lo ? 1 : (a.lo > b.hi ? 0 : -1); }
__device__ __forceinline__ int iv_le0(const Iv& a) { return a.hi <= 0.0f ? 1 : (a.lo > 0.0f ? 0 : -1); }
__device__ __forceinline__ int iv_lt(const Iv& a, const Iv& b) { return a.hi < b.lo ? 1 : (a.lo >= b.hi ? 0 : -1); }

__device__ __forceinline__ Iv iv_of(double x) { return Iv{__double2float_rd(x), __double2float_ru(x)}; }

struct World32 {
    float o[3], d[3], omax;
    // shared by every axis-aligned slab test of the lane: rcp(d~), f32(o~ r~), 12u |r~|, 12u |r~| omax
    float r[3], ro[3], P[3], Q[3];
};

// what the interval walk reads of a node, written into the generated kernel as a constexpr literal
// per node (no loads; the fields are WalkNode's)
struct Node32 {
    float cm[12];
    float cN, cT;
    float bb32[6], bmag[3];
    float aab[6], aathr[3], aabmax, aasig;
    float sph[4], sphc;  // round spheres: centre, radius (1 + 1e-6) rounded up, max |centre|
    int casts;
};

__device__ __forceinline__ float o_lo(const World32& w, int a) { return w.o[a]; }
__device__ __forceinline__ float o_hi(const World32& w, int a) { return w.o[a]; }

__device__ __forceinline__ void world32_finish(World32& w) {
    w.omax = fmaxf(fmaxf(fabsf(w.o[0]), fabsf(w.o[1])), fabsf(w.o[2]));
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w.r[a] = __builtin_amdgcn_rcpf(w.d[a]);
        w.ro[a] = w.o[a] * w.r[a];
        w.P[a] = kAaK0 * fabsf(w.r[a]);
        w.Q[a] = w.P[a] * w.omax;
    }
}

// ---- the shadow lane in 32-bit arithmetic ----
// One lane per (path node, light sample j), as shadow_lane (frt_shadow.hpp): the host launches at
// most 2^31 lanes per call, so the lane index is 32-bit and node = tid / spn is a multiply-shift
// (magic = ceil(2^shift / spn), shift = 32 + ceil(log2 spn): exact for every 32-bit tid).
struct Lane32 {
    uint32_t node;
    int light;
    bool valid, live;
    const double* lp;  // the light point (binary64)
    const double* op;  // the path node's over_point
};

__device__ __forceinline__ void lane32(const DevScene& S, const Batch& B, const ShadowHead* __restrict__ shead,
                                       uint32_t total, const int32_t* __restrict__ j_light,
                                       const int32_t* __restrict__ j_point, uint32_t spn, uint64_t magic,
                                       uint32_t shift, uint32_t tid, Lane32& L) {
    L.valid = tid < total;
    L.live = false;
    L.node = 0;
    L.light = 0;
    L.lp = L.op = nullptr;
    if (L.valid) {
        L.node = (uint32_t)(((uint64_t)tid * magic) >> shift);
        const uint32_t j = tid - L.node * spn;
        L.light = j_light[j];
        const int pt = j_point[j];
        const ShadowHead* nr = shead + L.node;
        if (nr->material >= 0) {
            L.live = true;
            const frt_light& lt = S.lights[L.light];
            const int row = light_row(lt, B.seed, nr->key, L.light, 0);
            L.lp = S.light_points + lt.points + 3 * ((int64_t)row * lt.num_samples + pt);
            L.op = nr->over_point;
        }
    }
}

// is_shadowed's ray (renderer.c:74-93) in binary32 with the bounds of the error model above; false
// when they cannot be given (non-finite or degenerate): the lane takes the binary64 walk
__device__ __forceinline__ bool ray32v(const double* lp, const double* op, World32& w, Iv& dist) {
    float vf[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        vf[a] = (float)(lp[a] - op[a]);
        w.o[a] = (float)op[a];
    }
    const float n2 = vf[0] * vf[0] + vf[1] * vf[1] + vf[2] * vf[2];
    const float rs = __builtin_amdgcn_rsqf(n2);
#pragma unroll
    for (int a = 0; a < 3; ++a) w.d[a] = vf[a] * rs;
    const float dl = n2 * rs;
    dist = Iv{dl * (1.0f - 8.0f * kU), dl * (1.0f + 8.0f * kU)};
    world32_finish(w);
    return n2 >= 0x1p-60f && n2 <= 0x1p100f && w.omax <= 0x1p100f;  // (false for NaN)
}

__device__ __forceinline__ bool ray32(const Lane32& L, World32& w, Iv& dist) { return ray32v(L.lp, L.op, w, dist); }

// (frt_jit_trace) a closest-hit ray in binary32: o~ = f32(o) as above, d~ = f32(d), within u of the reference's
// binary64 direction, inside the 6.6u the model above allows the world ray, for a direction of unit length
// (camera, reflected and refracted rays); false when that does not hold within 1e-6 or a value is not finite:
// the lane takes the generic walk
__device__ __forceinline__ bool ray32d(const Ray& r, World32& w) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w.o[a] = (float)r.o[a];
        w.d[a] = (float)r.d[a];
    }
    world32_finish(w);
    const double n2 = r.d[0] * r.d[0] + r.d[1] * r.d[1] + r.d[2] * r.d[2];
    return n2 > 1.0 - 1e-6 && n2 < 1.0 + 1e-6 && w.omax <= 0x1p100f;  // (false for NaN)
}

// the reference's binary64 ray, exactly as shadow_lane computes it. Every lane of a wave runs the
// blocks that call this (uniform branches), so lanes without a ray (padding, nodes without a hit)
// get a placeholder instead of reading through their null light point.
__device__ __forceinline__ void ray64(const Lane32& L, Ray& r, double& dist) {
    if (!L.live) {
        r = Ray{{0, 0, 0}, {0, 0, 1}};
        dist = 0.0;
        return;
    }
    double v[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        v[a] = L.lp[a] - L.op[a];
        r.o[a] = L.op[a];
    }
    dist = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    normalize3(v, r.d);
}

// ray64 on a lane's first request (leaves the interval walk evaluates in binary64)
__device__ __forceinline__ void ray64_once(const Lane32& L, bool& have, Ray& r, double& dist) {
    if (!have) {
        ray64(L, r, dist);
        have = true;
    }
}

// ---- the list of mixed (node, light) pairs ----
// The beam kernel appends the pairs it cannot decide to kMixSegs segments (block b to segment
// b % kMixSegs, one counter per 256-byte line: device-scope atomics on one address serialise); the
// per-ray kernel finds its pair from the segment counts with a wave scan and a binary search.
constexpr int kMixSegs = 64;
constexpr int kMixLine = 64;  // 32-bit words per counter line

// (the list's second half, at kMixSegs * segcap, holds each pair's resume value at the same slot)
__device__ __forceinline__ void mix_append(bool mix, uint32_t pair, uint32_t value, uint32_t* __restrict__ mixed,
                                           unsigned* __restrict__ mcount, uint32_t segcap, unsigned* __restrict__ err) {
    const unsigned long long mm = __ballot(mix);
    if (mm == 0) return;
    const int lane = threadIdx.x & 63;
    const int seg = (int)(blockIdx.x % kMixSegs);
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(mcount + seg * kMixLine, (unsigned)__popcll(mm));
    base = __shfl(base, 0, 64);
    if (mix) {
        const unsigned at = base + (unsigned)__popcll(mm & ((1ull << lane) - 1));
        if (at < segcap) {
            mixed[(size_t)seg * segcap + at] = pair;
            mixed[(size_t)kMixSegs * segcap + (size_t)seg * segcap + at] = value;
        } else {
            atomicOr(err, kErrQueueOverflow);
        }
    }
}

// The per-ray kernel's blocks by segment (host-built from the segment counts, passed by value): segment
// s holds count[s] mixed pairs and takes blocks [bstart[s], bstart[s + 1]) of the launch sequence, its
// pairs' lanes (lpp each) packed over them; a block finds its segment with a scalar binary search.
struct SegTable {
    uint32_t bstart[kMixSegs + 1];
    uint32_t count[kMixSegs];
};

// (wave-uniform) the segment of global block gb
__device__ __forceinline__ int seg_of_block(const SegTable& t, uint32_t gb) {
    int s = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1)
        if (t.bstart[s + step] <= gb) s += step;  // (s + step <= 63: the table's last entry is never read)
    return s;
}

// the lit lanes of each (node, light part) pair: a pair's lanes are lpp consecutive lanes (j = 0..lpp-1),
// so its head lane (j == 0, or the wave's first lane) adds the pair's lit lanes of this wave
__device__ __forceinline__ void count_part(const DevScene& S, const Lane32& L, bool lit, uint32_t j, uint32_t lpp,
                                           int32_t* counts) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lits = __ballot(lit);
    if (L.valid && (j == 0 || lane == 0)) {
        const uint32_t len = min(lpp - j, 64u - (uint32_t)lane);
        const unsigned long long seg = (len >= 64u ? ~0ull : ((1ull << len) - 1ull)) << lane;
        const int c = __popcll(lits & seg);
        if (c) atomicAdd(counts + L.node * (uint32_t)S.num_lights + (uint32_t)L.light, c);
    }
}

// The beam stages' decided lit pairs add their sample count to every node of their tile (sub-tile): lanes of one wave
// that share the tile — the sub-part stage's 16 samples of a tile pair, the tile stage's parts of one tile — first sum
// their counts, then the wave adds each (run, light) group's total with one atomic per node, the run's nodes spread
// over the lanes (one per lane for 64-node tiles), instead of one atomic per node and lit lane (up to 64 per lane on
// the same addresses). Integer sums: the counts are the same. (all lanes of the wave; base, len, lt: the run's first
// node, its length (uniform) and light)
__device__ __forceinline__ void add_run_counts(const ShadowHead* __restrict__ shead, int32_t* counts, uint32_t nl,
                                               bool add, uint32_t base, uint32_t len, uint32_t lt, int32_t amount,
                                               uint32_t nnodes) {
    const int lane = threadIdx.x & 63;
    unsigned long long pending = __ballot(add);
    while (pending) {
        const int ld = __builtin_ctzll(pending);
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)base, ld);
        const uint32_t l0 = (uint32_t)__builtin_amdgcn_readlane((int)lt, ld);
        const bool same = add && base == b0 && lt == l0;
        pending &= ~__ballot(same);
        int32_t v = same ? amount : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        for (uint32_t n = (uint32_t)lane; n < len; n += 64u) {
            const uint32_t nd = b0 + n;
            if (nd < nnodes && shead[nd].material >= 0) atomicAdd(counts + nd * nl + l0, v);
        }
    }
}

// the lit lanes of each run of consecutive valid lanes with the same (node, light) (the per-ray kernel's node-major
// lanes: a node's samples of several list entries side by side), one atomic per run by its first lane (all lanes of
// the wave)
__device__ __forceinline__ void count_runs(const DevScene& S, const Lane32& L, bool lit, int32_t* counts) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lits = __ballot(lit), valid = __ballot(L.valid);
    const uint32_t key = L.node * (uint32_t)S.num_lights + (uint32_t)L.light;
    const uint32_t prev = __shfl_up(key, 1, 64);
    const bool prev_valid = lane > 0 && ((valid >> (lane - 1)) & 1ull);
    const bool head = L.valid && (!prev_valid || prev != key);
    const unsigned long long heads = __ballot(head);
    if (head) {
        const unsigned long long after = lane == 63 ? 0ull : (~0ull << (lane + 1));
        const unsigned long long stops = (heads | ~valid) & after;
        const int next = stops ? __ffsll((long long)stops) - 1 : 64;
        const unsigned long long run = (next >= 64 ? ~0ull : ((1ull << next) - 1ull)) & (~0ull << lane);
        const int c = __popcll(lits & run);
        if (c) atomicAdd(counts + key, c);
    }
}

// (all lanes of the wave) mixed index m -> its slot in the segmented list
__device__ __forceinline__ size_t mix_slot(uint32_t m, const unsigned* __restrict__ mcount, uint32_t segcap) {
    const int lane = threadIdx.x & 63;
    const unsigned c = min(mcount[lane * kMixLine], segcap);  // (an overflowed segment keeps its capacity)
    unsigned incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    const unsigned excl = incl - c;
    int lo = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
        const int probe = lo + step;
        const unsigned e = __shfl(excl, probe & 63, 64);
        if (probe < 64 && e <= m) lo = probe;
    }
    return (size_t)lo * segcap + (m - __shfl(excl, lo, 64));
}

// FRT_JIT_STATS diagnostics: per node, the waves and the lanes that take its test (after the 64 x 32
// words of per-launch counters)
__device__ __forceinline__ void node_stat(unsigned long long* js, int k, bool act) {
    const unsigned long long m = __ballot(act);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(js + 2048 + 2 * k, 1ull);
        atomicAdd(js + 2048 + 2 * k + 1, (unsigned long long)__popcll(m));
    }
}

struct F32 {
    float o[3], d[3], eo, ed;
};

__device__ __forceinline__ void frame32i(const Node32& nd, const World32& w, F32& f) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float* c = nd.cm + 4 * r;
        f.o[r] = fmaf(c[0], w.o[0], fmaf(c[1], w.o[1], fmaf(c[2], w.o[2], c[3])));
        f.d[r] = fmaf(c[0], w.d[0], fmaf(c[1], w.d[1], c[2] * w.d[2]));
    }
    f.eo = kXfErr * fmaf(nd.cN, w.omax, nd.cT);
    f.ed = kXfErrD * nd.cN;
}

// the slab entries tmin / tmax of an axis-aligned node (WalkNode::aa) on the world ray; false when
// |d_a| may be below the reference's EPSILON in the node's frame. The two planes of an axis and the
// two ends of the intervals travel as pairs (v_pk_fma_f32 / v_pk_add_f32).
typedef float f2 __attribute__((ext_vector_type(2)));
template <bool kSig>
__device__ __forceinline__ bool aa_slab(const Node32& nd, const World32& w, Iv& tmin, Iv& tmax) {
    bool ok = true;
    f2 lo = {0.0f, 0.0f}, hi = {0.0f, 0.0f};  // (tmin, tmax) lower ends, (tmin, tmax) upper ends
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        ok = ok && fabsf(w.d[a]) >= nd.aathr[a];
        const f2 B = {nd.aab[a], nd.aab[a + 3]};
        const f2 t = __builtin_elementwise_fma(B, f2{w.r[a], w.r[a]}, f2{-w.ro[a], -w.ro[a]});
        const float k1 = kSig ? fmaf(nd.aasig, fabsf(w.r[a]), kAaK1) : kAaK1;
        // (the axis' own max|B| bounds its planes' error: slab computations of nodes that share an axis'
        // planes are the same expressions, which the compiler computes once)
        const float bm = fmaxf(fabsf(nd.aab[a]), fabsf(nd.aab[a + 3])) * (1.0f + 4.0f * kU);
        const float e = fmaf(fmaxf(fabsf(t.x), fabsf(t.y)), k1, fmaf(bm, w.P[a], w.Q[a]));
        const f2 m = {fminf(t.x, t.y), fmaxf(t.x, t.y)};
        const f2 l = m - f2{e, e}, h = m + f2{e, e};
        if (a == 0) {
            lo = l;
            hi = h;
        } else {
            lo = f2{fmaxf(lo.x, l.x), fminf(lo.y, l.y)};
            hi = f2{fmaxf(hi.x, h.x), fminf(hi.y, h.y)};
        }
    }
    tmin = Iv{lo.x, hi.x};
    tmax = Iv{lo.y, hi.y};
    return ok;
}

// ---- beams: every shadow ray of one (path node, light) at once ----
// The rays of a (node, light) pair share the origin o and end at the light's points p_j (one cache
// row). With D = p - o (unnormalised), the reference's t along the normalised direction is
// t = |D| s with s = t* / |D| = (B - o_a) / D_a for a slab plane B; |D| > 0 is common to every value
// of one ray, so the walk's decisions (t <= 0, t < distance = |D| (1 +- 2^-52), t_i <= t_j, tmin <=
// tmax) are decisions on s, with DIST = 1 +- 1e-7. Over the pair, D_a lies in [Dlo_a, Dhi_a] (the
// row's bounding box minus o, widened by the binary32 roundings); when that interval keeps one sign,
// s = N / D_a (N = B - o_a) lies between N / Dlo_a and N / Dhi_a, so the interval walk's code, fed
// with these intervals, takes a decision only when it holds for every ray of the pair. A decision it
// cannot take for all of them marks the pair "mixed": its rays are walked one by one.
//  * N~ = B~ - o~: |N~ - N| <= eN = 1.01u (max|B| + |o~_a|) + u |N~|; q = N~ rcp(D) within 4u |q|;
//    s within 1.02 (4u |q| + eN max|1 / D_a|) (1 + 3u) of N / D_a, plus the permutation remnants'
//    sigma (|o| + |s| |D|max) max|1 / D_a| (their |t| / |d_a| term in s units).
//  * EPSILON: |d'_a| = |c D_a| / |D| >= EPSILON for every ray when min|D_a| >= aathr_a |D|max.
struct Beam32 {
    float o[3], omax;
    float Dlo[3], Dhi[3];  // bounds of the rays' D_a, sign-definite when sgn[a]
    float ilo[3], ihi[3];  // rcp(Dlo), rcp(Dhi)
    float im[3];           // max |1 / D_a| (1 + 3u)
    float Dmin[3];         // min |D_a| (0 unless sign-definite)
    float M[3];            // max |D_a|
    float Dn, Dnmin;       // |D| <= Dn, |D| >= Dnmin
    bool sgn[3];
};

// the beam of origin op (binary64) and a light row's box [pl, ph] (binary32, rounded outward)
__device__ __forceinline__ void beam32(const double* op, const float* pl, const float* ph, Beam32& w) {
    float n2 = 0.0f, m2 = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w.o[a] = (float)op[a];
        const float x0 = pl[a] - w.o[a], x1 = ph[a] - w.o[a];
        const float eD = 2.0f * kU * (fabsf(w.o[a]) + fmaxf(fabsf(x0), fabsf(x1)));
        w.Dlo[a] = x0 - eD;
        w.Dhi[a] = x1 + eD;
        w.sgn[a] = w.Dlo[a] > 0.0f || w.Dhi[a] < 0.0f;
        w.ilo[a] = __builtin_amdgcn_rcpf(w.Dlo[a]);
        w.ihi[a] = __builtin_amdgcn_rcpf(w.Dhi[a]);
        w.im[a] = fmaxf(fabsf(w.ilo[a]), fabsf(w.ihi[a])) * (1.0f + 3.0f * kU);
        const float M = fmaxf(fabsf(w.Dlo[a]), fabsf(w.Dhi[a]));
        w.Dmin[a] = w.sgn[a] ? fminf(fabsf(w.Dlo[a]), fabsf(w.Dhi[a])) : 0.0f;
        w.M[a] = M;
        n2 = fmaf(M, M, n2);
        m2 = fmaf(w.Dmin[a], w.Dmin[a], m2);
    }
    w.omax = fmaxf(fmaxf(fabsf(w.o[0]), fabsf(w.o[1])), fabsf(w.o[2]));
    w.Dn = sqrtf(n2) * (1.0f + 8.0f * kU);
    w.Dnmin = sqrtf(m2) * (1.0f - 8.0f * kU);
}

// ---- tiles: the beams of a run of T consecutive path nodes at once ----
// The rays of a (tile, light part) beam start anywhere in the box [olo, ohi] of the tile's over_points
// (binary64, rounded outward to binary32) and end anywhere in the part's box. D = p - o then lies in
// [pl - ohi, ph - olo] and a slab numerator N = B - o_a in [B - ohi_a, B - olo_a]; the beam functions
// below take both ends where Beam32 has one origin (kBox), so every decision they take holds for every
// ray from every origin of the tile. s = t / |D| keeps its meaning ray by ray, DIST = 1 as before.
struct BeamBox32 {
    float olo[3], ohi[3], omax;
    float pl[3], ph[3];     // the light part's box
    float iDc[3][4];        // rcp of p - o at the corners (pl - olo, ph - olo, pl - ohi, ph - ohi), per axis
    float Dlo[3], Dhi[3];
    float ilo[3], ihi[3];
    float im[3];
    float Dmin[3];
    float M[3];
    float Dn, Dnmin;
    bool sgn[3];
};

// the ends of the origin along axis a (one point for Beam32)
__device__ __forceinline__ float o_lo(const Beam32& w, int a) { return w.o[a]; }
__device__ __forceinline__ float o_hi(const Beam32& w, int a) { return w.o[a]; }
__device__ __forceinline__ float o_lo(const BeamBox32& w, int a) { return w.olo[a]; }
__device__ __forceinline__ float o_hi(const BeamBox32& w, int a) { return w.ohi[a]; }
template <typename BW>
struct BeamKind {
    static constexpr bool kBox = false;
};
template <>
struct BeamKind<BeamBox32> {
    static constexpr bool kBox = true;
};

// the beam of a tile's origin box tb = {olo[3], ohi[3]} (binary32, rounded outward; olo > ohi: no live
// node) and a light row's part box [pl, ph]; false: no ray
__device__ __forceinline__ bool beam_box32(const float* tb, const float* pl, const float* ph, BeamBox32& w) {
    float n2 = 0.0f, m2 = 0.0f;
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w.olo[a] = tb[a];
        w.ohi[a] = tb[a + 3];
        ok = ok && w.olo[a] <= w.ohi[a];
        const float x0 = pl[a] - w.ohi[a], x1 = ph[a] - w.olo[a];
        const float om = fmaxf(fabsf(w.olo[a]), fabsf(w.ohi[a]));
        const float eD = 2.0f * kU * (om + fmaxf(fabsf(x0), fabsf(x1)));
        w.Dlo[a] = x0 - eD;
        w.Dhi[a] = x1 + eD;
        w.sgn[a] = w.Dlo[a] > 0.0f || w.Dhi[a] < 0.0f;
        w.ilo[a] = __builtin_amdgcn_rcpf(w.Dlo[a]);
        w.ihi[a] = __builtin_amdgcn_rcpf(w.Dhi[a]);
        w.im[a] = fmaxf(fabsf(w.ilo[a]), fabsf(w.ihi[a])) * (1.0f + 3.0f * kU);
        const float M = fmaxf(fabsf(w.Dlo[a]), fabsf(w.Dhi[a]));
        w.Dmin[a] = w.sgn[a] ? fminf(fabsf(w.Dlo[a]), fabsf(w.Dhi[a])) : 0.0f;
        w.M[a] = M;
        n2 = fmaf(M, M, n2);
        m2 = fmaf(w.Dmin[a], w.Dmin[a], m2);
        w.pl[a] = pl[a];
        w.ph[a] = ph[a];
        w.iDc[a][0] = __builtin_amdgcn_rcpf(pl[a] - w.olo[a]);
        w.iDc[a][1] = __builtin_amdgcn_rcpf(ph[a] - w.olo[a]);
        w.iDc[a][2] = __builtin_amdgcn_rcpf(pl[a] - w.ohi[a]);
        w.iDc[a][3] = __builtin_amdgcn_rcpf(ph[a] - w.ohi[a]);
    }
    w.omax = fmaxf(fmaxf(fmaxf(fabsf(w.olo[0]), fabsf(w.ohi[0])), fmaxf(fabsf(w.olo[1]), fabsf(w.ohi[1]))),
                   fmaxf(fabsf(w.olo[2]), fabsf(w.ohi[2])));
    w.Dn = sqrtf(n2) * (1.0f + 8.0f * kU);
    w.Dnmin = sqrtf(m2) * (1.0f - 8.0f * kU);
    return ok;
}

// the s intervals of a slab plane pair (B0, B1) on axis a: false when D_a may change sign or the
// reference's EPSILON branch may apply to some ray
// thr: the node's aathr_a (0: no EPSILON branch), bmax >= |B0|, |B1|, sig: the node's aasig
//  * an origin strictly inside the slab (N0 < 0 < N1 with the error margin): every ray has mn <= 0 <= mx
//    on this axis (for |d'_a| below EPSILON the reference's values are -inf / +inf), whatever the sign of
//    D_a: used when D_a may change sign or come near EPSILON. Rays with D_a > 0 have mn = N0 / D_a <=
//    N0 / M+ and mx = N1 / D_a >= N1 / M+ (M+ = max D_a), rays with D_a < 0 have mn <= -N1 / M- and
//    mx >= -N0 / M- (M- = max -D_a). Remnants: numerators shrink by sigma |o|, denominators grow by
//    sigma |D|.
//  * an origin strictly outside the slab (beam_axis_split): a ray moving away from it has a wholly negative
//    s range on this axis (or, below EPSILON, no range: numerators of one sign times infinity), a ray moving
//    towards it enters the slab at s >= snear = (distance to the near plane - rs) / (max |D_a| towards it);
//    aa_slab turns that into a certain miss when another axis certainly enters at s >= 0 (the away rays:
//    tmin >= 0 > tmax) and snear lies beyond every exit bound of the decided axes (the towards rays).
template <bool kSig, typename BW>
__device__ __forceinline__ bool beam_axis_split(float thr, float bmax, float sig, const BW& w, int a, float B0,
                                                float B1, float& snear) {
    // numerators over the origins: N0 in [N0lo, N0hi] = [Bl - ohi, Bl - olo], N1 likewise (one value each for
    // a point origin)
    const float Bl = fminf(B0, B1), Bh = fmaxf(B0, B1);
    const float N0lo = Bl - o_hi(w, a), N1hi = Bh - o_lo(w, a);
    const float N0hi = BeamKind<BW>::kBox ? Bl - o_lo(w, a) : N0lo, N1lo = BeamKind<BW>::kBox ? Bh - o_hi(w, a) : N1hi;
    const float om = BeamKind<BW>::kBox ? fmaxf(fabsf(o_lo(w, a)), fabsf(o_hi(w, a))) : fabsf(o_lo(w, a));
    const float nm = BeamKind<BW>::kBox ? fmaxf(fmaxf(fabsf(N0lo), fabsf(N0hi)), fmaxf(fabsf(N1lo), fabsf(N1hi)))
                                        : fmaxf(fabsf(N0lo), fabsf(N1hi));
    const float eN = fmaf(1.01f * kU, bmax + om, kU * nm);
    const float rs = eN + (kSig ? 1.01f * sig * w.omax : 0.0f);
    const float ds = kSig ? 1.01f * sig * w.Dn : 0.0f;
    const float f = 1.0f - 8.0f * kU;
    // lower bounds by reciprocal (within 3u of the quotient, inside f), the denominators raised to 2^-100
    // at least (a larger denominator keeps a lower bound, and no ray moving towards it, 0, becomes a finite
    // bound in place of +inf)
    if (N0lo - rs > 0.0f) {  // below the slab (every origin): D_a > 0 moves towards it
        snear = (N0lo - rs) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(w.Dhi[a], 0.0f) + ds, 0x1p-100f)) * f;
        return snear > 0.0f;
    }
    if (-N1hi - rs > 0.0f) {  // above
        snear = (-N1hi - rs) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(-w.Dlo[a], 0.0f) + ds, 0x1p-100f)) * f;
        return snear > 0.0f;
    }
    return false;
}

template <bool kSig, typename BW>
__device__ __forceinline__ bool beam_axis(float thr, float bmax, float sig, const BW& w, int a, float B0, float B1,
                                          Iv& mn, Iv& mx) {
    const bool ok = w.sgn[a] && w.Dmin[a] >= thr * w.Dn;
    const float Bl = fminf(B0, B1), Bh = fmaxf(B0, B1);
    const float N0lo = Bl - o_hi(w, a), N1hi = Bh - o_lo(w, a);
    const float N0hi = BeamKind<BW>::kBox ? Bl - o_lo(w, a) : N0lo, N1lo = BeamKind<BW>::kBox ? Bh - o_hi(w, a) : N1hi;
    const float om = BeamKind<BW>::kBox ? fmaxf(fabsf(o_lo(w, a)), fabsf(o_hi(w, a))) : fabsf(o_lo(w, a));
    const float nm = BeamKind<BW>::kBox ? fmaxf(fmaxf(fabsf(N0lo), fabsf(N0hi)), fmaxf(fabsf(N1lo), fabsf(N1hi)))
                                        : fmaxf(fabsf(N0lo), fabsf(N1hi));
    const float eN = fmaf(1.01f * kU, bmax + om, kU * nm);
    if (!ok) {
        // (every origin strictly inside the slab: the smallest distances to its two planes)
        const float rs = eN + (kSig ? 1.01f * sig * w.omax : 0.0f);
        const float r0 = -N0hi - rs, r1 = N1lo - rs;
        const float ds = kSig ? 1.01f * sig * w.Dn : 0.0f;
        // lower bounds by reciprocal, as in beam_axis_split (no ray of a sign: a finite bound in place of +inf)
        const float iMp = __builtin_amdgcn_rcpf(fmaxf(fmaxf(w.Dhi[a], 0.0f) + ds, 0x1p-100f));
        const float iMn = __builtin_amdgcn_rcpf(fmaxf(fmaxf(-w.Dlo[a], 0.0f) + ds, 0x1p-100f));
        const float f = 1.0f - 8.0f * kU;
        const float vmx = fminf(r1 * iMp, r0 * iMn) * f, vmn = fminf(r0 * iMp, r1 * iMn) * f;
        mn = Iv{-__builtin_huge_valf(), -vmn};
        mx = Iv{vmx, __builtin_huge_valf()};
        return r0 > 0.0f && r1 > 0.0f && vmx > 0.0f && vmn > 0.0f;  // (false for NaN)
    }
    float lo0, hi0, lo1, hi1, qm;
    if constexpr (BeamKind<BW>::kBox) {
        // s = (B - o) / (p - o) over o in [olo, ohi], p in [pl, ph]. Where N = B - o keeps its sign over the
        // origins and the plane lies outside the part's extent (B - p keeps its sign), s is monotone in o and in
        // p (ds/do = (B - p) / D^2, ds/dp = -N / D^2): its range is that of the four corners (o, p), each with
        // its own D (the corners' D are the beam's own exact binary32 values, rounded once: inside the same
        // error term). Elsewhere the quotient's range over the independent N and D intervals.
        const float eB = 1.01f * kU * bmax;
        auto range = [&](float B, float Nlo, float Nhi, float& lo, float& hi) {
            const bool mono = (Nlo > eN || Nhi < -eN) && (B + eB < w.pl[a] || B - eB > w.ph[a]);
            const float c0 = Nhi * (mono ? w.iDc[a][0] : w.ilo[a]), c1 = Nhi * (mono ? w.iDc[a][1] : w.ihi[a]);
            const float c2 = Nlo * (mono ? w.iDc[a][2] : w.ilo[a]), c3 = Nlo * (mono ? w.iDc[a][3] : w.ihi[a]);
            lo = fminf(fminf(c0, c1), fminf(c2, c3));
            hi = fmaxf(fmaxf(c0, c1), fmaxf(c2, c3));
        };
        range(Bl, N0lo, N0hi, lo0, hi0);
        range(Bh, N1lo, N1hi, lo1, hi1);
        qm = fmaxf(fmaxf(fabsf(lo0), fabsf(hi0)), fmaxf(fabsf(lo1), fabsf(hi1)));
    } else {
        const float q00 = N0lo * w.ilo[a], q01 = N0lo * w.ihi[a], q10 = N1hi * w.ilo[a], q11 = N1hi * w.ihi[a];
        qm = fmaxf(fmaxf(fabsf(q00), fabsf(q01)), fmaxf(fabsf(q10), fabsf(q11)));
        lo0 = fminf(q00, q01);
        hi0 = fmaxf(q00, q01);
        lo1 = fminf(q10, q11);
        hi1 = fmaxf(q10, q11);
    }
    float err = 1.02f * fmaf(4.0f * kU, qm, eN * w.im[a]);
    if (kSig) err = fmaf(sig * w.im[a], fmaf(qm, w.Dn, w.omax) * 1.01f, err);
    mn = Iv{fminf(lo0, lo1) - err, fminf(hi0, hi1) + err};
    mx = Iv{fmaxf(lo0, lo1) - err, fmaxf(hi0, hi1) + err};
    return ok;
}

// the three slabs [B0_a, B1_a] of a world box on the beam (beam_axis per axis, beam_axis_split's certain
// misses); thr: the EPSILON thresholds, bmax >= |B|, sig: the permutation remnants (kSig)
template <bool kSig, typename BW>
__device__ __forceinline__ bool beam_slabs(const float* thr, float bmax, float sig, const BW& w, const float* B0,
                                           const float* B1, Iv& tmin, Iv& tmax, Iv* amn = nullptr, Iv* amx = nullptr,
                                           bool* aok = nullptr) {
    bool ok = true, split_ok = true, any_ok = false;
    float snear = 0.0f;  // max over the split axes
    Iv smin{-__builtin_huge_valf(), -__builtin_huge_valf()}, smax{__builtin_huge_valf(), __builtin_huge_valf()};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        Iv mn, mx;
        const bool oka = beam_axis<kSig>(thr[a], bmax, sig, w, a, B0[a], B1[a], mn, mx);
        if (amn != nullptr) {  // (the axes' own intervals: cube_iv_meta)
            amn[a] = mn;
            amx[a] = mx;
            aok[a] = oka;
        }
        ok = oka && ok;
        if (oka) {  // the decided axes alone
            smin = Iv{fmaxf(smin.lo, mn.lo), fmaxf(smin.hi, mn.hi)};
            smax = Iv{fminf(smax.lo, mx.lo), fminf(smax.hi, mx.hi)};
            any_ok = true;
        } else {
            float sn = 0.0f;
            split_ok = beam_axis_split<kSig>(thr[a], bmax, sig, w, a, B0[a], B1[a], sn) && split_ok;
            snear = fmaxf(snear, sn);
        }
        if (a == 0) {
            tmin = mn;
            tmax = mx;
        } else {
            tmin = Iv{fmaxf(tmin.lo, mn.lo), fmaxf(tmin.hi, mn.hi)};
            tmax = Iv{fminf(tmax.lo, mx.lo), fminf(tmax.hi, mx.hi)};
        }
    }
    if (!ok && split_ok && any_ok && smin.lo >= 0.0f && snear > smax.hi) {  // a certain miss (beam_axis_split)
        tmin = Iv{1.0f, 1.0f};
        tmax = Iv{0.0f, 0.0f};
        return true;
    }
    return ok;
}

template <bool kSig>
__device__ __forceinline__ bool aa_slab(const Node32& nd, const Beam32& w, Iv& tmin, Iv& tmax) {
    return beam_slabs<kSig>(nd.aathr, nd.aabmax, nd.aasig, w, nd.aab, nd.aab + 3, tmin, tmax);
}
template <bool kSig>
__device__ __forceinline__ bool aa_slab(const Node32& nd, const BeamBox32& w, Iv& tmin, Iv& tmax) {
    return beam_slabs<kSig>(nd.aathr, nd.aabmax, nd.aasig, w, nd.aab, nd.aab + 3, tmin, tmax);
}

// frames that are not axis-aligned take no beam decision (their pairs are mixed)
__device__ __forceinline__ void frame32i_none(F32& f) {
#pragma unroll
    for (int a = 0; a < 3; ++a) f.o[a] = f.d[a] = 0.0f;
    f.eo = 0.0f;
    f.ed = __builtin_huge_valf();  // slab_iv: |d| - ed < EPSILON -> undecided
}
__device__ __forceinline__ void frame32i(const Node32&, const Beam32&, F32& f) { frame32i_none(f); }
__device__ __forceinline__ void frame32i(const Node32&, const BeamBox32&, F32& f) { frame32i_none(f); }

// "wholly behind": every ray's t = |D| s <= Dnmin s_hi < -1e-6 (1 + |t|) (walk()'s behind())
__device__ __forceinline__ bool behind_all(const Iv& tmax, const World32&) {
    return tmax.hi < -1e-6f * (1.0f + fabsf(tmax.hi));
}
__device__ __forceinline__ bool behind_all_beam(const Iv& tmax, float Dnmin) {
    const float T = Dnmin * tmax.hi * (1.0f - 4.0f * kU);
    return tmax.hi < 0.0f && T < -1.01e-6f * (1.0f + fabsf(T));
}
__device__ __forceinline__ bool behind_all(const Iv& tmax, const Beam32& w) { return behind_all_beam(tmax, w.Dnmin); }
__device__ __forceinline__ bool behind_all(const Iv& tmax, const BeamBox32& w) { return behind_all_beam(tmax, w.Dnmin); }

// a round sphere whose box every ray of the beam misses: the box, centre~ -+ (R' + 2u (|C~| + R') +
// 1e-6 R') with R' = nd.sph[3] >= R (1 + 1e-6), holds the ball of radius R (1 + 1e-6) around the true
// centre, so each line passes the centre at more than that (sphere_miss32's margin argument)
template <typename BW>
__device__ __forceinline__ bool sphere_miss32_beam(const Node32& nd, const BW& w) {
    // (the line misses the box: a direction component of 0 keeps the line out of a slab its origin is outside)
    const float h = nd.sph[3] + fmaf(2.0f * kU, nd.sphc + nd.sph[3], 1e-6f * nd.sph[3]);
    const float thr[3] = {0.0f, 0.0f, 0.0f};
    float B0[3], B1[3];
    bool near = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        B0[a] = nd.sph[a] - h;
        B1[a] = nd.sph[a] + h;
        near = near && fmaxf(fabsf(o_lo(w, a) - nd.sph[a]), fabsf(o_hi(w, a) - nd.sph[a])) < 1e4f * nd.sph[3];
    }
    Iv tmin, tmax;
    const bool ok = beam_slabs<false>(thr, nd.sphc + h, 0.0f, w, B0, B1, tmin, tmax);
    return ok && near && tmin.lo > tmax.hi && w.omax < 1e8f * nd.sph[3];
}
__device__ __forceinline__ bool sphere_miss32(const Node32& nd, const Beam32& w) { return sphere_miss32_beam(nd, w); }
__device__ __forceinline__ bool sphere_miss32(const Node32& nd, const BeamBox32& w) { return sphere_miss32_beam(nd, w); }

// a round sphere the beam may meet (a top-level leaf of the pair kernel's walk):
//  1  every ray of the beam hits it with its first root in (0, distance): the walk stops there, blocked
//     (leaf_top: entries, stop_here, blocked)
//  2  every root any ray can have lies before the ray's light point: the sphere can only stop the walk
//     blocked or leave it going (the caller goes on and keeps the pair only if the rest ends blocked)
//  0  neither is certain
// v = C~ - O~ stands for a = C - O (true centre and origin) within ea per axis (the centre's binary32
// rounding 2u (|C~| + R'), the origin's u max|o|, the subtraction's u |v|), 1.75 ea in the 2-norm;
// R' = nd.sph[3] >= R >= R' (1 - 1e-5). The reference's binary64 roots err by far less than the
// margins below (~1e-8 relative even at a tangent).
//  * before the light: any root t <= |a| + R <= |v| (1 + 4u) + 1.75 ea + R' < Dnmin (1 - 1e-5) <= |D|.
//  * hit: O outside, |a| >= |v| (1 - 4u) - 1.75 ea > 1.01 R'; every D in the beam's box lies in the
//    cone about v of half-angle asin(Rc / |v|), Rc = R' (1 - 1e-5) (1 - 1e-4) - 1.75 ea (the cone is
//    convex: its 8 corners decide, with a 1e-4 relative slack over their binary32 dot products), so each
//    line passes the true centre closer than R (1 - 1e-4): two roots, the first in (0, |a|], |a| < |D|.
// (o: the origin; h: for a tile, the largest distance of any origin of its box from o, else 0 — a line through
// another origin O' parallel to one through o lies within h of it, and |C - O'| within h of |C - o|)
__device__ __forceinline__ int sphere_beam32_at(const Node32& nd, const float* o, float omax, float h, const float* Dlo,
                                                const float* Dhi, float Dnmin) {
    float v[3], vv = 0.0f, vm = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        v[a] = nd.sph[a] - o[a];
        vv = fmaf(v[a], v[a], vv);
        vm = fmaxf(vm, fabsf(v[a]));
    }
    const float ea = 1.75f * fmaf(2.0f * kU, nd.sphc + nd.sph[3], kU * (omax + vm)) + h;
    const float vn = sqrtf(vv);
    const float Rp = nd.sph[3];
    const float near_hi = fmaf(vn, 1.0f + 4.0f * kU, ea);  // >= |a|
    const float lim = Dnmin * (1.0f - 1e-5f);
    const bool before = near_hi + Rp < lim && vm + h < 1e4f * Rp && omax < 1e8f * Rp;
    if (!before) return 0;
    const float Rc = fmaf(Rp, (1.0f - 1e-5f) * (1.0f - 1e-4f), -ea);
    bool hit = fmaf(vn, 1.0f - 4.0f * kU, -ea) > 1.01f * Rp && near_hi < lim && Rc > 0.0f;
    const float k2 = (vv - Rc * Rc) * (1.0f + 1e-4f);  // |v|^2 cos^2 of the half-angle
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float d0 = (j & 1) ? Dhi[0] : Dlo[0];
        const float d1 = (j & 2) ? Dhi[1] : Dlo[1];
        const float d2 = (j & 4) ? Dhi[2] : Dlo[2];
        const float dv = fmaf(d0, v[0], fmaf(d1, v[1], d2 * v[2]));
        const float dd = fmaf(d0, d0, fmaf(d1, d1, d2 * d2));
        hit = hit && dv > 0.0f && dv * dv > dd * k2;
    }
    return hit ? 1 : 2;
}
__device__ __forceinline__ int sphere_beam32(const Node32& nd, const Beam32& w) {
    return sphere_beam32_at(nd, w.o, w.omax, 0.0f, w.Dlo, w.Dhi, w.Dnmin);
}
// a tile's beam: from the centre of its origin box, h = the box's half diagonal (rounded up, with the centre's
// rounding); the D box covers every origin already
__device__ __forceinline__ int sphere_beam32(const Node32& nd, const BeamBox32& w) {
    float o[3], h2 = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        o[a] = 0.5f * (w.olo[a] + w.ohi[a]);
        const float e = fmaxf(w.ohi[a] - o[a], o[a] - w.olo[a]);
        h2 = fmaf(e, e, h2);
    }
    const float h = sqrtf(h2) * (1.0f + 8.0f * kU) + 2.0f * kU * w.omax;
    return sphere_beam32_at(nd, o, w.omax, h, w.Dlo, w.Dhi, w.Dnmin);
}

// the slab entries tmin / tmax as intervals; false when |d_a| may be below EPSILON
__device__ __forceinline__ bool slab_iv(const F32& f, const float* lo, const float* hi, float bmax, Iv& tmin,
                                        Iv& tmax) {
    bool ok = true;
    const float ab = (f.eo + bmax * kU) * kSlack;
    const float eds = f.ed * kSlack;
    float Ll = 0.0f, Lh = 0.0f, Hl = 0.0f, Hh = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float ad = fabsf(f.d[a]) - f.ed;
        ok = ok && ad >= kEps32;
        const float ir = __builtin_amdgcn_rcpf(ad);
        const float r = __builtin_amdgcn_rcpf(f.d[a]);
        const float k1 = fmaf(eds, ir, kSlabRel), k0 = ab * ir;
        const float t0 = (lo[a] - f.o[a]) * r, t1 = (hi[a] - f.o[a]) * r;
        const float e = fmaf(fmaxf(fabsf(t0), fabsf(t1)), k1, k0);
        const float mn = fminf(t0, t1), mx = fmaxf(t0, t1);
        if (a == 0) {  // (the first axis starts the max / min chains)
            Ll = mn - e;
            Lh = mn + e;
            Hl = mx - e;
            Hh = mx + e;
        } else {
            Ll = fmaxf(Ll, mn - e);
            Lh = fmaxf(Lh, mn + e);
            Hl = fminf(Hl, mx - e);
            Hh = fminf(Hh, mx + e);
        }
    }
    tmin = Iv{Ll, Lh};
    tmax = Iv{Hl, Hh};
    return ok;
}

// a composite's box (bounding_box.c:164-175) in its own frame: 1 enter, 0 skip, -1 undecided
__device__ __forceinline__ int box_enter32(const Node32& nd, const F32& f, bool skip_behind) {
    Iv tmin, tmax;
    const float bmax = fmaxf(fmaxf(nd.bmag[0], nd.bmag[1]), nd.bmag[2]);
    if (!slab_iv(f, nd.bb32, nd.bb32 + 3, bmax, tmin, tmax)) return -1;
    const int hit = iv_le(tmin, tmax);
    if (hit <= 0) return hit;
    // wholly behind the ray: an upper bound of tmax is behind (walk()'s behind(), in binary32)
    if (skip_behind && tmax.hi < -1e-6f * (1.0f + fabsf(tmax.hi))) return 0;
    return 1;
}

// A round sphere (WalkNode::sph_ok) that the lane's ray certainly misses: the reference's discriminant
// (sphere.c:14-39) is then negative. With v = centre - o and |d| = 1, the line's distance from the
// centre is |v x d|; in binary32, |v~ - v| <= u (|C| + |o|) + u |v~| and |d~ - d| <= 6.6u per
// component, so each component of v~ x d~ (three roundings) is within ec = 2u (|C| + |o|) + 21u max|v~|
// of v x d. |v~ x d~|^2 > (R' + 1.75 ec)^2 (1 + 16u) with R' >= R (1 + 1e-6) then proves a distance
// above R (1 + 1e-6): the exact discriminant is below -8e-6 |d'|^2 while the reference's binary64
// one errs by < 2^-47 |d'|^2 (|o'|^2 + 1), |o'| = |v| / R < 1e4 (and |o| / R < 1e8 for its transform).
__device__ __forceinline__ bool sphere_miss32(const Node32& nd, const World32& w) {
    float v[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = nd.sph[a] - w.o[a];
    const float vmax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fabsf(v[2]));
    const float cx = v[1] * w.d[2] - v[2] * w.d[1];
    const float cy = v[2] * w.d[0] - v[0] * w.d[2];
    const float cz = v[0] * w.d[1] - v[1] * w.d[0];
    const float c2 = cx * cx + cy * cy + cz * cz;
    const float ec = fmaf(21.0f * kU, vmax, 2.0f * kU * (nd.sphc + w.omax));
    const float t = fmaf(1.75f, ec, nd.sph[3]);
    return c2 > t * t * (1.0f + 16.0f * kU) && vmax < 1e4f * nd.sph[3] && w.omax < 1e8f * nd.sph[3];
}

// An origin strictly inside an axis-aligned composite's box enters it for every direction: on each axis
// the reference's slab values are (lo - o'_a) / d'_a < 0 < (hi - o'_a) / d'_a (or -inf / +inf in its
// EPSILON branch), so tmin < 0 < tmax: a hit, and not behind the ray. The world planes B (binary32, within
// u |B|), o~ (within u |o|), the subtraction's rounding, the reference's own binary64 roundings and the
// permutation's remnants (within 2 sigma max|o| in world units) stay inside the margin
// 8u (max|B| + max|o|) + 2.02 sigma max|o|. World32 and Beam32 (one origin per pair) alike.
template <int kAa, typename W>
__device__ __forceinline__ bool inside_aa(const Node32& nd, const W& w) {
    const float m = fmaf(8.0f * kU, nd.aabmax + w.omax, kAa == 2 ? 2.02f * nd.aasig * w.omax : 0.0f);
    bool in = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float lo = fminf(nd.aab[a], nd.aab[a + 3]), hi = fmaxf(nd.aab[a], nd.aab[a + 3]);
        in = in && o_lo(w, a) - lo > m && hi - o_hi(w, a) > m;
    }
    return in;
}

// kAa (per node, fixed by the generator): 0 the node's own frame (frame32i + slab_iv), 1 an
// axis-aligned frame (aa_slab on the world ray), 2 the same with the permutation's remnants (aasig)

// the composite box decision (box_enter32) for an axis-aligned composite, on the world ray
template <int kAa, typename W>
__device__ __forceinline__ int box_enter_aa(const Node32& nd, const W& w, bool skip_behind) {
    Iv tmin, tmax;
    if (!aa_slab<kAa == 2>(nd, w, tmin, tmax)) return -1;
    if (tmin.lo > tmax.hi) return 0;
    if (!(tmin.hi <= tmax.lo)) return -1;
    if (skip_behind && behind_all(tmax, w)) return 0;
    return 1;
}

// unit cube slab intervals (cube.c:56-77); false: |d_a| may be below EPSILON
template <int kAa, typename W>
__device__ __forceinline__ bool cube_slab(const Node32& nd, const W& w, Iv& t0, Iv& t1) {
    if (kAa) return aa_slab<kAa == 2>(nd, w, t0, t1);
    F32 f;
    frame32i(nd, w, f);
    const float lo[3] = {-1.0f, -1.0f, -1.0f}, hi[3] = {1.0f, 1.0f, 1.0f};
    return slab_iv(f, lo, hi, 1.0f, t0, t1);
}

// unit cube entries: ex = 1 two entries, 0 none, -1 undecided
template <int kAa, typename W>
__device__ __forceinline__ int cube_iv(const Node32& nd, const W& w, Iv& t0, Iv& t1) {
    if (!cube_slab<kAa>(nd, w, t0, t1)) return -1;
    return iv_le(t0, t1);
}

// ---- the order of two slab values on one axis (beams) ----
// Two cubes' entries (or exits) that come, for every ray of a beam, from slab planes on the same axis a are
// (B_i - o_a) / d_a and (B_j - o_a) / d_a for the same ray (axis-aligned frames: the local slab value is
// exactly that in real arithmetic, the reference's binary64 roundings ~2^-50 relative): their order is the
// sign of (B_j - B_i) d_a for every ray at once, however widely the beam spreads each value. The interval
// walk alone loses that correlation: on the headline frame the window wall's two slabs and its hole order
// their x-faces 0.001-0.0025 apart, less than the spread of one part's beam.
struct SlabMeta {
    int ax;    // the axis giving this entry / exit for every ray of the beam, -1 none known
    float B;   // its plane (world, binary32)
    bool pos;  // the beam's direction along it (sign-definite: a binding axis is)
};

// cube_iv on a beam, with the binding axes of the entry (m0) and the exit (m1): axis a binds the entry when
// its interval lies above every other axis's (the reference's max over axes is then a's value, or an equal
// one), the exit when below every other's
template <int kAa, typename BW>
__device__ __forceinline__ int cube_iv_meta(const Node32& nd, const BW& w, Iv& t0, Iv& t1, SlabMeta& m0, SlabMeta& m1) {
    m0.ax = m1.ax = -1;
    m0.B = m1.B = 0.0f;
    m0.pos = m1.pos = false;
    if (kAa == 0) {  // (own frames take no beam decision)
        t0 = t1 = Iv{0.0f, 0.0f};
        return -1;
    }
    Iv mn[3], mx[3];
    bool ok[3];
    // (the decision itself: beam_slabs, as aa_slab / cube_iv)
    if (!beam_slabs<kAa == 2>(nd.aathr, nd.aabmax, nd.aasig, w, nd.aab, nd.aab + 3, t0, t1, mn, mx, ok)) return -1;
    const int x = iv_le(t0, t1);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int b = a == 0 ? 1 : 0, c = a == 2 ? 1 : 2;
        const bool pos = w.Dlo[a] > 0.0f;
        const float Bl = fminf(nd.aab[a], nd.aab[a + 3]), Bh = fmaxf(nd.aab[a], nd.aab[a + 3]);
        if (ok[a] && mn[a].lo >= mn[b].hi && mn[a].lo >= mn[c].hi) {
            m0.ax = a;
            m0.B = pos ? Bl : Bh;
            m0.pos = pos;
        }
        if (ok[a] && mx[a].hi <= mx[b].lo && mx[a].hi <= mx[c].lo) {
            m1.ax = a;
            m1.B = pos ? Bh : Bl;
            m1.pos = pos;
        }
    }
    return x;
}

// the order of slab values a, b known by their planes: 1 certainly t_a <= t_b, 0 certainly t_a > t_b, -1
// unknown. The planes are binary32 roundings (u |B| each) of the reference's; the reference's own values err by
// ~2^-50 relative (slack: 2^-30 (|B| + max|o|)); a permutation's remnants move a slab value by up to
// 1.0001 sigma (|o| + |t|) / |d_a| (sigma = nd.aasig of either cube: both are passed as sig, the larger)
template <typename BW>
__device__ __forceinline__ int slab_order(const SlabMeta& a, const SlabMeta& b, float sig, float tmax, const BW& w) {
    if (a.ax < 0 || a.ax != b.ax) return -1;
    const float d = b.B - a.B;
    const float m = 1.02f * kU * (fabsf(a.B) + fabsf(b.B) + fabsf(d)) + 0x1p-30f * (fabsf(a.B) + fabsf(b.B) + w.omax) +
                    2.02f * sig * (w.omax + tmax * w.Dn);
    if (!(fabsf(d) > m)) return -1;
    return (d > 0.0f) == a.pos ? 1 : 0;  // (a.pos: no indexing of the beam by a lane value, which would spill it)
}

// a cube outside CSG units: leaf_top's decisions on intervals, as lane masks; undecided -> amb.
// With entries tmin <= tmax: the walk stops iff tmax > 0; the lane is blocked iff tmax < distance or
// 0 < tmin < distance (an entry in (0, distance), intersection.c:42-55).
template <int kAa, typename W>
__device__ __forceinline__ void cube_top32(const Node32& nd, const W& w, const Iv& dist, bool act, bool& alive,
                                           int& result, bool& any_entry, bool& amb) {
    Iv ta, tb;
    const bool ok = cube_slab<kAa>(nd, w, ta, tb);
    if (!act) return;
    const bool miss = ta.lo > tb.hi, hit = ta.hi <= tb.lo;
    const bool stop = tb.lo > 0.0f, nostop = tb.hi <= 0.0f;
    const bool max_in = tb.hi < dist.lo, max_out = tb.lo >= dist.hi;
    const bool min_pos = ta.lo > 0.0f, min_nonpos = ta.hi <= 0.0f;
    const bool min_in = ta.hi < dist.lo, min_out = ta.lo >= dist.hi;
    const bool blk_known = max_in || (max_out && (min_nonpos || (min_pos && (min_in || min_out))));
    if (!(ok && (miss || (hit && (nostop || (stop && blk_known)))))) {
        amb = true;
        alive = false;
        return;
    }
    if (miss) return;
    any_entry = true;
    if (stop) {  // an entry that is not <= 0 ends the walk
        result = (max_in || (min_pos && min_in)) && nd.casts ? 1 : 0;
        alive = false;
    }
}

// (pair kernel) an axis-aligned cube wholly before every light point of the beam: each entry t of each
// ray lies on the cube's surface (|t| <= the farthest corner's distance F from the origin; the EPSILON
// branch moves it by < 1e-5 |t|), so any entry > 0 is also < |D|. The world box is the node's slab planes
// (binary32, within u aabmax, remnants sigma (|o| + F)); o~ within u |o| per axis; 1.75 > sqrt(3).
template <int kAa, typename BW>
__device__ __forceinline__ bool cube_before_light(const Node32& nd, const BW& w) {
    if (kAa == 0) return false;
    float f2 = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // (over a tile's origin box: both of its ends)
        float m = fmaxf(fabsf(nd.aab[a] - o_lo(w, a)), fabsf(nd.aab[a + 3] - o_lo(w, a)));
        if (BeamKind<BW>::kBox) m = fmaxf(m, fmaxf(fabsf(nd.aab[a] - o_hi(w, a)), fabsf(nd.aab[a + 3] - o_hi(w, a))));
        f2 = fmaf(m, m, f2);
    }
    const float F = sqrtf(f2) * (1.0f + 8.0f * kU);
    const float e = 1.75f * kU * (2.0f * nd.aabmax + 2.0f * w.omax) + nd.aasig * (w.omax + F) * 1.75f;
    return (F + e) * (1.0f + 1e-4f) < w.Dnmin * (1.0f - 1e-5f);
}

// (pair kernel) cube_top32, but a cube the beam cannot decide that lies wholly before the light and casts
// shadows can only stop the walk blocked or leave it going: the lane goes on marked ms (maybe blocked)
template <int kAa, typename BW>
__device__ __forceinline__ void cube_top32_beam(const Node32& nd, const BW& w, const Iv& dist, bool act,
                                                bool& alive, int& result, bool& any_entry, bool& amb, bool& ms) {
    bool undecided = false;
    cube_top32<kAa>(nd, w, dist, act, alive, result, any_entry, undecided);
    if (!undecided) return;
    if (nd.casts && cube_before_light<kAa>(nd, w)) {
        ms = true;
        alive = true;  // (act: the lane was alive)
    } else {
        amb = true;
    }
}

// sorted entries of a non-cube leaf inside a CSG unit, exactly (binary64 ray of its parent frame)
// (frt_jit_trace) a leaf's first smallest positive entry in emission order, exactly (binary64), as an interval:
// ok false when it has none
template <int kType, bool kXf>
__device__ __forceinline__ void leaf_first_pos(const DevScene& S, const WalkNode& nd, const Ray& R, bool act, Iv& t,
                                               int& j, bool& ok) {
    const Ray lr = kXf ? xf_ray_walk(nd.m, R) : R;
    LeafHits H;
    leaf_hits<true>(kType, S.prim + nd.prim, lr, H);
    ok = false;
    j = 0;
    double best = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double x = H.t.at(k);
        if (k < H.t.n && x > 0 && (!ok || x < best)) {
            best = x;
            j = k;
            ok = true;
        }
    }
    ok = ok && act;
    t = iv_of(best);
}
// (frt_jit_trace) entry j of a leaf, exactly as the generic walk computes it
template <int kType, bool kXf>
__device__ __forceinline__ double leaf_entry(const DevScene& S, const WalkNode& nd, const Ray& R, int j) {
    const Ray lr = kXf ? xf_ray_walk(nd.m, R) : R;
    LeafHits H;
    leaf_hits<true>(kType, S.prim + nd.prim, lr, H);
    return H.t.at(j);
}

template <int kType, bool kXf>
__device__ __forceinline__ void leaf_slots_iv(const DevScene& S, const WalkNode& nd, const Ray& R, bool act, Iv& t0,
                                              Iv& t1, bool& v0, bool& v1) {
    double a, b;
    leaf_slots<kType, kXf>(S, nd, R, act, a, b, v0, v1);
    t0 = iv_of(a);
    t1 = iv_of(b);
}

}  // namespace jit
}  // namespace frt
