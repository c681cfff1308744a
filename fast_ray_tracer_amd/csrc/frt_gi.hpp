// frt-mi355x global illumination on the device: photon emission and the
// photon_hit decisions of the reference's photon tracer (photon_tracer.c),
// the k-nearest-photon irradiance estimate (pm.c:91-250) over a dense uniform
// grid, and the hemisphere sampling shared with the final gather
// (sampler.c:24-114, renderer.c:648-687).
//
// The reference draws from drand48 / rand(); the device uses the
// counter-based stream of frt_engine.hip (rng_uniform), so global
// illumination is statistically, not bitwise, equivalent.
#pragma once

#include "frt_shade.hpp"

namespace frt {

// ---- hemisphere sampling (sampler.c:24-114) ----

// create_coordinate_system (sampler.c:63-86)
__device__ inline void coordinate_system(const double* n, double* nt, double* nb) {
    double tmp[3];
    if (fabs(n[0]) > fabs(n[1])) {
        tmp[0] = n[2];
        tmp[1] = 0;
        tmp[2] = -n[0];
        const double s = sqrt(n[0] * n[0] + n[2] * n[2]);
        for (int k = 0; k < 3; ++k) tmp[k] *= s;
    } else {
        tmp[0] = 0;
        tmp[1] = -n[2];
        tmp[2] = n[1];
        const double s = sqrt(n[1] * n[1] + n[2] * n[2]);
        for (int k = 0; k < 3; ++k) tmp[k] *= s;
    }
    normalize3(tmp, nt);
    for (int k = 0; k < 3; ++k) nt[k] *= -1.0;
    cross3(n, nt, nb);
}

// cosine_weighted_sample_hemisphere (sampler.c:40-61) + sampler_hemisphere's
// change of basis (sampler.c:88-114)
__device__ inline void hemisphere_dir(const double* n, const double* nt, const double* nb, double r1, double r2,
                                      double* out) {
    const double r = sqrt(r2);
    const double theta = 2 * kPi * r1;
    double v[3] = {r * cos(theta), sqrt(fmax(0.0, 1.0 - r2)), r * sin(theta)}, s[3], t[3];
    normalize3(v, s);
    for (int k = 0; k < 3; ++k) t[k] = s[0] * nb[k] + s[1] * n[k] + s[2] * nt[k];
    normalize3(t, out);
}

// ---- wave-cooperative estimate ----
// pm_irradiance_estimate (pm.c:91-156) with the 64 lanes of a wave working on ONE query point
// (wave-uniform x), reproducing the reference's search (pm_locate_photons, pm.c:163-252) exactly:
//  * the photons it can reach: the host drops the heap positions whose parent is not below
//    half_stored = n/2 - 1 (pm.c:172, 372) from the grid (frt_engine.hip upload_photon_map);
//  * "within max_dist": the binary64 squared distance in the reference's order (p - x per axis) below
//    max_dist^2. Binary32 distances decide it when they are farther from the radius than their error
//    bound tol (below), the binary64 positions of the kd-tree the rest;
//  * the selection: with at most k photons in range, all of them and dist2[0] = max_dist^2. Otherwise
//    the first k photons found (the kd traversal, near child first, a node after its subtrees) fill
//    the candidate array and the (k+1)-th replaces the largest of them whatever its own distance
//    (dist2[0] is still max_dist^2 when it is tested), after which a photon enters only below the
//    heap's maximum: the result is the k nearest in range except m, the largest of the first k found.
//    m is one of the k nearest exactly when the traversal finds all k nearest before any other photon
//    in range; the result is then the k nearest without the k-th plus the (k+1)-th, and dist2[0] the
//    (k+1)-th distance, else the k-th (oracle/pm_oracle.py states both forms and checks them against
//    each other and the reference's dumps);
//  * the sums (pm.c:129-145) over the selected photons, the density over pi dist2[0].
// Ties of binary64 distances (the order among equal values inside the reference's heap) are not
// reproduced; the sums run in another order (the cone-filter weights from binary64 distances).
//
// Candidates come from the dense grid of PhotonMapDev (cell edge radius / 3): the grid rows (y, z)
// within reach of the sphere, each clipped in x to the sphere's chord, are concatenated and scanned 64
// photons at a time (coalesced binary32 positions); photons within the radius are compacted into the
// wave's LDS list (ballot + rank) with the histogram of the top byte of their 24-bit keys of
// d^2 / r^2 (binary32). The k-th and (k+1)-th keys are found by radix selects over the keys; the
// photons whose keys lie within the error margin of that pair ("band", usually 2-3) are ranked by
// their binary64 distances: the k-th and (k+1)-th exact distances and the (k+1)-th's heap index. The
// traversal order test needs no traversal: photon a comes before photon b iff a lies in b's subtree,
// or, at their lowest common ancestor, on the side the query's near-first order takes first; with
// b = the (k+1)-th, that side is one bit per ancestor of b (near_mask). The sum pass checks every
// selected photon against it; only when all come first (rare) is the last of them found and every
// other photon in range checked against it. A list longer than the wave's capacity (a dense caustic)
// is not stored: the passes then re-scan the rows.
constexpr int kEstCap = 1024;

constexpr unsigned kEstSel = 256;

struct EstLds {
    uint2* ent;       // cap: (24-bit key of d^2 / r^2, photon index) of the photons within the radius
    unsigned* hist;   // 256
    unsigned* sel;    // kEstSel: the photons the sum pass certainly takes (their records load together)
    unsigned cap;
};

__device__ __forceinline__ int est_lane() { return (int)(threadIdx.x & 63); }

// FRT_WALK_PROF builds: phase cycles and counters of the estimate (frt_engine.hip dump_walk_stats)
#ifdef FRT_WALK_PROF
#define EST_STAMP(k)                                                                      \
    do {                                                                                  \
        const unsigned long long t1_ = prof_stamp();                                      \
        if (lane == 0 && prof) atomicAdd(prof + (k), t1_ - est_t0);                      \
        est_t0 = t1_;                                                                     \
    } while (0)
#define EST_COUNT(k, v)                                   \
    do {                                                  \
        if (lane == 0 && prof) atomicAdd(prof + (k), (v)); \
    } while (0)
#define EST_LANES(k, pred)                                                          \
    do {                                                                            \
        const unsigned long long m_ = __ballot(pred);                              \
        if (est_lane() == 0 && prof) atomicAdd(prof + (k), (unsigned long long)__popcll(m_)); \
    } while (0)
#else
#define EST_STAMP(k)
#define EST_COUNT(k, v)
#define EST_LANES(k, pred)
#endif

__device__ __forceinline__ unsigned wave_incl_scan(unsigned v) {
    const int lane = est_lane();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double readlane_dd(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ unsigned est_key(float d2, float inv_r2) {
    const float q = d2 * inv_r2 * 16777216.0f;  // d^2 / r^2 as a 24-bit fixed-point key
    return q >= 16777215.0f ? 16777215u : (unsigned)q;
}

// The candidates of a query at x: every photon whose binary32 distance to x is
// below the radius lies within `re` of x (the radius widened by the binary32
// rounding of the positions), hence in a grid row (y, z) whose cell rectangle
// is within re of (x_y, x_z), at an x-cell within the chord sqrt(re^2 - d_yz^2).
// Rows are taken 64 at a time (lane l owns row l of the round); their photon
// ranges are concatenated and scanned in chunks of 64 consecutive candidates
// (the rows starting inside a chunk are read with scalar readlanes), so short
// rows leave no lanes idle. Calls f(p, in, d2) per
// chunk in uniform control flow; `in`: this lane's candidate exists and lies
// within the radius. The visiting order (rows in (z, y) order, photons in grid
// order) is the same in every pass.
// probe(candidates): called once, before any photon is loaded, with the number of candidates when the rows
// fit one round of 64 (the usual case); returning true abandons the scan (wave_scan_cells returns false).
template <typename F, typename P>
__device__ __forceinline__ bool wave_scan_cells(const PhotonMapDev& M, const double* x, double r, float r2f, F&& f,
                                                P&& probe, unsigned long long* prof = nullptr) {
    const int lane = est_lane();
    const double ax = fmax(fmax(fabs(x[0]), fabs(x[1])), fabs(x[2]));
    const double re = r * (1.0 + 1e-5) + 0x1p-20 * ax;
    int lo[3], hi[3];
    bool any = true;
    for (int k = 0; k < 3; ++k) {
        const double a = floor((x[k] - re - M.origin[k]) * M.inv_cell);
        const double b = floor((x[k] + re - M.origin[k]) * M.inv_cell);
        const double top = (double)(M.dims[k] - 1);
        any = any && b >= 0.0 && a <= top;  // (false for NaN)
        lo[k] = (int)fmin(fmax(a, 0.0), top);
        hi[k] = (int)fmin(fmax(b, 0.0), top);
    }
    if (!any) return true;
    const int ny = hi[1] - lo[1] + 1;
    const int nrows = ny * (hi[2] - lo[2] + 1);
    const float xf[3] = {(float)x[0], (float)x[1], (float)x[2]};
    for (int rb = 0; rb < nrows; rb += 64) {
        const int l = rb + lane;
        int32_t s = 0, cnt = 0;
        if (l < nrows) {
            const int iy = lo[1] + l % ny, iz = lo[2] + l / ny;
            const double ylo = M.origin[1] + (double)iy * M.cell, zlo = M.origin[2] + (double)iz * M.cell;
            const double dy = fmax(0.0, fmax(ylo - x[1], x[1] - (ylo + M.cell)));
            const double dz = fmax(0.0, fmax(zlo - x[2], x[2] - (zlo + M.cell)));
            const double h2 = re * re - dy * dy - dz * dz;
            if (h2 >= 0.0) {
                const double hx = sqrt(h2);
                const double a = floor((x[0] - hx - M.origin[0]) * M.inv_cell);
                const double b = floor((x[0] + hx - M.origin[0]) * M.inv_cell);
                const int x0 = (int)fmax(a, (double)lo[0]), x1 = (int)fmin(b, (double)hi[0]);
                if (x0 <= x1) {
                    const int64_t row = ((int64_t)iz * M.dims[1] + iy) * (int64_t)M.dims[0];
                    s = M.start[row + x0];
                    cnt = M.start[row + x1 + 1] - s;
                }
            }
        }
        const unsigned incl = wave_incl_scan((unsigned)cnt);
        const unsigned excl = incl - (unsigned)cnt;
        const int32_t off = s - (int32_t)excl;  // candidate g of this row is photon off + g
        const unsigned total = (unsigned)__builtin_amdgcn_readlane((int)incl, 63);
        if (nrows <= 64 && probe(total)) return false;
        // the row of each candidate: the non-empty rows are visited in order with scalar
        // reads of their start (no cross-lane permutes); cur_off = the row holding the
        // chunk's first candidate
        unsigned long long rest = __ballot(cnt > 0);
        int32_t cur_off = 0;
        auto chunk_photon = [&](unsigned base) {
            const unsigned g = base + (unsigned)lane;
            int32_t o = cur_off;
            while (rest) {
                const int r = __builtin_ctzll(rest);
                const unsigned st = (unsigned)__builtin_amdgcn_readlane((int)excl, r);
                if (st >= base + 64u) break;
                const int32_t ro = __builtin_amdgcn_readlane(off, r);
                if (g >= st) o = ro;
                cur_off = ro;
                rest &= rest - 1;
            }
            return o + (int32_t)g;
        };
        // kScanChunks chunks per step: their position loads are all in flight before any is used
#ifndef FRT_SCAN_CHUNKS
#define FRT_SCAN_CHUNKS 3  // (2: 1857 ms, 3: 1761 ms k_gather_est per cornell_gi_480x270_8x8 frame, profiles/r04_ab_gi_occupancy.txt)
#endif
        constexpr int kScanChunks = FRT_SCAN_CHUNKS;
        for (unsigned base = 0; base < total; base += 64u * kScanChunks) {
            int32_t pc[kScanChunks];
            bool inc[kScanChunks];
            float4 qc[kScanChunks];
#pragma unroll
            for (int c = 0; c < kScanChunks; ++c) {
                pc[c] = chunk_photon(base + 64u * c);
                inc[c] = base + 64u * c + (unsigned)lane < total;
                qc[c] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (inc[c]) qc[c] = reinterpret_cast<const float4*>(M.pos4)[pc[c]];
                EST_LANES(14, inc[c]);  // (FRT_WALK_PROF: candidate positions read)
            }
#pragma unroll
            for (int c = 0; c < kScanChunks; ++c) {
                if (base + 64u * c >= total) break;  // (uniform)
                float d2 = 0.0f;
                bool in = inc[c];
                if (in) {
                    const float dx = qc[c].x - xf[0], dy = qc[c].y - xf[1], dz = qc[c].z - xf[2];
                    d2 = dx * dx + dy * dy + dz * dz;
                    in = d2 < r2f;
                }
                f(pc[c], in, d2);
            }
        }
    }
    return true;
}

template <typename F>
__device__ __forceinline__ void wave_scan_cells(const PhotonMapDev& M, const double* x, double r, float r2f, F&& f,
                                                unsigned long long* prof = nullptr) {
    wave_scan_cells(M, x, r, r2f, f, [](unsigned) { return false; }, prof);
}

// one photon's 80-byte record (grid order): binary64 position, power, pm_photon_dir of its direction
// bytes, heap index. (A 32-byte record with a power palette and the direction tables was measured
// slower: the estimate is bound by instruction issue, and the palette / table lookups cost more
// instructions than the wider record's loads.)
struct PhotonRec {
    double2 r[5];
    __device__ __forceinline__ double d2(const double* x) const {  // pm.c:188-193, the reference's order
        double d = r[0].x - x[0];
        double v = d * d;
        d = r[0].y - x[1];
        v += d * d;
        d = r[1].x - x[2];
        v += d * d;
        return v;
    }
    __device__ __forceinline__ int32_t heap() const { return (int32_t)__double_as_longlong(r[4].y); }
};

__device__ __forceinline__ PhotonRec photon_rec(const PhotonMapDev& M, int32_t p) {
    const double2* q = reinterpret_cast<const double2*>(M.rec) + 5 * (int64_t)p;
    PhotonRec o;
#pragma unroll
    for (int j = 0; j < 5; ++j) o.r[j] = q[j];
    return o;
}

// the photon's power (pm_scale_photon_power'd)
__device__ __forceinline__ void photon_power(const PhotonMapDev&, const PhotonRec& pr, int32_t, double* pw) {
    pw[0] = pr.r[1].y;
    pw[1] = pr.r[2].x;
    pw[2] = pr.r[2].y;
}

// pm_photon_dir (pm.c:80-88) . normal < 0 in the reference's operation order (pm.c:134): the photon
// arrives from the side the normal faces away from
__device__ __forceinline__ bool photon_facing(const PhotonMapDev&, const PhotonRec& pr, const double* normal) {
    return (pr.r[3].x * normal[0] + pr.r[3].y * normal[1] + pr.r[4].x * normal[2]) < 0.0;
}

// the binary64 squared distance alone (the first 32 bytes of the record)
__device__ __forceinline__ double photon_d2(const PhotonMapDev& M, int32_t p, const double* x) {
    const double2* q = reinterpret_cast<const double2*>(M.rec) + 5 * (int64_t)p;
    const double2 a = q[0], b = q[1];
    double d = a.x - x[0];
    double v = d * d;
    d = a.y - x[1];
    v += d * d;
    d = b.x - x[2];
    v += d * d;
    return v;
}

// The sum passes' record prefetch (FRT_SUM_TOUCH=1 builds, A/B runs; off by default: k_gather_est 1266 -> 1285 ms
// per cornell_gi_480x270_8x8 frame with it, profiles/r06_ab_gi_touch.txt): the sum over a query's nearest photons
// reads one 64-lane chunk of 80-byte records per round trip (a second chunk in flight costs 20 VGPRs and spills),
// and the sum was 55.6 % of the estimate's cycles (profiles/r06_gi_est_phases.txt). While a chunk is summed, each
// lane loads one word from each 64-byte line of its record in the next chunk (two VGPRs), so that chunk's record
// loads would find their lines in the CU's vector L1; the touched words are folded together and read by an empty
// asm statement after the loop (sum_touch_keep). The records are L1 / L2 hits already: the round trips it hides
// cost less than its loads and the wait its loop-carried registers force at the end of every chunk.
#ifndef FRT_SUM_TOUCH
#define FRT_SUM_TOUCH 0
#endif
struct SumTouch {
    uint32_t a = 0, b = 0, keep = 0;
    // (every lane loads: a lane past the list's end touches its last entry, so no branch splits the loop body)
    __device__ __forceinline__ void next(const PhotonMapDev& M, int32_t p) {
        keep ^= a ^ b;  // (the previous chunk's words: loaded a whole chunk ago)
        const uint32_t* q = reinterpret_cast<const uint32_t*>(M.rec + 10 * (int64_t)p);
        a = q[0];
        b = q[19];
    }
};
// (an empty asm statement reads the folded words: the loads stay live, no instruction is emitted)
__device__ __forceinline__ void sum_touch_keep(uint32_t t) { asm volatile("" ::"v"(t)); }

__device__ __forceinline__ int32_t photon_heap(const PhotonMapDev& M, int32_t p) {
    return (int32_t)__double_as_longlong(M.rec[10 * (int64_t)p + 9]);
}

// the traversal of query x visits heap node c's right child first (pm.c:173-183: dist1 = x[plane] -
// p[plane] > 0); the node's 32 bytes in one round trip
__device__ __forceinline__ bool kd_right_first(const double* __restrict__ kd, int32_t c, const double* x) {
    const double2* q = reinterpret_cast<const double2*>(kd + 4 * (int64_t)c);
    const double2 a = q[0], b = q[1];
    const int ax = (int)b.y;
    const double split = ax == 0 ? a.x : (ax == 1 ? a.y : b.x);
    const double xa = ax == 0 ? x[0] : (ax == 1 ? x[1] : x[2]);
    return xa - split > 0.0;
}

// (all lanes) bit j: at the ancestor of heap node q at depth j (root 0), the query's traversal visits
// the right child first
__device__ __forceinline__ unsigned near_mask(const double* __restrict__ kd, int32_t q, const double* x) {
    const int dq = 31 - __clz(q), lane = est_lane();
    bool right = false;
    if (lane < dq) right = kd_right_first(kd, q >> (dq - lane), x);
    return (unsigned)__ballot(right);
}

// heap node a (!= q) is found before node q by the query's traversal; qmask = near_mask(q)
__device__ __forceinline__ bool found_before(int32_t a, int32_t q, unsigned qmask) {
    const int da = 31 - __clz(a), dq = 31 - __clz(q);
    if (da > dq && (a >> (da - dq)) == q) return true;   // in q's subtree: before q
    if (dq > da && (q >> (dq - da)) == a) return false;  // an ancestor of q: after it
    const int m = min(da, dq);
    const int32_t a2 = a >> (da - m), q2 = q >> (dq - m);
    const int up = 32 - __clz(a2 ^ q2);  // levels from depth m up to the common ancestor
    return ((a2 >> (up - 1)) & 1) == (int)((qmask >> (m - up)) & 1u);
}

// the same for any pair, the common ancestor's split read from the kd-tree (the rare full check)
__device__ __forceinline__ bool found_before_any(const double* __restrict__ kd, int32_t a, int32_t b, const double* x) {
    const int da = 31 - __clz(a), db = 31 - __clz(b);
    if (da > db && (a >> (da - db)) == b) return true;
    if (db > da && (b >> (db - da)) == a) return false;
    const int m = min(da, db);
    const int32_t a2 = a >> (da - m), b2 = b >> (db - m);
    const int up = 32 - __clz(a2 ^ b2);
    return ((a2 >> (up - 1)) & 1) == (kd_right_first(kd, a2 >> up, x) ? 1 : 0);
}

__device__ __forceinline__ unsigned wave_and(bool v) { return __ballot(!v) == 0ull ? 1u : 0u; }

// sqrt(x) for x >= 0 within a few ulps (v_rsq_f64 and two Newton steps): the cone filter's weights only
// scale the sums (which run in another order than the reference's anyway); every decision of the
// selection uses exact squared distances
#ifndef FRT_SQRTW_STEPS
#define FRT_SQRTW_STEPS 2
#endif
__device__ __forceinline__ double sqrt_w(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double s = x * y, h = 0.5 * y;
#pragma unroll
    for (int k = 0; k < FRT_SQRTW_STEPS; ++k) {
        const double r = fma(-s, s, x);
        s = fma(r, h, s);
    }
    return x > 0.0 ? s : 0.0;
}



// the digit of rank `need` (1-based) in a 256-bin histogram held 4 bins per lane: its bin, count, and
// the entries in lower bins (wave-uniform results)
__device__ __forceinline__ void radix_pick(const unsigned* c4, unsigned need, unsigned& bin, unsigned& cnt,
                                           unsigned& below) {
    const int lane = est_lane();
    unsigned local = c4[0] + c4[1] + c4[2] + c4[3];
    const unsigned incl = wave_incl_scan(local);
    const int owner = __builtin_ctzll(__ballot(incl >= need));
    unsigned b = incl - local, c = c4[3];
    int bi = 4 * lane + 3;
    for (int j = 0; j < 4; ++j) {
        if (b + c4[j] >= need) {
            bi = 4 * lane + j;
            c = c4[j];
            break;
        }
        b += c4[j];
    }
    bin = (unsigned)__builtin_amdgcn_readlane(bi, owner);
    cnt = (unsigned)__builtin_amdgcn_readlane((int)c, owner);
    below = (unsigned)__builtin_amdgcn_readlane((int)b, owner);
}

// the sum passes' record chunks in flight per round trip (80 bytes per lane each). 1 since round 5: with the final
// gather's requests in spatial order the records are L2 hits, and a second chunk's 20 VGPRs cost more than its
// overlap saves (k_gather_est 1401 -> 1293 ms per cornell_gi_480x270_8x8 frame, 27 -> 12 spilled VGPRs,
// profiles/r05_ab_gi_sort.txt); the lane's records are summed in the same order either way
#ifndef FRT_SUM_CHUNKS
#define FRT_SUM_CHUNKS 1
#endif
constexpr int kSumChunks = FRT_SUM_CHUNKS;

// all 64 lanes call with the same x / normal; returns the photons used (the reference's `found`) and
// the irradiance, in every lane
__device__ __forceinline__ int64_t wave_irradiance_estimate(const PhotonMapDev& M, const double* x, const double* normal,
                                                   double max_dist, int k, double cone_k, double* irrad,
                                                   const EstLds& L, unsigned long long* prof = nullptr) {
    irrad[0] = irrad[1] = irrad[2] = 0.0;
    if (M.count <= 0) return 0;
#ifdef FRT_WALK_PROF
    unsigned long long est_t0 = prof_stamp();
#endif
    const int lane = est_lane();
    EST_COUNT(12, 1ull);
    const double r2 = max_dist * max_dist;
    // error bound of a binary32 squared distance against the reference's binary64 one, for points
    // within reach of the radius: each difference within eb = 1.01u (2A + 2r) (A = max|x| + r: the two
    // positions' roundings and the subtraction's), the squares and sums adding 2 |d| eb + eb^2 and 3u d^2
    const double A = fmax(fmax(fabs(x[0]), fabs(x[1])), fabs(x[2])) + max_dist;
    const double eb = 1.01 * 0x1p-24 * (2.0 * A + 2.0 * max_dist);
    const double tol = 1.02 * (4.0 * max_dist * eb + 3.0 * eb * eb + 4.0 * 0x1p-24 * r2);
    const float lo_thr = __double2float_rd(r2 - tol), hi_thr = __double2float_ru(r2 + tol);
    const float inv_r2 = (float)(1.0 / r2);
    // keys closer than dk may belong to photons whose binary64 order differs from their keys' order
    // (2 tol, the key's own rounding (3u relative) and its truncation); dk < 2^16 for any sane radius
    const unsigned dk = min((unsigned)ceil((2.0 * tol + 8.0 * 0x1p-24 * r2) * (16777216.0 / r2)) + 3u, 65535u);
    // within the radius, exactly: binary32 away from it, binary64 near it (uniform control flow)
    auto in_range = [&](int32_t p, bool cand, float d2) {
        bool in = cand && d2 < lo_thr;
        const bool unc = cand && !in;
        if (__ballot(unc)) {
            if (unc) in = photon_d2(M, p, x) < r2;
        }
        return in;
    };
    // Dense queries take a reduced radius rho < max_dist: the k nearest and the (k+1)-th are all the
    // selection needs (the rare full traversal-order check re-scans the whole radius), so when the grid's
    // row counts (the probe of pass 1, before any photon is loaded) predict many more than k + 1 photons
    // in range (photons lie on surfaces: the count within rho scales as rho^2), only the photons within
    // rho are listed. Exactness: every photon whose binary32 d^2 is below rho^2 - tol lies within rho, so
    // at least k + 1 of those mean d^2_(k+1) < rho^2 exactly; every photon with exact d^2 < rho^2 has
    // binary32 d^2 below rho^2 + tol and is listed; and rho^2 + tol stays below the radius' certain
    // threshold (lo_thr), so every listed photon is in range. Otherwise (too few, or the list overflows)
    // the full pass 1 runs.
    unsigned total = 0, count = 0;
    bool listed = false, filtered = false;
#ifndef FRT_EST_REDUCE_ALPHA
#define FRT_EST_REDUCE_ALPHA 2.0  // rho^2 / r^2 = alpha (k + 1) / predicted count
#endif
#ifndef FRT_EST_REDUCE_MIN
#define FRT_EST_REDUCE_MIN 3.0  // reduce when the predicted count exceeds min (k + 1)
#endif
#ifndef FRT_EST_CAND_RATIO
#define FRT_EST_CAND_RATIO 0.45  // photons in range per candidate of the chord-clipped rows (surfaces)
#endif
    double rho2 = 0.0;
    bool probing = true;
    auto want_reduce = [&](unsigned cands) {
        if (!(probing && k >= 8 && FRT_EST_REDUCE_ALPHA > 0.0)) return false;
        const double t_est = FRT_EST_CAND_RATIO * (double)cands;
        if (!(t_est > FRT_EST_REDUCE_MIN * (double)(k + 1))) return false;
        rho2 = r2 * (FRT_EST_REDUCE_ALPHA * (double)(k + 1) / t_est);
        return __double2float_ru(rho2 + tol) < lo_thr;
    };
    // pass 1: the photons within the radius into the LDS list in scan order, and the histogram of their
    // keys' top byte (the radix selects' first digit)
    auto pass1 = [&]() {
        for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
        __builtin_amdgcn_wave_barrier();
        total = 0;
        const bool done = wave_scan_cells(M, x, max_dist, hi_thr, [&](int32_t p, bool cand, float d2) {
            const bool in = in_range(p, cand, d2);
            const unsigned long long m = __ballot(in);
            if (in) {
                const unsigned at = total + (unsigned)__popcll(m & ((1ull << lane) - 1));
                const unsigned key = est_key(d2, inv_r2);
                if (at < L.cap) L.ent[at] = make_uint2(key, (unsigned)p);
                atomicAdd(&L.hist[key >> 16], 1u);
            }
            total += (unsigned)__popcll(m);
        }, want_reduce, prof);
        __builtin_amdgcn_wave_barrier();
        count = total;
        listed = total <= L.cap;
        return done;
    };
    if (!pass1()) {
        const float rlo = __double2float_rd(rho2 - tol), rhi = __double2float_ru(rho2 + tol);
        for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
        __builtin_amdgcn_wave_barrier();
        unsigned n_in = 0, n_lo = 0;
        wave_scan_cells(M, x, sqrt((double)rhi), rhi, [&](int32_t p, bool in, float d2) {
            const unsigned long long m = __ballot(in);
            if (in) {
                const unsigned at = n_in + (unsigned)__popcll(m & ((1ull << lane) - 1));
                const unsigned key = est_key(d2, inv_r2);
                if (at < L.cap) L.ent[at] = make_uint2(key, (unsigned)p);
                atomicAdd(&L.hist[key >> 16], 1u);
            }
            n_in += (unsigned)__popcll(m);
            n_lo += (unsigned)__popcll(__ballot(in && d2 < rlo));
        }, prof);
        __builtin_amdgcn_wave_barrier();
        const bool reduced = n_lo >= (unsigned)k + 1u && n_in <= L.cap;
        EST_COUNT(10, 1ull);
        EST_COUNT(11, reduced ? 0ull : 1ull);
        if (reduced) {
            total = n_in;  // (> k: found = k)
            count = n_in;
            listed = filtered = true;
        } else {
            probing = false;
            pass1();
        }
    }
    EST_STAMP(0);
    const unsigned found = total < (unsigned)k ? total : (unsigned)k;
    if (found < 8) return found;
    unsigned h4[4];  // the first digit's histogram
    for (int j = 0; j < 4; ++j) h4[j] = L.hist[4 * lane + j];
    // the list: every photon in range or, when they overflow the wave's LDS and the heap decides,
    // those whose key's top digit is at most one beyond the (k+1)-th's (which covers the band, dk <
    // 2^16), stored by a second scan; only the rare traversal-order check needs the others (re-scan)
    if (!listed && total > (unsigned)k) {
        unsigned b1, c1, below1;
        radix_pick(h4, (unsigned)k + 1u, b1, c1, below1);
        const unsigned top = min(b1 + 1u, 255u);
        unsigned le = 0;
        for (int j = 0; j < 4; ++j) le += (unsigned)(4 * lane + j) <= top ? h4[j] : 0u;
        const unsigned n_le = (unsigned)__builtin_amdgcn_readlane((int)wave_incl_scan(le), 63);
        if (n_le <= L.cap) {
            unsigned at0 = 0;
            wave_scan_cells(M, x, max_dist, hi_thr, [&](int32_t p, bool cand, float d2) {
                const unsigned key = est_key(d2, inv_r2);
                const bool keep = in_range(p, cand, d2) && (key >> 16) <= top;
                const unsigned long long m = __ballot(keep);
                if (keep) L.ent[at0 + (unsigned)__popcll(m & ((1ull << lane) - 1))] = make_uint2(key, (unsigned)p);
                at0 += (unsigned)__popcll(m);
            }, prof);
            __builtin_amdgcn_wave_barrier();
            count = at0;
            listed = filtered = true;
        }
    }
    EST_COUNT(4, total > (unsigned)k ? 1ull : 0ull);
    EST_COUNT(5, listed ? 0ull : 1ull);
    EST_COUNT(8, (unsigned long long)total);
    // every pass visits the listed photons in the same order (the list, or a re-scan when unlisted);
    // visit_all also the ones a filtered list omits
    auto scan_all = [&](auto&& fn) {
        wave_scan_cells(M, x, max_dist, hi_thr, [&](int32_t p, bool cand, float d2) {
            fn(p, in_range(p, cand, d2), est_key(d2, inv_r2));
        }, prof);
    };
    auto visit = [&](auto&& fn) {
        if (listed) {
            for (unsigned base = 0; base < count; base += 64) {
                const unsigned i = base + (unsigned)lane;
                const bool in = i < count;
                const uint2 e = in ? L.ent[i] : make_uint2(0u, 0u);
                fn((int32_t)e.y, in, e.x);
            }
        } else {
            scan_all(fn);
        }
    };
    auto visit_all = [&](auto&& fn) {
        if (filtered) scan_all(fn);
        else visit(fn);
    };
    const double cone_r = cone_k * max_dist, inv_cone_r = 1.0 / cone_r;
    double acc[3] = {0.0, 0.0, 0.0};
    // pm.c:129-145 (weight = 1 - sqrt(dist2) / (k r), within a few ulps)
    auto photon_weighted = [&](const PhotonRec& pr, int32_t p, double dp, double* w) {
        const double weight = 1.0 - dp * inv_cone_r;
        const bool facing = photon_facing(M, pr, normal);
        double pw[3];
        photon_power(M, pr, p, pw);
        w[0] = facing ? pw[0] * weight : 0.0;
        w[1] = facing ? pw[1] * weight : 0.0;
        w[2] = facing ? pw[2] * weight : 0.0;
    };
    auto accumulate = [&](const PhotonRec& pr, int32_t p, double dp) {
        const double weight = 1.0 - dp * inv_cone_r;
        if (photon_facing(M, pr, normal)) {
            double pw[3];
            photon_power(M, pr, p, pw);
            acc[0] = fma(pw[0], weight, acc[0]);
            acc[1] = fma(pw[1], weight, acc[1]);
            acc[2] = fma(pw[2], weight, acc[2]);
        }
    };
    auto finish = [&](double d0) {
        for (int j = 0; j < 3; ++j) irrad[j] = wave_sum_d(acc[j]);
        // np.dist2[0] (pm.c:147)
        const double tmp = 1.0 / ((1.0 - 2.0 / (3.0 * cone_k)) * (kPi * d0));
        irrad[0] *= tmp;
        irrad[1] *= tmp;
        irrad[2] *= tmp;
    };
    if (total <= (unsigned)k) {  // every photon in range: no heap, dist2[0] = max_dist^2
        if (listed) {  // kSumChunks chunks of the list per round trip
            SumTouch tch;  // (FRT_SUM_TOUCH)
            for (unsigned base = 0; base < count; base += 64u * kSumChunks) {
                PhotonRec rc[kSumChunks];
                bool ok[kSumChunks];
                int32_t pc[kSumChunks];
#pragma unroll
                for (int c = 0; c < kSumChunks; ++c) {
                    const unsigned i = base + 64u * c + (unsigned)lane;
                    ok[c] = i < count;
                    pc[c] = ok[c] ? (int32_t)L.ent[i].y : 0;
                    EST_LANES(15, ok[c]);
                    if (ok[c]) rc[c] = photon_rec(M, pc[c]);
                }
                if (FRT_SUM_TOUCH) tch.next(M, (int32_t)L.ent[min(base + 64u * kSumChunks + (unsigned)lane, count - 1u)].y);
#pragma unroll
                for (int c = 0; c < kSumChunks; ++c)
                    if (ok[c]) accumulate(rc[c], pc[c], sqrt_w(rc[c].d2(x)));
            }
            if (FRT_SUM_TOUCH) sum_touch_keep(tch.keep ^ tch.a ^ tch.b);
        } else {
            visit([&](int32_t p, bool in, unsigned) {
                EST_LANES(15, in);
                if (in) {
                    const PhotonRec pr = photon_rec(M, p);
                    accumulate(pr, p, sqrt_w(pr.d2(x)));
                }
            });
        }
        finish(r2);
        EST_STAMP(2);
        return found;
    }
    // ---- the k-th and (k+1)-th keys: radix selects, 8 bits per digit, sharing a histogram pass while
    // both ranks lie under the same prefix ----
    unsigned need_s[2] = {(unsigned)k, (unsigned)k + 1u}, prefix[2], mask[2] = {0xFF0000u, 0xFF0000u};
    bool done[2];
    for (int s = 0; s < 2; ++s) {
        unsigned bin, cnt, below;
        radix_pick(h4, need_s[s], bin, cnt, below);
        need_s[s] -= below;
        prefix[s] = bin << 16;
        done[s] = cnt <= 64u;  // few enough: the band ranks them
    }
    for (int shift = 8; shift >= 0 && !(done[0] && done[1]); shift -= 8) {
        const bool shared = !done[0] && !done[1] && prefix[0] == prefix[1];
        unsigned c4[4];
        for (int s = 0; s < 2; ++s) {
            if (done[s]) continue;
            if (!(s == 1 && shared)) {
                for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
                __builtin_amdgcn_wave_barrier();
                const unsigned pf = prefix[s], mk = mask[s];
                visit([&](int32_t, bool in, unsigned key) {
                    if (in && (key & mk) == pf) atomicAdd(&L.hist[(key >> shift) & 255u], 1u);
                });
                __builtin_amdgcn_wave_barrier();
                for (int j = 0; j < 4; ++j) c4[j] = L.hist[4 * lane + j];
            }
            unsigned bin, cnt, below;
            radix_pick(c4, need_s[s], bin, cnt, below);
            need_s[s] -= below;
            prefix[s] |= bin << shift;
            mask[s] |= 255u << shift;
            done[s] = cnt <= 64u || shift == 0;
        }
    }
    const unsigned klo = prefix[0], k1hi = prefix[1] | (~mask[1] & 0xFFFFFFu);
    const unsigned blo = klo > dk ? klo - dk : 0u, bhi = min(k1hi + dk, 0xFFFFFFu);
    EST_STAMP(1);
    // ---- the band: ranked by binary64 distance ----
    // pass B: photons with keys in [blo, bhi] set aside (up to 64, in L.hist), the certain ones counted
    // and the certain ones' indices compacted into L.sel (while they fit)
    unsigned c_in = 0, nb = 0;
    visit([&](int32_t p, bool in, unsigned key) {
        const bool band = in && key >= blo && key <= bhi, cert = in && key < blo;
        const unsigned long long lt = (1ull << lane) - 1;
        const unsigned long long bm = __ballot(band), cm = __ballot(cert);
        if (band) {
            const unsigned at = nb + (unsigned)__popcll(bm & lt);
            if (at < 64u) L.hist[at] = (unsigned)p;
        }
        if (cert) {
            const unsigned at = c_in + (unsigned)__popcll(cm & lt);
            if (at < kEstSel) L.sel[at] = (unsigned)p;
        }
        nb += (unsigned)__popcll(bm);
        c_in += (unsigned)__popcll(cm);
    });
    __builtin_amdgcn_wave_barrier();
    const unsigned need = (unsigned)k - c_in;  // band ranks of the k-th (need - 1) and the (k+1)-th (need)
    double vk = r2, vk1 = r2;
    int32_t R = 1;
    bool mine_band = false;  // this lane holds a band photon (fast path)
    int32_t bh = 1;
    double bv = 0.0, bw[3] = {0.0, 0.0, 0.0};  // its binary64 distance, weighted power (0: facing away)
    unsigned brank = 0;
    const bool fast = nb <= 64u && need >= 1u && need + 1u <= nb;
    if (fast) {
        mine_band = (unsigned)lane < nb;
        EST_LANES(15, mine_band);
        if (mine_band) {
            const int32_t bp = (int32_t)L.hist[lane];
            const PhotonRec pr = photon_rec(M, bp);
            bv = pr.d2(x);
            bh = pr.heap();
            photon_weighted(pr, bp, sqrt_w(bv), bw);
        }
        for (unsigned j = 0; j < nb; ++j) {
            const double vj = readlane_dd(bv, (int)j);
            brank += (vj < bv || (vj == bv && j < (unsigned)lane)) ? 1u : 0u;
        }
        const int ok = __builtin_ctzll(__ballot(mine_band && brank == need - 1u));
        const int ok1 = __builtin_ctzll(__ballot(mine_band && brank == need));
        vk = readlane_dd(bv, ok);
        vk1 = readlane_dd(bv, ok1);
        R = __builtin_amdgcn_readlane(bh, ok1);
    } else {
        EST_COUNT(6, 1ull);
        // many photons in the band (a dense caustic): exact radix selects over the band's binary64
        // distances (their bit patterns order like the values), passes over the list
        auto exact_rank = [&](unsigned rk) {
            unsigned long long pf = 0, mk = 0;
            for (int shift = 56; shift >= 0; shift -= 8) {
                for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
                __builtin_amdgcn_wave_barrier();
                visit([&](int32_t p, bool in, unsigned key) {
                    const bool band = in && key >= blo && key <= bhi;
                    if (band) {
                        const unsigned long long b = (unsigned long long)__double_as_longlong(photon_d2(M, p, x));
                        if ((b & mk) == pf) atomicAdd(&L.hist[(unsigned)((b >> shift) & 255ull)], 1u);
                    }
                });
                __builtin_amdgcn_wave_barrier();
                unsigned c4[4], bin, cnt, below;
                for (int j = 0; j < 4; ++j) c4[j] = L.hist[4 * lane + j];
                radix_pick(c4, rk, bin, cnt, below);
                rk -= below;
                pf |= (unsigned long long)bin << shift;
                mk |= 255ull << shift;
            }
            return __longlong_as_double((long long)pf);
        };
        vk = exact_rank(need);
        vk1 = exact_rank(need + 1u);
        int32_t rh = 0;
        visit([&](int32_t p, bool in, unsigned key) {  // the (k+1)-th's heap index (first of equal distances)
            int32_t hx = 0;
            if (in && key >= blo && key <= bhi && photon_d2(M, p, x) == vk1) hx = photon_heap(M, p);
            const unsigned long long hm = __ballot(hx != 0);
            if (rh == 0 && hm) rh = __builtin_amdgcn_readlane(hx, __builtin_ctzll(hm));
        });
        R = rh != 0 ? rh : 1;
    }
    EST_STAMP(3);
    // ---- sum pass over the k nearest, checking that each comes before the (k+1)-th ----
    bool before_all = true;
    unsigned below_k = 0;  // (slow path) band photons strictly nearer than the k-th
    const bool compact = c_in <= kEstSel;
    // the certain photons from L.sel, two chunks' records in flight together; the first two chunks'
    // loads issue with near_mask's
    const unsigned qmask = near_mask(M.kd, R, x);
    if (compact) {
        SumTouch tch;  // (FRT_SUM_TOUCH)
        for (unsigned base = 0; base < c_in; base += 64u * kSumChunks) {
            PhotonRec rc[kSumChunks];
            bool ok[kSumChunks];
            int32_t pc[kSumChunks];
#pragma unroll
            for (int c = 0; c < kSumChunks; ++c) {
                const unsigned i = base + 64u * c + (unsigned)lane;
                ok[c] = i < c_in;
                pc[c] = ok[c] ? (int32_t)L.sel[i] : 0;
                EST_LANES(15, ok[c]);
                if (ok[c]) rc[c] = photon_rec(M, pc[c]);
            }
            if (FRT_SUM_TOUCH) tch.next(M, (int32_t)L.sel[min(base + 64u * kSumChunks + (unsigned)lane, c_in - 1u)]);
#pragma unroll
            for (int c = 0; c < kSumChunks; ++c)
                if (ok[c]) {
                    accumulate(rc[c], pc[c], sqrt_w(rc[c].d2(x)));
                    before_all = before_all && found_before(rc[c].heap(), R, qmask);
                }
        }
        if (FRT_SUM_TOUCH) sum_touch_keep(tch.keep ^ tch.a ^ tch.b);
    }
    if (!compact || !fast) visit([&](int32_t p, bool in, unsigned key) {
        const bool certain = in && key < blo && !compact;
        const bool band = in && key >= blo && key <= bhi && !fast;
        if (certain) {
            const PhotonRec pr = photon_rec(M, p);
            accumulate(pr, p, sqrt_w(pr.d2(x)));
            before_all = before_all && found_before(pr.heap(), R, qmask);
        }
        if (__ballot(band)) {  // (slow path) band photons: membership by their binary64 distance
            bool nearer = false;
            if (band) {
                const PhotonRec pr = photon_rec(M, p);
                const double v = pr.d2(x);
                nearer = v < vk;
                // those at the k-th's and the (k+1)-th's distance are added after the check
                if (nearer) accumulate(pr, p, sqrt_w(v));
                if (v <= vk && pr.heap() != R) before_all = before_all && found_before(pr.heap(), R, qmask);
            }
            below_k += (unsigned)__popcll(__ballot(nearer));
        }
    });
    if (fast && mine_band && brank < need) before_all = before_all && found_before(bh, R, qmask);
    bool quirk = false;
    EST_STAMP(2);
    if (wave_and(before_all)) {
        // every one of the k nearest precedes the (k+1)-th: the traversal may have found them first.
        // The last of them in traversal order, then every other photon in range against it.
        EST_COUNT(7, 1ull);
        int32_t last = 0;
        auto consider = [&](int32_t hx) {
            if (last == 0 || found_before_any(M.kd, last, hx, x)) last = hx;
        };
        visit([&](int32_t p, bool in, unsigned key) {
            if (in && key < blo) consider(photon_heap(M, p));
            if (in && key >= blo && key <= bhi && !fast && photon_d2(M, p, x) <= vk) consider(photon_heap(M, p));
        });
        if (fast && mine_band && brank < need) consider(bh);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int32_t other = __shfl_xor(last, o, 64);
            if (other != 0) consider(other);
        }
        const int32_t Lh = __builtin_amdgcn_readlane(last, 0);
        const unsigned lmask = near_mask(M.kd, Lh, x);
        bool after = true;
        visit_all([&](int32_t p, bool in, unsigned key) {
            bool other = in && key > bhi;
            if (in && key >= blo && key <= bhi && !fast) other = photon_d2(M, p, x) > vk;
            if (other) after = after && !found_before(photon_heap(M, p), Lh, lmask);
        });
        if (fast && mine_band && brank >= need) after = after && !found_before(bh, Lh, lmask);
        quirk = wave_and(after);
        EST_STAMP(9);
    }
    // the band's selected photons: ranks below need (the k-th excluded and the (k+1)-th included when
    // the traversal found the k nearest first)
    if (fast) {
        if (mine_band && (quirk ? (brank + 1u < need || brank == need) : brank < need))
            for (int j = 0; j < 3; ++j) acc[j] += bw[j];
    } else {
        // slow path: photons at the k-th's distance up to rank k (rank k - 1 when the (k+1)-th replaces
        // the k-th), then the (k+1)-th (ties: the first ones visited)
        unsigned take_k = need - below_k, take_k1 = 0;
        if (quirk && vk1 != vk) {  // (at equal distances the count at vk stays)
            take_k -= 1;
            take_k1 = 1;
        }
        visit([&](int32_t p, bool in, unsigned key) {
            const bool band = in && key >= blo && key <= bhi;
            if (__ballot(band)) {
                double v = -1.0;
                if (band) v = photon_d2(M, p, x);
                const bool ek = band && v == vk, ek1 = band && v == vk1 && vk1 != vk;
                const unsigned long long below = (1ull << lane) - 1;
                const unsigned long long mk = __ballot(ek), mk1 = __ballot(ek1);
                if ((ek && (unsigned)__popcll(mk & below) < take_k) || (ek1 && (unsigned)__popcll(mk1 & below) < take_k1))
                    accumulate(photon_rec(M, p), p, sqrt_w(v));
                take_k -= min(take_k, (unsigned)__popcll(mk));
                take_k1 -= min(take_k1, (unsigned)__popcll(mk1));
            }
        });
    }
    finish(quirk ? vk1 : vk);
    EST_STAMP(2);
    return found;
}

}  // namespace frt
