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
// pm_irradiance_estimate (pm.c:91-155) with the 64 lanes of a wave working on
// ONE query point (wave-uniform x): the k nearest photons within max_dist (the
// reference's max-heap in pm_locate_photons keeps exactly the k smallest
// squared distances), cone-filtered, photons arriving from the "normal" side
// only; zero below 8 photons, as in the reference.
//
// Candidates come from the dense grid of PhotonMapDev (cell edge radius / 3):
// the grid rows (y, z) within reach of the sphere, each clipped in x to the
// sphere's chord, are concatenated and scanned 64 photons at a time
// (coalesced binary32 positions); photons within the radius are compacted into
// the wave's LDS list (ballot + rank), the k-th smallest distance is found by a
// radix select over 24-bit keys of d^2 / r^2 (LDS histograms: the first digit's
// built during the scan; when the k-th falls in a bin of at most 64 photons they
// are ranked directly in the sum pass, else up to two more passes over the
// list), and the cone-filtered sum is one more pass with a wave reduction. A list longer than the wave's capacity (a dense caustic) is not stored: the
// select and sum passes then re-scan the rows. Distances are binary32 here (the
// estimate is a statistical quantity: the reference's photon maps come from
// drand48); the sums are binary64.
constexpr int kEstCap = 1024;

struct EstLds {
    uint2* ent;       // cap: (squared distance bits, photon index) of the photons within the radius
    unsigned* hist;   // 256
    unsigned cap;
};

__device__ __forceinline__ int est_lane() { return (int)(threadIdx.x & 63); }

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
template <typename F>
__device__ inline void wave_scan_cells(const PhotonMapDev& M, const double* x, double r, float r2f, F&& f) {
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
    if (!any) return;
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
        // two chunks per step: both position loads are in flight before either is used
        for (unsigned base = 0; base < total; base += 128) {
            const int32_t pa = chunk_photon(base), pb = chunk_photon(base + 64u);
            bool ina = base + (unsigned)lane < total, inb = base + 64u + (unsigned)lane < total;
            float4 qa = make_float4(0.0f, 0.0f, 0.0f, 0.0f), qb = qa;
            if (ina) qa = reinterpret_cast<const float4*>(M.pos4)[pa];
            if (inb) qb = reinterpret_cast<const float4*>(M.pos4)[pb];
            float d2a = 0.0f, d2b = 0.0f;
            if (ina) {
                const float dx = qa.x - xf[0], dy = qa.y - xf[1], dz = qa.z - xf[2];
                d2a = dx * dx + dy * dy + dz * dz;
                ina = d2a < r2f;
            }
            if (inb) {
                const float dx = qb.x - xf[0], dy = qb.y - xf[1], dz = qb.z - xf[2];
                d2b = dx * dx + dy * dy + dz * dz;
                inb = d2b < r2f;
            }
            f(pa, ina, d2a);
            f(pb, inb, d2b);
        }
    }
}

// all 64 lanes call with the same x / normal; returns the photons used (the
// reference's `found`) and the irradiance, in every lane
#ifdef FRT_WALK_PROF
#define EST_STAMP(k)                                                                      \
    do {                                                                                  \
        const unsigned long long t1_ = prof_stamp();                                      \
        if (lane == 0 && prof) atomicAdd(prof + (k), t1_ - est_t0);                      \
        est_t0 = t1_;                                                                     \
    } while (0)
#else
#define EST_STAMP(k)
#endif
__device__ inline int64_t wave_irradiance_estimate(const PhotonMapDev& M, const double* x, const double* normal,
                                                   double max_dist, int k, double cone_k, double* irrad,
                                                   const EstLds& L, unsigned long long* prof = nullptr) {
    irrad[0] = irrad[1] = irrad[2] = 0.0;
    if (M.count <= 0) return 0;
#ifdef FRT_WALK_PROF
    unsigned long long est_t0 = prof_stamp();
#endif
    const int lane = est_lane();
    const double r2 = max_dist * max_dist;
    const float r2f = (float)r2, inv_r2 = (float)(1.0 / r2);
    // pass 1: the photons within the radius, compacted into the LDS list in scan order, and the
    // histogram of their keys' top byte (the radix select's first digit)
    for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
    __builtin_amdgcn_wave_barrier();
    unsigned total = 0;
    wave_scan_cells(M, x, max_dist, r2f, [&](int32_t p, bool in, float d2) {
        const unsigned long long m = __ballot(in);
        if (in) {
            const unsigned at = total + (unsigned)__popcll(m & ((1ull << lane) - 1));
            if (at < L.cap) {
                L.ent[at] = make_uint2(__float_as_uint(d2), (unsigned)p);
            }
            atomicAdd(&L.hist[est_key(d2, inv_r2) >> 16], 1u);
        }
        total += (unsigned)__popcll(m);
    });
    EST_STAMP(0);
    const unsigned found = total < (unsigned)k ? total : (unsigned)k;
    if (found < 8) return found;
    const bool listed = total <= L.cap;
    // every pass visits the in-range photons in the same order: from the list, or a re-scan
    auto visit = [&](auto&& fn) {
        if (listed) {
            for (unsigned base = 0; base < total; base += 64) {
                const unsigned i = base + (unsigned)lane;
                const bool in = i < total;
                const uint2 e = in ? L.ent[i] : make_uint2(0u, 0u);
                fn((int32_t)e.y, in, __uint_as_float(e.x));
            }
        } else {
            wave_scan_cells(M, x, max_dist, r2f, fn);
        }
    };
    // the k-th smallest key: radix select, 8 bits per pass
    unsigned prefix = 0, mask = 0, need = found;
    bool resolved = total <= (unsigned)k;  // every photon in range is used
    bool few_ties = false;  // the k-th lies among <= 64 photons of one bin: ranked directly in the sum pass
    for (int shift = 16; shift >= 0 && !resolved; shift -= 8) {
        if (shift != 16) {  // (the first digit's histogram came with pass 1)
            for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
            __builtin_amdgcn_wave_barrier();
            visit([&](int32_t, bool in, float d2) {
                const unsigned key = est_key(d2, inv_r2);
                if (in && (key & mask) == prefix) atomicAdd(&L.hist[(key >> shift) & 255u], 1u);
            });
        }
        __builtin_amdgcn_wave_barrier();
        unsigned h4[4], local = 0;
        for (int j = 0; j < 4; ++j) {
            h4[j] = L.hist[4 * lane + j];
            local += h4[j];
        }
        const unsigned incl = wave_incl_scan(local);
        const unsigned long long hit = __ballot(incl >= need);
        const int owner = __builtin_ctzll(hit);
        // the owner lane walks its four bins
        unsigned below = incl - local;
        int bin = 4 * lane + 3;
        unsigned cnt = h4[3];
        for (int j = 0; j < 4; ++j) {
            if (below + h4[j] >= need) {
                bin = 4 * lane + j;
                cnt = h4[j];
                break;
            }
            below += h4[j];
        }
        bin = __builtin_amdgcn_readlane(bin, owner);
        cnt = __builtin_amdgcn_readlane(cnt, owner);
        below = __builtin_amdgcn_readlane(below, owner);
        need -= below;
        prefix |= (unsigned)bin << shift;
        mask |= 255u << shift;
        resolved = cnt == need;
        if (!resolved && cnt <= 64u) {
            few_ties = true;
            break;
        }
    }
    EST_STAMP(1);
    // sum pass (pm.c:125-145): keys below the k-th are in; at the k-th key the first `need` met
    const double cone_r = cone_k * max_dist;
    double acc[3] = {0.0, 0.0, 0.0};
    float dmax = 0.0f;
    unsigned ties = 0;
    const bool all = total <= (unsigned)k;
    // few_ties: the bin's photons (the "ties" at the selected prefix) are set aside in L.hist
    // (index, d^2, key at scan position r < 64) and the `need` smallest by (key, scan order) taken
    // after the pass: the same photons as a further select pass would keep
    auto decide = [&](int32_t p, bool in, float d2) {
        const unsigned key = est_key(d2, inv_r2);
        const bool lower = in && (all || (key & mask) < prefix);
        const bool tie = in && !all && (key & mask) == prefix;
        const unsigned long long tm = __ballot(tie);
        const unsigned r = ties + (unsigned)__popcll(tm & ((1ull << lane) - 1));
        bool take = lower;
        if (few_ties) {
            if (tie) {
                L.hist[r] = (unsigned)p;
                L.hist[64 + r] = __float_as_uint(d2);
                L.hist[128 + r] = key;
            }
        } else {
            take = take || (tie && (resolved || r < need));
        }
        ties += (unsigned)__popcll(tm);
        return take;
    };
    // one 48-byte record per photon: power x, y, z, direction x, y, z
    auto record = [&](int32_t p, double2* r) {
        const double2* rec = reinterpret_cast<const double2*>(M.pwdir) + 3 * (int64_t)p;
        r[0] = rec[0];
        r[1] = rec[1];
        r[2] = rec[2];
    };
    auto accumulate = [&](float d2, const double2* r) {
        dmax = fmaxf(dmax, d2);
        const double weight = 1.0 - (double)sqrtf(d2) / cone_r;
        if ((r[1].y * normal[0] + r[2].x * normal[1] + r[2].y * normal[2]) < 0.0) {
            acc[0] += r[0].x * weight;
            acc[1] += r[0].y * weight;
            acc[2] += r[1].x * weight;
        }
    };
    if (listed) {  // two chunks per step: both record loads in flight together
        for (unsigned base = 0; base < total; base += 128) {
            const unsigned ia = base + (unsigned)lane, ib = ia + 64u;
            const bool ina = ia < total, inb = ib < total;
            const uint2 ea = ina ? L.ent[ia] : make_uint2(0u, 0u), eb = inb ? L.ent[ib] : make_uint2(0u, 0u);
            const int32_t pa = (int32_t)ea.y, pb = (int32_t)eb.y;
            const float d2a = __uint_as_float(ea.x), d2b = __uint_as_float(eb.x);
            const bool ta = decide(pa, ina, d2a), tb = decide(pb, inb, d2b);
            double2 ra[3], rb[3];
            if (ta) record(pa, ra);
            if (tb) record(pb, rb);
            if (ta) accumulate(d2a, ra);
            if (tb) accumulate(d2b, rb);
        }
    } else {
        wave_scan_cells(M, x, max_dist, r2f, [&](int32_t p, bool in, float d2) {
            if (decide(p, in, d2)) {
                double2 r[3];
                record(p, r);
                accumulate(d2, r);
            }
        });
    }
    if (few_ties) {
        __builtin_amdgcn_wave_barrier();
        const bool mine = (unsigned)lane < ties;
        const unsigned kl = mine ? L.hist[128 + lane] : 0xffffffffu;
        unsigned rank = 0;
        for (unsigned m = 0; m < ties; ++m) {
            const unsigned km = (unsigned)__builtin_amdgcn_readlane((int)kl, (int)m);
            rank += (km < kl || (km == kl && m < (unsigned)lane)) ? 1u : 0u;
        }
        if (mine && rank < need) {
            const float d2 = __uint_as_float(L.hist[64 + lane]);
            double2 r[3];
            record((int32_t)L.hist[lane], r);
            accumulate(d2, r);
        }
    }
    for (int j = 0; j < 3; ++j) irrad[j] = wave_sum_d(acc[j]);
    dmax = wave_max_f(dmax);
    EST_STAMP(2);
    // np.dist2[0]: max_dist^2 until the heap filled, then its largest entry (pm.c:244)
    const double d0 = all ? r2 : (double)dmax;
    const double tmp = 1.0 / ((1.0 - 2.0 / (3.0 * cone_k)) * (kPi * d0));
    irrad[0] *= tmp;
    irrad[1] *= tmp;
    irrad[2] *= tmp;
    return found;
}

}  // namespace frt
