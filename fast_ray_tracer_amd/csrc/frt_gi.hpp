// frt-mi355x global illumination on the device: photon emission and the
// photon_hit decisions of the reference's photon tracer (photon_tracer.c),
// the k-nearest-photon irradiance estimate (pm.c:91-250) over a hashed
// uniform grid, and the hemisphere sampling shared with the final gather
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

// ---- photon maps on the device ----

__device__ __forceinline__ uint32_t grid_bucket(int64_t ix, int64_t iy, int64_t iz, int32_t nb) {
    const uint64_t h = (uint64_t)ix * 73856093ull ^ (uint64_t)iy * 19349663ull ^ (uint64_t)iz * 83492791ull;
    return (uint32_t)(mix64(h) & (uint64_t)(nb - 1));
}

// Visit every photon within distance^2 < r2 of x exactly once: the 27 cells
// around x's cell (cell edge >= radius), each bucket once even when cells
// collide in the hash. f(index, d2) is called per photon inside the sphere.
template <typename F>
__device__ inline void for_photons_within(const PhotonMapDev& M, const double* x, double r2, F&& f) {
    int64_t c[3];
    for (int k = 0; k < 3; ++k) c[k] = (int64_t)floor((x[k] - M.origin[k]) / M.cell);
    uint32_t seen[27];
    int nseen = 0;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                const uint32_t b = grid_bucket(c[0] + dx, c[1] + dy, c[2] + dz, M.num_buckets);
                bool dup = false;
                for (int q = 0; q < nseen; ++q) dup = dup || seen[q] == b;
                if (dup) continue;
                seen[nseen++] = b;
                const int32_t e = M.start[b + 1];
                for (int32_t p = M.start[b]; p < e; ++p) {
                    const double* pp = M.pos + 3 * (int64_t)p;
                    // pm_locate_photons' distance (pm.c:185-191)
                    double d1 = pp[0] - x[0];
                    double d2 = d1 * d1;
                    d1 = pp[1] - x[1];
                    d2 += d1 * d1;
                    d1 = pp[2] - x[2];
                    d2 += d1 * d1;
                    if (d2 < r2) f(p, d2);
                }
            }
}

// pm_irradiance_estimate (pm.c:91-155): the k nearest photons within
// max_dist (the reference's max-heap in pm_locate_photons keeps exactly the k
// smallest squared distances), cone-filtered, photons arriving from the
// "normal" side only. The k-th distance is found by histogram refinement over
// [0, max_dist^2) (a few passes over the candidates, bounded registers), the
// sum is taken in one more pass. Returns the number of photons used; irradiance
// is zero when fewer than 8 were found, as in the reference.
__device__ inline int64_t irradiance_estimate(const PhotonMapDev& M, const double* x, const double* normal,
                                              double max_dist, int k, double cone_k, double* irrad) {
    irrad[0] = irrad[1] = irrad[2] = 0.0;
    if (M.count <= 0) return 0;
    const double r2 = max_dist * max_dist;
    constexpr int kBins = 16;
    // pass 1: count and histogram over [0, r2)
    int64_t total = 0;
    int32_t hist[kBins];
    for (int b = 0; b < kBins; ++b) hist[b] = 0;
    double lo = 0.0, hi = r2;
    for_photons_within(M, x, r2, [&](int32_t, double d2) {
        ++total;
        int b = (int)(d2 / r2 * kBins);
        b = b < 0 ? 0 : (b >= kBins ? kBins - 1 : b);
        ++hist[b];
    });
    int64_t found = total < (int64_t)k ? total : (int64_t)k;
    if (found < 8) return found;
    // select: photons with d2 < lo are all in; `need` more come from [lo, hi)
    int64_t need = found;
    bool all_in_range = total <= (int64_t)k;
    for (int level = 0; level < 12 && !all_in_range; ++level) {
        int64_t cum = 0;
        int b = 0;
        for (; b < kBins; ++b) {
            if (cum + hist[b] >= need) break;
            cum += hist[b];
        }
        const double w = (hi - lo) / kBins;
        const double nlo = lo + w * b, nhi = (b == kBins - 1) ? hi : lo + w * (b + 1);
        need -= cum;
        lo = nlo;
        hi = nhi;
        if (hist[b] == need || !(hi > lo)) {
            all_in_range = hist[b] == need;
            break;
        }
        for (int q = 0; q < kBins; ++q) hist[q] = 0;
        const double llo = lo, lhi = hi, lw = hi - lo;
        for_photons_within(M, x, r2, [&](int32_t, double d2) {
            if (d2 >= llo && d2 < lhi) {
                int q = (int)((d2 - llo) / lw * kBins);
                q = q < 0 ? 0 : (q >= kBins ? kBins - 1 : q);
                ++hist[q];
            }
        });
    }
    // sum pass (pm.c:125-145); exact ties at the boundary: the first `need` met are taken
    int64_t taken_in_range = 0;
    double dmax = 0.0;
    const double llo = total <= (int64_t)k ? r2 : lo;
    const double lhi = total <= (int64_t)k ? r2 : hi;
    const double cone_r = cone_k * max_dist;
    const double* pw = M.power;
    const double* pd = M.dir;
    const double* ps = M.pos;
    for_photons_within(M, x, r2, [&](int32_t p, double d2) {
        bool take = d2 < llo;
        if (!take && d2 >= llo && d2 < lhi && taken_in_range < need) {
            take = true;
            ++taken_in_range;
        }
        if (total <= (int64_t)k) take = true;
        if (!take) return;
        if (d2 > dmax) dmax = d2;
        const double* pp = ps + 3 * (int64_t)p;
        const double dp = sqrt((x[0] - pp[0]) * (x[0] - pp[0]) + (x[1] - pp[1]) * (x[1] - pp[1]) +
                               (x[2] - pp[2]) * (x[2] - pp[2]));
        const double weight = 1.0 - dp / cone_r;
        const double* dd = pd + 3 * (int64_t)p;
        if ((dd[0] * normal[0] + dd[1] * normal[1] + dd[2] * normal[2]) < 0.0) {
            const double* w3 = pw + 3 * (int64_t)p;
            irrad[0] += w3[0] * weight;
            irrad[1] += w3[1] * weight;
            irrad[2] += w3[2] * weight;
        }
    });
    // np.dist2[0]: max_dist^2 until the heap filled, then its largest entry (pm.c:244)
    const double d0 = total < (int64_t)k ? r2 : (total == (int64_t)k ? r2 : dmax);
    const double tmp = 1.0 / ((1.0 - 2.0 / (3.0 * cone_k)) * (kPi * d0));
    irrad[0] *= tmp;
    irrad[1] *= tmp;
    irrad[2] *= tmp;
    return found;
}

// ---- wave-cooperative estimate ----
// pm_irradiance_estimate with the 64 lanes of a wave working on ONE query
// point (wave-uniform x): the neighbour cells' photons are scanned with
// consecutive lanes on consecutive photons (coalesced binary32 positions),
// those within the radius are compacted into the wave's LDS list, the k-th
// smallest distance is found by a radix select over 24-bit keys of d^2 / r^2
// (LDS histograms, at most three passes over the list), and the cone-filtered
// sum is one more pass with a wave reduction. A list longer than kEstCap (a
// dense caustic) is not stored: the select and sum passes then re-scan the
// cells. Distances are binary32 here — the estimate is a statistical quantity
// (the reference's photon maps come from drand48), the per-lane version
// above keeps binary64.
constexpr int kEstCap = 1024;

struct EstLds {
    float* d2;        // kEstCap: squared distances of the photons within the radius
    int32_t* idx;     // kEstCap: their photon indices
    unsigned* hist;   // 256
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

// the neighbour cells (lane c < 27 owns cell c, dz outer, dx inner; each bucket once):
// calls f(p, in, d2) for every chunk of up to 64 consecutive photons of a cell, in
// uniform control flow; `in`: this lane's photon exists and lies within the radius
template <typename F>
__device__ inline void wave_scan_cells(const PhotonMapDev& M, const double* x, float r2f, F&& f) {
    const int lane = est_lane();
    const int ci = lane < 27 ? lane : 0;
    int64_t c[3];
    for (int k = 0; k < 3; ++k) c[k] = (int64_t)floor((x[k] - M.origin[k]) / M.cell);
    const uint32_t b = grid_bucket(c[0] + ci % 3 - 1, c[1] + (ci / 3) % 3 - 1, c[2] + ci / 9 - 1, M.num_buckets);
    bool dup = false;
    for (int j = 0; j < 26; ++j) {
        const uint32_t bj = (uint32_t)__shfl((int)b, j, 64);
        dup = dup || (j < ci && bj == b);
    }
    const bool keep = lane < 27 && !dup;
    const int32_t s0 = keep ? M.start[b] : 0, e0 = keep ? M.start[b + 1] : 0;
    const float xf[3] = {(float)x[0], (float)x[1], (float)x[2]};
    for (int q = 0; q < 27; ++q) {
        const int32_t s = __builtin_amdgcn_readlane(s0, q), e = __builtin_amdgcn_readlane(e0, q);
        for (int32_t base = s; base < e; base += 64) {
            const int32_t p = base + lane;
            bool in = p < e;
            float d2 = 0.0f;
            if (in) {
                const float4 pp = reinterpret_cast<const float4*>(M.pos4)[p];
                const float dx = pp.x - xf[0], dy = pp.y - xf[1], dz = pp.z - xf[2];
                d2 = dx * dx + dy * dy + dz * dz;
                in = d2 < r2f;
            }
            f(p, in, d2);
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
    // pass 1: the photons within the radius, compacted into the LDS list in scan order
    unsigned total = 0;
    wave_scan_cells(M, x, r2f, [&](int32_t p, bool in, float d2) {
        const unsigned long long m = __ballot(in);
        if (in) {
            const unsigned at = total + (unsigned)__popcll(m & ((1ull << lane) - 1));
            if (at < (unsigned)kEstCap) {
                L.d2[at] = d2;
                L.idx[at] = p;
            }
        }
        total += (unsigned)__popcll(m);
    });
    EST_STAMP(0);
    const unsigned found = total < (unsigned)k ? total : (unsigned)k;
    if (found < 8) return found;
    const bool listed = total <= (unsigned)kEstCap;
    // every pass visits the in-range photons in the same order: from the list, or a re-scan
    auto visit = [&](auto&& fn) {
        if (listed) {
            for (unsigned base = 0; base < total; base += 64) {
                const unsigned i = base + (unsigned)lane;
                const bool in = i < total;
                fn(in ? L.idx[i] : 0, in, in ? L.d2[i] : 0.0f);
            }
        } else {
            wave_scan_cells(M, x, r2f, fn);
        }
    };
    // the k-th smallest key: radix select, 8 bits per pass
    unsigned prefix = 0, mask = 0, need = found;
    bool resolved = total <= (unsigned)k;  // every photon in range is used
    for (int shift = 16; shift >= 0 && !resolved; shift -= 8) {
        for (int j = 0; j < 4; ++j) L.hist[4 * lane + j] = 0u;
        __builtin_amdgcn_wave_barrier();
        visit([&](int32_t, bool in, float d2) {
            const unsigned key = est_key(d2, inv_r2);
            if (in && (key & mask) == prefix) atomicAdd(&L.hist[(key >> shift) & 255u], 1u);
        });
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
    }
    EST_STAMP(1);
    // sum pass (pm.c:125-145): keys below the k-th are in; at the k-th key the first `need` met
    const double cone_r = cone_k * max_dist;
    double acc[3] = {0.0, 0.0, 0.0};
    float dmax = 0.0f;
    unsigned ties = 0;
    const bool all = total <= (unsigned)k;
    visit([&](int32_t p, bool in, float d2) {
        const unsigned key = est_key(d2, inv_r2);
        const bool lower = in && (all || (key & mask) < prefix);
        const bool tie = in && !all && (key & mask) == prefix;
        const unsigned long long tm = __ballot(tie);
        const bool take = lower || (tie && (resolved || ties + (unsigned)__popcll(tm & ((1ull << lane) - 1)) < need));
        ties += (unsigned)__popcll(tm);
        if (take) {
            dmax = fmaxf(dmax, d2);
            const double weight = 1.0 - sqrt((double)d2) / cone_r;
            const double* dd = M.dir + 3 * (int64_t)p;
            if ((dd[0] * normal[0] + dd[1] * normal[1] + dd[2] * normal[2]) < 0.0) {
                const double* w3 = M.power + 3 * (int64_t)p;
                acc[0] += w3[0] * weight;
                acc[1] += w3[1] * weight;
                acc[2] += w3[2] * weight;
            }
        }
    });
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
