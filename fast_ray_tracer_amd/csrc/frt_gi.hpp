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

}  // namespace frt
