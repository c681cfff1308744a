// frt-mi355x camera rays and the ray / hit records of the level queues, shared by the engine
// (frt_engine.hip: k_trace, k_prepare) and the scene-specialised closest-hit kernel (frt_jit.hip
// frt_jit_trace), which generates its level-0 rays in place as k_trace does.
#pragma once

#include "frt_shadow.hpp"

namespace frt {

// one queued ray of a level (segmented queues: frt_shadow.hpp queue_slot)
struct QueuedRay {
    double o[3];
    double d[3];
    uint64_t key;
    int32_t parent;
    int32_t slot;
};

// a ray's closest hit (k_trace -> k_prepare)
// (the refractive indices either side of a hit, from the containers, go to an array of their own (n12, two per
// ray), written only where a scene has indices other than one: most scenes write and read 16 bytes per hit)
struct HitRec {
    double t;
    int32_t node;  // -1: miss
    int32_t pad;
};

// ---- stochastic camera sampling (counter-based RNG; the reference draws drand48) ----
// Uniform double in [0, 1) for draw d of stream (seed, key): 53 bits of a splitmix64 hash.
__device__ __forceinline__ double rng_uniform(uint64_t seed, uint64_t key, uint64_t d) {
    const uint64_t h = mix64(seed ^ mix64(key * 0x9e3779b97f4a7c15ULL + d * 0xd1b54a32d192ed03ULL + 0x632be59bd9b4e019ULL));
    return (double)(h >> 11) * 0x1.0p-53;
}

// Jittered correlated multi-jittered sub-pixel point (u, v) of one pixel: the
// reference's sampler_reset_2d (sampler.c:411-470: canonical pattern with a
// drand48 jitter per cell, then the x rows and y columns shuffled with
// drand48) evaluated for one cell by tracing the two shuffles backwards.
// Draw numbering: canonical cell (j, i) -> x: 2(jV+i), y: 2(jV+i)+1;
// x-row shuffle step j -> 2UV + j; y-column shuffle step i -> 2UV + V + i.
__device__ inline void cmj_point(uint64_t seed, uint64_t pixel, int U, int V, int u, int v, double* out) {
    const uint64_t base = 2ull * (uint64_t)U * (uint64_t)V;
    // x: rows j < V of length U are permuted (sampler.c:442-450, n = steps[1] = V, m = steps[0] = U)
    int p = v;
    for (int j = V - 1; j >= 0; --j) {
        const int k = (int)(j + rng_uniform(seed, pixel, base + j) * (double)(V - j));
        if (p == j) p = k;
        else if (p == k) p = j;
    }
    {
        const int f = p * U + u;           // flat index of the source cell
        const int jj = f / V, ii = f % V;  // canonical layout idx = j * V + i (sampler.c:419-427)
        const double r = rng_uniform(seed, pixel, 2ull * (uint64_t)f);
        out[0] = (ii + (jj + r) / (double)U) / (double)V;
    }
    // y: columns i < U are permuted (sampler.c:452-460)
    p = u;
    for (int i = U - 1; i >= 0; --i) {
        const int k = (int)(i + rng_uniform(seed, pixel, base + (uint64_t)V + i) * (double)(U - i));
        if (p == i) p = k;
        else if (p == k) p = i;
    }
    {
        const int f = v * U + p;
        const int jj = f / V, ii = f % V;
        const double r = rng_uniform(seed, pixel, 2ull * (uint64_t)f + 1);
        out[1] = (jj + (ii + r) / (double)V) / (double)U;
    }
}

// aperture_fn (camera.c:11-82): rejection sampling on [0,1)^2; point-like types give the centre
__device__ inline void aperture_point(const frt_camera& cam, uint64_t seed, uint64_t sample, double* xy,
                                      unsigned& err) {
    const double* a = cam.aperture_args;
    const int type = cam.aperture_type;
    if (type == 6 || type == 4 || type == 5 || type == 8 || type < 0 || type > 8) {  // point / not-implemented types
        xy[0] = 0.5;
        xy[1] = 0.5;
        return;
    }
    for (int attempt = 0; attempt < 4096; ++attempt) {
        const double x = rng_uniform(seed ^ 0xa5e7u, sample, 2ull * attempt);
        const double y = rng_uniform(seed ^ 0xa5e7u, sample, 2ull * attempt + 1);
        const double u = 2 * x - 1, v = 2 * y - 1;
        bool ok;
        switch (type) {
        case 0: ok = !(u * u + v * v > a[0]); break;                                    // circle r1
        case 1: ok = ((u > a[0]) && (u <= a[1])) || ((v > a[2]) && (v <= a[3])); break;  // cross x1 x2 y1 y2
        case 2:                                                                           // diamond b1..b4
            ok = (u <= 0) ? (-u + a[0] <= v) && (v < u + a[1]) : (0 <= x) ? (u + a[2] <= v) && (v < -u + a[3]) : false;
            break;
        case 3: {  // doughnut r1 r2
            const double mag = u * u + v * v;
            ok = !(mag > a[0] || mag < a[1]);
            break;
        }
        default: ok = true; break;  // square
        }
        if (ok) {
            xy[0] = x;
            xy[1] = y;
            return;
        }
    }
    err |= kErrAperture;  // the reference would loop forever
    xy[0] = 0.5;
    xy[1] = 0.5;
}

__device__ __forceinline__ void ray_for_pixel(const frt_camera& cam, double px, double py, const double* jit,
                                              const double* ap, Ray& r) {
    // renderer.c:95-129; ap = aperture_fn's point in [0,1)^2 (sample_aperture subtracts 0.5, camera.c:85-90)
    double xoff = (px + jit[0]) * cam.pixel_size;
    double yoff = (py + jit[1]) * cam.pixel_size;
    double wx = cam.half_width - xoff, wy = cam.half_height - yoff;
    double p[3] = {wx, wy, -cam.canvas_distance}, pixel[3], origin[3];
    xf_point(cam.inv, p, pixel);
    double q[3] = {(ap[0] - 0.5) * cam.aperture_size, (ap[1] - 0.5) * cam.aperture_size, 0.0};
    xf_point(cam.inv, q, origin);
    double v[3] = {pixel[0] - origin[0], pixel[1] - origin[1], pixel[2] - origin[2]};
    r.o[0] = origin[0];
    r.o[1] = origin[1];
    r.o[2] = origin[2];
    normalize3(v, r.d);
}

// camera ray of sample s of a batch (k_trace level 0 and k_prepare level 0)
__device__ __forceinline__ void camera_ray(const DevScene& S, const Batch& B, int64_t s, Ray& r, uint64_t& key,
                                           unsigned& err) {
    const int64_t pix = B.pixel_begin + s / B.spp;
    const int sub = (int)(s % B.spp);  // sub = v * usteps + u
    const int64_t hs = S.cam.hsize;
    const int64_t row = B.row_begin + (pix / hs) * B.row_stride;
    const int64_t col = pix % hs;
    const uint64_t global_pixel = (uint64_t)(row * hs + col);
    const uint64_t global_sample = global_pixel * (uint64_t)B.spp + (uint64_t)sub;
    double jit[2], ap[2] = {0.5, 0.5};
    if (S.cam.jitter) {
        const int U = (int)S.cam.usteps, V = (int)S.cam.vsteps;
        cmj_point(B.seed, global_pixel, U, V, sub % U, sub / U, jit);
    } else {
        jit[0] = S.sample_table[2 * sub];
        jit[1] = S.sample_table[2 * sub + 1];
    }
    if (S.cam.aperture_size != 0.0) aperture_point(S.cam, B.seed, global_sample, ap, err);
    ray_for_pixel(S.cam, (double)col, (double)row, jit, ap, r);
    key = (global_sample << 12) | 1ull;
}

}  // namespace frt
