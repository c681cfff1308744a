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

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "frt_device.h"
#include "frt_shade.hpp"

namespace frt {

constexpr int kBlock = 256;

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

// what k_shadow reads of a path node, one 64-byte line per node (the shadow
// pass re-reads it from 100 lanes; keeping it apart from the 216-byte NodeRec
// keeps the pass's HBM traffic at one line per node)
struct alignas(64) ShadowHead {
    double over_point[3];
    uint64_t key;
    int32_t material;  // -1: the ray missed
    int32_t pad[5];
};
static_assert(sizeof(ShadowHead) == 64, "ShadowHead layout");

struct QueuedRay {
    double o[3];
    double d[3];
    uint64_t key;
    int32_t parent;
    int32_t slot;
};

enum NodeFlags : int32_t { kReflApplies = 1, kRefrApplies = 2, kMix = 4, kDissolve = 8 };

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
__device__ __forceinline__ int light_row(const frt_light& L, uint64_t seed, uint64_t key, int light, int draw) {
    if (L.rows <= 1) return 0;
    uint64_t h = mix64(seed ^ mix64(key * 0x9e3779b97f4a7c15ULL + (uint64_t)(light * 2 + draw + 1)));
    return (int)(h % (uint64_t)L.rows);
}

struct Batch {
    int64_t sample_begin;  // first global sample index of the batch
    int64_t pixel_begin;   // first pixel (in render order) of the batch
    int64_t num_samples;
    int64_t row_begin, row_stride;
    uint64_t seed;
    int32_t spp, level;
    int32_t remaining;     // path_length - level
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

struct HitRec {
    double t;
    int32_t node;  // -1: miss
    int32_t pad;
    double n1, n2;  // refractive indices either side of the hit (containers)
};

extern __shared__ __align__(16) char frt_walk_smem[];

// closest hit of every ray of one level (level 0: camera rays generated in place)
template <int kFeat>
__global__ void __launch_bounds__(kTraceBlock) k_trace(DevScene S, Batch B, const QueuedRay* __restrict__ q, int64_t n,
                                                       HitRec* __restrict__ hits, unsigned* err) {
    // every lane of the wave takes part in the (wave-coherent) walk
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n;
    Ray r{{0, 0, 0}, {0, 0, 1}};
    unsigned e = 0;
    if (live) {
        if (q == nullptr) {
            uint64_t key;
            camera_ray(S, B, i, r, key, e);
        } else {
            const QueuedRay& qr = q[i];
            for (int k = 0; k < 3; ++k) {
                r.o[k] = qr.o[k];
                r.d[k] = qr.d[k];
            }
        }
    }
    double t;
    double n12[2];
    const int node = walk<false, kFeat>(S, r, 0.0, live, t, frt_walk_smem, e, n12);
    if (live) hits[i] = HitRec{t, node, 0, n12[0], n12[1]};
    if (e) atomicOr(err, e);
}

// prepare_computations + spawn of the reflection / refraction rays (renderer.c:369-605)
__global__ void __launch_bounds__(kBlock) k_prepare(DevScene S, Batch B, const QueuedRay* __restrict__ q, int64_t n,
                                                    const HitRec* __restrict__ hits, NodeRec* __restrict__ rec,
                                                    ShadowHead* __restrict__ heads,
                                                    QueuedRay* __restrict__ next_q, int64_t next_cap,
                                                    unsigned long long* next_count, unsigned long long* counters,
                                                    unsigned* err) {
    const int64_t node = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (node >= n) return;
    Ray r;
    uint64_t key;
    int32_t parent = -1, slot = 0;
    if (q == nullptr) {
        unsigned ce = 0;
        camera_ray(S, B, node, r, key, ce);
    } else {
        const QueuedRay& qr = q[node];
        for (int k = 0; k < 3; ++k) {
            r.o[k] = qr.o[k];
            r.d[k] = qr.d[k];
        }
        key = qr.key;
        parent = qr.parent;
        slot = qr.slot;
    }
    const HitRec hr = hits[node];
    if (hr.node < 0) {
        rec[node].material = -1;
        rec[node].parent = parent;
        rec[node].slot = slot;
        heads[node].material = -1;
        return;
    }
    Hit h{hr.t, -1, -1, hr.node};
    Comps c;
    prepare(S, r, h, c);
    c.n1 = hr.n1;
    c.n2 = hr.n2;
    atomicAdd(counters + 1, 1ull);  // shaded path nodes
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
        if (reflect_applies && (c.refl[0] != 0.0 || c.refl[1] != 0.0 || c.refl[2] != 0.0)) {
            unsigned long long at = atomicAdd(next_count, 1ull);
            if ((int64_t)at < next_cap) {
                QueuedRay qo;
                for (int k = 0; k < 3; ++k) {
                    qo.o[k] = c.over_point[k];
                    qo.d[k] = c.reflectv[k];
                }
                qo.key = base | ((code * 2) & 0xFFFull);
                qo.parent = (int32_t)node;
                qo.slot = 0;
                next_q[at] = qo;
            } else {
                atomicOr(err, kErrQueueOverflow);
            }
        } else if (reflect_applies) {
            atomicAdd(counters, 1ull);
        }
        const bool tf_zero = M.Tf[0] == 0.0 && M.Tf[1] == 0.0 && M.Tf[2] == 0.0;
        if (refract_applies && !tf_zero) {
            unsigned long long at = atomicAdd(next_count, 1ull);
            if ((int64_t)at < next_cap) {
                QueuedRay qo;
                for (int k = 0; k < 3; ++k) {
                    qo.o[k] = c.under_point[k];
                    qo.d[k] = refr_dir[k];
                }
                qo.key = base | ((code * 2 + 1) & 0xFFFull);
                qo.parent = (int32_t)node;
                qo.slot = 1;
                next_q[at] = qo;
            } else {
                atomicOr(err, kErrQueueOverflow);
            }
        } else if (refract_applies) {
            atomicAdd(counters, 1ull);
        }
    }
    nr.flags = flags;
    rec[node] = nr;
    ShadowHead hd;
    for (int k = 0; k < 3; ++k) hd.over_point[k] = c.over_point[k];
    hd.key = key;
    hd.material = c.material;
    for (int k = 0; k < 5; ++k) hd.pad[k] = 0;
    heads[node] = hd;
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
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = tid < n * samples_per_node;
    int64_t node = 0;
    int light = 0;
    bool live = false;
    Ray r{{0, 0, 0}, {0, 0, 1}};
    double distance = 0.0;
    if (valid) {
        node = tid / samples_per_node;
        const int j = (int)(tid % samples_per_node);
        light = j_light[j];
        const int pt = j_point[j];
        const ShadowHead* nr = shead + node;
        if (nr->material >= 0) {
            live = true;
            const frt_light& L = S.lights[light];
            const int row = light_row(L, B.seed, nr->key, light, 0);
            const double* lp = S.light_points + L.points + 3 * ((int64_t)row * L.num_samples + pt);
            // is_shadowed (renderer.c:74-93)
            double v[3] = {lp[0] - nr->over_point[0], lp[1] - nr->over_point[1], lp[2] - nr->over_point[2]};
            distance = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            r.o[0] = nr->over_point[0];
            r.o[1] = nr->over_point[1];
            r.o[2] = nr->over_point[2];
            normalize3(v, r.d);
        }
    }
    // every lane of the wave takes part in the (wave-coherent) walk
    unsigned e = 0;
    double unused;
#ifdef FRT_EXPERIMENT_NOWALK
    const bool lit = live && distance > 0.5;
#else
    const bool lit = walk<true, kFeat>(S, r, distance, live, unused, frt_walk_smem, e) == 0 && live;
#endif
    if (e) atomicOr(err, e);
    // segmented wave reduction: lanes with the same (node, light) are contiguous
    const int lane = threadIdx.x & 63;
    const int64_t key = valid ? node * S.num_lights + light : -1 - (int64_t)lane;
    const int64_t prev = __shfl_up(key, 1, 64);
    const bool head = lane == 0 || prev != key;
    const unsigned long long heads = __ballot(head);
    const unsigned long long lits = __ballot(lit);
    if (valid && head) {
        const unsigned long long above = lane == 63 ? 0ull : (heads >> (lane + 1)) << (lane + 1);
        const int next = above ? __ffsll((long long)above) - 1 : 64;
        const unsigned long long seg = (next >= 64 ? ~0ull : ((1ull << next) - 1)) & ~((1ull << lane) - 1);
        const int c = __popcll(lits & seg);
        if (c) atomicAdd(counts + key, c);
    }
}

// lighting_microfacet (renderer.c:895-979) per light, summed as shade_hit does (renderer.c:704-725)
__global__ void __launch_bounds__(kBlock) k_shade(DevScene S, Batch B, const NodeRec* __restrict__ rec, int64_t n,
                                                  const int32_t* __restrict__ counts, double* __restrict__ surface) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NodeRec& nr = rec[i];
    if (nr.material < 0) return;
    double sA[3] = {0, 0, 0}, sD[3] = {0, 0, 0}, sS[3] = {0, 0, 0};
    if (S.cfg.include_direct) {
        for (int li = 0; li < S.num_lights; ++li) {
            const frt_light& L = S.lights[li];
            double inten;
            if (L.type == FRT_AREA_LIGHT || L.type == FRT_CIRCLE_LIGHT) {
                inten = (double)counts[i * S.num_lights + li] / (double)L.num_samples;  // light.c:229-242
            } else {
                inten = counts[i * S.num_lights + li] ? 1.0 : 0.0;  // light.c:245-251
            }
            double amb[3], cA[3] = {0, 0, 0}, cD[3] = {0, 0, 0}, cS[3] = {0, 0, 0};
            for (int k = 0; k < 3; ++k) amb[k] = nr.Ka[k] * L.intensity[k];
            if (!feq(inten, 0.0)) {
                if (S.cfg.include_diffuse || S.cfg.include_spec_highlight) {
                    const int row = light_row(L, B.seed, nr.key, li, 1);
                    const double* pts = S.light_points + L.points + 3 * (int64_t)row * L.num_samples;
                    double ned = 0.0;
                    if (S.cfg.include_spec_highlight) ned = dot3(nr.normalv, nr.eyev);
                    double dacc[3] = {0, 0, 0}, sacc[3] = {0, 0, 0};
                    for (int p = 0; p < L.num_samples; ++p) {
                        const double* lp = pts + 3 * p;
                        double diff[3] = {lp[0] - nr.over_point[0], lp[1] - nr.over_point[1], lp[2] - nr.over_point[2]};
                        double lv[3];
                        normalize3(diff, lv);
                        double ldn = dot3(lv, nr.normalv);
                        if (S.cfg.include_diffuse && ldn >= 0.0) {
                            for (int k = 0; k < 3; ++k) {
                                double cc = nr.Kd[k] * L.intensity[k];
                                cc *= ldn;
                                dacc[k] += cc;
                            }
                        }
                        if (S.cfg.include_spec_highlight && ldn >= 0.0) {
                            double ndl = dot3(nr.normalv, lv);
                            double tmp[3] = {lv[0] + nr.eyev[0], lv[1] + nr.eyev[1], lv[2] + nr.eyev[2]}, hv[3];
                            normalize3(tmp, hv);
                            double ndh = fmax(0.0, dot3(nr.normalv, hv));
                            double edh_inv = 1.0 / fmax(0.0, dot3(nr.eyev, hv));
                            double ldh = dot3(lv, hv);
                            double dist_term = (nr.Ns + 2) * pow(ndh, nr.Ns) * 0.5 * k1Pi;
                            double gc = 2.0 * ndh * edh_inv;
                            double geo = fmin(1.0, fmin(gc * ned, gc * ndl));
                            double factor = pow(1.0 - ldh, 5.0);
                            double brdf = dist_term * geo / (4.0 * ndl * ned);
                            for (int k = 0; k < 3; ++k) {
                                double f = nr.Ks[k] + (1.0 - nr.Ks[k]) * factor;
                                sacc[k] += f * L.intensity[k] * brdf;
                            }
                        }
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
    double* out = surface + 12 * i;
    for (int k = 0; k < 3; ++k) {
        out[k] = sA[k];
        out[4 + k] = sD[k];
        out[8 + k] = sS[k];
    }
    out[3] = out[7] = out[11] = 0.0;
}

// bottom-up combine of one level (shade_hit's specular block, renderer.c:773-822)
__global__ void __launch_bounds__(kBlock) k_combine(const NodeRec* __restrict__ rec, int64_t n,
                                                    const double* __restrict__ surface,
                                                    const double* __restrict__ child,
                                                    double* __restrict__ parent_child, double* __restrict__ sample_out,
                                                    const frt_material* __restrict__ mats, int32_t include_specular) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NodeRec& nr = rec[i];
    double col[12];
    if (nr.material < 0) {
        for (int k = 0; k < 12; ++k) col[k] = 0.0;
    } else {
        const double* s = surface + 12 * i;
        for (int k = 0; k < 12; ++k) col[k] = s[k];
        if (include_specular) {
            const frt_material& M = mats[nr.material];
            const double* R = child + 24 * i;
            const double* T = R + 12;
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
    double* dst = nr.parent >= 0 ? parent_child + 24 * (int64_t)nr.parent + 12 * nr.slot : sample_out + 12 * i;
    if (nr.parent >= 0 && nr.material < 0) return;  // a missed child leaves its zeroed slot
    for (int k = 0; k < 12; ++k) dst[k] = col[k];
}

// pixel_multi_sample + render_multi_helper's (A+D+S)/3 (renderer.c:132-181, 216-233)
__global__ void __launch_bounds__(kBlock) k_resolve(const double* __restrict__ sample_col, int64_t npix, int32_t spp,
                                                    double* __restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    double acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const double* s = sample_col + 12 * p * spp;
    for (int k = 0; k < spp; ++k)
        for (int c = 0; c < 12; ++c) acc[c] += s[12 * k + c];
    const double total = (double)spp;
    for (int c = 0; c < 12; ++c) acc[c] *= 1.0 / total;
    double* o = out + 4 * p;
    for (int k = 0; k < 3; ++k) {
        double v = 0.0 + acc[k];
        v += acc[4 + k];
        v += acc[8 + k];
        v *= 1.0 / 3.0;
        o[k] = v;
    }
    o[3] = 0.0;
}

}  // namespace frt

// ======================================================================
// host side: scene upload, buffer management, frame driver, C ABI
// ======================================================================

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
    // work buffers (grow on demand)
    struct Level {
        frt::NodeRec* rec = nullptr;
        frt::ShadowHead* head = nullptr;
        frt::QueuedRay* q = nullptr;
        double* surface = nullptr;
        double* child = nullptr;
        int32_t* counts = nullptr;
        int64_t cap = 0;
    };
    std::vector<Level> levels;
    frt::HitRec* hits = nullptr;  // closest hits of the level being traced
    int64_t hits_cap = 0;
    double* sample_col = nullptr;
    int64_t sample_cap = 0;
    double* out_dev = nullptr;
    int64_t out_cap = 0;
    unsigned long long* counters = nullptr;  // [0..15] queue counts per level, [16] pruned
    unsigned* err = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct Mark {
        int slot;
        size_t a, b;
    };
    std::vector<hipEvent_t> ev_pool;
    std::vector<Mark> ev_marks;
    size_t ev_used = 0;
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

extern "C" {

int frt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* frt_last_error(void) { return g_last_error.c_str(); }

int frt_scene_upload(const frt_scene* sc, int device, frt_scene_handle** out) {
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
    }
    if (rc) {
        frt_scene_release(h);
        return -1;
    }
    {
        // walk visit records (frt_traverse.hpp WalkNode)
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
        std::vector<frt::WalkNode> wn((size_t)std::max(1, sc->num_nodes));
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
            for (int k = 0; k < 6; ++k) w.bbox[k] = nd.bbox[k];
            const double* mi = nd.xform >= 0 ? sc->xforms + 16 * (size_t)nd.xform : nullptr;
            if (mi)
                for (int k = 0; k < 12; ++k) w.m[k] = mi[k];
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
        S.wn = upload(h, wn.data(), wn.size(), rc);
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
        h->lds_bytes = (size_t)frt::walk_lds_bytes(list_cap, comp_depth, xf_depth);
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
#ifdef FRT_WALK_STATS
    if (hipMalloc((void**)&h->S.dbg, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(h->S.dbg, 0, 16 * sizeof(unsigned long long)) != hipSuccess) {
        frt_scene_release(h);
        return fail("frt_scene_upload: debug counters");
    }
#endif
    if (hipStreamCreate(&h->stream) != hipSuccess || hipMalloc((void**)&h->counters, 32 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void**)&h->err, sizeof(unsigned)) != hipSuccess || hipEventCreate(&h->ev[0]) != hipSuccess ||
        hipEventCreate(&h->ev[1]) != hipSuccess) {
        frt_scene_release(h);
        return fail("frt_scene_upload: stream / counter allocation failed");
    }
    h->levels.resize((size_t)std::max(1, sc->config.path_length + 2));
    *out = h;
    return 0;
}

void frt_scene_release(frt_scene_handle* h) {
    if (!h) return;
    hip_ignore(hipSetDevice(h->device));
    for (void* p : h->owned) hip_ignore(hipFree(p));
    for (auto& L : h->levels) {
        hip_ignore(hipFree(L.rec));
        hip_ignore(hipFree(L.head));
        hip_ignore(hipFree(L.q));
        hip_ignore(hipFree(L.surface));
        hip_ignore(hipFree(L.child));
        hip_ignore(hipFree(L.counts));
    }
    hip_ignore(hipFree(h->hits));
    hip_ignore(hipFree(h->sample_col));
    hip_ignore(hipFree(h->out_dev));
    hip_ignore(hipFree(h->counters));
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
    hip_ignore(hipFree(L.rec));
    hip_ignore(hipFree(L.head));
    L.head = nullptr;
    hip_ignore(hipFree(L.q));
    hip_ignore(hipFree(L.surface));
    hip_ignore(hipFree(L.child));
    hip_ignore(hipFree(L.counts));
    L.rec = nullptr;
    L.q = nullptr;
    L.surface = nullptr;
    L.child = nullptr;
    L.counts = nullptr;
    FRT_HIP(hipMalloc((void**)&L.rec, nc * sizeof(frt::NodeRec)));
    FRT_HIP(hipMalloc((void**)&L.head, nc * sizeof(frt::ShadowHead)));
    FRT_HIP(hipMalloc((void**)&L.q, nc * sizeof(frt::QueuedRay)));
    FRT_HIP(hipMalloc((void**)&L.surface, nc * 12 * sizeof(double)));
    FRT_HIP(hipMalloc((void**)&L.child, nc * 24 * sizeof(double)));
    FRT_HIP(hipMalloc((void**)&L.counts, nc * std::max(1, h->S.num_lights) * sizeof(int32_t)));
    L.cap = nc;
    return 0;
}

static inline unsigned grid_for(int64_t n, int block = frt::kBlock) { return (unsigned)((n + block - 1) / block); }

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
        st->kernel_ms[m.slot] += ms;
        st->kernel_launches[m.slot] += 1;
    }
    h->ev_marks.clear();
    h->ev_used = 0;
}

}  // extern "C"

// scene-specialised traversal kernels: the template instance without CSG
// frames / the quartic keeps register pressure down for scenes that lack them
template <int F>
static void launch_trace_f(frt_scene_handle* h, const frt::Batch& B, const frt::QueuedRay* q, int64_t n) {
    hipLaunchKernelGGL(frt::k_trace<F>, dim3(grid_for(n, frt::kTraceBlock)), dim3(frt::kTraceBlock), h->lds_bytes,
                       h->stream, h->S, B, q, n, h->hits, h->err);
}

static void launch_trace(frt_scene_handle* h, const frt::Batch& B, const frt::QueuedRay* q, int64_t n) {
    switch (h->S.features & 3) {
    case 0: launch_trace_f<0>(h, B, q, n); break;
    case 1: launch_trace_f<1>(h, B, q, n); break;
    case 2: launch_trace_f<2>(h, B, q, n); break;
    default: launch_trace_f<3>(h, B, q, n); break;
    }
}

template <int F>
static void launch_shadow_f(frt_scene_handle* h, const frt::Batch& B, const frt::ShadowHead* rec, int64_t n, int32_t* counts) {
    const int64_t work = n * h->samples_per_node;
    hipLaunchKernelGGL(frt::k_shadow<F>, dim3(grid_for(work, frt::kTraceBlock)), dim3(frt::kTraceBlock), h->lds_bytes,
                       h->stream, h->S, B, rec, n, h->j_light, h->j_point, h->samples_per_node, counts, h->err);
}

static void launch_shadow(frt_scene_handle* h, const frt::Batch& B, const frt::ShadowHead* rec, int64_t n, int32_t* counts) {
    switch (h->S.features & 3) {
    case 0: launch_shadow_f<0>(h, B, rec, n, counts); break;
    case 1: launch_shadow_f<1>(h, B, rec, n, counts); break;
    case 2: launch_shadow_f<2>(h, B, rec, n, counts); break;
    default: launch_shadow_f<3>(h, B, rec, n, counts); break;
    }
}

extern "C" {

#ifdef FRT_WALK_STATS
// debug builds: dump the walk counters accumulated so far to stderr
static void dump_walk_stats(frt_scene_handle* h) {
    unsigned long long c[16];
    if (hipMemcpy(c, h->S.dbg, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return;
    const char* names[8] = {"composite_visits", "leaf_visits", "active_lane_visits", "jumps", "walks", "live_lanes",
                            "prefilter_rejects", "lanes_tested"};
    for (int k = 0; k < 2; ++k) {
        std::fprintf(stderr, "walk stats (%s):", k == 0 ? "shadow" : "closest");
        for (int j = 0; j < 8; ++j) std::fprintf(stderr, " %s=%llu", names[j], c[8 * k + j]);
        std::fprintf(stderr, "\n");
    }
}
#endif

static int render_impl(frt_scene_handle* h, const frt_frame_params* P, double* dev_out, frt_frame_stats* st) {
    using namespace frt;
    FRT_HIP(hipSetDevice(h->device));
    const int64_t hs = h->S.cam.hsize;
    const int64_t stride = P->row_stride > 0 ? P->row_stride : 1;
    int64_t nrows = 0;
    for (int64_t r = P->row_begin; r < P->row_end; r += stride) nrows++;
    const int64_t npix = nrows * hs;
    const int32_t spp = (int32_t)(h->S.cam.usteps * h->S.cam.vsteps);
    if (spp <= 0) return fail("render: usteps*vsteps must be positive");
    int64_t batch = P->batch_samples > 0 ? P->batch_samples : (int64_t)1 << 21;
    int64_t pix_per_batch = std::max<int64_t>(1, batch / spp);
    const int path = h->S.cfg.path_length;
    if (st) {
        std::memset(st, 0, sizeof(*st));
        (void)hipEventRecord(h->ev[0], h->stream);
    }
    FRT_HIP(hipMemsetAsync(h->err, 0, sizeof(unsigned), h->stream));
    FRT_HIP(hipMemsetAsync(h->counters, 0, 32 * sizeof(unsigned long long), h->stream));
    unsigned long long host_counters[32];
    for (int64_t p0 = 0; p0 < npix; p0 += pix_per_batch) {
        const int64_t bp = std::min<int64_t>(pix_per_batch, npix - p0);
        const int64_t ns = bp * spp;
        if (grow(&h->sample_col, h->sample_cap, ns * 12)) return -1;
        if (ensure_level(h, 0, ns)) return -1;
        Batch B;
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
        std::vector<int64_t> count(path + 2, 0);
        count[0] = ns;
        FRT_HIP(hipMemsetAsync(h->counters, 0, 16 * sizeof(unsigned long long), h->stream));
        for (int d = 0; d <= path; ++d) {
            const int64_t n = count[d];
            if (n == 0) break;
            B.level = d;
            B.remaining = path - d;
            auto& L = h->levels[d];
            if (ensure_level(h, d + 1, std::max<int64_t>(2 * n, 1024))) return -1;
            auto& N = h->levels[d + 1];
            FRT_HIP(hipMemsetAsync(L.child, 0, (size_t)n * 24 * sizeof(double), h->stream));
            FRT_HIP(hipMemsetAsync(L.counts, 0, (size_t)n * std::max(1, h->S.num_lights) * sizeof(int32_t), h->stream));
            if (grow(&h->hits, h->hits_cap, n)) return -1;
            const QueuedRay* q = d == 0 ? nullptr : L.q;
            {
                KTimer t(h, st, d == 0 ? 5 : 0);
                launch_trace(h, B, q, n);
                FRT_HIP(hipGetLastError());
            }
            {
                KTimer t(h, st, 6);
                hipLaunchKernelGGL(k_prepare, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, q, n, h->hits,
                                   L.rec, L.head, N.q, N.cap, h->counters + d + 1, h->counters + 16, h->err);
                FRT_HIP(hipGetLastError());
            }
            if (h->S.cfg.include_direct && h->samples_per_node > 0) {
                KTimer t(h, st, 1);
                launch_shadow(h, B, L.head, n, L.counts);
                FRT_HIP(hipGetLastError());
            }
            {
                KTimer t(h, st, 2);
                hipLaunchKernelGGL(k_shade, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->S, B, L.rec, n, L.counts,
                                   L.surface);
                FRT_HIP(hipGetLastError());
            }
            FRT_HIP(hipMemcpyAsync(host_counters, h->counters, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                   h->stream));
            FRT_HIP(hipStreamSynchronize(h->stream));
            int64_t next = (int64_t)host_counters[d + 1];
            if (next > N.cap) {
                unsigned e = kErrQueueOverflow;
                FRT_HIP(hipMemcpyAsync(h->err, &e, sizeof(unsigned), hipMemcpyHostToDevice, h->stream));
                next = N.cap;
            }
            count[d + 1] = d < path ? next : 0;
            if (st) {
                if (d > 0) st->secondary_rays += (uint64_t)n;
                else st->primary_rays += (uint64_t)n;
            }
        }
        for (int d = path; d >= 0; --d) {
            const int64_t n = count[d];
            if (n == 0) continue;
            KTimer t(h, st, 3);
            double* parent_child = d > 0 ? h->levels[d - 1].child : nullptr;
            hipLaunchKernelGGL(k_combine, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, h->levels[d].rec, n,
                               h->levels[d].surface, h->levels[d].child, parent_child, h->sample_col, h->S.materials,
                               h->S.cfg.include_specular);
            FRT_HIP(hipGetLastError());
        }
        {
            KTimer t(h, st, 4);
            hipLaunchKernelGGL(k_resolve, dim3(grid_for(bp)), dim3(kBlock), 0, h->stream, h->sample_col, bp, spp,
                               dev_out + 4 * p0);
            FRT_HIP(hipGetLastError());
        }
    }
    FRT_HIP(hipMemcpyAsync(host_counters, h->counters, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    unsigned err = 0;
    FRT_HIP(hipMemcpyAsync(&err, h->err, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    if (st) (void)hipEventRecord(h->ev[1], h->stream);
    FRT_HIP(hipStreamSynchronize(h->stream));
    if (st) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
        st->render_ms = ms;
        st->pruned_secondary = host_counters[16];
        st->hits = host_counters[17];
        st->shadow_rays = h->S.cfg.include_direct ? host_counters[17] * (uint64_t)h->samples_per_node : 0;
        // DESIGN.md byte model: per shaded node its 64-byte ShadowHead read + one 4-byte count per light written
        st->shadow_kernel_bytes =
            h->S.cfg.include_direct && h->samples_per_node > 0 ? (double)host_counters[17] * (64.0 + 4.0 * h->S.num_lights) : 0.0;
        st->errors = err;
        collect_timings(h, st);
    }
#ifdef FRT_WALK_STATS
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

}  // extern "C"
