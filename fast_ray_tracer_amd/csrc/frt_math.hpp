// frt-mi355x device math: binary64 vector helpers and the analytic
// primitive tests, in the reference's operation order so that device results
// match the reference bit for bit wherever only + - * / sqrt are involved.
// Compiled with -ffp-contract=off (no FMA fusion), like the reference's
// ISO-C build.
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (frt_jit.cpp) provides the HIP runtime and fixed-width types itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "frt_device.h"

namespace frt {

constexpr double kEps = 0.00001;       // reference linalg.h:7
constexpr double kEqnEps = 1e-9;       // reference Roots3And4.c:36
constexpr double kPi = 3.14159265358979323846;
constexpr double k1Pi = 0.31830988618379067154;

struct Ray {
    double o[3];  // w = 1 implicitly
    double d[3];  // w = 0 implicitly
};

struct Hit {
    double t, u, v;
    int node;
};

__device__ __forceinline__ bool feq(double a, double b) { return fabs(a - b) < kEps; }

__device__ __forceinline__ double dot3(const double* a, const double* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// The compiler's own correctly rounded binary64 sqrt(x) and 1 / y sequences for gfx950 (v_rsq_f64 / v_rcp_f64
// and their Newton steps, instruction for instruction) without their range steps: sqrt's scaling of
// x < 2^-767 and its +-0 / +inf pass-through, division's v_div_scale (no scaling: the exponents are far
// from the limits), v_div_fmas (a plain fma without scaling) and v_div_fixup (no special value, a positive
// normal quotient). For x in [2^-600, 2^600] (so y = sqrt(x) in [2^-300, 2^300]) they return the same
// values as sqrt() and 1.0 / y; frt_math_selftest compares them on the device.
__device__ __forceinline__ double sqrt_core(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double h = x * r, g = r * 0.5;
    const double e = __builtin_fma(-g, h, 0.5);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(g, e, g);
    double d = __builtin_fma(-h, h, x);
    h = __builtin_fma(d, g, h);
    d = __builtin_fma(-h, h, x);
    return __builtin_fma(d, g, h);
}
__device__ __forceinline__ double recip_core(double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-y, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double rem = __builtin_fma(-y, r, 1.0);  // (the quotient 1.0 * r is r)
    return __builtin_fma(rem, r, r);
}

// vector_normalize (reference linalg.c:141-148): multiply by the reciprocal of the magnitude
__device__ __forceinline__ void normalize3_ref(const double* v, double* r) {
    double inv = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double x = v[0], y = v[1], z = v[2];
    r[0] = x * inv;
    r[1] = y * inv;
    r[2] = z * inv;
}
// the same values; a wave whose squared magnitudes all lie in [2^-600, 2^600] takes the core sequences
__device__ __forceinline__ void normalize3(const double* v, double* r) {
    const double m2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    double inv;
    if (__ballot(!(m2 >= 0x1p-600 && m2 <= 0x1p600)) == 0ull)
        inv = recip_core(sqrt_core(m2));
    else
        inv = 1.0 / sqrt(m2);
    double x = v[0], y = v[1], z = v[2];
    r[0] = x * inv;
    r[1] = y * inv;
    r[2] = z * inv;
}

// ---- shading-only approximations (lighting_microfacet's per-light-point terms) ----
// The shading's per-light-point terms (lighting_microfacet) take hardware estimates refined by Newton
// steps instead of the correctly rounded operations: the reciprocal magnitude of a normalisation from
// v_rsq_f64, reciprocals and the BRDF quotient from v_rcp_f64, FRT_SHADE_NEWTON steps each (1: relative
// error below 2^-46, 2: within a few ulps; k_math_selftest bounds them on the device) — far inside the
// 1e-4 canvas tolerance; no decision of any walk uses them. A lane whose operand lies outside [2^-600,
// 2^600] (overflow, underflow or a special value in the steps) takes the IEEE operation instead — per
// lane, so a node's result never depends on which other nodes share its wave (the lit-node list's order
// is not deterministic). (FRT_SHADE_FAST=0 builds: the IEEE operations only, A/B runs)
#ifndef FRT_SHADE_FAST
#define FRT_SHADE_FAST 1
#endif
#ifndef FRT_SHADE_NEWTON
#define FRT_SHADE_NEWTON 1
#endif
__device__ __forceinline__ bool shade_in_range(double x) { return x >= 0x1p-600 && x <= 0x1p600; }
// 1 / sqrt(x): v_rsq_f64 (~2^-24) and Newton steps r += r (1/2 - x r^2 / 2)
__device__ __forceinline__ double rsqrt_nr(double x) {
    double r = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int k = 0; k < FRT_SHADE_NEWTON; ++k) {
        const double t = x * r, g = r * 0.5;
        r = __builtin_fma(r, __builtin_fma(-g, t, 0.5), r);
    }
    return r;
}
// 1 / y: v_rcp_f64 (~2^-24) and Newton steps r += r (1 - y r)
__device__ __forceinline__ double rcp_nr(double y) {
    double r = __builtin_amdgcn_rcp(y);
#pragma unroll
    for (int k = 0; k < FRT_SHADE_NEWTON; ++k) r = __builtin_fma(r, __builtin_fma(-y, r, 1.0), r);
    return r;
}
// 1 / sqrt(m2) with the IEEE operations where the estimate's steps may leave range. (The slow paths below sit
// behind a wave-uniform branch: the compiler would otherwise if-convert them and every lane would pay for the
// IEEE division in every light point.)
__device__ __forceinline__ double rsqrt_shade(double m2) {
    if (!FRT_SHADE_FAST) return 1.0 / sqrt(m2);
    double inv = rsqrt_nr(m2);
    const bool slow = !shade_in_range(m2);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) inv = 1.0 / sqrt(m2);
    }
    return inv;
}
// vector_normalize (linalg.c:141-148) with the approximate reciprocal magnitude
__device__ __forceinline__ void normalize3_shade(const double* v, double* r) {
    const double m2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double inv = rsqrt_shade(m2);
    r[0] = v[0] * inv;
    r[1] = v[1] * inv;
    r[2] = v[2] * inv;
}
// 1 / y and a / b (a >= 0)
__device__ __forceinline__ double recip_shade(double y) {
    if (!FRT_SHADE_FAST) return 1.0 / y;
    double r = rcp_nr(y);
    const bool slow = !shade_in_range(y);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) r = 1.0 / y;
    }
    return r;
}
__device__ __forceinline__ double div_shade(double a, double b) {
    if (!FRT_SHADE_FAST) return a / b;
    double q = a * rcp_nr(b);
    const bool slow = !(shade_in_range(b) && (a == 0.0 || shade_in_range(a)));
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) q = a / b;
    }
    return q;
}
// lighting_microfacet's brdf_factor (renderer.c:952-963): D G / (4 (n.l)(n.e)), G = min(1, gc (n.e), gc (n.l)),
// gc = 2 (n.h) / (e.h). FRT_SHADE_MERGE (default 1) takes one reciprocal where the reference divides twice: the
// three candidates of G scaled by e.h > 0 keep their order, so G (e.h) = min(e.h, 2 (n.h)(n.e), 2 (n.h)(n.l)) and
// brdf = D min(..) / ((e.h) 4 (n.l)(n.e)) — a few ulps from the two-quotient form, like the estimates above. A lane
// whose operands leave [2^-600, 2^600] (e.h = 0 among them: the reference's 1 / (e.h) is inf there and G = 1)
// takes the reference's form with IEEE quotients. (FRT_SHADE_MERGE=0 builds: a reciprocal and a quotient, A/B runs)
#ifndef FRT_SHADE_MERGE
#define FRT_SHADE_MERGE 1
#endif
__device__ __forceinline__ double brdf_shade(double D, double ndh, double edh, double ndl, double ned) {
    if (FRT_SHADE_MERGE && FRT_SHADE_FAST) {
        const double g2 = 2.0 * ndh;
        const double a = D * fmin(edh, fmin(g2 * ned, g2 * ndl)), b = edh * (4.0 * ndl * ned);
        double q = a * rcp_nr(b);
        const bool slow = !(shade_in_range(edh) && shade_in_range(b) && (a == 0.0 || shade_in_range(a)));
        if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
            if (slow) {
                const double gc = 2.0 * ndh * (1.0 / edh);
                q = (D * fmin(1.0, fmin(gc * ned, gc * ndl))) / (4.0 * ndl * ned);
            }
        }
        return q;
    }
    const double gc = 2.0 * ndh * recip_shade(edh);
    const double geo = fmin(1.0, fmin(gc * ned, gc * ndl));
    return div_shade(D * geo, 4.0 * ndl * ned);
}

__device__ __forceinline__ void cross3(const double* a, const double* b, double* r) {
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    r[0] = x;
    r[1] = y;
    r[2] = z;
}

// matrix_point_multiply with w = 1 (the m[i3]*1.0 term is exact)
__device__ __forceinline__ void xf_point(const double* m, const double* p, double* r) {
    double x = ((m[0] * p[0] + m[1] * p[1]) + m[2] * p[2]) + m[3];
    double y = ((m[4] * p[0] + m[5] * p[1]) + m[6] * p[2]) + m[7];
    double z = ((m[8] * p[0] + m[9] * p[1]) + m[10] * p[2]) + m[11];
    r[0] = x;
    r[1] = y;
    r[2] = z;
}

// matrix_vector_multiply with w = +0 (kept: it can only change the sign of a zero)
__device__ __forceinline__ void xf_vector(const double* m, const double* v, double* r) {
    double x = ((m[0] * v[0] + m[1] * v[1]) + m[2] * v[2]) + m[3] * 0.0;
    double y = ((m[4] * v[0] + m[5] * v[1]) + m[6] * v[2]) + m[7] * 0.0;
    double z = ((m[8] * v[0] + m[9] * v[1]) + m[10] * v[2]) + m[11] * 0.0;
    r[0] = x;
    r[1] = y;
    r[2] = z;
}

// transpose(m) * n with n.w = 0 (shape_normal_to_world, shapes.c:92-114)
__device__ __forceinline__ void xf_normal_t(const double* m, const double* n, double* r) {
    double x = ((m[0] * n[0] + m[4] * n[1]) + m[8] * n[2]) + m[12] * 0.0;
    double y = ((m[1] * n[0] + m[5] * n[1]) + m[9] * n[2]) + m[13] * 0.0;
    double z = ((m[2] * n[0] + m[6] * n[1]) + m[10] * n[2]) + m[14] * 0.0;
    r[0] = x;
    r[1] = y;
    r[2] = z;
}

// ray transform of the traversal: drops the m[i3] * 0.0 terms of the direction,
// which can only flip the sign of a zero component; the walk's only uses of
// direction components are |d| < EPSILON guards, products and sums, none of
// which can see that sign in a t value or a hit / miss decision
__device__ __forceinline__ Ray xf_ray_walk(const double* m, const Ray& r) {
    Ray t;
    xf_point(m, r.o, t.o);
    t.d[0] = (m[0] * r.d[0] + m[1] * r.d[1]) + m[2] * r.d[2];
    t.d[1] = (m[4] * r.d[0] + m[5] * r.d[1]) + m[6] * r.d[2];
    t.d[2] = (m[8] * r.d[0] + m[9] * r.d[1]) + m[10] * r.d[2];
    return t;
}

__device__ __forceinline__ Ray xf_ray(const double* m, const Ray& r) {
    Ray t;
    xf_point(m, r.o, t.o);
    xf_vector(m, r.d, t.d);
    return t;
}

// check_axis / bbox_check_axis (cube.c:16-53, bounding_box.c:124-162)
// max / min of slab values, which are never NaN (finite quotients or the +-inf
// of the EPSILON branch): fmax / fmin as in the reference, one v_max_f64 /
// v_min_f64 each (arithmetic results need no IEEE-mode canonicalisation)
__device__ __forceinline__ double max2(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ double min2(double a, double b) { return __builtin_fmin(a, b); }

// check_axis / bbox_check_axis (cube.c:16-53, bounding_box.c:124-162), branch-free:
// for |d| < EPSILON the reference takes n * INFINITY with NaN (n == 0) mapped to
// (n < 0 ? -inf : inf) — i.e. exactly (n < 0 ? -inf : inf) for every n
__device__ __forceinline__ void slab(double o, double d, double lo, double hi, double& a, double& b) {
    const double nl = lo - o, nh = hi - o;
    double t0 = nl / d, t1 = nh / d;
    if (!(fabs(d) >= kEps)) {
        t0 = nl < 0 ? -__builtin_inf() : __builtin_inf();
        t1 = nh < 0 ? -__builtin_inf() : __builtin_inf();
    }
    a = min2(t0, t1);  // the reference's "if (t0 > t1) swap" for NaN-free values
    b = max2(t0, t1);
}

// bbox_intersect (bounding_box.c:164-177); also reports the entry / exit t
__device__ __forceinline__ bool box_range(const double* bb, const Ray& r, double& tmin, double& tmax) {
    double x0, x1, y0, y1, z0, z1;
    slab(r.o[0], r.d[0], bb[0], bb[3], x0, x1);
    slab(r.o[1], r.d[1], bb[1], bb[4], y0, y1);
    slab(r.o[2], r.d[2], bb[2], bb[5], z0, z1);
    tmin = max2(max2(x0, y0), z0);
    tmax = min2(min2(x1, y1), z1);
    return tmin <= tmax;
}

// ---- filtered box tests (decisions only; no IEEE division on the fast path) ----
// v_rcp_f64 is good to ~2^-24 (tools/microbench/rcp_accuracy.hip); each Newton
// step squares the error: one step <= 2^-48, two steps correctly rounded on 4M samples.
template <int kSteps>
__device__ __forceinline__ double recip(double d) {
    double r = __builtin_amdgcn_rcp(d);
#pragma unroll
    for (int k = 0; k < kSteps; ++k) r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    return r;
}

__device__ __forceinline__ double finite_abs(double x) { return __builtin_isinf(x) ? 0.0 : fabs(x); }

constexpr double kFilterRel = 0x1p-40;  // decision margin; the approximations are good to 2^-47

// The reference's box decision (bounding_box_intersects, bounding_box.c:164-175),
// exactly: slab t values from an approximate reciprocal (rc[a] ~ 1/d[a], one
// Newton step), the |d| < EPSILON branch exact as in slab(); the comparison is
// trusted when it clears a margin far above the approximation error, otherwise
// the IEEE-division box_range() decides. tmin / tmax return the approximate values.
__device__ __forceinline__ bool box_decide(const double* bb, const Ray& r, const double* rc, double& tmin,
                                           double& tmax) {
    double lo3[3], hi3[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double nl = bb[a] - r.o[a], nh = bb[a + 3] - r.o[a];
        double t0 = nl * rc[a], t1 = nh * rc[a];
        if (!(fabs(r.d[a]) >= kEps)) {
            t0 = nl < 0 ? -__builtin_inf() : __builtin_inf();
            t1 = nh < 0 ? -__builtin_inf() : __builtin_inf();
        }
        lo3[a] = min2(t0, t1);
        hi3[a] = max2(t0, t1);
    }
    tmin = max2(max2(lo3[0], lo3[1]), lo3[2]);
    tmax = min2(min2(hi3[0], hi3[1]), hi3[2]);
    const double margin = kFilterRel * (finite_abs(tmin) + finite_abs(tmax));
    if (tmin <= tmax - margin) return true;
    if (tmin > tmax + margin) return false;
    double a, b;
    return box_range(bb, r, a, b);
}

// pow(x, y) of the microfacet distribution term (renderer.c:966): an integral
// exponent (the usual Ns) by binary exponentiation — a few ulps from the
// reference's libm pow, like the device pow it replaces, at a fraction of its
// cost; other exponents through pow
__device__ __attribute__((noinline)) double pow_general(double x, double y) { return pow(x, y); }

__device__ __forceinline__ double pow_ns(double x, double y) {
    if (y >= 0.0 && y < 4096.0 && y == __builtin_floor(y)) {
        const unsigned e = (unsigned)y;
        double r = 1.0, b = x;
        const unsigned e0 = (unsigned)__builtin_amdgcn_readfirstlane((int)e);
        if (__ballot(e != e0) == 0ull) {
            // one exponent in the whole wave (one material's Ns): a scalar loop over its bits, the same
            // products in the same order as below, without the selects, the first product (1 x b is exact)
            // and the squaring past the top bit
            bool first = true;
            for (unsigned k = 0; (e0 >> k) != 0u; ++k) {
                if ((e0 >> k) & 1u) {
                    r = first ? b : r * b;
                    first = false;
                }
                if ((e0 >> (k + 1)) == 0u) break;
                b *= b;
            }
            return r;
        }
        // several exponents: every lane runs the squarings of the wave's largest one (uniform trip count)
        unsigned emax = e;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) emax = max(emax, (unsigned)__shfl_xor((int)emax, o, 64));
        const unsigned bits = 32u - (unsigned)__clz((int)emax);
#pragma nounroll
        for (unsigned k = 0; k < bits; ++k) {
            r = (e >> k) & 1u ? r * b : r;
            b *= b;
        }
        return r;
    }
    return pow_general(x, y);
}

// pow_ns's exponent analysis hoisted out of a loop whose exponent stays the same (the shading's light points:
// the node's Ns). pow_plan runs where every lane of the loop is active; pow_apply(x, y, P) returns pow_ns(x, y)
// bit for bit: the same products in the same order, by the one-exponent scalar loop when every lane of the wave
// has the same integral exponent, else by the several-exponent loop (the squarings of the wave's largest
// exponent: squarings past a lane's top bit leave its product alone), pow_general for the rest.
struct PowPlan {
    bool uniform;   // every lane: an integral exponent in [0, 4096), the same one (e0)
    bool integral;  // this lane's exponent is integral and in range
    unsigned e0;    // (uniform) the exponent
    unsigned bits;  // (several) bit length of the wave's largest integral exponent
};
__device__ __forceinline__ PowPlan pow_plan(double y) {
    PowPlan P;
    P.integral = y >= 0.0 && y < 4096.0 && y == __builtin_floor(y);
    const unsigned e = P.integral ? (unsigned)y : 0u;
    P.e0 = (unsigned)__builtin_amdgcn_readfirstlane((int)e);
    P.uniform = __ballot(!P.integral || e != P.e0) == 0ull;
    P.bits = 0;
    if (!P.uniform) {
        unsigned emax = e;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) emax = max(emax, (unsigned)__shfl_xor((int)emax, o, 64));
        P.bits = 32u - (unsigned)__clz((int)emax);
    }
    return P;
}
__device__ __forceinline__ double pow_apply(double x, double y, const PowPlan& P) {
    double r = 1.0, b = x;
    if (P.uniform) {
        // over the set bits (scalar control only: squarings up to the next set bit, then one product; no
        // per-lane selects, which the bit-by-bit loop compiled to)
        unsigned m = P.e0;
        if (m == 0u) return 1.0;
        unsigned pos = (unsigned)__builtin_ctz(m);
        for (unsigned k = 0; k < pos; ++k) b *= b;
        r = b;  // (the first product, 1 x b, is exact)
        m &= m - 1u;
        while (m != 0u) {
            const unsigned k = (unsigned)__builtin_ctz(m);
            for (; pos < k; ++pos) b *= b;
            r *= b;
            m &= m - 1u;
        }
        return r;
    }
    if (P.integral) {
        const unsigned e = (unsigned)y;
#pragma nounroll
        for (unsigned k = 0; k < P.bits; ++k) {
            r = (e >> k) & 1u ? r * b : r;
            b *= b;
        }
        return r;
    }
    return pow_general(x, y);
}

// ---- wave-aggregated counters ----
// One atomic per wave instead of one per lane: a single shared counter taking
// an atomic from every path node serialises at its L2 channel (the queue
// appends of k_prepare cost more than the rest of the kernel). Every active
// lane of the wave must call it at the same point; returns this lane's slot
// (base + rank among the lanes with want), meaningless where want is false.
__device__ __forceinline__ unsigned long long wave_append(unsigned long long* ctr, bool want) {
    const unsigned long long m = __ballot(want);
    if (m == 0) return 0;
    const int leader = __builtin_ctzll(m);
    const int lane = (int)(threadIdx.x & 63);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)base, leader);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(base >> 32), leader);
    return (((unsigned long long)hi << 32) | lo) + (unsigned long long)__popcll(m & ((1ull << lane) - 1));
}

// statistics counter: one atomic per wave whose result nobody waits for
__device__ __forceinline__ void wave_count(unsigned long long* ctr, bool cond) {
    const unsigned long long m = __ballot(cond);
    if (m != 0 && (int)(threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(ctr, (unsigned long long)__popcll(m));
}

// ---- binary32 box decisions with a rigorous error bound ----
// The reference decides a box hit as tmin <= tmax over binary64 slab quotients
// (lo - o) / d (bounding_box.c:124-175). Here the quotients come from binary32
// operands: o' = f32(o), lo' = f32(lo), r = v_rcp_f32(f32(d)) (1 ulp), t' = (lo' - o') * r.
// Per axis |t' - t| <= (|lo' - lo| + |o' - o| + u|lo - o|)/|d| + |t|(|r d - 1|) + u|t'|
//                  <= (2.01 + 3.01 + 1.01) u (|lo| + |o|) / |d| + O(u^2)     (|t| <= (|lo|+|o|)/|d|)
// with u = 2^-24, so with mag = max(|lo|, |hi|) rounded up, every slab value and
// hence tmin / tmax (max / min of them) are within E = 7u max_a (mag_a + |o'_a|) |r_a|
// of the reference's. tmax' - tmin' > 2.01 E proves a hit, < -2.01 E a miss; in
// between the binary64 test decides. The |d| < EPSILON branch (infinite slabs) is
// never taken here: a frame whose f32 direction has a component below kEps32 is
// decided in binary64 throughout (Frame32::exact).
constexpr float kEps32 = 1.00001e-5f;  // |f32(d)| >= kEps32  =>  |d| >= EPSILON
constexpr float kBox32Err = 7.0f * 0x1p-24f;

struct Frame32 {
    float o[3];  // f32(origin)
    float r[3];  // v_rcp_f32(f32(direction))
    bool exact;  // a direction component may be below EPSILON: binary64 decisions only
};

__device__ __forceinline__ void frame32(const Ray& ray, Frame32& f) {
    bool ex = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        f.o[a] = (float)ray.o[a];
        const float d = (float)ray.d[a];
        f.r[a] = __builtin_amdgcn_rcpf(d);
        ex = ex || !(fabsf(d) >= kEps32);
    }
    f.exact = ex;
}

// 1: hit, 0: miss, -1: undecided (take the binary64 test). tmin / tmax: the f32
// estimates, err: their error bound E.
__device__ __forceinline__ int box32(const float* bb, const float* mag, const Frame32& f, float& tmin, float& tmax,
                                     float& err) {
    float lo3[3], hi3[3], e = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t0 = (bb[a] - f.o[a]) * f.r[a];
        const float t1 = (bb[a + 3] - f.o[a]) * f.r[a];
        lo3[a] = fminf(t0, t1);
        hi3[a] = fmaxf(t0, t1);
        e = fmaxf(e, (mag[a] + fabsf(f.o[a])) * fabsf(f.r[a]));
    }
    tmin = fmaxf(fmaxf(lo3[0], lo3[1]), lo3[2]);
    tmax = fminf(fminf(hi3[0], hi3[1]), hi3[2]);
    err = kBox32Err * e + 1e-30f;
    const float diff = tmax - tmin;
    if (diff > 2.01f * err) return 1;
    if (-diff > 2.01f * err) return 0;
    return -1;
}

// Conservative line-vs-box test for the prefilter: false only when the exact
// line misses bb (an inflated parent-space bound of a node) by far more than
// the approximation error. Direction components below 1e-200 count as parallel.
__device__ __forceinline__ bool box_may_hit(const double* bb, const Ray& r, const double* rc, double& tmin,
                                            double& tmax) {
    double lo3[3], hi3[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double nl = bb[a] - r.o[a], nh = bb[a + 3] - r.o[a];
        double t0 = nl * rc[a], t1 = nh * rc[a];
        if (!(fabs(r.d[a]) >= 1e-200)) {  // parallel: inside the slab iff nl <= 0 <= nh
            t0 = nl <= 0 ? -__builtin_inf() : __builtin_inf();
            t1 = nh >= 0 ? __builtin_inf() : -__builtin_inf();
        }
        lo3[a] = min2(t0, t1);
        hi3[a] = max2(t0, t1);
    }
    tmin = max2(max2(lo3[0], lo3[1]), lo3[2]);
    tmax = min2(min2(hi3[0], hi3[1]), hi3[2]);
    return !(tmin > tmax + kFilterRel * (finite_abs(tmin) + finite_abs(tmax)));
}

// origin strictly inside the box: every slab gives t0 < 0 < t1 (signs of IEEE
// quotients are exact; the EPSILON branch gives -inf / +inf), so the reference's
// box test reports a hit with tmin < 0 < tmax — decided without any slab arithmetic
// (all six comparisons evaluated: no short-circuit chain of dependent loads)
__device__ __forceinline__ bool origin_inside(const double* bb, const Ray& r) {
    return (bb[0] < r.o[0]) & (r.o[0] < bb[3]) & (bb[1] < r.o[1]) & (r.o[1] < bb[4]) & (bb[2] < r.o[2]) &
           (r.o[2] < bb[5]);
}

// Could a local direction component (row a of the node's inverse transform
// applied to the parent-frame direction) fall below EPSILON, where the
// reference's slab test switches to its infinite-slab branch? Float estimate
// with an error bound: rows / L1 norms from the upload, df = float(d), dmax = max |df|.
__device__ __forceinline__ bool quirk_possible(const float* mrow, const float* l1, const float* df, float dmax) {
    bool q = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float v = (mrow[3 * a] * df[0] + mrow[3 * a + 1] * df[1]) + mrow[3 * a + 2] * df[2];
        q = q || fabsf(v) < 1.0001e-5f + 0x1p-19f * l1[a] * dmax;
    }
    return q;
}

__device__ __forceinline__ bool box_hit(const double* bb, const Ray& r) {
    double a, b;
    return box_range(bb, r, a, b);
}

// ---- up to four values in registers: appended / read with constant-index
// selects only, so no per-lane scratch array is ever materialised ----
struct Vals4 {
    double v0, v1, v2, v3;
    int n;
    __device__ __forceinline__ void push(double x) {
        v0 = n == 0 ? x : v0;
        v1 = n == 1 ? x : v1;
        v2 = n == 2 ? x : v2;
        v3 = n == 3 ? x : v3;
        ++n;
    }
    __device__ __forceinline__ double at(int i) const { return i == 0 ? v0 : i == 1 ? v1 : i == 2 ? v2 : v3; }
};

// ---- quartic (reference Roots3And4.c:43-244) ----
__device__ __forceinline__ bool is_zero(double x) { return x > -kEqnEps && x < kEqnEps; }

// SolveQuadric (Roots3And4.c:43-71): roots appended to R
__device__ __forceinline__ void solve_quadric(double c0, double c1, double c2, Vals4& R) {
    double p = c1 / (2 * c2);
    double q = c0 / c2;
    double D = p * p - q;
    if (is_zero(D)) {
        R.push(-p);
        return;
    }
    if (D < 0) return;
    double sd = sqrt(D);
    R.push(sd - p);
    R.push(-sd - p);
}

// SolveCubic (Roots3And4.c:74-134) for c[3] = 1 callers: roots appended to R (R.n = 0 on entry)
__device__ __forceinline__ void solve_cubic(double c0, double c1, double c2, double c3, Vals4& R) {
    double A = c2 / c3, B = c1 / c3, C = c0 / c3;
    double sq_A = A * A;
    double p = 1.0 / 3 * (-1.0 / 3 * sq_A + B);
    double q = 1.0 / 2 * (2.0 / 27 * A * sq_A - 1.0 / 3 * A * B + C);
    double cb_p = p * p * p;
    double D = q * q + cb_p;
    double s0, s1 = 0, s2 = 0;
    int num;
    if (is_zero(D)) {
        if (is_zero(q)) {
            s0 = 0;
            num = 1;
        } else {
            double u = cbrt(-q);
            s0 = 2 * u;
            s1 = -u;
            num = 2;
        }
    } else if (D < 0) {
        double phi = 1.0 / 3 * acos(-q / sqrt(-cb_p));
        double t = 2 * sqrt(-p);
        s0 = t * cos(phi);
        s1 = -t * cos(phi + kPi / 3);
        s2 = -t * cos(phi - kPi / 3);
        num = 3;
    } else {
        double sd = sqrt(D);
        double u = cbrt(sd - q);
        double v = -cbrt(sd + q);
        s0 = u + v;
        num = 1;
    }
    double sub = 1.0 / 3 * A;
    R.push(s0 - sub);
    if (num > 1) R.push(s1 - sub);
    if (num > 2) R.push(s2 - sub);
}

// SolveQuartic (Roots3And4.c:137-244) with c[4] the leading coefficient
__device__ __forceinline__ void solve_quartic(double c0, double c1, double c2, double c3, double c4, Vals4& R) {
    R.n = 0;
    double A = c3 / c4, B = c2 / c4, C = c1 / c4, D = c0 / c4;
    double sq_A = A * A;
    double p = -3.0 / 8 * sq_A + B;
    double q = 1.0 / 8 * sq_A * A - 1.0 / 2 * A * B + C;
    double r = -3.0 / 256 * sq_A * sq_A + 1.0 / 16 * sq_A * B - 1.0 / 4 * A * C + D;
    if (is_zero(r)) {
        solve_cubic(q, p, 0, 1, R);
        R.push(0);
    } else {
        Vals4 cub{0, 0, 0, 0, 0};
        solve_cubic(1.0 / 2 * r * p - 1.0 / 8 * q * q, -r, -1.0 / 2 * p, 1, cub);
        double z = cub.v0;
        double u = z * z - r;
        double v = 2 * z - p;
        if (is_zero(u)) u = 0;
        else if (u > 0) u = sqrt(u);
        else return;
        if (is_zero(v)) v = 0;
        else if (v > 0) v = sqrt(v);
        else return;
        solve_quadric(z - u, q < 0 ? -v : v, 1, R);
        solve_quadric(z + u, q < 0 ? v : -v, 1, R);
    }
    double sub = 1.0 / 4 * A;
    R.v0 -= sub;  // unused slots are never read
    R.v1 -= sub;
    R.v2 -= sub;
    R.v3 -= sub;
}

// ---- primitive intersections: hit t values appended in the reference's
// emission order (H.n <= 4); triangles also report the hit's (u, v) ----
struct LeafHits {
    Vals4 t;
    double u, v;
};

// type: enum frt_node_type; p: the leaf's parameters in prim_data
template <bool kTorus = true>
__device__ __forceinline__ void leaf_hits(int type, const double* __restrict__ p, const Ray& r, LeafHits& H) {
    H.t.n = 0;
    H.t.v0 = H.t.v1 = H.t.v2 = H.t.v3 = 0.0;
    switch (type) {
    case FRT_SPHERE: {  // sphere.c:14-39
        double a = dot3(r.d, r.d);
        double b = 2 * dot3(r.d, r.o);
        double c = dot3(r.o, r.o) - 1.0;
        double disc = b * b - 4 * a * c;
        if (disc < 0) return;
        disc = sqrt(disc);
        a = 1.0 / (2 * a);
        H.t.v0 = (-b - disc) * a;
        H.t.v1 = (-b + disc) * a;
        H.t.n = 2;
        return;
    }
    case FRT_CUBE: {  // cube.c:56-77
        double x0, x1, y0, y1, z0, z1;
        slab(r.o[0], r.d[0], -1, 1, x0, x1);
        slab(r.o[1], r.d[1], -1, 1, y0, y1);
        slab(r.o[2], r.d[2], -1, 1, z0, z1);
        double tmin = max2(max2(x0, y0), z0), tmax = min2(min2(x1, y1), z1);
        if (tmin > tmax) return;
        H.t.v0 = tmin;
        H.t.v1 = tmax;
        H.t.n = 2;
        return;
    }
    case FRT_PLANE:  // plane.c:11-24
        if (fabs(r.d[1]) < kEps) return;
        H.t.v0 = -r.o[1] / r.d[1];
        H.t.n = 1;
        return;
    case FRT_TRIANGLE:
    case FRT_SMOOTH_TRIANGLE: {  // triangle.c:11-44
        double dce2[3], p1o[3], oce1[3];
        cross3(r.d, p + FRT_TRI_E2, dce2);
        double det = dot3(p + FRT_TRI_E1, dce2);
        if (fabs(det) < kEps) return;
        double f = 1.0 / det;
        p1o[0] = r.o[0] - p[0];
        p1o[1] = r.o[1] - p[1];
        p1o[2] = r.o[2] - p[2];
        double u = f * dot3(p1o, dce2);
        if (u < 0 || u > 1) return;
        cross3(p1o, p + FRT_TRI_E1, oce1);
        double v = f * dot3(r.d, oce1);
        if (v < 0 || (u + v) > 1) return;
        H.t.v0 = f * dot3(p + FRT_TRI_E2, oce1);
        H.t.n = 1;
        H.u = u;
        H.v = v;
        return;
    }
    case FRT_CYLINDER: {  // cylinder.c:11-87
        double mn = p[0], mx = p[1];
        double a = r.d[0] * r.d[0] + r.d[2] * r.d[2];
        double b = 2 * (r.o[0] * r.d[0] + r.o[2] * r.d[2]);
        double c = r.o[0] * r.o[0] + r.o[2] * r.o[2] - 1;
        if (!feq(a, 0.0)) {
            double disc = b * b - 4 * a * c;
            if (disc < 0) return;
            double sq = sqrt(disc);
            double t0 = (-b - sq) / (2 * a), t1 = (-b + sq) / (2 * a);
            if (t0 > t1) {
                double tt = t0;
                t0 = t1;
                t1 = tt;
            }
            double y0 = r.o[1] + t0 * r.d[1];
            if (mn <= y0 && y0 <= mx) H.t.push(t0);
            double y1 = r.o[1] + t1 * r.d[1];
            if (mn <= y1 && y1 <= mx) H.t.push(t1);
        }
        if (p[2] == 0.0 || feq(r.d[1], 0.0)) return;
        double ta = (mn - r.o[1]) / r.d[1];
        double tb = (mx - r.o[1]) / r.d[1];
        double xa = r.o[0] + ta * r.d[0], za = r.o[2] + ta * r.d[2];
        if (xa * xa + za * za <= 1) H.t.push(ta);
        double xb = r.o[0] + tb * r.d[0], zb = r.o[2] + tb * r.d[2];
        if (xb * xb + zb * zb <= 1) H.t.push(tb);
        return;
    }
    case FRT_CONE: {  // cone.c:11-96
        double mn = p[0], mx = p[1];
        double a = r.d[0] * r.d[0] + r.d[2] * r.d[2] - r.d[1] * r.d[1];
        double b = 2 * (r.o[0] * r.d[0] + r.o[2] * r.d[2] - r.o[1] * r.d[1]);
        double c = r.o[0] * r.o[0] + r.o[2] * r.o[2] - r.o[1] * r.o[1];
        if (feq(a, 0.0)) {
            if (!feq(b, 0.0)) H.t.push(-c / (2 * b));
        } else {
            double disc = b * b - 4 * a * c;
            if (disc < 0) return;
            double sq = sqrt(disc);
            double t0 = (-b - sq) / (2 * a), t1 = (-b + sq) / (2 * a);
            if (t0 > t1) {
                double tt = t0;
                t0 = t1;
                t1 = tt;
            }
            double y0 = r.o[1] + t0 * r.d[1];
            if (mn < y0 && y0 < mx) H.t.push(t0);
            double y1 = r.o[1] + t1 * r.d[1];
            if (mn < y1 && y1 < mx) H.t.push(t1);
        }
        if (p[2] == 0.0 || feq(r.d[1], 0.0)) return;
        double ta = (mn - r.o[1]) / r.d[1];
        double xa = r.o[0] + ta * r.d[0], za = r.o[2] + ta * r.d[2];
        if (xa * xa + za * za <= fabs(mn)) H.t.push(ta);
        double tb = (mx - r.o[1]) / r.d[1];
        double xb = r.o[0] + tb * r.d[0], zb = r.o[2] + tb * r.d[2];
        if (xb * xb + zb * zb <= fabs(mx)) H.t.push(tb);
        return;
    }
    case FRT_TOROID: {  // toroid.c:15-52
        if constexpr (!kTorus) return;
        double r1 = p[0], r2 = p[1];
        double ox = r.o[0], oy = r.o[1], oz = r.o[2];
        double dx = r.d[0], dy = r.d[1], dz = r.d[2];
        double sum_d_sq = dx * dx + dy * dy + dz * dz;
        double e = ox * ox + oy * oy + oz * oz - r1 * r1 - r2 * r2;
        double f = ox * dx + oy * dy + oz * dz;
        double four_a_sq = 4.0 * r1 * r1;
        Vals4 sol;
        solve_quartic(e * e - four_a_sq * (r2 * r2 - oy * oy), 4.0 * f * e + 2.0 * four_a_sq * oy * dy,
                      2.0 * sum_d_sq * e + 4.0 * f * f + four_a_sq * dy * dy, 4.0 * sum_d_sq * f,
                      sum_d_sq * sum_d_sq, sol);
        // the reference appends the roots last to first
        const int n = sol.n;
        H.t.v0 = sol.at(n - 1);
        H.t.v1 = sol.at(n - 2);
        H.t.v2 = sol.at(n - 3);
        H.t.v3 = sol.at(n - 4);
        H.t.n = n;
        return;
    }
    default:
        return;
    }
}

// Cube entries for a shadow-ray decision (cube.c:56-77 + the stop / blocked
// tests of the caller): slab quotients from a one-Newton-step reciprocal
// instead of IEEE divisions. The approximate (tmin, tmax) are returned only
// when every comparison the caller makes with them — tmin <= tmax, t <= 0,
// t < distance — clears a margin far above their error, so the decisions are
// the exact ones; otherwise the exact cube test runs.
__device__ __forceinline__ void cube_hits_for_decisions(const Ray& r, double distance, LeafHits& H) {
    double lo3[3], hi3[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double nl = -1.0 - r.o[a], nh = 1.0 - r.o[a];
        const double rc = recip<1>(r.d[a]);
        double t0 = nl * rc, t1 = nh * rc;
        if (!(fabs(r.d[a]) >= kEps)) {
            t0 = nl < 0 ? -__builtin_inf() : __builtin_inf();
            t1 = nh < 0 ? -__builtin_inf() : __builtin_inf();
        }
        lo3[a] = min2(t0, t1);
        hi3[a] = max2(t0, t1);
    }
    const double tmin = max2(max2(lo3[0], lo3[1]), lo3[2]);
    const double tmax = min2(min2(hi3[0], hi3[1]), hi3[2]);
    const double m = kFilterRel * (finite_abs(tmin) + finite_abs(tmax) + distance);
    const bool entries = tmin <= tmax;
    bool robust = fabs(tmin - tmax) > m;
    if (entries)
        robust = robust && fabs(tmin) > m && fabs(tmax) > m && fabs(tmin - distance) > m && fabs(tmax - distance) > m;
    H.t.v2 = H.t.v3 = 0.0;
    if (robust) {
        H.t.n = entries ? 2 : 0;
        H.t.v0 = tmin;
        H.t.v1 = tmax;
    } else {
        leaf_hits<false>(FRT_CUBE, nullptr, r, H);
    }
}

}  // namespace frt
