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

}  // namespace jit
}  // namespace frt
