// frt-mi355x device traversal over the pre-order node array.
//
// Closest hit (intersect_world(stop=false) + hit(), reference world.c:163-197,
// group.c:92-147, intersection.c:42-55): the reference visits every child of
// every group whose box the ray crosses, concatenates the children's sorted
// lists and stably sorts them, then takes the first t > 0. That equals the
// minimum positive t with ties going to the entry emitted first in DFS order,
// so the kernel walks the nodes in pre-order and keeps the first strictly
// smaller t — no per-ray lists except inside CSG subtrees.
//
// Shadow any-hit (stop=true, renderer.c:74-93): a group stops visiting
// children after the first child whose list holds a t that is not <= 0, so
// the whole walk ends at the first leaf / CSG "unit" that produces one; the
// point is shadowed iff that unit holds a shadow-casting t in (0, distance).
// Non-casting objects hit first therefore shield what lies behind them,
// exactly as in the reference.
//
// CSG (csg.c:74-125) needs the full sorted lists of both operands, negative t
// included: a CSG subtree is evaluated into a small per-lane list with
// compile-time-bounded recursion (stable insertion sort = glibc's stable
// merge sort permutation, then the inside/outside filter).
#pragma once

#include "frt_math.hpp"

namespace frt {

struct DevScene {
    const frt_node* __restrict__ nodes;
    const int32_t* __restrict__ roots;
    const double* __restrict__ xforms;
    const double* __restrict__ prim;
    const frt_material* __restrict__ materials;
    const frt_pattern* __restrict__ patterns;
    const frt_texture* __restrict__ textures;
    const double* __restrict__ texels;
    const frt_light* __restrict__ lights;
    const double* __restrict__ light_points;
    const double* __restrict__ sample_table;
    int32_t num_nodes, num_roots, num_lights, num_patterns;
    frt_camera cam;
    frt_config cfg;
};

constexpr int kCsgListCap = 48;
constexpr int kCsgDepth = 6;
constexpr int kMaxXformDepth = 8;

enum ErrBits : unsigned {
    kErrCsgOverflow = 1u,
    kErrCsgDepth = 2u,
    kErrXformDepth = 4u,
    kErrQueueOverflow = 8u,
    kErrContainer = 16u,
};

__device__ __forceinline__ const double* xform_of(const DevScene& S, int x) { return S.xforms + 16 * (size_t)x; }

__device__ __forceinline__ void sort_hits(Hit* a, int n) {
    // stable insertion sort with the reference comparator (l - r < 0 / > 0)
    for (int i = 1; i < n; ++i) {
        Hit cur = a[i];
        int j = i;
        while (j > 0 && (a[j - 1].t - cur.t) > 0) {
            a[j] = a[j - 1];
            --j;
        }
        a[j] = cur;
    }
}

__device__ __forceinline__ bool csg_allowed(int op, bool lhit, bool inl, bool inr) {
    if (op == 0) return (lhit && !inr) || (!lhit && !inl);  // union
    if (op == 1) return (lhit && inr) || (!lhit && inl);    // intersect
    if (op == 2) return (lhit && !inr) || (!lhit && inl);   // difference
    return false;
}

__device__ __forceinline__ int csg_filter(int op, int left_begin, int left_end, Hit* a, int n) {
    bool inl = false, inr = false;
    int kept = 0;
    for (int i = 0; i < n; ++i) {
        bool lhit = a[i].node >= left_begin && a[i].node < left_end;  // csg_includes = subtree range
        if (csg_allowed(op, lhit, inl, inr)) a[kept++] = a[i];
        if (lhit) inl = !inl;
        else inr = !inr;
    }
    return kept;
}

__device__ __noinline__ int leaf_hits_call(const frt_node& nd, int ni, const double* prim, const Ray& r, Hit* h) {
    return leaf_hits(nd, ni, prim, r, h);
}

// Append the (sorted / filtered, as the reference returns it) list of node ni
// for a ray given in ni's parent space. Used for CSG subtrees only.
template <int D>
__device__ int eval_list(const DevScene& S, int ni, const Ray& pr, bool stop, Hit* L, int n, unsigned& err) {
    const frt_node nd = S.nodes[ni];
    const Ray r = nd.xform >= 0 ? xf_ray(xform_of(S, nd.xform), pr) : pr;
    if (nd.type == FRT_GROUP) {
        if (!box_hit(nd.bbox, r)) return n;
        const int start = n;
        for (int c = ni + 1; c < nd.skip; c = S.nodes[c].skip) {
            const int cs = n;
            if constexpr (D > 0) {
                n = eval_list<D - 1>(S, c, r, stop, L, n, err);
            } else {
                err |= kErrCsgDepth;
            }
            if (stop) {
                bool go_on = true;
                for (int k = cs; go_on && k < n; ++k) go_on = L[k].t <= 0;
                if (!go_on) break;
            }
        }
        sort_hits(L + start, n - start);
        return n;
    }
    if (nd.type == FRT_CSG) {
        if (!box_hit(nd.bbox, r)) return n;
        const int start = n;
        int mid = n;
        if constexpr (D > 0) {
            n = eval_list<D - 1>(S, ni + 1, r, stop, L, n, err);
            mid = n;
            n = eval_list<D - 1>(S, nd.right, r, stop, L, n, err);
        } else {
            err |= kErrCsgDepth;
        }
        const int nl = mid - start, nr = n - mid;
        if (nl + nr == 0) return start;
        int kept;
        if (nl == 0) {
            kept = csg_filter(nd.prim, ni + 1, nd.right, L + mid, nr);
            for (int k = 0; k < kept; ++k) L[start + k] = L[mid + k];
        } else if (nr == 0) {
            kept = csg_filter(nd.prim, ni + 1, nd.right, L + start, nl);
        } else {
            sort_hits(L + start, nl + nr);
            kept = csg_filter(nd.prim, ni + 1, nd.right, L + start, nl + nr);
        }
        return start + kept;
    }
    Hit h[4];
    const int k = leaf_hits_call(nd, ni, S.prim, r, h);
    for (int j = 0; j < k; ++j) {
        if (n < kCsgListCap) L[n++] = h[j];
        else err |= kErrCsgOverflow;
    }
    return n;
}

// Transform-frame bookkeeping shared by both walks: frames are pushed when a
// transformed group is entered and popped once the walk leaves its subtree;
// the ray is then rebuilt from the world ray through the remaining frames
// (transformed groups are rare and shallow; no ray copies are stored).
struct Frames {
    int end[kMaxXformDepth];
    int xf[kMaxXformDepth];
    int sp;
};

__device__ __forceinline__ void pop_frames(const DevScene& S, Frames& F, int i, const Ray& world, Ray& cur) {
    if (F.sp == 0 || i < F.end[F.sp - 1]) return;
    while (F.sp > 0 && i >= F.end[F.sp - 1]) F.sp--;
    cur = world;
    for (int k = 0; k < F.sp; ++k) cur = xf_ray(xform_of(S, F.xf[k]), cur);
}

__device__ __forceinline__ void consider(const Hit& h, Hit& best, bool& found) {
    if (h.t > 0 && (!found || h.t < best.t)) {
        best = h;
        found = true;
    }
}

__device__ bool closest_hit(const DevScene& S, const Ray& world, Hit& best, unsigned& err) {
    bool found = false;
    for (int ri = 0; ri < S.num_roots; ++ri) {
        const int root = S.roots[ri];
        const int end = S.nodes[root].skip;
        Frames F;
        F.sp = 0;
        Ray cur = world;
        int i = root;
        while (i < end) {
            pop_frames(S, F, i, world, cur);
            const frt_node nd = S.nodes[i];
            if (nd.type == FRT_GROUP) {
                const Ray lr = nd.xform >= 0 ? xf_ray(xform_of(S, nd.xform), cur) : cur;
                if (!box_hit(nd.bbox, lr)) {
                    i = nd.skip;
                    continue;
                }
                if (nd.xform >= 0) {
                    if (F.sp < kMaxXformDepth) {
                        F.end[F.sp] = nd.skip;
                        F.xf[F.sp] = nd.xform;
                        F.sp++;
                        cur = lr;
                    } else {
                        err |= kErrXformDepth;
                        i = nd.skip;
                        continue;
                    }
                }
                ++i;
                continue;
            }
            if (nd.type == FRT_CSG) {
                Hit L[kCsgListCap];
                const int n = eval_list<kCsgDepth>(S, i, cur, false, L, 0, err);
                for (int k = 0; k < n; ++k) consider(L[k], best, found);
                i = nd.skip;
                continue;
            }
            const Ray lr = nd.xform >= 0 ? xf_ray(xform_of(S, nd.xform), cur) : cur;
            Hit h[4];
            const int k = leaf_hits(nd, i, S.prim, lr, h);
            for (int j = 0; j < k; ++j) consider(h[j], best, found);
            ++i;
        }
    }
    return found;
}

// any-hit with the reference's stop rule; returns is_shadowed()
__device__ bool shadowed(const DevScene& S, const Ray& world, double distance, unsigned& err) {
    for (int ri = 0; ri < S.num_roots; ++ri) {
        const int root = S.roots[ri];
        const int end = S.nodes[root].skip;
        Frames F;
        F.sp = 0;
        Ray cur = world;
        bool any_entry = false;
        int i = root;
        while (i < end) {
            pop_frames(S, F, i, world, cur);
            const frt_node nd = S.nodes[i];
            if (nd.type == FRT_GROUP) {
                const Ray lr = nd.xform >= 0 ? xf_ray(xform_of(S, nd.xform), cur) : cur;
                if (!box_hit(nd.bbox, lr)) {
                    i = nd.skip;
                    continue;
                }
                if (nd.xform >= 0) {
                    if (F.sp < kMaxXformDepth) {
                        F.end[F.sp] = nd.skip;
                        F.xf[F.sp] = nd.xform;
                        F.sp++;
                        cur = lr;
                    } else {
                        err |= kErrXformDepth;
                        i = nd.skip;
                        continue;
                    }
                }
                ++i;
                continue;
            }
            if (nd.type == FRT_CSG) {
                Hit L[kCsgListCap];
                const int n = eval_list<kCsgDepth>(S, i, cur, true, L, 0, err);
                i = nd.skip;
                if (n > 0) any_entry = true;
                bool stop_here = false;
                for (int k = 0; k < n; ++k) stop_here = stop_here || !(L[k].t <= 0);
                if (stop_here) {
                    for (int k = 0; k < n; ++k) {
                        const double t = L[k].t;
                        if (t > 0 && t < distance && S.materials[S.nodes[L[k].node].material].casts_shadow) return true;
                    }
                    return false;
                }
                continue;
            }
            const Ray lr = nd.xform >= 0 ? xf_ray(xform_of(S, nd.xform), cur) : cur;
            Hit h[4];
            const int n = leaf_hits(nd, i, S.prim, lr, h);
            ++i;
            if (n > 0) {
                any_entry = true;
                bool stop_here = false;
                for (int k = 0; k < n; ++k) stop_here = stop_here || !(h[k].t <= 0);
                if (stop_here) {
                    if (!S.materials[nd.material].casts_shadow) return false;
                    for (int k = 0; k < n; ++k) {
                        const double t = h[k].t;
                        if (t > 0 && t < distance) return true;
                    }
                    return false;
                }
            }
        }
        if (any_entry) return false;  // intersect_world(stop) ends after the first shape with entries
    }
    return false;
}

}  // namespace frt
