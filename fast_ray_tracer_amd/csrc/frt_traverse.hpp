// frt-mi355x device traversal over the pre-order node array.
//
// Closest hit (intersect_world(stop=false) + hit(), reference world.c:163-197,
// group.c:92-147, intersection.c:42-55): the reference visits every child of
// every group whose box the ray crosses, concatenates the children's sorted
// lists and stably sorts them, then takes the first t > 0. That equals the
// minimum positive t with ties going to the entry emitted first in DFS order,
// so the walk visits the nodes in pre-order and keeps the first strictly
// smaller t. A subtree whose box lies wholly behind the ray, or wholly beyond
// the best t so far, cannot change that answer and is skipped.
//
// Shadow any-hit (stop=true, renderer.c:74-93): a group stops visiting
// children after the first child whose list holds a t that is not <= 0, so
// the whole walk ends at the first leaf / CSG "unit" that produces one; the
// point is shadowed iff that unit holds a shadow-casting t in (0, distance).
// Non-casting objects hit first therefore shield what lies behind them,
// exactly as in the reference. Order matters
// here, so only subtrees wholly behind the ray are skipped (in the last world
// shape, where the "first world shape with entries" rule no longer applies).
//
// CSG (csg.c:74-125) needs the full sorted lists of both operands, negative t
// included. The same loop evaluates a CSG subtree iteratively: composites
// (groups / CSGs) inside it open a frame {node, list start, mid/child start};
// leaves append (t, node) entries; a closing group stably sorts its range
// (glibc's merge-sort permutation == stable insertion sort) and a closing CSG
// applies the reference's sort-unless-one-side-is-empty + inside/outside
// filter. Lists, composite frames and transform frames live in LDS,
// lane-interleaved ([k * kTraceBlock + lane], consecutive banks), sized per
// scene at upload (frt_scene_handle::lds_bytes) — one leaf-test call site in
// the whole walk, no recursion, no scratch memory.
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
    const uint8_t* __restrict__ casts;  // per node: material casts shadows (leaves)
    int32_t num_nodes, num_roots, num_lights, num_patterns;
    // per-lane LDS capacities of the walk (computed from the tree at upload)
    int32_t list_cap;    // CSG list entries
    int32_t comp_depth;  // open composites inside a CSG unit
    int32_t xf_depth;    // open transformed composites
    int32_t features;    // FeatureBits present in the scene
    frt_camera cam;
    frt_config cfg;
};

enum FeatureBits : int { kFeatCsg = 1, kFeatTorus = 2 };

constexpr int kTraceBlock = 128;  // lanes per block of the traversal kernels

enum ErrBits : unsigned {
    kErrCsgOverflow = 1u,
    kErrCsgDepth = 2u,
    kErrXformDepth = 4u,
    kErrQueueOverflow = 8u,
    kErrContainer = 16u,
};

__device__ __forceinline__ const double* xform_of(const DevScene& S, int x) { return S.xforms + 16 * (size_t)x; }

// Dynamic LDS of a traversal block. Per lane ([k * kTraceBlock + lane]):
// the CSG list (t, node) and each open composite's list start / mid. Per wave
// (uniform, [wave * depth + k]): the node of each open composite frame and of
// each open transform frame.
struct WalkLds {
    double* lt;  // list t          (per lane)
    int* ln;     // list node       (per lane)
    int* cs;     // composite frame: list start (per lane)
    int* ca;     // composite frame: CSG mid / group current-child start (per lane)
    int* cn;     // composite frame: node (per wave)
    int* xn;     // transform frame: node (per wave)
    __device__ __forceinline__ double& T(int k) const { return lt[k * kTraceBlock]; }
    __device__ __forceinline__ int& N(int k) const { return ln[k * kTraceBlock]; }
};

__host__ __device__ constexpr int walk_lds_bytes(int list_cap, int comp_depth, int xf_depth) {
    return (12 * list_cap + 8 * comp_depth) * kTraceBlock + 4 * (comp_depth + xf_depth) * (kTraceBlock / 64);
}

__device__ __forceinline__ WalkLds walk_lds(const DevScene& S, char* smem) {
    const int l = threadIdx.x, w = threadIdx.x >> 6;
    const int L = S.list_cap, C = S.comp_depth, X = S.xf_depth;
    WalkLds v;
    double* lt = (double*)smem;
    int* ints = (int*)(lt + L * kTraceBlock);
    v.lt = lt + l;
    v.ln = ints + l;
    v.cs = ints + L * kTraceBlock + l;
    v.ca = v.cs + C * kTraceBlock;
    int* wave = ints + (L + 2 * C) * kTraceBlock;
    v.cn = wave + w * C;
    v.xn = wave + (kTraceBlock / 64) * C + w * X;
    return v;
}

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return uniform(x);
}

__device__ __forceinline__ void sort_range(const WalkLds& W, int b, int e) {
    // stable insertion sort with the reference comparator (l - r < 0 / > 0)
    for (int i = b + 1; i < e; ++i) {
        const double ct = W.T(i);
        const int cn = W.N(i);
        int j = i;
        while (j > b && (W.T(j - 1) - ct) > 0) {
            W.T(j) = W.T(j - 1);
            W.N(j) = W.N(j - 1);
            --j;
        }
        W.T(j) = ct;
        W.N(j) = cn;
    }
}

// intersection_allowed (csg.c:27-40)
__device__ __forceinline__ bool csg_allowed(int op, bool lhit, bool inl, bool inr) {
    if (op == 0) return (lhit && !inr) || (!lhit && !inl);  // union
    if (op == 1) return (lhit && inr) || (!lhit && inl);    // intersect
    if (op == 2) return (lhit && !inr) || (!lhit && inl);   // difference
    return false;
}

// csg_filter_intersections (csg.c:42-71) over entries [b, e), kept ones written from `to`; returns the new end
__device__ __forceinline__ int csg_filter(const WalkLds& W, int op, int left_begin, int left_end, int b, int e, int to) {
    bool inl = false, inr = false;
    for (int i = b; i < e; ++i) {
        const double t = W.T(i);
        const int n = W.N(i);
        const bool lhit = n >= left_begin && n < left_end;  // csg_includes = subtree range
        if (csg_allowed(op, lhit, inl, inr)) {
            W.T(to) = t;
            W.N(to) = n;
            ++to;
        }
        if (lhit) inl = !inl;
        else inr = !inr;
    }
    return to;
}

// close a composite: group -> sort (group.c:144); CSG -> csg_local_intersect's tail (csg.c:93-121).
// Returns the lane's new list end.
__device__ __forceinline__ int close_composite(const frt_node& nd, int node, const WalkLds& W, int start, int mid,
                                               int n) {
    if (nd.type == FRT_GROUP) {
        sort_range(W, start, n);
        return n;
    }
    const int right = nd.right, op = nd.prim;
    if (n == start) return start;
    if (mid == start) return csg_filter(W, op, node + 1, right, mid, n, start);  // left empty: right list as is
    if (n == mid) return csg_filter(W, op, node + 1, right, start, mid, start);  // right empty
    sort_range(W, start, n);
    return csg_filter(W, op, node + 1, right, start, n, start);
}

__device__ __forceinline__ bool behind(double tmax) { return tmax < -1e-6 * (1.0 + fabs(tmax)); }

constexpr int kDone = 0x7fffffff;  // resume index of a lane whose walk has finished

// One wave-coherent walk for both ray kinds. The wave visits the pre-order
// nodes together (node index, frames and box / leaf decisions of the wave
// are uniform, so node records and transforms come in through scalar loads);
// each lane carries its own ray, result and `resume` index: a lane whose ray
// misses a composite's box (or that has finished) sits out until the walk
// reaches `resume`. A composite is entered if any lane enters it; when no lane
// is active the walk jumps to the smallest resume index.
//   kShadow = false: returns the closest-hit leaf (-1 = miss), its t in best_t.
//   kShadow = true:  returns 1 if shadowed (is_shadowed), else 0.
// Lanes that should not trace pass live = false (they still take part).
template <bool kShadow, int kFeat>
__device__ int walk(const DevScene& S, const Ray& world, double distance, bool live, double& best_t, char* smem,
                    unsigned& err) {
    constexpr bool kCsg = (kFeat & kFeatCsg) != 0;
    constexpr bool kTorus = (kFeat & kFeatTorus) != 0;
    const WalkLds W = walk_lds(S, smem);
    int best = -1;
    int result = 0;
    best_t = 0.0;
    for (int ri = 0; ri < S.num_roots; ++ri) {
        if (__ballot(live) == 0) break;
        const int root = S.roots[ri];
        const int end = S.nodes[root].skip;
        const bool may_skip_behind = !kShadow || ri == S.num_roots - 1;
        int sp = 0;  // open transform frames (uniform)
        int cp = 0;  // open composite frames inside a CSG unit (uniform)
        int n = 0;   // list entries of the open CSG unit (per lane)
        int resume = live ? 0 : kDone;
        bool any_entry = false;
        Ray cur = world;
        int i = root;
        while (true) {
            // ---- close the composites the walk has left ----
            if constexpr (kCsg) {
                while (cp > 0) {
                    const int top = uniform(W.cn[cp - 1]);
                    const frt_node& tn = S.nodes[top];
                    if (i < tn.skip) {
                        // group_local_intersect's stop rule (group.c:114-121) for a group inside the unit
                        if (kShadow && tn.type == FRT_GROUP && i > top + 1 && i >= resume) {
                            bool go_on = true;
                            for (int k = W.ca[(cp - 1) * kTraceBlock]; go_on && k < n; ++k) go_on = W.T(k) <= 0;
                            if (!go_on) resume = tn.skip;
                        }
                        break;
                    }
                    n = close_composite(tn, top, W, W.cs[(cp - 1) * kTraceBlock], W.ca[(cp - 1) * kTraceBlock], n);
                    --cp;
                    if (cp == 0) {
                        // a CSG unit of the main walk is complete: the lane's list is [0, n)
                        if (resume != kDone) {
                            if (!kShadow) {
                                for (int k = 0; k < n; ++k) {
                                    const double t = W.T(k);
                                    if (t > 0 && (best < 0 || t < best_t)) {
                                        best_t = t;
                                        best = W.N(k);
                                    }
                                }
                            } else if (n > 0) {
                                any_entry = true;
                                bool stop_here = false;
                                for (int k = 0; k < n; ++k) stop_here = stop_here || !(W.T(k) <= 0);
                                if (stop_here) {
                                    bool blocked = false;
                                    for (int k = 0; k < n; ++k) {
                                        const double t = W.T(k);
                                        blocked = blocked || (t > 0 && t < distance && S.casts[W.N(k)]);
                                    }
                                    result = blocked ? 1 : 0;
                                    resume = kDone;
                                }
                            }
                        }
                        n = 0;
                    }
                }
            }
            // ---- pop transform frames, rebuild the ray from the world ray ----
            if (sp > 0 && i >= S.nodes[uniform(W.xn[sp - 1])].skip) {
                do {
                    --sp;
                } while (sp > 0 && i >= S.nodes[uniform(W.xn[sp - 1])].skip);
                cur = world;
                for (int k = 0; k < sp; ++k) cur = xf_ray(xform_of(S, S.nodes[uniform(W.xn[k])].xform), cur);
            }
            if (i >= end) break;
            const bool active = i >= resume;
            if (__ballot(active) == 0) {
                // every inactive lane has resume > i; max() only guards progress
                i = min(end, max(wave_min(resume), i + 1));
                continue;
            }
            if constexpr (kCsg) {
                if (cp > 0) {
                    const int top = uniform(W.cn[cp - 1]);
                    const frt_node& tn = S.nodes[top];
                    if (tn.type == FRT_GROUP || i == tn.right) W.ca[(cp - 1) * kTraceBlock] = n;
                }
            }
            // ---- visit node i (uniform) ----
            const frt_node& nd = S.nodes[i];
            const int type = nd.type;
            const int xf = nd.xform;
            const Ray lr = xf >= 0 ? xf_ray(xform_of(S, xf), cur) : cur;
            if (type == FRT_GROUP || type == FRT_CSG) {
                bool enter = false;
                if (active) {
                    double tmin, tmax;
                    enter = box_range(nd.bbox, lr, tmin, tmax);
                    if (cp == 0) {  // skips that cannot change this lane's answer (see header)
                        if (may_skip_behind && behind(tmax)) enter = false;
                        if (!kShadow && best >= 0 && tmin > best_t + 1e-6 * (1.0 + fabs(best_t))) enter = false;
                    }
                    if (!enter) resume = nd.skip;
                }
                if (__ballot(enter) == 0) {
                    i = nd.skip;
                    continue;
                }
                if (xf >= 0) {
                    if (sp >= S.xf_depth) {  // cannot happen: xf_depth is exact (upload)
                        err |= kErrXformDepth;
                        resume = kDone;
                        i = nd.skip;
                        continue;
                    }
                    if ((threadIdx.x & 63) == 0) W.xn[sp] = i;
                    ++sp;
                    cur = lr;
                }
                if constexpr (kCsg) {
                    if (type == FRT_CSG || cp > 0) {
                        if (cp >= S.comp_depth) {  // cannot happen: comp_depth is exact (upload)
                            err |= kErrCsgDepth;
                            resume = kDone;
                            i = nd.skip;
                            continue;
                        }
                        if ((threadIdx.x & 63) == 0) W.cn[cp] = i;
                        W.cs[cp * kTraceBlock] = n;
                        W.ca[cp * kTraceBlock] = n;
                        ++cp;
                    }
                }
                ++i;
                continue;
            }
            if (active) {
                LeafHits H;
                leaf_hits<kTorus>(nd, S.prim, lr, H);
                if (kCsg && cp > 0) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (j < H.t.n) {
                            if (n < S.list_cap) {
                                W.T(n) = H.t.at(j);
                                W.N(n) = i;
                                ++n;
                            } else {
                                err |= kErrCsgOverflow;
                            }
                        }
                    }
                } else if (!kShadow) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const double t = H.t.at(j);
                        if (j < H.t.n && t > 0 && (best < 0 || t < best_t)) {
                            best_t = t;
                            best = i;
                        }
                    }
                } else if (H.t.n > 0) {
                    any_entry = true;
                    bool stop_here = false;
                    bool blocked = false;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const double t = H.t.at(j);
                        if (j < H.t.n) {
                            stop_here = stop_here || !(t <= 0);
                            blocked = blocked || (t > 0 && t < distance);
                        }
                    }
                    if (stop_here) {
                        result = blocked && S.casts[i] ? 1 : 0;
                        resume = kDone;
                    }
                }
            }
            ++i;
        }
        if (kShadow && live && resume != kDone && any_entry) live = false;  // first world shape with entries ends it
        if (resume == kDone) live = false;
    }
    return kShadow ? result : best;
}

// recompute a leaf's local ray (through every transformed ancestor, root first,
// exactly as the walk composed it) — used to recover triangle (u, v)
__device__ inline Ray leaf_local_ray(const DevScene& S, int leaf, const Ray& world) {
    const int first = S.nodes[leaf].xform >= 0 ? leaf : S.nodes[leaf].tparent;
    int n = 0;
    for (int x = first; x >= 0; x = S.nodes[x].tparent) n++;
    Ray r = world;
    for (int k = n - 1; k >= 0; --k) {
        int x = first;
        for (int j = 0; j < k; ++j) x = S.nodes[x].tparent;
        r = xf_ray(xform_of(S, S.nodes[x].xform), r);
    }
    return r;
}

}  // namespace frt
