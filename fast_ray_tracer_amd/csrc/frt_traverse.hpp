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

// bytes of dynamic LDS per lane for a scene's capacities (host and device agree)
__host__ __device__ constexpr int walk_lds_bytes_per_lane(int list_cap, int comp_depth, int xf_depth) {
    return 12 * list_cap + 12 * comp_depth + 4 * xf_depth;
}

// per-lane views into the dynamic LDS of a traversal block
struct WalkLds {
    double* lt;  // list t          [k * kTraceBlock]
    int* ln;     // list node
    int* cn;     // composite frame: node
    int* cs;     // composite frame: list start
    int* ca;     // composite frame: CSG mid / group current-child start
    int* xn;     // transform frame: node
    __device__ __forceinline__ double& T(int k) const { return lt[k * kTraceBlock]; }
    __device__ __forceinline__ int& N(int k) const { return ln[k * kTraceBlock]; }
};

__device__ __forceinline__ WalkLds walk_lds(const DevScene& S, char* smem) {
    const int l = threadIdx.x;
    const int L = S.list_cap, C = S.comp_depth;
    WalkLds w;
    double* lt = (double*)smem;
    int* ints = (int*)(lt + L * kTraceBlock);
    w.lt = lt + l;
    w.ln = ints + l;
    w.cn = ints + L * kTraceBlock + l;
    w.cs = w.cn + C * kTraceBlock;
    w.ca = w.cs + C * kTraceBlock;
    w.xn = w.ca + C * kTraceBlock;
    return w;
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

// close the composite at frame top: group -> sort; CSG -> csg_local_intersect's tail. Returns the new list end.
__device__ __forceinline__ int close_composite(const DevScene& S, const WalkLds& W, int node, int start, int aux, int n) {
    const frt_node& nd = S.nodes[node];
    if (nd.type == FRT_GROUP) {
        sort_range(W, start, n);
        return n;
    }
    const int mid = aux, right = nd.right, op = nd.prim;
    if (n == start) return start;
    if (mid == start) return csg_filter(W, op, node + 1, right, mid, n, start);  // left empty: right list as is
    if (n == mid) return csg_filter(W, op, node + 1, right, start, mid, start);  // right empty
    sort_range(W, start, n);
    return csg_filter(W, op, node + 1, right, start, n, start);
}

// rebuild the current ray from the world ray through the open transform frames
__device__ __forceinline__ void rebuild_ray(const DevScene& S, const WalkLds& W, int sp, const Ray& world, Ray& cur) {
    cur = world;
    for (int k = 0; k < sp; ++k) cur = xf_ray(xform_of(S, S.nodes[W.xn[k * kTraceBlock]].xform), cur);
}

__device__ __forceinline__ bool behind(double tmax) { return tmax < -1e-6 * (1.0 + fabs(tmax)); }

// One walk for both ray kinds.
//   kShadow = false: returns the closest-hit leaf (-1 = miss), its t in best_t.
//   kShadow = true:  returns 1 if shadowed (is_shadowed), else 0.
template <bool kShadow, int kFeat>
__device__ int walk(const DevScene& S, const Ray& world, double distance, double& best_t, char* smem, unsigned& err) {
    constexpr bool kCsg = (kFeat & kFeatCsg) != 0;
    constexpr bool kTorus = (kFeat & kFeatTorus) != 0;
    const WalkLds W = walk_lds(S, smem);
    int best = -1;
    best_t = 0.0;
    for (int ri = 0; ri < S.num_roots; ++ri) {
        const int root = S.roots[ri];
        const int end = S.nodes[root].skip;
        const bool may_skip_behind = !kShadow || ri == S.num_roots - 1;
        int sp = 0;  // open transform frames
        int cp = 0;  // open composite frames (inside a CSG unit)
        int n = 0;   // list entries of the open CSG unit
        bool any_entry = false;
        Ray cur = world;
        int i = root;
        while (true) {
            // ---- close what the walk has left ----
            if constexpr (kCsg) {
                bool unit_done = false;
                while (cp > 0) {
                    const int top = W.cn[(cp - 1) * kTraceBlock];
                    const frt_node& tn = S.nodes[top];
                    if (i < tn.skip) {
                        // group_local_intersect's stop rule for a group inside the unit
                        if (kShadow && tn.type == FRT_GROUP && i > top + 1) {
                            bool go_on = true;
                            for (int k = W.ca[(cp - 1) * kTraceBlock]; go_on && k < n; ++k) go_on = W.T(k) <= 0;
                            if (!go_on) {
                                i = tn.skip;
                                continue;
                            }
                        }
                        break;
                    }
                    n = close_composite(S, W, top, W.cs[(cp - 1) * kTraceBlock], W.ca[(cp - 1) * kTraceBlock], n);
                    --cp;
                    unit_done = cp == 0;
                }
                if (unit_done) {
                    // a CSG unit of the main walk is complete: its list is [0, n)
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
                            for (int k = 0; k < n; ++k) {
                                const double t = W.T(k);
                                if (t > 0 && t < distance && S.casts[W.N(k)]) return 1;
                            }
                            return 0;
                        }
                    }
                    n = 0;
                }
            }
            if (sp > 0 && i >= S.nodes[W.xn[(sp - 1) * kTraceBlock]].skip) {
                do {
                    --sp;
                } while (sp > 0 && i >= S.nodes[W.xn[(sp - 1) * kTraceBlock]].skip);
                rebuild_ray(S, W, sp, world, cur);
            }
            if (i >= end) break;
            if constexpr (kCsg) {
                if (cp > 0) {
                    const int top = W.cn[(cp - 1) * kTraceBlock];
                    const frt_node& tn = S.nodes[top];
                    if (tn.type == FRT_GROUP || i == tn.right) W.ca[(cp - 1) * kTraceBlock] = n;
                }
            }
            // ---- visit node i ----
            const frt_node& nd = S.nodes[i];
            const int type = nd.type;
            const int xf = nd.xform;
            const Ray lr = xf >= 0 ? xf_ray(xform_of(S, xf), cur) : cur;
            if (type == FRT_GROUP || type == FRT_CSG) {
                double tmin, tmax;
                bool enter = box_range(nd.bbox, lr, tmin, tmax);
                if (cp == 0) {  // skips that cannot change this walk's answer (see header)
                    if (may_skip_behind && behind(tmax)) enter = false;
                    if (!kShadow && best >= 0 && tmin > best_t + 1e-6 * (1.0 + fabs(best_t))) enter = false;
                }
                if (!enter) {
                    i = nd.skip;
                    continue;
                }
                if (xf >= 0) {
                    if (sp >= S.xf_depth) {
                        err |= kErrXformDepth;
                        i = nd.skip;
                        continue;
                    }
                    W.xn[sp * kTraceBlock] = i;
                    ++sp;
                    cur = lr;
                }
                if constexpr (kCsg) {
                    if (type == FRT_CSG || cp > 0) {
                        if (cp >= S.comp_depth) {
                            err |= kErrCsgDepth;
                            i = nd.skip;
                            continue;
                        }
                        W.cn[cp * kTraceBlock] = i;
                        W.cs[cp * kTraceBlock] = n;
                        W.ca[cp * kTraceBlock] = n;
                        ++cp;
                    }
                }
                ++i;
                continue;
            }
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
                if (stop_here) return blocked && S.casts[i];
            }
            ++i;
        }
        if (kShadow && any_entry) return 0;  // intersect_world(stop) ends after the first shape with entries
    }
    return kShadow ? 0 : best;
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
