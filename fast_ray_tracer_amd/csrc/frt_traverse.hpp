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

// Device visit record of one node for the walk (built at upload): everything a
// visit reads sits in one 176-byte record, fetched with independent scalar loads
// once the (wave-uniform) node index is known — no node -> transform chain.
struct alignas(16) WalkNode {
    int32_t type, skip, right, op;     // op: CSG operation
    int32_t has_xf, casts, prim;       // prim: offset of the leaf's parameters in prim_data
    int32_t pre;                       // bit0: pbox prefilter applies, bit1: check the EPSILON quirk first
    double bbox[6];                    // composites: own-space bounds
    double m[12];                      // inverse transform, rows 0-2 (has_xf)
    double pbox[6];                    // prefilter: inflated bound of the node in its parent's frame
    float mrow[9];                     // rows of m's 3x3 part (identity without transform), as float
    float mrow_l1[3];                  // their L1 norms
    float bb32[6];                     // composites: f32(bbox) (box32)
    float bmag[3];                     // composites: max(|lo_a|, |hi_a|) rounded up (box32's error bound)
    int32_t parent;                    // parent node (-1: a world shape)
    // world -> this node's frame as one affine map (the product of the inverse transforms from the
    // world shape down to this node, composed in binary64 at upload), rounded to binary32, with the
    // bounds frt_jit_rt.hpp's interval walk needs: cN = max row L1 norm of the 3x3 part, cT = max
    // |translation|, both rounded up
    float cm[12];
    float cN, cT;
    // axis-aligned frames (the 3x3 part of the composed map a signed permutation up to entries below
    // 2^-30 of their row's largest; written as if diagonal below, c_aa != 0): the node's slab
    // planes in world coordinates, B = (b - c_a3) / c_aa for its two bounds b per axis (cube: -1 / +1,
    // composite: its own-space box), rounded to binary32 — the slab test then runs on the world ray
    // (frt_jit_rt.hpp aa_slab) without a frame or a reciprocal per node. aathr_a: |f32(d_a)| >= aathr_a
    // proves the local |d_a| >= EPSILON (the reference's slab branch); aabmax >= every |B|; aasig >=
    // 1.02 x (the other entries of a row / its largest), the relative error they add to t per |r_a|.
    float aab[6];
    float aathr[3];
    float aabmax, aasig;
    int32_t aa;
    // spheres whose frame is an exact signed permutation with one scale (a round sphere in the
    // world): centre and radius x (1 + 1e-6) rounded up, for the interval walk's certain-miss test
    // (frt_jit_rt.hpp sphere_miss32); sph_ok = 0 otherwise
    int32_t sph_ok;
    float sph[4];
};

// per-frame cache of the current ray: reciprocal direction (two Newton steps),
// float direction and its largest magnitude (prefilter / quirk check)
struct FrameCache {
    double rc[3];
    float df[3];
    float dmax;
};

__device__ __forceinline__ void frame_cache(const Ray& r, FrameCache& c) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        c.rc[a] = recip<2>(r.d[a]);
        c.df[a] = (float)r.d[a];
    }
    c.dmax = fmaxf(fmaxf(fabsf(c.df[0]), fabsf(c.df[1])), fabsf(c.df[2]));
}

// one photon map (frt_gi.hpp): photons sorted by cell of a dense uniform grid
// (x fastest, so a row of cells is one contiguous photon range), built on the
// host after tracing
struct PhotonMapDev {
    const float* pos4;    // 4 per photon: binary32 x, y, z, 0 (the estimate's candidate scan)
    const double* rec;    // 10 per photon (80 bytes, grid order like pos4): binary64 x, y, z, power (scaled by
                          // 1 / photon_count), pm_photon_dir of the stored theta / phi bytes (pm.c:80-88),
                          // the heap index (int64 bits)
    const int32_t* start; // cell -> first photon, cells + 1 entries
    const double* kd;     // 4 per heap index (pm_balance's kd-tree, frt_engine.hip pm_balance_heap): binary64
                          // x, y, z and the split plane (the traversal order of the estimate's selection)
    int64_t count;        // photons in the grid (those the reference's search reaches)
    int32_t dims[3];      // cells per axis
    int32_t pad;
    double origin[3];     // grid origin (the photons' lower bounding-box corner)
    double cell;          // cell edge: radius / 3, doubled until the grid fits kMaxGridCells
    double inv_cell;
};

// A mesh: a group subtree of groups and triangles only (no transforms below its root, no CSG around it)
// gets a BVH of its own at upload (frt_engine.hip build_meshes): binary32 boxes rounded outward, two
// children per node, the smallest pre-order index below each child. The walk searches it per lane
// (mesh_closest / mesh_first) instead of visiting the reference's group tree node by node.
struct MeshNode {
    float b[12];        // child 0 lo xyz, hi xyz; child 1 lo xyz, hi xyz
    int32_t child[2];   // >= 0: node; < 0: leaf, ~child = first << 3 | (count - 1) in tris
    int32_t mindfs[2];  // the smallest pre-order index of the triangles below each child
};
struct MeshDesc {
    const MeshNode* nodes;  // node 0: the root
    const int2* tris;       // (pre-order index, prim_data offset) per leaf entry
    int32_t root;           // the mesh's root group in the node array
    int32_t last_root;      // inside the last world shape (the shadow search applies)
};

struct DevScene {
    const WalkNode* __restrict__ wn;
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
    const int4* __restrict__ xchain;    // per node: {n, ids}: its transform chain, root-most first (xf_chain)
    int32_t num_nodes, num_roots, num_lights, num_patterns;
    // per-lane LDS capacities of the walk (computed from the tree at upload)
    int32_t list_cap;    // CSG list entries
    int32_t comp_depth;  // open composites inside a CSG unit
    int32_t xf_depth;    // open transformed composites
    int32_t features;    // FeatureBits present in the scene
    unsigned long long* dbg;  // walk statistics (FRT_WALK_STATS builds only)
    int32_t walk_flags;       // FRT_WALK_FLAGS (A/B experiments): bit0 no prefilter, bit1 exact box decisions, bit2 exact cubes
    frt_camera cam;
    frt_config cfg;
    PhotonMapDev pmaps[2];  // 0 caustic, 1 global (global illumination only)
    const MeshDesc* meshes;  // WalkNode::op - 1 of a mesh's root group (0: not a mesh)
    int32_t num_meshes;
    int32_t mesh_stack;      // per-lane LDS stack entries of the mesh searches (0: no meshes)
};

enum FeatureBits : int { kFeatCsg = 1, kFeatTorus = 2 };

// FRT_WALK_STATS builds: 16 global counters + per node (first kDbgNodes) {wave visits, active lanes} x 2 walks
constexpr int kDbgNodes = 64;
constexpr int kDbgSlots = 16 + 4 * kDbgNodes + 32;
constexpr int kDbgProf = 16 + 4 * kDbgNodes;  // FRT_WALK_PROF builds: s_memtime cycles per walk region (shadow)

#ifdef FRT_WALK_PROF
__device__ __forceinline__ unsigned long long prof_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define FRT_PROF_DECL unsigned long long prof_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_last = prof_stamp();
#define FRT_PROF(k)                              \
    do {                                         \
        const unsigned long long now_ = prof_stamp(); \
        prof_acc[k] += now_ - prof_last;         \
        prof_last = now_;                        \
    } while (0)
#define FRT_PROF_FLUSH                                                                  \
    do {                                                                                \
        if (kShadow && (threadIdx.x & 63) == 0)                                         \
            for (int k_ = 0; k_ < 8; ++k_) atomicAdd(S.dbg + kDbgProf + k_, prof_acc[k_]); \
    } while (0)
#else
#define FRT_PROF_DECL
#define FRT_PROF(k) \
    do {            \
    } while (0)
#define FRT_PROF_FLUSH \
    do {               \
    } while (0)
#endif

constexpr int kTraceBlock = 128;  // lanes per block of the traversal kernels

#ifndef FRT_PREFILTER
#define FRT_PREFILTER 0  // parent-frame bound prefilter for leaves (costs registers; off by default)
#endif

enum ErrBits : unsigned {
    kErrCsgOverflow = 1u,
    kErrCsgDepth = 2u,
    kErrXformDepth = 4u,
    kErrQueueOverflow = 8u,
    kErrContainer = 16u,
    kErrAperture = 32u,
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
    int* ms;     // mesh search stack (per lane)
    __device__ __forceinline__ double& T(int k) const { return lt[k * kTraceBlock]; }
    __device__ __forceinline__ int& N(int k) const { return ln[k * kTraceBlock]; }
};

__host__ __device__ constexpr int walk_lds_bytes(int list_cap, int comp_depth, int xf_depth, int mesh_stack = 0) {
    return (12 * list_cap + 8 * comp_depth + 4 * mesh_stack) * kTraceBlock +
           4 * (comp_depth + xf_depth) * (kTraceBlock / 64);
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
    v.ms = wave + (kTraceBlock / 64) * (C + X) + l;
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
__device__ __forceinline__ int close_composite(int type, int node, int right, int op, const WalkLds& W, int start,
                                               int mid, int n) {
    if (type == FRT_GROUP) {
        sort_range(W, start, n);
        return n;
    }
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
// Refractive containers (prepare_computations, renderer.c:404-447) for the
// closest hit: the reference walks the full sorted list up to the hit,
// toggling objects in and out of an ordered container. Every entry before the
// hit has t <= 0 (the hit is the first positive one), and all entries of an
// object are emitted together, so the container at the hit is determined by,
// per object, the parity of its t <= 0 entries and the sort key (t, node,
// index) of its last one: the container's last element is the present object
// with the greatest key. The walk keeps the two greatest present objects.
struct ContainerTop2 {
    double t1, t2;
    int n1, i1, n2, i2;  // node -1: none
    __device__ __forceinline__ void init() {
        n1 = n2 = -1;
        t1 = t2 = 0.0;
        i1 = i2 = 0;
    }
    __device__ __forceinline__ static bool greater(double ta, int na, int ia, double tb, int nb, int ib) {
        return ta > tb || (ta == tb && (na > nb || (na == nb && ia > ib)));
    }
    __device__ __forceinline__ void offer(double t, int node, int idx) {
        if (n1 < 0 || greater(t, node, idx, t1, n1, i1)) {
            t2 = t1;
            n2 = n1;
            i2 = i1;
            t1 = t;
            n1 = node;
            i1 = idx;
        } else if (n2 < 0 || greater(t, node, idx, t2, n2, i2)) {
            t2 = t;
            n2 = node;
            i2 = idx;
        }
    }
};

__device__ __forceinline__ double node_ni(const DevScene& S, int node) {
    return node >= 0 ? S.materials[S.nodes[node].material].Ni : 1.0;
}

// ---- mesh searches (MeshDesc) ----
// The reference visits a group's children only when the ray passes the group's box test; the mesh BVH's
// boxes contain every triangle (binary32, rounded outward) and its box test below is conservative (it
// never rejects a box the ray meets), so the triangles it reaches include every triangle the reference
// reaches; triangle t values come from the reference's own arithmetic (leaf_hits). The search's answer is
// therefore the reference's answer exactly when its winning triangle is one the reference reaches: every
// group between the mesh root and the triangle passes the reference's box test (mesh_reachable, the walk's
// own decision). When it does not (a ray grazing a box, in binary64), or the search's stack overflows, the
// walk descends the mesh's group tree node by node instead.

// the walk's decision to enter group nd (no transform) with ray r: box32 where it decides, else binary64
__device__ __forceinline__ bool ref_group_enter(const DevScene& S, const WalkNode& nd, const Ray& r) {
    Frame32 lf;
    frame32(r, lf);
    float tmin32 = -1.0f, tmax32 = 1.0f, err32 = 0.0f;
    const int dec = (lf.exact || (S.walk_flags & 2)) ? -1 : box32(nd.bb32, nd.bmag, lf, tmin32, tmax32, err32);
    if (dec >= 0) return dec != 0;
    if (origin_inside(nd.bbox, r)) return true;
    double tmin = -1.0, tmax = 1.0;
    if (S.walk_flags & 2) return box_range(nd.bbox, r, tmin, tmax);
    double rc[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) rc[a] = recip<1>(r.d[a]);
    return box_decide(nd.bbox, r, rc, tmin, tmax);
}

__device__ __forceinline__ bool mesh_reachable(const DevScene& S, const MeshDesc& M, int leaf, const Ray& r) {
    for (int a = S.nodes[leaf].parent; a != M.root && a >= 0; a = S.nodes[a].parent)
        if (!ref_group_enter(S, S.wn[a], r)) return false;
    return true;
}

// the ray in binary32 for the conservative box test: origin, clamped reciprocal direction and the absolute
// error bound of a slab parameter from the origin's and the reciprocal's roundings
struct MeshRay {
    float o[3], inv[3], E;
};

__device__ __forceinline__ void mesh_ray(const Ray& r, MeshRay& m) {
    float om = 0.0f, im = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        m.o[a] = (float)r.o[a];
        const float d = (float)r.d[a];
        m.inv[a] = fabsf(d) < 1e-30f ? copysignf(1e30f, d) : 1.0f / d;
        om = fmaxf(om, fabsf(m.o[a]));
        im = fmaxf(im, fabsf(m.inv[a]));
    }
    m.E = 8.0f * 0x1p-24f * om * im;
}

// child box c of N: may the ray meet it within [0 - slack, tlim]? tnear: its (lowered) entry
__device__ __forceinline__ bool mesh_box(const float* b, const MeshRay& m, float tlim, float& tnear) {
    float t0 = -__builtin_huge_valf(), t1 = __builtin_huge_valf();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float x = (b[a] - m.o[a]) * m.inv[a], y = (b[3 + a] - m.o[a]) * m.inv[a];
        t0 = fmaxf(t0, fminf(x, y));
        t1 = fminf(t1, fmaxf(x, y));
    }
    const float s = fmaf(16.0f * 0x1p-24f, fmaxf(fabsf(t0), fabsf(t1)), m.E);
    tnear = t0 - s;
    return t0 - s <= t1 + s && t1 + s >= 0.0f && t0 - s <= tlim;  // (false for NaN)
}

// closest hit among the mesh's triangles, against (best_t, best) from the walk so far (pre-order ties: the
// smaller index wins). false: the walk must descend the mesh itself (answer unconfirmed)
__device__ inline bool mesh_closest(const DevScene& S, const MeshDesc& M, const Ray& r, double& best_t, int& best,
                                    int* stack) {
    MeshRay m;
    mesh_ray(r, m);
    double ct = best >= 0 ? best_t : __builtin_huge_val();
    int cn = best >= 0 ? best : 0x7fffffff;
    bool mine = false;  // the current best is a triangle of this mesh
    auto tlim = [&]() { return ct < 3e38 ? (float)ct * (1.0f + 32.0f * 0x1p-24f) + m.E : __builtin_huge_valf(); };
    auto leaf = [&](int ref) {
        const int code = ~ref, first = code >> 3, cnt = (code & 7) + 1;
        for (int k = 0; k < cnt; ++k) {
            const int2 tri = M.tris[first + k];
            LeafHits H;
            leaf_hits<false>(FRT_TRIANGLE, S.prim + tri.y, r, H);
            const double t = H.t.v0;
            if (H.t.n && t > 0 && (t < ct || (t == ct && tri.x < cn))) {
                ct = t;
                cn = tri.x;
                mine = true;
            }
        }
    };
    int sp = 0, node = 0;
    bool ok = true;
    while (true) {
        const MeshNode& N = M.nodes[node];
        const float tl = tlim();
        float tn0, tn1;
        const bool h0 = mesh_box(N.b, m, tl, tn0), h1 = mesh_box(N.b + 6, m, tl, tn1);
        const int c0 = N.child[0], c1 = N.child[1];
        if (h0 && c0 < 0) leaf(c0);
        if (h1 && c1 < 0) leaf(c1);
        const bool g0 = h0 && c0 >= 0, g1 = h1 && c1 >= 0;
        if (g0 && g1) {
            const bool near0 = tn0 <= tn1;
            if (sp >= S.mesh_stack) {
                ok = false;
                break;
            }
            stack[sp * kTraceBlock] = near0 ? c1 : c0;
            ++sp;
            node = near0 ? c0 : c1;
        } else if (g0) {
            node = c0;
        } else if (g1) {
            node = c1;
        } else {
            if (sp == 0) break;
            --sp;
            node = stack[sp * kTraceBlock];
        }
    }
    if (!ok) return false;
    if (mine) {
        if (!mesh_reachable(S, M, cn, r)) return false;
        best_t = ct;
        best = cn;
    }
    return true;
}

// the shadow walk inside a mesh: it ends at the first triangle in pre-order that the ray reaches with an
// entry t > 0 (group.c:114-121, every enclosing group stops there): the smallest pre-order index among
// those. found: such a triangle exists (its index and t); false: the walk must descend the mesh itself
__device__ inline bool mesh_first(const DevScene& S, const MeshDesc& M, const Ray& r, int& found, double& ft,
                                  int* stack) {
    MeshRay m;
    mesh_ray(r, m);
    int cn = 0x7fffffff;
    double ct = 0.0;
    auto leaf = [&](int ref) {
        const int code = ~ref, first = code >> 3, cnt = (code & 7) + 1;
        for (int k = 0; k < cnt; ++k) {
            const int2 tri = M.tris[first + k];
            if (tri.x >= cn) continue;
            LeafHits H;
            leaf_hits<false>(FRT_TRIANGLE, S.prim + tri.y, r, H);
            if (H.t.n && !(H.t.v0 <= 0)) {  // the walk's stop rule: an entry that is not <= 0
                cn = tri.x;
                ct = H.t.v0;
            }
        }
    };
    const float inf = __builtin_huge_valf();
    int sp = 0, node = 0;
    bool ok = true;
    while (true) {
        const MeshNode& N = M.nodes[node];
        float tn0, tn1;
        const int c0 = N.child[0], c1 = N.child[1];
        const bool h0 = N.mindfs[0] < cn && mesh_box(N.b, m, inf, tn0);
        const bool h1 = N.mindfs[1] < cn && mesh_box(N.b + 6, m, inf, tn1);
        // children in pre-order of their first triangle; leaves first when they come first
        const bool first0 = N.mindfs[0] <= N.mindfs[1];
        if (first0) {
            if (h0 && c0 < 0) leaf(c0);
            if (h1 && c1 < 0 && N.mindfs[1] < cn) leaf(c1);
        } else {
            if (h1 && c1 < 0) leaf(c1);
            if (h0 && c0 < 0 && N.mindfs[0] < cn) leaf(c0);
        }
        const bool g0 = h0 && c0 >= 0 && N.mindfs[0] < cn, g1 = h1 && c1 >= 0 && N.mindfs[1] < cn;
        if (g0 && g1) {
            if (sp >= S.mesh_stack) {
                ok = false;
                break;
            }
            stack[sp * kTraceBlock] = first0 ? c1 : c0;
            ++sp;
            node = first0 ? c0 : c1;
        } else if (g0) {
            node = c0;
        } else if (g1) {
            node = c1;
        } else {
            // pop, skipping entries that can no longer hold an earlier triangle (their mindfs is not kept:
            // the child's box test runs again when the node is visited)
            if (sp == 0) break;
            --sp;
            node = stack[sp * kTraceBlock];
        }
    }
    if (!ok) return false;
    found = cn == 0x7fffffff ? -1 : cn;
    ft = ct;
    if (found >= 0 && !mesh_reachable(S, M, found, r)) return false;
    return true;
}

template <bool kShadow, int kFeat>
__device__ int walk(const DevScene& S, const Ray& world, double distance, bool live, double& best_t, char* smem,
                    unsigned& err, double* n12 = nullptr, bool filter_casts = false) {
    // filter_casts (closest hit only): hit(xs, true) of the photon tracer (photon_tracer.c:185),
    // the first positive entry whose material casts shadows
    constexpr bool kCsg = (kFeat & kFeatCsg) != 0;
    constexpr bool kTorus = (kFeat & kFeatTorus) != 0;
    constexpr int kNone = 0x7fffffff;
    const WalkLds W = walk_lds(S, smem);
    int best = -1;
    int result = 0;
    best_t = 0.0;
    const bool cont = !kShadow && !S.cfg.all_ni_one;  // refractive containers needed
    ContainerTop2 ct;
    ct.init();
    bool best_present = false;
    FRT_PROF_DECL
#ifdef FRT_WALK_STATS
    {
        const unsigned long long lv = __ballot(live);
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {
            atomicAdd(S.dbg + (kShadow ? 0 : 8) + 4, 1ull);
            atomicAdd(S.dbg + (kShadow ? 0 : 8) + 5, (unsigned long long)__popcll(lv));
        }
    }
#endif
    for (int ri = 0; ri < S.num_roots; ++ri) {
        if (__ballot(live) == 0) break;
        const int root = S.roots[ri];
        const int end = S.wn[root].skip;
        // entries behind the origin matter for the containers (closest hit) and, for shadow
        // rays, for the "first world shape with entries" rule before the last world shape
        const bool may_skip_behind = kShadow ? ri == S.num_roots - 1 : !cont;
        // uniform walk state; the tops of both frame stacks are cached here
        int sp = 0, xf_end = kNone;                             // transform frames
        int cp = 0, c_node = 0, c_skip = kNone, c_right = 0;   // composite frames (inside a CSG unit)
        int c_type = 0, c_op = 0;
        int n = 0;  // list entries of the open CSG unit (per lane)
        int resume = live ? 0 : kDone;
        bool any_entry = false;
        Ray cur = world;
#if FRT_PREFILTER
        FrameCache fc;
        frame_cache(cur, fc);
#endif
        int i = root;
        FRT_PROF(0);
        while (true) {
            FRT_PROF(7);
            // ---- close the composites the walk has left ----
            if constexpr (kCsg) {
                while (cp > 0) {
                    if (i < c_skip) {
                        // group_local_intersect's stop rule (group.c:114-121) for a group inside the unit
                        if (kShadow && c_type == FRT_GROUP && i > c_node + 1 && i >= resume) {
                            bool go_on = true;
                            for (int k = W.ca[(cp - 1) * kTraceBlock]; go_on && k < n; ++k) go_on = W.T(k) <= 0;
                            if (!go_on) resume = c_skip;
                        }
                        break;
                    }
                    n = close_composite(c_type, c_node, c_right, c_op, W, W.cs[(cp - 1) * kTraceBlock],
                                        W.ca[(cp - 1) * kTraceBlock], n);
                    --cp;
                    if (cp > 0) {
                        c_node = uniform(W.cn[cp - 1]);
                        const WalkNode& tn = S.wn[c_node];
                        c_skip = tn.skip;
                        c_right = tn.right;
                        c_type = tn.type;
                        c_op = tn.op;
                        continue;
                    }
                    c_skip = kNone;
                    // a CSG unit of the main walk is complete: the lane's list is [0, n)
                    if (resume != kDone) {
                        if (!kShadow) {
                            int unit_best = -1;
                            for (int k = 0; k < n; ++k) {
                                const double t = W.T(k);
                                if (t > 0 && (best < 0 || t < best_t) && (!filter_casts || S.casts[W.N(k)])) {
                                    best_t = t;
                                    best = W.N(k);
                                    unit_best = best;
                                }
                            }
                            if (cont) {
                                // per node of the unit: parity of its t <= 0 entries and its last one
                                for (int k = 0; k < n; ++k) {
                                    const int nk = W.N(k);
                                    int cnt = 0, last = -1;
                                    for (int q = 0; q < n; ++q) {
                                        if (W.N(q) == nk && W.T(q) <= 0) {
                                            ++cnt;
                                            if (last < 0 || W.T(q) > W.T(last) || (W.T(q) == W.T(last) && q > last))
                                                last = q;
                                        }
                                    }
                                    if (last == k && (cnt & 1)) ct.offer(W.T(k), nk, k);
                                }
                                if (unit_best >= 0) {
                                    int cnt = 0;
                                    for (int q = 0; q < n; ++q) cnt += (W.N(q) == unit_best && W.T(q) <= 0) ? 1 : 0;
                                    best_present = (cnt & 1) != 0;
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
            FRT_PROF(1);
            // ---- pop transform frames, rebuild the ray from the world ray ----
            if (i >= xf_end) {
                do {
                    --sp;
                    xf_end = sp > 0 ? S.wn[uniform(W.xn[sp - 1])].skip : kNone;
                } while (i >= xf_end);
                cur = world;
                for (int k = 0; k < sp; ++k) cur = xf_ray_walk(S.wn[uniform(W.xn[k])].m, cur);
#if FRT_PREFILTER
                frame_cache(cur, fc);
#endif
            }
            FRT_PROF(2);
            if (i >= end) break;
            const bool active = i >= resume;
            if (__ballot(active) == 0) {
#ifdef FRT_WALK_STATS
                if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) atomicAdd(S.dbg + (kShadow ? 0 : 8) + 3, 1ull);
#endif
                // every inactive lane has resume > i; max() only guards progress
                i = min(end, max(wave_min(resume), i + 1));
                continue;
            }
            if constexpr (kCsg) {
                if (cp > 0 && (c_type == FRT_GROUP || i == c_right)) W.ca[(cp - 1) * kTraceBlock] = n;
            }
            // ---- visit node i (uniform) ----
            const WalkNode& nd = S.wn[i];
            const int type = nd.type;
#ifdef FRT_WALK_STATS
            {
                const unsigned long long av = __ballot(active);
                if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {
                    atomicAdd(S.dbg + (kShadow ? 0 : 8) + ((type == FRT_GROUP || type == FRT_CSG) ? 0 : 1), 1ull);
                    atomicAdd(S.dbg + (kShadow ? 0 : 8) + 2, (unsigned long long)__popcll(av));
                    if (i < kDbgNodes) {
                        unsigned long long* pn = S.dbg + 16 + ((kShadow ? 0 : kDbgNodes) + i) * 2;
                        atomicAdd(pn, 1ull);
                        atomicAdd(pn + 1, (unsigned long long)__popcll(av));
                    }
                }
            }
#endif
            // prefilter: a lane whose ray cannot meet the node's parent-frame bound
            // (and cannot take the EPSILON branch in its local test) skips the node
            // A leaf of the main walk (outside CSG units) whose bound lies wholly
            // behind the ray, or (closest hit) beyond the best t, has no entry
            // that could matter either.
            bool may = active;
#if FRT_PREFILTER
            if ((nd.pre & 1) && !(S.walk_flags & 1)) {
                if (may) {
                    double pt0, pt1;
                    may = box_may_hit(nd.pbox, cur, fc.rc, pt0, pt1);
                    if (may && cp == 0 && type != FRT_GROUP && type != FRT_CSG) {
                        if (may_skip_behind && behind(pt1)) may = false;
                        if (!kShadow && best >= 0 && pt0 > best_t + 1e-6 * (1.0 + fabs(best_t))) may = false;
                    }
                    if (!may && (nd.pre & 2)) may = quirk_possible(nd.mrow, nd.mrow_l1, fc.df, fc.dmax);
                }
            }
#endif
#ifdef FRT_WALK_STATS
            {
                const unsigned long long pv = __ballot(active && !may), fv = __ballot(may);
                if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {
                    atomicAdd(S.dbg + (kShadow ? 0 : 8) + 6, (unsigned long long)__popcll(pv));
                    atomicAdd(S.dbg + (kShadow ? 0 : 8) + 7, (unsigned long long)__popcll(fv));
                }
            }
#endif
            if (type == FRT_GROUP || type == FRT_CSG) {
                bool enter = false;
                if (may) {
                    const Ray lr = nd.has_xf ? xf_ray_walk(nd.m, cur) : cur;
                    Frame32 lf;
                    frame32(lr, lf);
                    // binary32 decision with an error bound (box32), binary64 where it cannot decide
                    float tmin32 = -1.0f, tmax32 = 1.0f, err32 = 0.0f;
                    const int dec = (lf.exact || (S.walk_flags & 2)) ? -1 : box32(nd.bb32, nd.bmag, lf, tmin32, tmax32, err32);
                    double tmin = -1.0, tmax = 1.0;
                    if (dec >= 0) {
                        enter = dec != 0;
                        tmin = (double)tmin32 - (double)err32;  // bounds on the reference's tmin / tmax
                        tmax = (double)tmax32 + (double)err32;
                    } else if (origin_inside(nd.bbox, lr)) {
                        enter = true;
                    } else if (S.walk_flags & 2) {
                        enter = box_range(nd.bbox, lr, tmin, tmax);
                    } else {
                        double lrc[3];
#pragma unroll
                        for (int a = 0; a < 3; ++a) lrc[a] = recip<1>(lr.d[a]);
                        enter = box_decide(nd.bbox, lr, lrc, tmin, tmax);
                    }
                    if (cp == 0) {  // skips that cannot change this lane's answer (see header)
                        if (may_skip_behind && behind(tmax)) enter = false;
                        if (!kShadow && best >= 0 && tmin > best_t + 1e-6 * (1.0 + fabs(best_t))) enter = false;
                    }
                }
                if (active && !enter) resume = nd.skip;
                FRT_PROF(3);
                if (__ballot(enter) == 0) {
                    i = nd.skip;
                    continue;
                }
                if (nd.has_xf) {
                    if (sp >= S.xf_depth) {  // cannot happen: xf_depth is exact (upload)
                        err |= kErrXformDepth;
                        resume = kDone;
                        i = nd.skip;
                        continue;
                    }
                    if ((threadIdx.x & 63) == 0) W.xn[sp] = i;
                    ++sp;
                    xf_end = nd.skip;
                    cur = xf_ray_walk(nd.m, cur);
#if FRT_PREFILTER
                    frame_cache(cur, fc);
#endif
                }
                // a mesh (MeshDesc): each entering lane searches its BVH; the wave descends the group tree only
                // for lanes whose answer the search cannot confirm
                if (type == FRT_GROUP && nd.op > 0 && cp == 0 && (kShadow || (!cont && !filter_casts))) {
                    const MeshDesc& M = S.meshes[nd.op - 1];
                    if (!kShadow || M.last_root) {
                        bool fb = false;
                        if (enter) {
                            if constexpr (!kShadow) {
                                fb = !mesh_closest(S, M, cur, best_t, best, W.ms);
                            } else {
                                int f = -1;
                                double ft = 0.0;
                                fb = !mesh_first(S, M, cur, f, ft, W.ms);
                                if (!fb && f >= 0) {
                                    any_entry = true;
                                    result = (ft > 0 && ft < distance && S.casts[f]) ? 1 : 0;
                                    resume = kDone;
                                }
                            }
                            if (!fb && resume != kDone) resume = nd.skip;
                        }
                        if (__ballot(fb) == 0) {
                            i = nd.skip;
                            continue;
                        }
                    }
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
                        c_node = i;
                        c_skip = nd.skip;
                        c_right = nd.right;
                        c_type = type;
                        c_op = nd.op;
                    }
                }
                ++i;
                continue;
            }
            if (may) {
                const Ray lr = nd.has_xf ? xf_ray_walk(nd.m, cur) : cur;
                LeafHits H;
                FRT_PROF(4);
                if (kShadow && cp == 0 && type == FRT_CUBE && !(S.walk_flags & 4)) cube_hits_for_decisions(lr, distance, H);
                else leaf_hits<kTorus>(type, S.prim + nd.prim, lr, H);
                FRT_PROF(5);
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
                    bool took = false;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const double t = H.t.at(j);
                        if (j < H.t.n && t > 0 && (best < 0 || t < best_t) && (!filter_casts || nd.casts)) {
                            best_t = t;
                            best = i;
                            took = true;
                        }
                    }
                    if (cont) {
                        int cnt = 0, last = -1;
                        double tl = 0.0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const double t = H.t.at(j);
                            if (j < H.t.n && t <= 0) {
                                ++cnt;
                                if (last < 0 || t >= tl) {
                                    tl = t;
                                    last = j;
                                }
                            }
                        }
                        if (cnt & 1) ct.offer(tl, i, last);
                        if (took) best_present = (cnt & 1) != 0;
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
                        result = blocked && nd.casts ? 1 : 0;
                        resume = kDone;
                    }
                }
            }
            FRT_PROF(6);
            ++i;
        }
        if (kShadow && live && resume != kDone && any_entry) live = false;  // first world shape with entries ends it
        if (resume == kDone) live = false;
    }
    FRT_PROF_FLUSH;
    if (!kShadow && n12 != nullptr) {
        n12[0] = 1.0;
        n12[1] = 1.0;
        if (cont && best >= 0) {
            n12[0] = node_ni(S, ct.n1);
            n12[1] = best_present ? (best == ct.n1 ? node_ni(S, ct.n2) : n12[0]) : node_ni(S, best);
        }
    }
    return kShadow ? result : best;
}

// a node's transform chain (its own transform, then its transformed ancestors' through the tparent links):
// {n, the xform ids root-most first} for chains of up to three, n = -1 for deeper ones (the links then). One
// 16-byte load instead of the links' dependent loads (built at upload, frt_engine.hip)
__device__ __forceinline__ int4 xf_chain(const DevScene& S, int leaf) { return S.xchain[leaf]; }
__device__ __forceinline__ int xf_chain_id(const int4& c, int k) { return k == 0 ? c.y : k == 1 ? c.z : c.w; }

// recompute a leaf's local ray (through every transformed ancestor, root first,
// exactly as the walk composed it) — used to recover triangle (u, v)
__device__ inline Ray leaf_local_ray(const DevScene& S, int leaf, const Ray& world) {
    const int4 c = xf_chain(S, leaf);
    if (c.x >= 0) {
        Ray r = world;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < c.x) r = xf_ray(xform_of(S, xf_chain_id(c, k)), r);
        return r;
    }
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
