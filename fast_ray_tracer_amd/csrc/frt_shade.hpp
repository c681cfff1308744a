// frt-mi355x device shading: surface normals, patterns / textures,
// prepare_computations and the microfacet light model.
//
// Restates reference src/shapes/shapes.c:63-131 (normal_at with the parent
// chain and bump maps), src/pattern/pattern.c (every pattern kind and UV map),
// src/renderer/renderer.c:369-495 (prepare_computations) and :895-979
// (lighting_microfacet), in binary64 and in the reference's operation order.
#pragma once

#include "frt_traverse.hpp"

namespace frt {

// ---- transform chains (nearest transformed ancestors, tparent links) ----
__device__ __forceinline__ int first_xf(const DevScene& S, int leaf) {
    return S.nodes[leaf].xform >= 0 ? leaf : S.nodes[leaf].tparent;
}

// shape_world_to_object (shapes.c:117-131): root-most transform first; w0: the point's w is 0
// (a perturbed pattern's point, see pattern_at_shape), so no transform adds its translation
__device__ inline void world_to_object(const DevScene& S, int leaf, const double* p, double* out, bool w0 = false) {
    double q[3] = {p[0], p[1], p[2]};
    const int4 c = xf_chain(S, leaf);
    if (c.x >= 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k < c.x) {
                double t[3];
                if (w0) xf_vector(xform_of(S, xf_chain_id(c, k)), q, t);
                else xf_point(xform_of(S, xf_chain_id(c, k)), q, t);
                q[0] = t[0];
                q[1] = t[1];
                q[2] = t[2];
            }
        }
        out[0] = q[0];
        out[1] = q[1];
        out[2] = q[2];
        return;
    }
    const int first = first_xf(S, leaf);
    int n = 0;
    for (int x = first; x >= 0; x = S.nodes[x].tparent) n++;
    for (int k = n - 1; k >= 0; --k) {
        int x = first;
        for (int j = 0; j < k; ++j) x = S.nodes[x].tparent;
        double t[3];
        if (w0) xf_vector(xform_of(S, S.nodes[x].xform), q, t);
        else xf_point(xform_of(S, S.nodes[x].xform), q, t);
        q[0] = t[0];
        q[1] = t[1];
        q[2] = t[2];
    }
    out[0] = q[0];
    out[1] = q[1];
    out[2] = q[2];
}

// shape_normal_to_world (shapes.c:92-114): leaf-most transform first, each one
// followed by a normalize; identity levels copy without normalizing
__device__ inline void normal_to_world(const DevScene& S, int leaf, double* n) {
    const int4 c = xf_chain(S, leaf);
    if (c.x >= 0) {
#pragma unroll
        for (int k = 2; k >= 0; --k) {
            if (k < c.x) {
                double t[3];
                xf_normal_t(xform_of(S, xf_chain_id(c, k)), n, t);
                normalize3(t, n);
            }
        }
        return;
    }
    for (int x = first_xf(S, leaf); x >= 0; x = S.nodes[x].tparent) {
        double t[3];
        xf_normal_t(xform_of(S, S.nodes[x].xform), n, t);
        normalize3(t, n);
    }
}

__device__ inline void local_normal(const DevScene& S, int leaf, const double* lp, const Hit& h, double* n) {
    const frt_node& nd = S.nodes[leaf];
    n[0] = n[1] = n[2] = 0.0;
    switch (nd.type) {
    case FRT_SPHERE:
        n[0] = lp[0];
        n[1] = lp[1];
        n[2] = lp[2];
        return;
    case FRT_PLANE:
        n[1] = 1;
        return;
    case FRT_CUBE: {  // cube.c:80-96
        double ax = fabs(lp[0]), ay = fabs(lp[1]), az = fabs(lp[2]);
        double mx = fmax(fmax(ax, ay), az);
        if (feq(mx, ax)) n[0] = lp[0];
        else if (feq(mx, ay)) n[1] = lp[1];
        else n[2] = lp[2];
        return;
    }
    case FRT_CYLINDER:
    case FRT_CONE: {  // cylinder.c:90-105, cone.c:99-118
        const double* p = S.prim + nd.prim;
        double dist = lp[0] * lp[0] + lp[2] * lp[2];
        if (dist < 1 && ((p[1] - kEps) <= lp[1])) {
            n[1] = 1;
        } else if (dist < 1 && ((p[0] + kEps) >= lp[1])) {
            n[1] = -1;
        } else if (nd.type == FRT_CYLINDER) {
            n[0] = lp[0];
            n[2] = lp[2];
        } else {
            double y = sqrt(dist);
            if (lp[1] > 0) y = -y;
            n[0] = lp[0];
            n[1] = y;
            n[2] = lp[2];
        }
        return;
    }
    case FRT_TOROID: {  // toroid.c:55-65
        const double* p = S.prim + nd.prim;
        double r1 = p[0], r2 = p[1];
        double p_sq = r1 * r1 + r2 * r2;
        double mag = lp[0] * lp[0] + lp[1] * lp[1] + lp[2] * lp[2];
        double rv[3] = {4.0 * lp[0] * (mag - p_sq), 4.0 * lp[1] * (mag - p_sq + 2.0 * r1 * r1),
                        4.0 * lp[2] * (mag - p_sq)};
        normalize3(rv, n);
        return;
    }
    case FRT_TRIANGLE: {
        const double* p = S.prim + nd.prim + FRT_TRI_N;
        n[0] = p[0];
        n[1] = p[1];
        n[2] = p[2];
        return;
    }
    case FRT_SMOOTH_TRIANGLE: {  // triangle.c:158-174
        const double* p = S.prim + nd.prim;
        double w = 1.0 - h.u - h.v;
        for (int k = 0; k < 3; ++k) {
            double a = p[FRT_TRI_N2 + k] * h.u, b = p[FRT_TRI_N3 + k] * h.v;
            n[k] = p[FRT_TRI_N + k] * w + (a + b);
        }
        return;
    }
    default:
        return;
    }
}

// ---- patterns ----
__device__ inline void gradient_at(const frt_pattern& P, const double* ca, const double* cb, const double* pt, double* out) {
    double fr = pt[0] - floor(pt[0]);
    for (int k = 0; k < 3; ++k) {
        double dist = cb[k] - ca[k];
        out[k] = ca[k] + dist * fr;
    }
}

__device__ inline void radial_at(const double* ca, const double* cb, const double* pt, double* out) {
    double mag = sqrt(pt[0] * pt[0] + pt[2] * pt[2]);
    double fr = mag - floor(mag);
    for (int k = 0; k < 3; ++k) {
        double dist = cb[k] - ca[k];
        out[k] = ca[k] + dist * fr;
    }
}

__device__ inline void copy3(const double* a, double* o) {
    o[0] = a[0];
    o[1] = a[1];
    o[2] = a[2];
}

__device__ inline void uv_pattern_at(const DevScene& S, const frt_pattern& P, double u, double v, double* out) {
    switch (P.type) {
    case 5: {  // UV_ALIGN_CHECKER (pattern.c:238-258)
        const double* c = P.color[0];
        if (v > 0.8) {
            if (u < 0.2) c = P.color[1];
            else if (u > 0.8) c = P.color[2];
        } else if (v < 0.2) {
            if (u < 0.2) c = P.color[3];
            else if (u > 0.8) c = P.color[4];
        }
        copy3(c, out);
        return;
    }
    case 6: {  // UV_CHECKER (pattern.c:252-265)
        int u2 = (int)floor(u * (double)P.width);
        int v2 = (int)floor(v * (double)P.height);
        copy3(((u2 + v2) % 2 == 0) ? P.color[0] : P.color[1], out);
        return;
    }
    case 7: {  // UV_GRADIENT
        double pt[3] = {u, v, 0.0};
        gradient_at(P, P.color[0], P.color[1], pt, out);
        return;
    }
    case 8: {  // UV_RADIAL_GRADIENT
        double pt[3] = {u, v, 0.0};
        radial_at(P.color[0], P.color[1], pt, out);
        return;
    }
    case 9: {  // UV_TEXTURE (pattern.c:287-298): texel (round(u*(w-1)), round((1-v)*(h-1)))
        const frt_texture& T = S.textures[P.texture];
        double vv = 1 - v;
        double fc = round(u * (double)(T.width - 1));
        double fr = round(vv * (double)(T.height - 1));
        long col = (long)fc, row = (long)fr;
        col = col < 0 ? 0 : (col >= T.width ? T.width - 1 : col);  // out-of-range is UB in the reference
        row = row < 0 ? 0 : (row >= T.height ? T.height - 1 : row);
        copy3(S.texels + T.offset + 3 * ((size_t)row * T.width + col), out);
        return;
    }
    default:
        out[0] = u;
        out[1] = v;
        out[2] = 0;
        return;
    }
}

__device__ inline int uv_map(const DevScene& S, int leaf, int type, const double* pt, double& u, double& v) {
    const frt_node& nd = S.nodes[leaf];
    switch (type) {
    case 0: {  // CUBE_UV_MAP (pattern.c:311-356)
        double ax = fabs(pt[0]), ay = fabs(pt[1]), az = fabs(pt[2]);
        double coord = fmax(fmax(ax, ay), az);
        int face = feq(coord, pt[0]) ? 0 : feq(coord, -pt[0]) ? 1 : feq(coord, pt[1]) ? 2
                 : feq(coord, -pt[1]) ? 3 : feq(coord, pt[2]) ? 4 : 5;
        switch (face) {
        case 0: u = fmod((1.0 - pt[2]), 2.0) / 2.0; v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        case 1: u = fmod((pt[2] + 1.0), 2.0) / 2.0; v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        case 2: u = fmod((pt[0] + 1.0), 2.0) / 2.0; v = fmod((1.0 - pt[2]), 2.0) / 2.0; break;
        case 3: u = fmod((pt[0] + 1.0), 2.0) / 2.0; v = fmod((pt[2] + 1.0), 2.0) / 2.0; break;
        case 4: u = fmod((pt[0] + 1.0), 2.0) / 2.0; v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        default: u = fmod((1.0 - pt[0]), 2.0) / 2.0; v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        }
        return face;
    }
    case 1: {  // CYLINDER_UV_MAP (pattern.c:358-389)
        double mn = 0.0, mx = 0.0;
        if (nd.type == FRT_CYLINDER || nd.type == FRT_CONE) {
            mn = S.prim[nd.prim];
            mx = S.prim[nd.prim + 1];
        }
        int face = (mx - kEps) <= pt[1] ? 1 : (mn + kEps) >= pt[1] ? 2 : 0;
        if (face == 0) {
            double theta = atan2(pt[0], pt[2]);
            double raw_u = theta / (2.0 * kPi);
            u = 1.0 - (raw_u + 0.5);
            v = fmod(pt[1], 1.0);
        } else if (face == 1) {
            u = fmod((pt[0] + 1.0), 2.0) / 2.0;
            v = fmod((1.0 - pt[2]), 2.0) / 2.0;
        } else {
            u = fmod((pt[0] + 1.0), 2.0) / 2.0;
            v = fmod((pt[2] + 1.0), 2.0) / 2.0;
        }
        return face;
    }
    case 5: {  // TRIANGLE_UV_MAP (pattern.c:391-440)
        if (nd.type != FRT_TRIANGLE && nd.type != FRT_SMOOTH_TRIANGLE) {
            u = v = 0.0;
            return 0;
        }
        const double* p = S.prim + nd.prim;
        const double* e1 = p + FRT_TRI_E1;
        const double* e2 = p + FRT_TRI_E2;
        double v2[3] = {pt[0] - p[0], pt[1] - p[1], pt[2] - p[2]};
        double d00 = dot3(e1, e1), d01 = dot3(e1, e2), d11 = dot3(e2, e2);
        double d20 = dot3(v2, e1), d21 = dot3(v2, e2);
        double denom = 1.0 / (d00 * d11 - d01 * d01);
        double bv = fmod((d11 * d20 - d01 * d21) * denom, 1.0);
        double bw = fmod((d00 * d21 - d01 * d20) * denom, 1.0);
        double bu = 1.0 - bv - bw;
        const double* t = p + (nd.type == FRT_SMOOTH_TRIANGLE ? FRT_TRI_UV_SMOOTH : FRT_TRI_UV_FLAT);
        if (t[6] != 0.0) {
            double a0 = t[0] * bu, a1 = t[1] * bu;
            double b0 = t[2] * bv, b1 = t[3] * bv;
            double w = 1.0 - bu - bv;
            double c0 = t[4] * w, c1 = t[5] * w;
            a0 += b0 + c0;
            a1 += b1 + c1;
            u = fmod(a0, 1.0);
            v = fmod(a1, 1.0);
        } else {
            u = bu;
            v = bv;
        }
        if (u < 0) u += 1.0;
        if (v < 0) v += 1.0;
        return 0;
    }
    case 2: {  // PLANE_UV_MAP (pattern.c:442-457)
        double uu = fmod(pt[0], 1.0), vv = fmod(pt[2], 1.0);
        if (uu < 0) uu += 1.0;
        if (vv < 0) vv += 1.0;
        u = uu;
        v = vv;
        return 0;
    }
    case 3: {  // SPHERE_UV_MAP (pattern.c:459-475)
        double theta = atan2(pt[0], pt[2]);
        double radius = sqrt(pt[0] * pt[0] + pt[1] * pt[1] + pt[2] * pt[2]);
        double phi = acos(pt[1] / radius);
        double raw_u = theta / (2 * kPi);
        u = 1 - (raw_u + 0.5);
        v = 1 - phi / kPi;
        return 0;
    }
    case 4: {  // TOROID_UV_MAP (pattern.c:477-488)
        double r1 = nd.type == FRT_TOROID ? S.prim[nd.prim] : 0.0;
        u = (1.0 - (atan2(pt[2], pt[0]) + kPi) / (2 * kPi));
        double len = sqrt(pt[0] * pt[0] + pt[2] * pt[2]);
        double x = len - r1;
        v = (atan2(pt[1], x) + kPi) / (2 * kPi);
        return 0;
    }
    default:
        u = pt[0];
        v = pt[1];
        return 0;
    }
}

// pattern_at for the "base" kinds, with the two concrete colors overridable
// (nested patterns substitute them, pattern.c:41-78)
__device__ inline void base_pattern_at(const DevScene& S, const frt_pattern& P, int leaf, const double* pt,
                                       const double* ca, const double* cb, double* out) {
    switch (P.type) {
    case 0: {  // CHECKER (pattern.c:140-153)
        int t = (int)floor(pt[0]) + (int)floor(pt[1]) + (int)floor(pt[2]);
        copy3(t % 2 == 0 ? ca : cb, out);
        return;
    }
    case 1:
        gradient_at(P, ca, cb, pt, out);
        return;
    case 2:
        radial_at(ca, cb, pt, out);
        return;
    case 3: {  // RING
        int t = (int)floor(sqrt(pt[0] * pt[0] + pt[2] * pt[2]));
        copy3(t % 2 == 0 ? ca : cb, out);
        return;
    }
    case 4: {  // STRIPE
        int t = (int)floor(pt[0]);
        copy3(t % 2 == 0 ? ca : cb, out);
        return;
    }
    case 15: {  // TEXTURE_MAP (pattern.c:198-217): face from pt, uv from the face-transformed pt
        double u, v;
        int face = uv_map(S, leaf, P.uv_map, pt, u, v);
        const frt_pattern& F = S.patterns[P.faces + face];
        double q[3];
        if (F.transform_identity) copy3(pt, q);
        else xf_point(F.inv, pt, q);
        (void)uv_map(S, leaf, P.uv_map, q, u, v);
        uv_pattern_at(S, F, u, v, out);
        return;
    }
    default:
        copy3(pt, out);  // base_pattern_at returns the point (pattern.c:118-123)
        return;
    }
}

__device__ inline double noise3(int x, int y, int z, int octave, int seed) {
    unsigned n = (unsigned)x * 1919u + (unsigned)y * 31337u + (unsigned)z * 7669u + (unsigned)octave * 3463u +
                 (unsigned)seed * 13397u;
    n = (n << 13) ^ n;
    unsigned m = (n * (n * n * 15731u + 789221u) + 1376312589u) & 0x7fffffffu;
    return 1.0 - (double)(int)m / 1073741824.0;
}

__device__ inline double interp(double a, double b, double x) {
    double f = (1.0 - cos(x * kPi)) * 0.5;
    return a * (1.0 - f) + b * f;
}

__device__ inline double pnoise3(double x, double y, double z, double persistence, double frequency, int octaves, int seed) {
    double total = 0.0, amplitude = 1.0;
    for (int i = 0; i < octaves; ++i) {
        double X = x * frequency, Y = y * frequency, Z = z * frequency;
        int ix = (int)(X < 0 ? -X : X), iy = (int)(Y < 0 ? -Y : Y), iz = (int)(Z < 0 ? -Z : Z);
        double fx = X - ix, fy = Y - iy, fz = Z - iz;
        double i1 = interp(noise3(ix, iy, iz, i, seed), noise3(ix + 1, iy, iz, i, seed), fx);
        double i2 = interp(noise3(ix, iy + 1, iz, i, seed), noise3(ix + 1, iy + 1, iz, i, seed), fx);
        double i3 = interp(noise3(ix, iy, iz + 1, i, seed), noise3(ix + 1, iy, iz + 1, i, seed), fx);
        double i4 = interp(noise3(ix, iy + 1, iz + 1, i, seed), noise3(ix + 1, iy + 1, iz + 1, i, seed), fx);
        total += interp(interp(i1, i2, fy), interp(i3, i4, fy), fz) * amplitude;
        frequency /= 2.0;
        amplitude *= persistence;
    }
    return total;
}

// pattern_at_shape for world point wp (pattern.c:10-116); w0: wp's w component is 0 (below)
template <int D>
__device__ void pattern_at_shape(const DevScene& S, int pi, int leaf, const double* wp, double* out,
                                 const double* ov_a = nullptr, const double* ov_b = nullptr, bool w0 = false) {
    const frt_pattern& P = S.patterns[pi];
    if constexpr (D > 0) {
        if (P.type == 10) {  // BLENDED
            double c1[3], c2[3];
            pattern_at_shape<D - 1>(S, P.child[0], leaf, wp, c1, nullptr, nullptr, w0);
            pattern_at_shape<D - 1>(S, P.child[1], leaf, wp, c2, nullptr, nullptr, w0);
            for (int k = 0; k < 3; ++k) out[k] = (c1[k] + c2[k]) / 2.0;
            return;
        }
        if (P.type == 11) {  // NESTED
            double c1[3], c2[3];
            pattern_at_shape<D - 1>(S, P.child[1], leaf, wp, c1, nullptr, nullptr, w0);
            pattern_at_shape<D - 1>(S, P.child[2], leaf, wp, c2, nullptr, nullptr, w0);
            const frt_pattern& prim = S.patterns[P.child[0]];
            if (prim.type <= 4) pattern_at_shape<D - 1>(S, P.child[0], leaf, wp, out, c1, c2, w0);
            else pattern_at_shape<D - 1>(S, P.child[0], leaf, wp, out, nullptr, nullptr, w0);
            return;
        }
        if (P.type == 12) {  // PERTURBED
            double x = wp[0], y = wp[1], z = wp[2];
            double q[3];
            q[0] = wp[0] + P.scale_factor * pnoise3(x, y, z, P.persistence, P.frequency, P.octaves, P.seed);
            if (z < 0) z -= 1.0;
            else z += 1.0;
            q[1] = wp[1] + P.scale_factor * pnoise3(x, y, z, P.persistence, P.frequency, P.octaves, P.seed);
            if (z < 0) z -= 1.0;
            else z += 1.0;
            q[2] = wp[2] + P.scale_factor * pnoise3(x, y, z, P.persistence, P.frequency, P.octaves, P.seed);
            // the reference leaves the perturbed point's w uninitialised (pattern.c:110-113) and its
            // build reads it as 0 (pinned by the patterns_160x80 golden): the object and pattern
            // transforms then apply without their translations
            pattern_at_shape<D - 1>(S, P.child[0], leaf, q, out, nullptr, nullptr, true);
            return;
        }
    }
    double op[3], pp[3];
    world_to_object(S, leaf, wp, op, w0);
    if (P.transform_identity) copy3(op, pp);
    else if (w0) xf_vector(P.inv, op, pp);
    else xf_point(P.inv, op, pp);
    base_pattern_at(S, P, leaf, pp, ov_a ? ov_a : P.color[0], ov_b ? ov_b : P.color[1], out);
}

constexpr int kPatternDepth = 3;

// ---- prepare_computations (renderer.c:369-495) ----
struct Comps {
    double p[3], over_point[3], under_point[3], normalv[3], eyev[3], reflectv[3];
    double Ka[3], Kd[3], Ks[3], refl[3];
    double Ns, over_d, n1, n2;
    int leaf, material;
};

// kPat = false: the scene has no patterns (every map_* is -1), so the pattern
// code — most of prepare's registers and its scratch — is compiled out
template <bool kPat = true>
__device__ inline void normal_at(const DevScene& S, int leaf, const double* wp, const Hit& h, double* n) {
    double lp[3], ln[3];
    world_to_object(S, leaf, wp, lp);
    local_normal(S, leaf, lp, h, ln);
    normal_to_world(S, leaf, ln);
    const frt_material& M = S.materials[S.nodes[leaf].material];
    if (kPat && M.map_bump >= 0) {
        double tmp[3];
        pattern_at_shape<kPatternDepth>(S, M.map_bump, leaf, wp, tmp);
        for (int k = 0; k < 3; ++k) {
            tmp[k] *= 2.0;
            ln[k] += tmp[k] - 1.0;
        }
    }
    normalize3(ln, n);
}

template <bool kPat = true>
__device__ inline void prepare(const DevScene& S, const Ray& r, Hit h, Comps& c) {
    if (S.nodes[h.node].type == FRT_TRIANGLE || S.nodes[h.node].type == FRT_SMOOTH_TRIANGLE) {
        // the walk keeps (t, node) only; the triangle's (u, v) are recomputed with the same ray
        LeafHits H;
        const Ray lr = leaf_local_ray(S, h.node, r);
        leaf_hits<false>(S.nodes[h.node].type, S.prim + S.nodes[h.node].prim, lr, H);
        if (H.t.n > 0) {
            h.u = H.u;
            h.v = H.v;
        }
    }
    c.leaf = h.node;
    c.material = S.nodes[h.node].material;
    for (int k = 0; k < 3; ++k) c.p[k] = r.o[k] + r.d[k] * h.t;
    normal_at<kPat>(S, h.node, c.p, h, c.normalv);
    for (int k = 0; k < 3; ++k) c.eyev[k] = r.d[k] * -1.0;
    if (dot3(c.normalv, c.eyev) < 0) {
        for (int k = 0; k < 3; ++k) c.normalv[k] *= -1;
    }
    double dd = 2 * dot3(r.d, c.normalv);
    for (int k = 0; k < 3; ++k) c.reflectv[k] = r.d[k] - c.normalv[k] * dd;
    for (int k = 0; k < 3; ++k) {
        c.over_point[k] = c.p[k] + c.normalv[k] * kEps;
        c.under_point[k] = c.p[k] - c.normalv[k] * kEps;
    }
    c.n1 = 1.0;
    c.n2 = 1.0;
    const frt_material& M = S.materials[c.material];
    if (kPat && M.map_Ka >= 0) pattern_at_shape<kPatternDepth>(S, M.map_Ka, c.leaf, c.over_point, c.Ka);
    else copy3(M.Ka, c.Ka);
    if (kPat && M.map_Kd >= 0) pattern_at_shape<kPatternDepth>(S, M.map_Kd, c.leaf, c.over_point, c.Kd);
    else copy3(M.Kd, c.Kd);
    if (kPat && M.map_Ks >= 0) pattern_at_shape<kPatternDepth>(S, M.map_Ks, c.leaf, c.over_point, c.Ks);
    else copy3(M.Ks, c.Ks);
    if (kPat && M.map_refl >= 0) pattern_at_shape<kPatternDepth>(S, M.map_refl, c.leaf, c.over_point, c.refl);
    else copy3(M.refl, c.refl);
    if (kPat && M.map_Ns >= 0) {
        double tmp[3];
        pattern_at_shape<kPatternDepth>(S, M.map_Ns, c.leaf, c.over_point, tmp);
        c.Ns = tmp[0];
    } else {
        c.Ns = M.Ns;
    }
    if (kPat && M.map_d >= 0) {
        double tmp[3];
        pattern_at_shape<kPatternDepth>(S, M.map_d, c.leaf, c.over_point, tmp);
        c.over_d = tmp[0];
    } else {
        c.over_d = 1.0 - M.Tr;
    }
}

// schlick (renderer.c:607-624)
__device__ inline double schlick(const double* eyev, const double* normalv, double n1, double n2) {
    double co = dot3(eyev, normalv);
    if (n1 > n2) {
        double n = n1 / n2;
        double sin2_t = n * n * (1.0 - co * co);
        if (sin2_t > 1.0) return 1.0;
        co = sqrt(1.0 - sin2_t);
    }
    double r0 = (n1 - n2) / (n1 + n2);
    r0 = r0 * r0;
    return r0 + (1.0 - r0) * (1.0 - co) * (1.0 - co) * (1.0 - co) * (1.0 - co) * (1.0 - co);
}

}  // namespace frt
