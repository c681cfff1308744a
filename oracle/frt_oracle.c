/*
 * TEST INFRASTRUCTURE ONLY — see frt_oracle.h. Never linked into the product.
 *
 * Plain-C restatement of the reference's render recursion over the host scene
 * graph. Each function cites the reference code it restates; operation order
 * follows the reference so results are bit-identical on deterministic scenes
 * (gcc, -O2 -ffp-contract=off; glibc libm, as the reference uses).
 */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "frt_oracle.h"
#include "src/pattern/pattern.h"
#include "src/material/material.h"

typedef struct oray {
    double o[4];
    double d[4];
} oray;

typedef struct ohit {
    double t, u, v;
    Shape obj;
} ohit;

typedef struct hitlist {
    ohit *v;
    size_t n, cap;
} hitlist;

typedef struct octx {
    World w;
    hitlist xs;      /* scratch for one intersect_world call chain */
    Shape *container;
    size_t container_cap;
    frt_oracle_stats st;
    /* setup_config statics (renderer.c:54-71) */
    bool include_direct, include_ambient, include_diffuse, include_spec_highlight, include_specular;
    size_t path_length;
} octx;

static void
hl_push(hitlist *l, double t, double u, double v, Shape obj)
{
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 256;
        l->v = (ohit *)realloc(l->v, l->cap * sizeof(ohit));
    }
    l->v[l->n].t = t;
    l->v[l->n].u = u;
    l->v[l->n].v = v;
    l->v[l->n].obj = obj;
    l->n++;
}

/* qsort comparator semantics of sort_intersections_asc (intersection.c:108-119);
 * glibc qsort is a stable merge sort at these sizes, so a stable insertion sort
 * gives the same permutation. */
static int
cmp_t(double l, double r)
{
    return (l - r < 0) ? -1 : ((l - r > 0) ? 1 : 0);
}

static void
sort_range(ohit *a, size_t n)
{
    for (size_t i = 1; i < n; ++i) {
        ohit cur = a[i];
        size_t j = i;
        while (j > 0 && cmp_t(a[j - 1].t, cur.t) > 0) {
            a[j] = a[j - 1];
            --j;
        }
        a[j] = cur;
    }
}

static void
mat_apply4(const double *m, const double *in, double *out)
{
    double r[4];
    for (int k = 0; k < 4; ++k) {
        r[k] = m[4 * k + 0] * in[0] + m[4 * k + 1] * in[1] + m[4 * k + 2] * in[2] + m[4 * k + 3] * in[3];
    }
    memcpy(out, r, sizeof(r));
}

static double dot3(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static void
normalize3(const double *v, double *res)
{
    double inv = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double x = v[0], y = v[1], z = v[2];
    res[0] = x * inv;
    res[1] = y * inv;
    res[2] = z * inv;
    res[3] = 0.0;
}

static void
cross3(const double *a, const double *b, double *res)
{
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    res[0] = x;
    res[1] = y;
    res[2] = z;
    res[3] = 0.0;
}

/* ---------------- quartic (reference src/libs/quartic/Roots3And4.c) ---------------- */

#define EQN_EPS 1e-9
#define IS_ZERO(x) ((x) > -EQN_EPS && (x) < EQN_EPS)

static int
solve_quadric(const double c[3], double s[2])
{
    double p = c[1] / (2 * c[2]);
    double q = c[0] / c[2];
    double D = p * p - q;
    if (IS_ZERO(D)) {
        s[0] = -p;
        return 1;
    }
    if (D < 0) {
        return 0;
    }
    double sd = sqrt(D);
    s[0] = sd - p;
    s[1] = -sd - p;
    return 2;
}

static int
solve_cubic(const double c[4], double s[3])
{
    double A = c[2] / c[3], B = c[1] / c[3], C = c[0] / c[3];
    double sq_A = A * A;
    double p = 1.0 / 3 * (-1.0 / 3 * sq_A + B);
    double q = 1.0 / 2 * (2.0 / 27 * A * sq_A - 1.0 / 3 * A * B + C);
    double cb_p = p * p * p;
    double D = q * q + cb_p;
    int num;
    if (IS_ZERO(D)) {
        if (IS_ZERO(q)) {
            s[0] = 0;
            num = 1;
        } else {
            double u = cbrt(-q);
            s[0] = 2 * u;
            s[1] = -u;
            num = 2;
        }
    } else if (D < 0) {
        double phi = 1.0 / 3 * acos(-q / sqrt(-cb_p));
        double t = 2 * sqrt(-p);
        s[0] = t * cos(phi);
        s[1] = -t * cos(phi + M_PI / 3);
        s[2] = -t * cos(phi - M_PI / 3);
        num = 3;
    } else {
        double sd = sqrt(D);
        double u = cbrt(sd - q);
        double v = -cbrt(sd + q);
        s[0] = u + v;
        num = 1;
    }
    double sub = 1.0 / 3 * A;
    for (int i = 0; i < num; ++i) {
        s[i] -= sub;
    }
    return num;
}

static int
solve_quartic(const double c[5], double s[4])
{
    double coeffs[4];
    double A = c[3] / c[4], B = c[2] / c[4], C = c[1] / c[4], D = c[0] / c[4];
    double sq_A = A * A;
    double p = -3.0 / 8 * sq_A + B;
    double q = 1.0 / 8 * sq_A * A - 1.0 / 2 * A * B + C;
    double r = -3.0 / 256 * sq_A * sq_A + 1.0 / 16 * sq_A * B - 1.0 / 4 * A * C + D;
    int num;
    if (IS_ZERO(r)) {
        coeffs[0] = q;
        coeffs[1] = p;
        coeffs[2] = 0;
        coeffs[3] = 1;
        num = solve_cubic(coeffs, s);
        s[num++] = 0;
    } else {
        coeffs[0] = 1.0 / 2 * r * p - 1.0 / 8 * q * q;
        coeffs[1] = -r;
        coeffs[2] = -1.0 / 2 * p;
        coeffs[3] = 1;
        (void)solve_cubic(coeffs, s);
        double z = s[0];
        double u = z * z - r;
        double v = 2 * z - p;
        if (IS_ZERO(u)) {
            u = 0;
        } else if (u > 0) {
            u = sqrt(u);
        } else {
            return 0;
        }
        if (IS_ZERO(v)) {
            v = 0;
        } else if (v > 0) {
            v = sqrt(v);
        } else {
            return 0;
        }
        double q1[3] = {z - u, q < 0 ? -v : v, 1};
        num = solve_quadric(q1, s);
        double q2[3] = {z + u, q < 0 ? v : -v, 1};
        num += solve_quadric(q2, s + num);
    }
    double sub = 1.0 / 4 * A;
    for (int i = 0; i < num; ++i) {
        s[i] -= sub;
    }
    return num;
}

/* ---------------- primitive intersections ---------------- */

static void
axis_slab(double o, double d, double lo, double hi, double *a, double *b)
{
    /* check_axis (cube.c:16-53) / bbox_check_axis (bounding_box.c:124-162) */
    double nl = lo - o, nh = hi - o, t0, t1;
    if (fabs(d) >= EPSILON) {
        t0 = nl / d;
        t1 = nh / d;
    } else {
        t0 = nl * INFINITY;
        if (isnan(t0)) t0 = nl < 0 ? -INFINITY : INFINITY;
        t1 = nh * INFINITY;
        if (isnan(t1)) t1 = nh < 0 ? -INFINITY : INFINITY;
    }
    if (t0 > t1) {
        *a = t1;
        *b = t0;
    } else {
        *a = t0;
        *b = t1;
    }
}

static bool
box_hit(const Bounding_box *bx, const oray *r)
{
    double x0, x1, y0, y1, z0, z1;
    axis_slab(r->o[0], r->d[0], bx->min[0], bx->max[0], &x0, &x1);
    axis_slab(r->o[1], r->d[1], bx->min[1], bx->max[1], &y0, &y1);
    axis_slab(r->o[2], r->d[2], bx->min[2], bx->max[2], &z0, &z1);
    return fmax(fmax(x0, y0), z0) <= fmin(fmin(x1, y1), z1);
}

static void
local_leaf(Shape s, const oray *r, hitlist *out)
{
    switch (s->type) {
    case SHAPE_SPHERE: { /* sphere.c:14-39 */
        double a = dot3(r->d, r->d);
        double b = 2 * dot3(r->d, r->o);
        double c = dot3(r->o, r->o) - 1.0;
        double disc = b * b - 4 * a * c;
        if (disc < 0) return;
        disc = sqrt(disc);
        a = 1.0 / (2 * a);
        hl_push(out, (-b - disc) * a, -1, -1, s);
        hl_push(out, (-b + disc) * a, -1, -1, s);
        return;
    }
    case SHAPE_PLANE: /* plane.c:11-24 */
        if (fabs(r->d[1]) < EPSILON) return;
        hl_push(out, -r->o[1] / r->d[1], -1, -1, s);
        return;
    case SHAPE_CUBE: { /* cube.c:56-77 */
        double x0, x1, y0, y1, z0, z1;
        axis_slab(r->o[0], r->d[0], -1, 1, &x0, &x1);
        axis_slab(r->o[1], r->d[1], -1, 1, &y0, &y1);
        axis_slab(r->o[2], r->d[2], -1, 1, &z0, &z1);
        double tmin = fmax(fmax(x0, y0), z0), tmax = fmin(fmin(x1, y1), z1);
        if (tmin > tmax) return;
        hl_push(out, tmin, -1, -1, s);
        hl_push(out, tmax, -1, -1, s);
        return;
    }
    case SHAPE_CYLINDER: { /* cylinder.c:11-87 */
        const struct cone_cylinder_fields *f = &s->fields.cylinder;
        double a = r->d[0] * r->d[0] + r->d[2] * r->d[2];
        double b = 2 * (r->o[0] * r->d[0] + r->o[2] * r->d[2]);
        double c = r->o[0] * r->o[0] + r->o[2] * r->o[2] - 1;
        if (!equal(a, 0.0)) {
            double disc = b * b - 4 * a * c;
            if (disc < 0) return;
            double sq = sqrt(disc);
            double t0 = (-b - sq) / (2 * a), t1 = (-b + sq) / (2 * a);
            if (t0 > t1) {
                double tt = t0;
                t0 = t1;
                t1 = tt;
            }
            double y0 = r->o[1] + t0 * r->d[1];
            if (f->minimum <= y0 && y0 <= f->maximum) hl_push(out, t0, -1, -1, s);
            double y1 = r->o[1] + t1 * r->d[1];
            if (f->minimum <= y1 && y1 <= f->maximum) hl_push(out, t1, -1, -1, s);
        }
        if (!f->closed || equal(r->d[1], 0.0)) return;
        double ta = (f->minimum - r->o[1]) / r->d[1];
        double tb = (f->maximum - r->o[1]) / r->d[1];
        double xa = r->o[0] + ta * r->d[0], za = r->o[2] + ta * r->d[2];
        if (xa * xa + za * za <= 1) hl_push(out, ta, -1, -1, s);
        double xb = r->o[0] + tb * r->d[0], zb = r->o[2] + tb * r->d[2];
        if (xb * xb + zb * zb <= 1) hl_push(out, tb, -1, -1, s);
        return;
    }
    case SHAPE_CONE: { /* cone.c:11-96 */
        const struct cone_cylinder_fields *f = &s->fields.cone;
        double a = r->d[0] * r->d[0] + r->d[2] * r->d[2] - r->d[1] * r->d[1];
        double b = 2 * (r->o[0] * r->d[0] + r->o[2] * r->d[2] - r->o[1] * r->d[1]);
        double c = r->o[0] * r->o[0] + r->o[2] * r->o[2] - r->o[1] * r->o[1];
        if (equal(a, 0.0)) {
            if (!equal(b, 0.0)) hl_push(out, -c / (2 * b), -1, -1, s);
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
            double y0 = r->o[1] + t0 * r->d[1];
            if (f->minimum < y0 && y0 < f->maximum) hl_push(out, t0, -1, -1, s);
            double y1 = r->o[1] + t1 * r->d[1];
            if (f->minimum < y1 && y1 < f->maximum) hl_push(out, t1, -1, -1, s);
        }
        if (!f->closed || equal(r->d[1], 0.0)) return;
        double ta = (f->minimum - r->o[1]) / r->d[1];
        double xa = r->o[0] + ta * r->d[0], za = r->o[2] + ta * r->d[2];
        if (xa * xa + za * za <= fabs(f->minimum)) hl_push(out, ta, -1, -1, s);
        double tb = (f->maximum - r->o[1]) / r->d[1];
        double xb = r->o[0] + tb * r->d[0], zb = r->o[2] + tb * r->d[2];
        if (xb * xb + zb * zb <= fabs(f->maximum)) hl_push(out, tb, -1, -1, s);
        return;
    }
    case SHAPE_TOROID: { /* toroid.c:15-52 */
        double ox = r->o[0], oy = r->o[1], oz = r->o[2];
        double dx = r->d[0], dy = r->d[1], dz = r->d[2];
        double r1 = s->fields.toroid.r1, r2 = s->fields.toroid.r2;
        double sum_d_sq = dx * dx + dy * dy + dz * dz;
        double e = ox * ox + oy * oy + oz * oz - r1 * r1 - r2 * r2;
        double f = ox * dx + oy * dy + oz * dz;
        double four_a_sq = 4.0 * r1 * r1;
        double coeffs[5] = {e * e - four_a_sq * (r2 * r2 - oy * oy),
                            4.0 * f * e + 2.0 * four_a_sq * oy * dy,
                            2.0 * sum_d_sq * e + 4.0 * f * f + four_a_sq * dy * dy,
                            4.0 * sum_d_sq * f,
                            sum_d_sq * sum_d_sq};
        double sol[4];
        int n = solve_quartic(coeffs, sol);
        for (; n > 0; n--) hl_push(out, sol[n - 1], -1, -1, s);
        return;
    }
    case SHAPE_TRIANGLE:
    case SHAPE_SMOOTH_TRIANGLE: { /* triangle.c:11-44 / 122-155 */
        const struct triangle_fields *tf = &s->fields.triangle;
        double dce2[4], p1o[4], oce1[4];
        cross3(r->d, tf->e2, dce2);
        double det = dot3(tf->e1, dce2);
        if (fabs(det) < EPSILON) return;
        double fi = 1.0 / det;
        p1o[0] = r->o[0] - tf->p1[0];
        p1o[1] = r->o[1] - tf->p1[1];
        p1o[2] = r->o[2] - tf->p1[2];
        double u = fi * dot3(p1o, dce2);
        if (u < 0 || u > 1) return;
        cross3(p1o, tf->e1, oce1);
        double v = fi * dot3(r->d, oce1);
        if (v < 0 || (u + v) > 1) return;
        double t = fi * dot3(tf->e2, oce1);
        hl_push(out, t, u, v, s);
        return;
    }
    default:
        return;
    }
}

static bool
csg_allowed(enum csg_ops_enum op, bool lhit, bool inl, bool inr)
{
    /* csg.c:28-40 */
    if (op == CSG_UNION) return (lhit && !inr) || (!lhit && !inl);
    if (op == CSG_INTERSECT) return (lhit && inr) || (!lhit && inl);
    if (op == CSG_DIFFERENCE) return (lhit && !inr) || (!lhit && inl);
    return false;
}

static size_t
csg_filter(Shape s, ohit *a, size_t n)
{
    /* csg.c:43-71 */
    bool inl = false, inr = false;
    size_t kept = 0;
    for (size_t i = 0; i < n; ++i) {
        bool lhit = shape_includes(s->fields.csg.left, a[i].obj);
        if (csg_allowed(s->fields.csg.op, lhit, inl, inr)) {
            a[kept++] = a[i];
        }
        if (lhit) inl = !inl;
        else inr = !inr;
    }
    return kept;
}

static void intersect_shape(Shape s, const oray *r, bool stop, hitlist *out);

static void
local_intersect(Shape s, const oray *r, bool stop, hitlist *out)
{
    if (s->type == SHAPE_GROUP) { /* group.c:92-147 */
        Bounding_box box;
        shape_bounds(s, &box);
        if (!box_hit(&box, r)) return;
        size_t start = out->n;
        for (size_t i = 0; i < s->fields.group.num_children; ++i) {
            size_t cs = out->n;
            intersect_shape(s->fields.group.children + i, r, stop, out);
            if (stop) {
                bool go_on = true;
                for (size_t k = cs; go_on && k < out->n; ++k) go_on = out->v[k].t <= 0;
                if (!go_on) break;
            }
        }
        if (out->n - start > 0) sort_range(out->v + start, out->n - start);
        return;
    }
    if (s->type == SHAPE_CSG) { /* csg.c:74-125 */
        Bounding_box box;
        shape_bounds(s, &box);
        if (!box_hit(&box, r)) return;
        size_t start = out->n;
        intersect_shape(s->fields.csg.left, r, stop, out);
        size_t mid = out->n;
        intersect_shape(s->fields.csg.right, r, stop, out);
        size_t end = out->n;
        size_t nl = mid - start, nr = end - mid;
        if (nl + nr == 0) return;
        if (nl == 0) {
            size_t k = csg_filter(s, out->v + mid, nr);
            memmove(out->v + start, out->v + mid, k * sizeof(ohit));
            out->n = start + k;
        } else if (nr == 0) {
            out->n = start + csg_filter(s, out->v + start, nl);
        } else {
            sort_range(out->v + start, nl + nr);
            out->n = start + csg_filter(s, out->v + start, nl + nr);
        }
        return;
    }
    local_leaf(s, r, out);
}

static void
intersect_shape(Shape s, const oray *r, bool stop, hitlist *out)
{
    /* shape_intersect (shapes.c:42-56): transform unless the transform is ~identity */
    if (s->transform_identity) {
        local_intersect(s, r, stop, out);
    } else {
        oray t;
        mat_apply4(s->transform_inverse, r->o, t.o);
        mat_apply4(s->transform_inverse, r->d, t.d);
        local_intersect(s, &t, stop, out);
    }
}

static void
intersect_world(octx *cx, const oray *r, bool stop)
{
    /* world.c:163-197 */
    hitlist *xs = &cx->xs;
    xs->n = 0;
    for (size_t i = 0; i < cx->w->shapes_num; ++i) {
        size_t before = xs->n;
        intersect_shape(cx->w->shapes + i, r, stop, xs);
        if (xs->n > before && stop) break;
    }
    if (xs->n > 1) sort_range(xs->v, xs->n);
}

static long
hit_index(const hitlist *xs, bool shadow)
{
    /* hit (intersection.c:42-55) */
    for (size_t i = 0; i < xs->n; ++i) {
        if (xs->v[i].t > 0 && (!shadow || xs->v[i].obj->material->casts_shadow)) return (long)i;
    }
    return -1;
}

static bool
is_shadowed(octx *cx, const double *light_pos, const double *pt)
{
    /* renderer.c:74-93 */
    double v[4], dir[4];
    v[0] = light_pos[0] - pt[0];
    v[1] = light_pos[1] - pt[1];
    v[2] = light_pos[2] - pt[2];
    v[3] = 0.0;
    double distance = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    normalize3(v, dir);
    oray r;
    memcpy(r.o, pt, 4 * sizeof(double));
    memcpy(r.d, dir, 4 * sizeof(double));
    cx->st.shadow_rays++;
    intersect_world(cx, &r, true);
    long h = hit_index(&cx->xs, true);
    return h >= 0 && cx->xs.v[h].t < distance;
}

/* ---------------- normals ---------------- */

static void
world_to_object(Shape s, const double *pt, double *res)
{
    /* shapes.c:117-131 */
    double tmp[4];
    if (s->parent) world_to_object(s->parent, pt, tmp);
    else memcpy(tmp, pt, sizeof(tmp));
    if (s->transform_identity) memcpy(res, tmp, sizeof(tmp));
    else mat_apply4(s->transform_inverse, tmp, res);
}

static void
normal_to_world(Shape s, const double *n, double *res)
{
    /* shapes.c:92-114 */
    double nn[4];
    if (s->transform_identity) {
        memcpy(nn, n, sizeof(nn));
    } else {
        double tr[16], un[4];
        matrix_transpose(s->transform_inverse, tr);
        mat_apply4(tr, n, un);
        normalize3(un, nn);
    }
    if (s->parent) normal_to_world(s->parent, nn, res);
    else memcpy(res, nn, sizeof(nn));
}

static void
local_normal(Shape s, const double *lp, const ohit *h, double *res)
{
    memset(res, 0, 4 * sizeof(double));
    switch (s->type) {
    case SHAPE_SPHERE:
        res[0] = lp[0];
        res[1] = lp[1];
        res[2] = lp[2];
        return;
    case SHAPE_PLANE:
        res[1] = 1;
        return;
    case SHAPE_CUBE: { /* cube.c:80-96 */
        double ax = fabs(lp[0]), ay = fabs(lp[1]), az = fabs(lp[2]);
        double mx = fmax(fmax(ax, ay), az);
        if (equal(mx, ax)) res[0] = lp[0];
        else if (equal(mx, ay)) res[1] = lp[1];
        else res[2] = lp[2];
        return;
    }
    case SHAPE_CYLINDER:
    case SHAPE_CONE: { /* cylinder.c:90-105, cone.c:99-118 */
        const struct cone_cylinder_fields *f = &s->fields.cylinder;
        double dist = lp[0] * lp[0] + lp[2] * lp[2];
        if (dist < 1 && ((f->maximum - EPSILON) <= lp[1])) {
            res[1] = 1;
        } else if (dist < 1 && ((f->minimum + EPSILON) >= lp[1])) {
            res[1] = -1;
        } else if (s->type == SHAPE_CYLINDER) {
            res[0] = lp[0];
            res[2] = lp[2];
        } else {
            double y = sqrt(dist);
            if (lp[1] > 0) y = -y;
            res[0] = lp[0];
            res[1] = y;
            res[2] = lp[2];
        }
        return;
    }
    case SHAPE_TOROID: { /* toroid.c:55-65 */
        double r1 = s->fields.toroid.r1, r2 = s->fields.toroid.r2;
        double p_sq = r1 * r1 + r2 * r2;
        double mag = lp[0] * lp[0] + lp[1] * lp[1] + lp[2] * lp[2];
        double rv[4] = {4.0 * lp[0] * (mag - p_sq), 4.0 * lp[1] * (mag - p_sq + 2.0 * r1 * r1),
                        4.0 * lp[2] * (mag - p_sq), 0.0};
        normalize3(rv, res);
        return;
    }
    case SHAPE_TRIANGLE:
        memcpy(res, s->fields.triangle.u_normals.normal, 4 * sizeof(double));
        return;
    case SHAPE_SMOOTH_TRIANGLE: { /* triangle.c:158-174 */
        const double *n1 = s->fields.triangle.u_normals.s_normals.n1;
        const double *n2 = s->fields.triangle.u_normals.s_normals.n2;
        const double *n3 = s->fields.triangle.u_normals.s_normals.n3;
        double w = 1.0 - h->u - h->v;
        for (int k = 0; k < 3; ++k) {
            double a = n2[k] * h->u, b = n3[k] * h->v;
            res[k] = n1[k] * w + (a + b);
        }
        res[3] = n1[3];
        return;
    }
    default:
        return;
    }
}

static void pattern_at_shape(Pattern p, Shape s, const double *pt, double *res);

static void
normal_at(Shape s, const double *wp, const ohit *h, double *res)
{
    /* shape_normal_at (shapes.c:63-89) */
    double lp[4], ln[4], wn[4];
    world_to_object(s, wp, lp);
    local_normal(s, lp, h, ln);
    normal_to_world(s, ln, wn);
    if (s->material->map_bump) {
        double tmp[4];
        pattern_at_shape(s->material->map_bump, s, wp, tmp);
        for (int k = 0; k < 3; ++k) {
            tmp[k] *= 2.0;
            wn[k] += tmp[k] - 1.0;
        }
    }
    normalize3(wn, res);
}

/* ---------------- patterns (pattern.c) ---------------- */

static void
gradient_at(const Pattern p, const double *pt, double *res)
{
    double dist[3] = {p->fields.concrete.b[0] - p->fields.concrete.a[0], p->fields.concrete.b[1] - p->fields.concrete.a[1],
                      p->fields.concrete.b[2] - p->fields.concrete.a[2]};
    double fr = pt[0] - floor(pt[0]);
    for (int k = 0; k < 3; ++k) res[k] = p->fields.concrete.a[k] + dist[k] * fr;
}

static void
radial_at(const Pattern p, const double *pt, double *res)
{
    double dist[3] = {p->fields.concrete.b[0] - p->fields.concrete.a[0], p->fields.concrete.b[1] - p->fields.concrete.a[1],
                      p->fields.concrete.b[2] - p->fields.concrete.a[2]};
    double mag = sqrt(pt[0] * pt[0] + pt[2] * pt[2]);
    double fr = mag - floor(mag);
    for (int k = 0; k < 3; ++k) res[k] = p->fields.concrete.a[k] + dist[k] * fr;
}

static void
uv_pattern_at(const Pattern p, double u, double v, double *res)
{
    switch (p->type) {
    case UV_ALIGN_CHECKER_PATTERN: { /* pattern.c:238-258 */
        const double *c = p->fields.uv_align_check.main;
        if (v > 0.8) {
            if (u < 0.2) c = p->fields.uv_align_check.ul;
            else if (u > 0.8) c = p->fields.uv_align_check.ur;
        } else if (v < 0.2) {
            if (u < 0.2) c = p->fields.uv_align_check.bl;
            else if (u > 0.8) c = p->fields.uv_align_check.br;
        }
        memcpy(res, c, sizeof(Color));
        return;
    }
    case UV_CHECKER_PATTERN: { /* pattern.c:252-265 */
        int u2 = (int)floor(u * (double)p->fields.uv_check.width);
        int v2 = (int)floor(v * (double)p->fields.uv_check.height);
        memcpy(res, ((u2 + v2) % 2 == 0) ? p->fields.uv_check.a : p->fields.uv_check.b, sizeof(Color));
        return;
    }
    case UV_GRADIENT_PATTERN: {
        double pt[4] = {u, v, 0.0, 1.0};
        gradient_at(p, pt, res);
        return;
    }
    case UV_RADIAL_GRADIENT_PATTERN: {
        double pt[4] = {u, v, 0.0, 1.0};
        radial_at(p, pt, res);
        return;
    }
    case UV_TEXTURE_PATTERN: { /* pattern.c:287-298 */
        Canvas cv = p->fields.uv_texture.canvas;
        double vv = 1 - v;
        size_t col = (size_t)round(u * (double)(cv->width - 1));
        size_t row = (size_t)round(vv * (double)(cv->height - 1));
        canvas_pixel_at(cv, (int)col, (int)row, res);
        return;
    }
    default:
        res[0] = u;
        res[1] = v;
        res[2] = 0;
        return;
    }
}

static int
uv_map(Shape s, enum uv_map_type type, const double *pt, double *u, double *v)
{
    switch (type) {
    case CUBE_UV_MAP: { /* pattern.c:311-356 */
        double ax = fabs(pt[0]), ay = fabs(pt[1]), az = fabs(pt[2]);
        double coord = fmax(fmax(ax, ay), az);
        int face = equal(coord, pt[0]) ? 0 : equal(coord, -pt[0]) ? 1 : equal(coord, pt[1]) ? 2
                 : equal(coord, -pt[1]) ? 3 : equal(coord, pt[2]) ? 4 : 5;
        switch (face) {
        case 0: *u = fmod((1.0 - pt[2]), 2.0) / 2.0; *v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        case 1: *u = fmod((pt[2] + 1.0), 2.0) / 2.0; *v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        case 2: *u = fmod((pt[0] + 1.0), 2.0) / 2.0; *v = fmod((1.0 - pt[2]), 2.0) / 2.0; break;
        case 3: *u = fmod((pt[0] + 1.0), 2.0) / 2.0; *v = fmod((pt[2] + 1.0), 2.0) / 2.0; break;
        case 4: *u = fmod((pt[0] + 1.0), 2.0) / 2.0; *v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        default: *u = fmod((1.0 - pt[0]), 2.0) / 2.0; *v = fmod((pt[1] + 1.0), 2.0) / 2.0; break;
        }
        return face;
    }
    case CYLINDER_UV_MAP: { /* pattern.c:358-389 */
        int face = (s->fields.cylinder.maximum - EPSILON) <= pt[1] ? 1 : (s->fields.cylinder.minimum + EPSILON) >= pt[1] ? 2 : 0;
        if (face == 0) {
            double theta = atan2(pt[0], pt[2]);
            double raw_u = theta / (2.0 * M_PI);
            *u = 1.0 - (raw_u + 0.5);
            *v = fmod(pt[1], 1.0);
        } else if (face == 1) {
            *u = fmod((pt[0] + 1.0), 2.0) / 2.0;
            *v = fmod((1.0 - pt[2]), 2.0) / 2.0;
        } else {
            *u = fmod((pt[0] + 1.0), 2.0) / 2.0;
            *v = fmod((pt[2] + 1.0), 2.0) / 2.0;
        }
        return face;
    }
    case TRIANGLE_UV_MAP: { /* pattern.c:391-440 */
        const struct triangle_fields *tf = &s->fields.triangle;
        double v2[4] = {pt[0] - tf->p1[0], pt[1] - tf->p1[1], pt[2] - tf->p1[2], 0.0};
        double d00 = dot3(tf->e1, tf->e1), d01 = dot3(tf->e1, tf->e2), d11 = dot3(tf->e2, tf->e2);
        double d20 = dot3(v2, tf->e1), d21 = dot3(v2, tf->e2);
        double denom = 1.0 / (d00 * d11 - d01 * d01);
        double bv = fmod((d11 * d20 - d01 * d21) * denom, 1.0);
        double bw = fmod((d00 * d21 - d01 * d20) * denom, 1.0);
        double bu = 1.0 - bv - bw;
        if (tf->use_textures) {
            double a[3], b[3], c[3];
            for (int k = 0; k < 3; ++k) {
                a[k] = tf->t1[k] * bu;
                b[k] = tf->t2[k] * bv;
                c[k] = tf->t3[k] * (1.0 - bu - bv);
                a[k] += b[k] + c[k];
            }
            *u = fmod(a[0], 1.0);
            *v = fmod(a[1], 1.0);
        } else {
            *u = bu;
            *v = bv;
        }
        if (*u < 0) *u += 1.0;
        if (*v < 0) *v += 1.0;
        return 0;
    }
    case PLANE_UV_MAP: { /* pattern.c:442-457 */
        double uu = fmod(pt[0], 1.0), vv = fmod(pt[2], 1.0);
        if (uu < 0) uu += 1.0;
        if (vv < 0) vv += 1.0;
        *u = uu;
        *v = vv;
        return 0;
    }
    case SPHERE_UV_MAP: { /* pattern.c:459-475 */
        double theta = atan2(pt[0], pt[2]);
        double radius = sqrt(pt[0] * pt[0] + pt[1] * pt[1] + pt[2] * pt[2]);
        double phi = acos(pt[1] / radius);
        double raw_u = theta / (2 * M_PI);
        *u = 1 - (raw_u + 0.5);
        *v = 1 - phi / M_PI;
        return 0;
    }
    case TOROID_UV_MAP: { /* pattern.c:477-488 */
        *u = (1.0 - (atan2(pt[2], pt[0]) + M_PI) / (2 * M_PI));
        double len = sqrt(pt[0] * pt[0] + pt[2] * pt[2]);
        double x = len - s->fields.toroid.r1;
        *v = (atan2(pt[1], x) + M_PI) / (2 * M_PI);
        return 0;
    }
    default:
        *u = pt[0];
        *v = pt[1];
        return 0;
    }
}

static void
pattern_at(Pattern p, Shape s, const double *pt, double *res)
{
    switch (p->type) {
    case CHECKER_PATTERN: { /* pattern.c:140-153 */
        int t = (int)floor(pt[0]) + (int)floor(pt[1]) + (int)floor(pt[2]);
        memcpy(res, t % 2 == 0 ? p->fields.concrete.a : p->fields.concrete.b, sizeof(Color));
        return;
    }
    case GRADIENT_PATTERN:
        gradient_at(p, pt, res);
        return;
    case RADIAL_GRADIENT_PATTERN:
        radial_at(p, pt, res);
        return;
    case RING_PATTERN: {
        int t = (int)floor(sqrt(pt[0] * pt[0] + pt[2] * pt[2]));
        memcpy(res, t % 2 == 0 ? p->fields.concrete.a : p->fields.concrete.b, sizeof(Color));
        return;
    }
    case STRIPE_PATTERN: {
        int t = (int)floor(pt[0]);
        memcpy(res, t % 2 == 0 ? p->fields.concrete.a : p->fields.concrete.b, sizeof(Color));
        return;
    }
    case TEXTURE_MAP_PATTERN: { /* pattern.c:198-217 */
        double u, v, q[4];
        int face = uv_map(s, p->fields.uv_map.type, pt, &u, &v);
        Pattern f = p->fields.uv_map.uv_faces + face;
        if (f->transform_identity) memcpy(q, pt, sizeof(q));
        else mat_apply4(f->transform_inverse, pt, q);
        (void)uv_map(s, p->fields.uv_map.type, q, &u, &v);
        uv_pattern_at(f, u, v, res);
        return;
    }
    default: /* base_pattern_at: the reference prints and returns the point */
        memcpy(res, pt, sizeof(Color));
        return;
    }
}

static double
noise3(int x, int y, int z, int octave, int seed)
{
    /* perlin.c:9-24 with two's-complement wrap-around */
    unsigned int n = (unsigned int)x * 1919u + (unsigned int)y * 31337u + (unsigned int)z * 7669u +
                     (unsigned int)octave * 3463u + (unsigned int)seed * 13397u;
    n = (n << 13) ^ n;
    unsigned int m = (n * (n * n * 15731u + 789221u) + 1376312589u) & 0x7fffffffu;
    return 1.0 - (double)(int)m / 1073741824.0;
}

static double
interp(double a, double b, double x)
{
    double f = (1.0 - cos(x * M_PI)) * 0.5;
    return a * (1.0 - f) + b * f;
}

static double
smooth3(double x, double y, double z, int octave, int seed)
{
    int ix = (int)(x < 0 ? -x : x), iy = (int)(y < 0 ? -y : y), iz = (int)(z < 0 ? -z : z);
    double fx = x - ix, fy = y - iy, fz = z - iz;
    double v1 = noise3(ix, iy, iz, octave, seed), v2 = noise3(ix + 1, iy, iz, octave, seed);
    double v3 = noise3(ix, iy + 1, iz, octave, seed), v4 = noise3(ix + 1, iy + 1, iz, octave, seed);
    double v5 = noise3(ix, iy, iz + 1, octave, seed), v6 = noise3(ix + 1, iy, iz + 1, octave, seed);
    double v7 = noise3(ix, iy + 1, iz + 1, octave, seed), v8 = noise3(ix + 1, iy + 1, iz + 1, octave, seed);
    double i1 = interp(v1, v2, fx), i2 = interp(v3, v4, fx), i3 = interp(v5, v6, fx), i4 = interp(v7, v8, fx);
    return interp(interp(i1, i2, fy), interp(i3, i4, fy), fz);
}

static double
pnoise3(double x, double y, double z, double persistence, double frequency, int octaves, int seed)
{
    double total = 0.0, amplitude = 1.0;
    for (int i = 0; i < octaves; ++i) {
        total += smooth3(x * frequency, y * frequency, z * frequency, i, seed) * amplitude;
        frequency /= 2.0;
        amplitude *= persistence;
    }
    return total;
}

static void
pattern_at_shape(Pattern p, Shape s, const double *pt, double *res)
{
    switch (p->type) {
    case BLENDED_PATTERN: { /* pattern.c:30-38 */
        double c1[4], c2[4];
        pattern_at_shape(p->fields.blended.pattern1, s, pt, c1);
        pattern_at_shape(p->fields.blended.pattern2, s, pt, c2);
        for (int k = 0; k < 3; ++k) res[k] = (c1[k] + c2[k]) / 2.0;
        return;
    }
    case NESTED_PATTERN: { /* pattern.c:41-78: substitutes colors into a concrete primary */
        double c1[4], c2[4];
        pattern_at_shape(p->fields.nested.pattern2, s, pt, c1);
        pattern_at_shape(p->fields.nested.pattern3, s, pt, c2);
        /* the reference writes c1 / c2 into the shared primary pattern and then evaluates it (a data
         * race between its render threads, "TODO not threadsafe"); single-threaded that is the primary
         * evaluated with colors (c1, c2), which a private copy gives without the race */
        struct pattern prim = *p->fields.nested.pattern1;
        if (prim.type <= STRIPE_PATTERN) {
            memcpy(prim.fields.concrete.a, c1, sizeof(Color));
            memcpy(prim.fields.concrete.b, c2, sizeof(Color));
        }
        pattern_at_shape(&prim, s, pt, res);
        return;
    }
    case PERTURBED_PATTERN: { /* pattern.c:80-116 */
        const struct perturbed_pattern_fields *f = &p->fields.perturbed;
        double x = pt[0], y = pt[1], z = pt[2];
        double q[4];
        q[0] = pt[0] + f->scale_factor * pnoise3(x, y, z, f->persistence, f->frequency, (int)f->octaves, f->seed);
        if (z < 0) z -= 1.0;
        else z += 1.0;
        q[1] = pt[1] + f->scale_factor * pnoise3(x, y, z, f->persistence, f->frequency, (int)f->octaves, f->seed);
        if (z < 0) z -= 1.0;
        else z += 1.0;
        q[2] = pt[2] + f->scale_factor * pnoise3(x, y, z, f->persistence, f->frequency, (int)f->octaves, f->seed);
        /* the reference leaves the perturbed point's w uninitialised (pattern.c:110-113); its build reads it
         * as 0.0 (pinned by the patterns_160x80 golden), which drops the translations of the
         * object and pattern transforms applied to it */
        q[3] = 0.0;
        pattern_at_shape(f->pattern1, s, q, res);
        return;
    }
    default: { /* base_pattern_at_shape (pattern.c:10-28) */
        double op[4], pp[4];
        world_to_object(s, pt, op);
        if (p->transform_identity) memcpy(pp, op, sizeof(pp));
        else mat_apply4(p->transform_inverse, op, pp);
        double c[4] = {0, 0, 0, 0};
        pattern_at(p, s, pp, c);
        memcpy(res, c, 3 * sizeof(double));
        res[3] = 0.0;
        return;
    }
    }
}

/* ---------------- shading (renderer.c) ---------------- */

typedef struct comps {
    double t, n1, n2, over_d, over_Ns;
    bool inside;
    Shape obj;
    double p[4], over_point[4], under_point[4], eyev[4], normalv[4], reflectv[4];
    double over_Ka[4], over_Kd[4], over_Ks[4], over_refl[4];
} comps;

static void
prepare_computations(octx *cx, long hi, const oray *r, comps *c)
{
    /* renderer.c:369-495 */
    const hitlist *xs = &cx->xs;
    const ohit *h = &xs->v[hi];
    c->t = h->t;
    c->obj = h->obj;
    for (int k = 0; k < 3; ++k) c->p[k] = r->o[k] + r->d[k] * h->t;
    c->p[3] = r->o[3];
    normal_at(c->obj, c->p, h, c->normalv);
    for (int k = 0; k < 3; ++k) c->eyev[k] = r->d[k] * -1.0;
    c->eyev[3] = r->d[3];
    c->inside = false;
    if (dot3(c->normalv, c->eyev) < 0) {
        c->inside = true;
        for (int k = 0; k < 3; ++k) c->normalv[k] *= -1;
    }
    {
        double dd = 2 * dot3(r->d, c->normalv);
        for (int k = 0; k < 3; ++k) c->reflectv[k] = r->d[k] - c->normalv[k] * dd;
        c->reflectv[3] = 0.0;
    }
    for (int k = 0; k < 3; ++k) {
        c->over_point[k] = c->p[k] + c->normalv[k] * EPSILON;
        c->under_point[k] = c->p[k] - c->normalv[k] * EPSILON;
    }
    c->over_point[3] = c->under_point[3] = 1.0;

    c->n1 = 1.0;
    c->n2 = 1.0;
    if (cx->container_cap < xs->n + 1) {
        cx->container_cap = 2 * (xs->n + 1);
        cx->container = (Shape *)realloc(cx->container, cx->container_cap * sizeof(Shape));
    }
    size_t len = 0;
    for (size_t j = 0; j < xs->n; ++j) {
        const ohit *x = &xs->v[j];
        if ((long)j == hi && len > 0) c->n1 = cx->container[len - 1]->material->Ni;
        size_t k = 0;
        while (k < len && cx->container[k] != x->obj) k++;
        if (k < len) {
            --len;
            for (; k < len; ++k) cx->container[k] = cx->container[k + 1];
        } else {
            cx->container[len++] = x->obj;
        }
        if ((long)j == hi) {
            if (len > 0) c->n2 = cx->container[len - 1]->material->Ni;
            break;
        }
    }

    Material m = c->obj->material;
    if (m->map_Ka) pattern_at_shape(m->map_Ka, c->obj, c->over_point, c->over_Ka);
    else memcpy(c->over_Ka, m->Ka, sizeof(Color));
    if (m->map_Kd) pattern_at_shape(m->map_Kd, c->obj, c->over_point, c->over_Kd);
    else memcpy(c->over_Kd, m->Kd, sizeof(Color));
    if (m->map_Ks) pattern_at_shape(m->map_Ks, c->obj, c->over_point, c->over_Ks);
    else memcpy(c->over_Ks, m->Ks, sizeof(Color));
    if (m->map_refl) pattern_at_shape(m->map_refl, c->obj, c->over_point, c->over_refl);
    else memcpy(c->over_refl, m->refl, sizeof(Color));
    if (m->map_Ns) {
        double tmp[4];
        pattern_at_shape(m->map_Ns, c->obj, c->over_point, tmp);
        c->over_Ns = tmp[0];
    } else {
        c->over_Ns = m->Ns;
    }
    if (m->map_d) {
        double tmp[4];
        pattern_at_shape(m->map_d, c->obj, c->over_point, tmp);
        c->over_d = tmp[0];
    } else {
        c->over_d = 1.0 - m->Tr;
    }
}

static const Points
light_row(const struct light *l)
{
    /* area_light_surface_points (light.c:193-198): rand() % cache_len */
    if (l->type == AREA_LIGHT || l->type == CIRCLE_LIGHT) {
        int choice = rand() % (int)l->surface_points_cache_len;
        return l->surface_points_cache + choice;
    }
    return l->surface_points_cache;
}

static double
intensity_at(octx *cx, const struct light *l, const double *p)
{
    if (l->type == AREA_LIGHT || l->type == CIRCLE_LIGHT) { /* light.c:229-242 */
        Points pts = light_row(l);
        double total = 0.0;
        for (size_t i = 0; i < pts->points_num; ++i) {
            if (!is_shadowed(cx, pts->points[i], p)) total += 1.0;
        }
        return total / (double)l->num_samples;
    }
    return is_shadowed(cx, frt_light_position(l), p) ? 0.0 : 1.0; /* light.c:245-251 */
}

static void
lighting_microfacet(octx *cx, const comps *c, const struct light *l, double intensity, double *res)
{
    /* renderer.c:895-979 */
    double amb[4];
    for (int k = 0; k < 3; ++k) amb[k] = c->over_Ka[k] * l->intensity[k];
    if (equal(intensity, 0.0)) {
        if (cx->include_ambient) for (int k = 0; k < 3; ++k) res[k] += amb[k];
        return;
    }
    if (cx->include_diffuse || cx->include_spec_highlight) {
        Points pts = light_row(l);
        double ned = 0.0;
        if (cx->include_spec_highlight) ned = dot3(c->normalv, c->eyev);
        double dacc[3] = {0, 0, 0}, sacc[3] = {0, 0, 0};
        for (size_t i = 0; i < pts->points_num; ++i) {
            double diff[4], lv[4];
            diff[0] = pts->points[i][0] - c->over_point[0];
            diff[1] = pts->points[i][1] - c->over_point[1];
            diff[2] = pts->points[i][2] - c->over_point[2];
            diff[3] = 0.0;
            normalize3(diff, lv);
            double ldn = dot3(lv, c->normalv);
            if (cx->include_diffuse && ldn >= 0.0) {
                for (int k = 0; k < 3; ++k) {
                    double cc = c->over_Kd[k] * l->intensity[k];
                    cc *= ldn;
                    dacc[k] += cc;
                }
            }
            if (cx->include_spec_highlight && ldn >= 0.0) {
                double ndl = dot3(c->normalv, lv);
                double tmp[4] = {lv[0] + c->eyev[0], lv[1] + c->eyev[1], lv[2] + c->eyev[2], 0.0}, hv[4];
                normalize3(tmp, hv);
                double ndh = fmax(0.0, dot3(c->normalv, hv));
                double edh_inv = 1.0 / fmax(0.0, dot3(c->eyev, hv));
                double ldh = dot3(lv, hv);
                double dist_term = (c->over_Ns + 2) * pow(ndh, c->over_Ns) * 0.5 * M_1_PI;
                double gc = 2.0 * ndh * edh_inv;
                double geo = fmin(1.0, fmin(gc * ned, gc * ndl));
                double factor = pow(1.0 - ldh, 5.0);
                double brdf = dist_term * geo / (4.0 * ndl * ned);
                for (int k = 0; k < 3; ++k) {
                    double f = c->over_Ks[k] + (1.0 - c->over_Ks[k]) * factor;
                    sacc[k] += f * l->intensity[k] * brdf;
                }
            }
        }
        double scaling = intensity / (double)l->num_samples;
        for (int k = 0; k < 3; ++k) {
            res[4 + k] += dacc[k];
            res[8 + k] += sacc[k];
            res[4 + k] *= scaling;
            res[8 + k] *= scaling;
        }
    }
    if (cx->include_ambient) for (int k = 0; k < 3; ++k) res[k] += amb[k];
}

static void color_at(octx *cx, const oray *r, size_t remaining, double *res);

static double
schlick(const comps *c)
{
    /* renderer.c:607-624 */
    double co = dot3(c->eyev, c->normalv);
    if (c->n1 > c->n2) {
        double n = c->n1 / c->n2;
        double sin2_t = n * n * (1.0 - co * co);
        if (sin2_t > 1.0) return 1.0;
        co = sqrt(1.0 - sin2_t);
    }
    double r0 = (c->n1 - c->n2) / (c->n1 + c->n2);
    r0 = r0 * r0;
    return r0 + (1.0 - r0) * (1.0 - co) * (1.0 - co) * (1.0 - co) * (1.0 - co) * (1.0 - co);
}

static void
shade_hit(octx *cx, const comps *c, size_t remaining, double *res)
{
    /* renderer.c:690-827 (global-illumination block not restated: refused upstream) */
    double surface[12] = {0};
    if (cx->include_direct) {
        for (size_t i = 0; i < cx->w->lights_num; ++i) {
            const struct light *l = cx->w->lights + i;
            double lc[12] = {0};
            double inten = intensity_at(cx, l, c->over_point);
            lighting_microfacet(cx, c, l, inten, lc);
            for (int k = 0; k < 12; ++k) surface[k] += lc[k];
        }
    }
    if (cx->include_specular) {
        Material m = c->obj->material;
        double refl[12] = {0}, refr[12] = {0};
        if (!(remaining == 0 || !m->reflective)) { /* reflected_color 498-532 */
            double cc[12] = {0};
            oray rr;
            memcpy(rr.o, c->over_point, sizeof(rr.o));
            memcpy(rr.d, c->reflectv, sizeof(rr.d));
            cx->st.secondary_rays++;
            color_at(cx, &rr, remaining - 1, cc);
            for (int t = 0; t < 12; t += 4)
                for (int k = 0; k < 3; ++k) cc[t + k] *= c->over_refl[k];
            for (int k = 0; k < 12; ++k) refl[k] += cc[k];
        }
        if (!(remaining == 0 || c->over_d <= 0.0)) { /* refracted_color 535-605 */
            double n_ratio = c->n1 / c->n2;
            double cos_i = dot3(c->eyev, c->normalv);
            double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
            if (!(sin2_t > 1.0)) {
                double cos_t = sqrt(1.0 - sin2_t);
                double s1 = n_ratio * cos_i - cos_t;
                oray rr;
                memcpy(rr.o, c->under_point, sizeof(rr.o));
                for (int k = 0; k < 3; ++k) {
                    double t1 = c->normalv[k] * s1;
                    double t2 = c->eyev[k] * n_ratio;
                    rr.d[k] = t1 - t2;
                }
                rr.d[3] = 0.0;
                double cc[12] = {0};
                cx->st.secondary_rays++;
                if (m->Tf[0] * c->over_d == 0.0 && m->Tf[1] * c->over_d == 0.0 && m->Tf[2] * c->over_d == 0.0)
                    cx->st.zero_weight_secondary++;
                color_at(cx, &rr, remaining - 1, cc);
                for (int t = 0; t < 12; t += 4)
                    for (int k = 0; k < 3; ++k) cc[t + k] *= m->Tf[k];
                for (int t = 0; t < 12; t += 4)
                    for (int k = 0; k < 3; ++k) cc[t + k] *= c->over_d;
                for (int k = 0; k < 12; ++k) refr[k] += cc[k];
            }
        }
        if (m->reflective && c->over_d < 1.0) {
            double rf = schlick(c);
            for (int t = 0; t < 12; t += 4)
                for (int k = 0; k < 3; ++k) {
                    refl[t + k] *= rf;
                    refr[t + k] *= 1.0 - rf;
                }
        }
        for (int t = 0; t < 12; t += 4)
            for (int k = 0; k < 3; ++k) surface[t + k] += refl[t + k];
        if (m->Tr > 0.0 && c->over_d > 0.0) {
            for (int t = 0; t < 12; t += 4)
                for (int k = 0; k < 3; ++k) surface[t + k] *= 1.0 - c->over_d;
        }
        for (int t = 0; t < 12; t += 4)
            for (int k = 0; k < 3; ++k) surface[t + k] += refr[t + k];
    }
    memcpy(res, surface, sizeof(surface));
}

static void
color_at(octx *cx, const oray *r, size_t remaining, double *res)
{
    /* renderer.c:347-366 */
    double c[12] = {0};
    intersect_world(cx, r, false);
    long hi = hit_index(&cx->xs, false);
    if (hi >= 0) {
        comps cp;
        prepare_computations(cx, hi, r, &cp);
        shade_hit(cx, &cp, remaining, c);
    }
    memcpy(res, c, sizeof(c));
}

static void
ray_for_pixel(Camera cam, size_t px, size_t py, const double *jit, oray *res)
{
    /* renderer.c:95-129 */
    double xoff = ((double)px + jit[0]) * cam->pixel_size;
    double yoff = ((double)py + jit[1]) * cam->pixel_size;
    double wx = cam->half_width - xoff, wy = cam->half_height - yoff;
    double p[4] = {wx, wy, -cam->canvas_distance, 1.0}, pixel[4], origin[4];
    mat_apply4(cam->transform_inverse, p, pixel);
    double ap[2] = {0, 0};
    sample_aperture(ap, px, py, &cam->aperture);
    p[0] = ap[0] * cam->aperture.size;
    p[1] = ap[1] * cam->aperture.size;
    p[2] = 0;
    mat_apply4(cam->transform_inverse, p, origin);
    double v[4] = {pixel[0] - origin[0], pixel[1] - origin[1], pixel[2] - origin[2], 0.0};
    memcpy(res->o, origin, sizeof(origin));
    normalize3(v, res->d);
}

struct job {
    Camera cam;
    World w;
    size_t usteps, vsteps, row_begin, row_end, row_stride;
    bool jitter;
    double *out;
    atomic_size_t next_row; /* job index j: row row_begin + j * row_stride */
    pthread_mutex_t stats_lock;
    frt_oracle_stats stats;
};

static void *
worker(void *arg)
{
    struct job *jb = (struct job *)arg;
    octx cx;
    memset(&cx, 0, sizeof(cx));
    cx.w = jb->w;
    const struct illumination_config *ic = &jb->w->global_config->illumination;
    cx.include_direct = ic->include_direct;
    cx.include_ambient = ic->di.include_ambient;
    cx.include_diffuse = ic->di.include_diffuse;
    cx.include_spec_highlight = ic->di.include_specular_highlight;
    cx.include_specular = ic->di.include_specular;
    cx.path_length = ic->di.path_length;
    Camera cam = jb->cam;
    double total = (double)jb->usteps * (double)jb->vsteps;
    for (;;) {
        const size_t j = atomic_fetch_add(&jb->next_row, 1);
        const size_t row = jb->row_begin + j * jb->row_stride;
        if (row >= jb->row_end) break;
        struct sampler smp; /* one table per row job (renderer.c:211) */
        sampler_2d(jb->jitter, jb->usteps, jb->vsteps, sampler_default_constraint, &smp);
        for (size_t px = 0; px < cam->hsize; ++px) {
            double acc[12] = {0};
            sampler_reset_2d(&smp); /* pixel_multi_sample (renderer.c:145) */
            for (size_t v = 0; v < jb->vsteps; ++v) {
                for (size_t u = 0; u < jb->usteps; ++u) {
                    size_t idx[2] = {u, v};
                    double jit[2];
                    sampler_get_point_2d(&smp, idx, jit);
                    oray r;
                    ray_for_pixel(cam, px, row, jit, &r);
                    double c[12];
                    cx.st.primary_rays++;
                    color_at(&cx, &r, cx.path_length, c);
                    for (int k = 0; k < 12; ++k) acc[k] += c[k];
                }
            }
            for (int k = 0; k < 12; ++k) acc[k] *= 1.0 / total;
            double *o = jb->out + 4 * (j * cam->hsize + px);
            double pix[3];
            for (int k = 0; k < 3; ++k) {
                pix[k] = 0.0 + acc[k];
                pix[k] += acc[4 + k];
                pix[k] += acc[8 + k];
                pix[k] *= 1.0 / 3.0;
            }
            o[0] = pix[0];
            o[1] = pix[1];
            o[2] = pix[2];
            o[3] = 0.0;
        }
        sampler_free(&smp);
    }
    pthread_mutex_lock(&jb->stats_lock);
    jb->stats.primary_rays += cx.st.primary_rays;
    jb->stats.secondary_rays += cx.st.secondary_rays;
    jb->stats.shadow_rays += cx.st.shadow_rays;
    jb->stats.zero_weight_secondary += cx.st.zero_weight_secondary;
    pthread_mutex_unlock(&jb->stats_lock);
    free(cx.xs.v);
    free(cx.container);
    return NULL;
}

static void
warm_bounds(Shape s)
{
    /* compute every lazily cached bound once, before worker threads read them */
    Bounding_box b;
    shape_bounds(s, &b);
    if (s->type == SHAPE_GROUP) {
        for (size_t i = 0; i < s->fields.group.num_children; ++i) warm_bounds(s->fields.group.children + i);
    } else if (s->type == SHAPE_CSG) {
        warm_bounds(s->fields.csg.left);
        warm_bounds(s->fields.csg.right);
    }
}

int
frt_oracle_render_rows_strided(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter,
                               size_t row_begin, size_t row_end, size_t row_stride, int nthreads, double *out,
                               frt_oracle_stats *stats)
{
    if (w->global_config == NULL) return -1;
    if (w->global_config->illumination.include_global || w->global_config->illumination.debug_visualize_photon_map) {
        fprintf(stderr, "frt oracle: global illumination is not restated\n");
        return -2;
    }
    for (size_t i = 0; i < w->shapes_num; ++i) warm_bounds(w->shapes + i);
    struct job jb;
    memset(&jb, 0, sizeof(jb));
    jb.cam = cam;
    jb.w = w;
    jb.usteps = usteps;
    jb.vsteps = vsteps;
    jb.row_begin = row_begin;
    jb.row_end = row_end;
    jb.row_stride = row_stride > 0 ? row_stride : 1;
    jb.jitter = jitter;
    jb.out = out;
    atomic_init(&jb.next_row, 0);
    pthread_mutex_init(&jb.stats_lock, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads == 1) {
        worker(&jb);
    } else {
        pthread_t *th = (pthread_t *)malloc((size_t)nthreads * sizeof(pthread_t));
        for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, worker, &jb);
        for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
        free(th);
    }
    pthread_mutex_destroy(&jb.stats_lock);
    if (stats) *stats = jb.stats;
    return 0;
}

/* rows row_begin, row_begin + 1, ... (out: one row after another) */
int
frt_oracle_render_rows(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter,
                       size_t row_begin, size_t row_end, int nthreads, double *out, frt_oracle_stats *stats)
{
    return frt_oracle_render_rows_strided(cam, w, usteps, vsteps, jitter, row_begin, row_end, 1, nthreads, out,
                                          stats);
}
