/*
 * frt-mi355x host: vector / matrix / ray / AABB arithmetic.
 *
 * Every routine keeps the reference's operation order (reference
 * src/libs/linalg/linalg.c, src/renderer/ray.c, src/shapes/bounding_box.c)
 * so host-side transforms, inverses and BVH bounds are bit-identical to the
 * reference build. Compiled with -ffp-contract=off.
 */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "src/libs/linalg/linalg.h"
#include "src/renderer/ray.h"
#include "src/shapes/bounding_box.h"

int
frt_matrix_is_identity(const Matrix m)
{
    /* reference: matrix_equal(m, MATRIX_IDENTITY), linalg.h:14-30 (|a-b| < EPSILON per entry) */
    for (int k = 0; k < 16; ++k) {
        if (!equal(m[k], MATRIX_IDENTITY[k])) {
            return 0;
        }
    }
    return 1;
}

static void
print4(const char *name, const double *a)
{
    printf("%s: [%f %f %f %f]\n", name, a[0], a[1], a[2], a[3]);
}

void point_print(Point p) { print4("Point", p); }
void vector_print(Vector v) { print4("Vector", v); }

void
matrix_print(Matrix m)
{
    for (int r = 0; r < 4; ++r) {
        print4("row", m + 4 * r);
    }
}

void point_copy(Point to, Point from) { memcpy(to, from, sizeof(Point)); }
void vector_copy(Vector to, Vector from) { memcpy(to, from, sizeof(Vector)); }
void matrix_copy(const Matrix m, Matrix res) { memcpy(res, m, sizeof(Matrix)); }

void
matrix(double aa, double ab, double ac, double ad,
       double ba, double bb, double bc, double bd,
       double ca, double cb, double cc, double cd,
       double da, double db, double dc, double dd,
       Matrix res)
{
    const double v[16] = {aa, ab, ac, ad, ba, bb, bc, bd, ca, cb, cc, cd, da, db, dc, dd};
    memcpy(res, v, sizeof(v));
}

void
vector_from_points(Point pt1, Point pt2, Vector res)
{
    res[0] = pt1[0] - pt2[0];
    res[1] = pt1[1] - pt2[1];
    res[2] = pt1[2] - pt2[2];
    res[3] = 0.0;
}

double
vector_dot(Vector a, Vector b)
{
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

double
vector_magnitude(Vector v)
{
    return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
}

void
vector_scale(Vector input, double scalar)
{
    input[0] *= scalar;
    input[1] *= scalar;
    input[2] *= scalar;
}

void
vector_normalize(Vector v, Vector res)
{
    /* reference linalg.c:141-148: multiply by the reciprocal, w forced to 0 */
    double inv = 1.0 / vector_magnitude(v);
    double x = v[0], y = v[1], z = v[2];
    res[0] = x * inv;
    res[1] = y * inv;
    res[2] = z * inv;
    res[3] = 0.0;
}

void
vector_cross(Vector a, Vector b, Vector res)
{
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    res[0] = x;
    res[1] = y;
    res[2] = z;
    res[3] = 0.0;
}

void
vector_reflect(Vector a, Vector n, Vector res)
{
    double k = 2 * vector_dot(a, n);
    double x = a[0] - n[0] * k, y = a[1] - n[1] * k, z = a[2] - n[2] * k;
    res[0] = x;
    res[1] = y;
    res[2] = z;
    res[3] = 0.0;
}

void
matrix_translate(double x, double y, double z, Matrix res)
{
    matrix_identity(res);
    res[3] = x;
    res[7] = y;
    res[11] = z;
}

void
matrix_scale(double x, double y, double z, Matrix res)
{
    matrix_identity(res);
    res[0] = x;
    res[5] = y;
    res[10] = z;
}

void
matrix_rotate_x(double rad, Matrix res)
{
    matrix_identity(res);
    res[5] = res[10] = cos(rad);
    res[6] = -sin(rad);
    res[9] = sin(rad);
}

void
matrix_rotate_y(double rad, Matrix res)
{
    matrix_identity(res);
    res[0] = res[10] = cos(rad);
    res[8] = -sin(rad);
    res[2] = sin(rad);
}

void
matrix_rotate_z(double rad, Matrix res)
{
    matrix_identity(res);
    res[0] = res[5] = cos(rad);
    res[1] = -sin(rad);
    res[4] = sin(rad);
}

void
matrix_shear(double xy, double xz, double yx, double yz, double zx, double zy, Matrix res)
{
    matrix_identity(res);
    res[1] = xy;
    res[2] = xz;
    res[4] = yx;
    res[6] = yz;
    res[8] = zx;
    res[9] = zy;
}

void
matrix_multiply(const Matrix a, const Matrix b, Matrix res)
{
    Matrix out;
    for (int r = 0; r < 4; ++r) {
        for (int c = 0; c < 4; ++c) {
            out[4 * r + c] = a[4 * r + 0] * b[c] + a[4 * r + 1] * b[4 + c] +
                             a[4 * r + 2] * b[8 + c] + a[4 * r + 3] * b[12 + c];
        }
    }
    memcpy(res, out, sizeof(Matrix));
}

void
transform_chain(const Matrix a, Matrix b)
{
    /* b <- a * b (reference linalg.c:252-258) */
    matrix_multiply(a, b, b);
}

void
matrix_array_multiply(const Matrix a, const double b[4], double res[4])
{
    double out[4];
    for (int r = 0; r < 4; ++r) {
        out[r] = a[4 * r + 0] * b[0] + a[4 * r + 1] * b[1] + a[4 * r + 2] * b[2] + a[4 * r + 3] * b[3];
    }
    memcpy(res, out, sizeof(out));
}

void matrix_point_multiply(const Matrix a, const Point b, Point res) { matrix_array_multiply(a, b, res); }
void matrix_vector_multiply(const Matrix a, const Vector b, Vector res) { matrix_array_multiply(a, b, res); }

void
matrix_transpose(const Matrix m, Matrix res)
{
    Matrix t;
    for (int r = 0; r < 4; ++r) {
        for (int c = 0; c < 4; ++c) {
            t[4 * c + r] = m[4 * r + c];
        }
    }
    memcpy(res, t, sizeof(Matrix));
}

void
matrix_inverse(const Matrix m, Matrix res)
{
    /*
     * Cofactor expansion along the first row with 2x2 sub-determinants, the
     * same grouping as reference linalg.c:306-392, so inverses agree bit for
     * bit. Cof[r][c] below are the signed-off minors M(r,c).
     */
    const double s05 = m[10] * m[15] - m[11] * m[14];
    const double s06 = m[9] * m[15] - m[11] * m[13];
    const double s07 = m[9] * m[14] - m[10] * m[13];
    const double s16 = m[8] * m[15] - m[11] * m[12];
    const double s17 = m[8] * m[14] - m[10] * m[12];
    const double s27 = m[8] * m[13] - m[9] * m[12];

    const double c00 = m[5] * s05 - m[6] * s06 + m[7] * s07;
    const double c01 = m[4] * s05 - m[6] * s16 + m[7] * s17;
    const double c02 = m[4] * s06 - m[5] * s16 + m[7] * s27;
    const double c03 = m[4] * s07 - m[5] * s17 + m[6] * s27;

    const double c10 = m[1] * s05 - m[2] * s06 + m[3] * s07;
    const double c11 = m[0] * s05 - m[2] * s16 + m[3] * s17;
    const double c12 = m[0] * s06 - m[1] * s16 + m[3] * s27;
    const double c13 = m[0] * s07 - m[1] * s17 + m[2] * s27;

    const double t81 = m[6] * m[15] - m[7] * m[14];
    const double t82 = m[5] * m[15] - m[7] * m[13];
    const double t83 = m[5] * m[14] - m[6] * m[13];
    const double t92 = m[4] * m[15] - m[7] * m[12];
    const double t93 = m[4] * m[14] - m[6] * m[12];
    const double tA3 = m[4] * m[13] - m[5] * m[12];

    const double c20 = m[1] * t81 - m[2] * t82 + m[3] * t83;
    const double c21 = m[0] * t81 - m[2] * t92 + m[3] * t93;
    const double c22 = m[0] * t82 - m[1] * t92 + m[3] * tA3;
    const double c23 = m[0] * t83 - m[1] * t93 + m[2] * tA3;

    const double u1 = m[6] * m[11] - m[7] * m[10];
    const double u2 = m[5] * m[11] - m[7] * m[9];
    const double u3 = m[5] * m[10] - m[6] * m[9];
    const double v2 = m[4] * m[11] - m[7] * m[8];
    const double v3 = m[4] * m[10] - m[6] * m[8];
    const double w3 = m[4] * m[9] - m[5] * m[8];

    const double c30 = m[1] * u1 - m[2] * u2 + m[3] * u3;
    const double c31 = m[0] * u1 - m[2] * v2 + m[3] * v3;
    const double c32 = m[0] * u2 - m[1] * v2 + m[3] * w3;
    const double c33 = m[0] * u3 - m[1] * v3 + m[2] * w3;

    const double det = m[0] * c00 - m[1] * c01 + m[2] * c02 - m[3] * c03;
    if (equal(det, 0.0)) {
        printf("determinant is zero\n");
    }

    Matrix out;
    out[0] = c00 / det;   out[4] = -c01 / det;  out[8] = c02 / det;   out[12] = -c03 / det;
    out[1] = -c10 / det;  out[5] = c11 / det;   out[9] = -c12 / det;  out[13] = c13 / det;
    out[2] = c20 / det;   out[6] = -c21 / det;  out[10] = c22 / det;  out[14] = -c23 / det;
    out[3] = -c30 / det;  out[7] = c31 / det;   out[11] = -c32 / det; out[15] = c33 / det;
    memcpy(res, out, sizeof(Matrix));
}

/* ---- rays (reference src/renderer/ray.c) ---- */

void
ray_array(Point origin, Vector direction, Ray ray)
{
    memcpy(ray->origin, origin, sizeof(Point));
    memcpy(ray->direction, direction, sizeof(Vector));
}

void
ray_transform(Ray original, Matrix m, Ray res)
{
    matrix_point_multiply(m, original->origin, res->origin);
    matrix_vector_multiply(m, original->direction, res->direction);
}

void
ray_position(Ray ray, double t, Point position)
{
    position[0] = ray->origin[0] + ray->direction[0] * t;
    position[1] = ray->origin[1] + ray->direction[1] * t;
    position[2] = ray->origin[2] + ray->direction[2] * t;
    position[3] = ray->origin[3];
}

/* ---- axis-aligned boxes (reference src/shapes/bounding_box.c) ---- */

void
bounding_box(Bounding_box *box)
{
    for (int k = 0; k < 3; ++k) {
        box->min[k] = INFINITY;
        box->max[k] = -INFINITY;
    }
    box->min[3] = box->max[3] = 1.0;
}

void
bounding_box_add_array(Bounding_box *box, double p[4])
{
    /* strict comparisons: NaN coordinates never widen a box (bounding_box.c:24-56) */
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = p[k] < box->min[k] ? p[k] : box->min[k];
        hi[k] = p[k] > box->max[k] ? p[k] : box->max[k];
    }
    for (int k = 0; k < 3; ++k) {
        box->min[k] = lo[k];
        box->max[k] = hi[k];
    }
}

void
bounding_box_add_box(Bounding_box *box, Bounding_box *other)
{
    if (box != other) {
        bounding_box_add_array(box, other->min);
        bounding_box_add_array(box, other->max);
    }
}

bool
bounding_box_contains_array(Bounding_box *box, double p[4])
{
    return box->min[0] <= p[0] && p[0] <= box->max[0] &&
           box->min[1] <= p[1] && p[1] <= box->max[1] &&
           box->min[2] <= p[2] && p[2] <= box->max[2];
}

bool
bounding_box_contains_box(Bounding_box *box, Bounding_box *other)
{
    return box == other ||
           (bounding_box_contains_array(box, other->min) && bounding_box_contains_array(box, other->max));
}

void
bounding_box_transform(Bounding_box *box, const Matrix m, Bounding_box *res)
{
    /* corner order x-major, then y, then z (bounding_box.c:97-108) */
    Bounding_box in = *box;
    bounding_box(res);
    for (int k = 0; k < 8; ++k) {
        double corner[4] = {(k & 4) ? in.max[0] : in.min[0],
                            (k & 2) ? in.max[1] : in.min[1],
                            (k & 1) ? in.max[2] : in.min[2], 1.0};
        double out[4];
        matrix_point_multiply(m, corner, out);
        bounding_box_add_array(res, out);
    }
}

static void
slab(double origin, double direction, double lo, double hi, double *tmin, double *tmax)
{
    double num_lo = lo - origin;
    double num_hi = hi - origin;
    double a, b;
    if (fabs(direction) >= EPSILON) {
        a = num_lo / direction;
        b = num_hi / direction;
    } else {
        a = num_lo * INFINITY;
        if (isnan(a)) {
            a = num_lo < 0 ? -INFINITY : INFINITY;
        }
        b = num_hi * INFINITY;
        if (isnan(b)) {
            b = num_hi < 0 ? -INFINITY : INFINITY;
        }
    }
    if (a > b) {
        *tmin = b;
        *tmax = a;
    } else {
        *tmin = a;
        *tmax = b;
    }
}

bool
bounding_box_intersects(Bounding_box *box, struct ray *r)
{
    double x0, x1, y0, y1, z0, z1;
    slab(r->origin[0], r->direction[0], box->min[0], box->max[0], &x0, &x1);
    slab(r->origin[1], r->direction[1], box->min[1], box->max[1], &y0, &y1);
    slab(r->origin[2], r->direction[2], box->min[2], box->max[2], &z0, &z1);
    double tmin = fmax(fmax(x0, y0), z0);
    double tmax = fmin(fmin(x1, y1), z1);
    return tmin <= tmax;
}

void
bounding_box_split_bounds(Bounding_box *box, Bounding_box *left_res, Bounding_box *right_res)
{
    /* split the longest axis at its midpoint (bounding_box.c:177-214) */
    double d[3] = {fabs(box->max[0] - box->min[0]), fabs(box->max[1] - box->min[1]), fabs(box->max[2] - box->min[2])};
    double greatest = fmax(fmax(d[0], d[1]), d[2]);
    int axis = equal(greatest, d[0]) ? 0 : (equal(greatest, d[1]) ? 1 : 2);
    double mid = box->min[axis] + d[axis] / 2.0;

    *left_res = *box;
    *right_res = *box;
    left_res->max[axis] = mid;
    right_res->min[axis] = mid;
}
