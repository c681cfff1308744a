/*
 * frt-mi355x host API: 4-vector / 4x4 matrix helpers.
 *
 * Source-compatible with the names the reference's YAML->C codegen emits
 * (reference: src/libs/linalg/linalg.h:7-33 types and macros,
 * yaml_parser/transform.py:17-30 for the matrix_* calls). All arithmetic is
 * IEEE binary64 with no contraction (-ffp-contract=off), operation order as in
 * the reference so host-built transforms are bit-identical.
 */
#ifndef FRT_LINALG_H
#define FRT_LINALG_H

#include <stdio.h>
#include <stddef.h>
#include <string.h>
#include <math.h>

#define EPSILON 0.00001
#define equal(a, b) (fabs((a) - (b)) < EPSILON)

typedef double Point[4];
typedef double Vector[4];
typedef double Matrix[16];

typedef struct pts {
    Point *points;
    size_t points_num;
} *Points;

static const Point POINT_IDENTITY = {0.0, 0.0, 0.0, 1.0};
static const Vector VECTOR_IDENTITY = {0.0, 0.0, 0.0, 0.0};
static const Matrix MATRIX_IDENTITY = {
    1.0, 0.0, 0.0, 0.0,
    0.0, 1.0, 0.0, 0.0,
    0.0, 0.0, 1.0, 0.0,
    0.0, 0.0, 0.0, 1.0};

#define matrix_identity(m) memcpy((m), MATRIX_IDENTITY, sizeof(Matrix))
#define point_default(p) memcpy((p), POINT_IDENTITY, sizeof(Point))
#define vector_default(v) memcpy((v), VECTOR_IDENTITY, sizeof(Vector))

#define point(x, y, z, _res) (_res)[0] = (x); (_res)[1] = (y); (_res)[2] = (z); (_res)[3] = 1.0
#define vector(x, y, z, _res) (_res)[0] = (x); (_res)[1] = (y); (_res)[2] = (z); (_res)[3] = 0.0
#define vector_init(x, y, z) { (x), (y), (z), 0.0 }

int frt_matrix_is_identity(const Matrix m);

void point_print(Point p);
void vector_print(Vector v);
void matrix_print(Matrix m);

void point_copy(Point to, Point from);
void vector_copy(Vector to, Vector from);
void matrix(double aa, double ab, double ac, double ad,
            double ba, double bb, double bc, double bd,
            double ca, double cb, double cc, double cd,
            double da, double db, double dc, double dd,
            Matrix res);
void matrix_copy(const Matrix m, Matrix res);

void vector_from_points(Point pt1, Point pt2, Vector res);
void vector_cross(Vector a, Vector b, Vector res);
double vector_magnitude(Vector v);
void vector_normalize(Vector v, Vector res);
double vector_dot(Vector a, Vector b);
void vector_reflect(Vector a, Vector b, Vector res);
void vector_scale(Vector input, double scalar);

void matrix_translate(double x, double y, double z, Matrix res);
void matrix_scale(double x, double y, double z, Matrix res);
void matrix_rotate_x(double rad, Matrix res);
void matrix_rotate_y(double rad, Matrix res);
void matrix_rotate_z(double rad, Matrix res);
void matrix_shear(double xy, double xz, double yx, double yz, double zx, double zy, Matrix res);

void matrix_multiply(const Matrix a, const Matrix b, Matrix res);
void transform_chain(const Matrix a, Matrix b);
void matrix_array_multiply(const Matrix a, const double b[4], double res[4]);
void matrix_vector_multiply(const Matrix a, const Vector b, Vector res);
void matrix_point_multiply(const Matrix a, const Point b, Point res);
void matrix_transpose(const Matrix m, Matrix res);
void matrix_inverse(const Matrix m, Matrix res);

#endif
