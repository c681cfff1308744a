/*
 * frt-mi355x host: correlated multi-jitter sample tables.
 *
 * Restates reference src/libs/sampler/sampler.c:401-535. A table holds
 * usteps*vsteps 2-D points; the canonical arrangement is followed by the two
 * correlated row/column shuffles. With jitter off every draw is 0.5, so the
 * table is a fixed function of (usteps, vsteps); with jitter on the draws come
 * from glibc drand48() in the reference's exact order, which keeps host-side
 * light caches identical to a reference run.
 *
 * Index quirk kept from the reference: the canonical pass treats
 * steps[0] as the row count and steps[1] as the column count, the shuffle and
 * the lookup the other way round (they only differ when usteps != vsteps).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "src/libs/sampler/sampler.h"

static double
draw(const struct sampler *s)
{
    return s->jittered ? drand48() : 0.5;
}

static void
swap_d(double *a, double *b)
{
    double t = *a;
    *a = *b;
    *b = t;
}

static void
canonical_2d(Sampler s)
{
    size_t rows = s->steps_by_dimension[0];
    size_t cols = s->steps_by_dimension[1];
    for (size_t j = 0; j < rows; ++j) {
        for (size_t i = 0; i < cols; ++i) {
            double *p = s->arr + 2 * (j * cols + i);
            p[0] = ((double)i + ((double)j + draw(s)) / (double)rows) / (double)cols;
            p[1] = ((double)j + ((double)i + draw(s)) / (double)cols) / (double)rows;
        }
    }
}

static void
shuffle_2d(Sampler s)
{
    size_t m = s->steps_by_dimension[0];
    size_t n = s->steps_by_dimension[1];
    for (size_t j = 0; j < n; ++j) {
        int k = (int)((double)j + draw(s) * (double)(n - j));
        for (size_t i = 0; i < m; ++i) {
            swap_d(s->arr + 2 * (j * m + i), s->arr + 2 * ((size_t)k * m + i));
        }
    }
    for (size_t i = 0; i < m; ++i) {
        int k = (int)((double)i + draw(s) * (double)(m - i));
        for (size_t j = 0; j < n; ++j) {
            swap_d(s->arr + 2 * (j * m + i) + 1, s->arr + 2 * (j * m + (size_t)k) + 1);
        }
    }
}

void
sampler_reset_2d(Sampler s)
{
    canonical_2d(s);
    shuffle_2d(s);
    s->needs_hemi_coords = true;
    memset(s->nt, 0, sizeof(Vector));
    memset(s->nb, 0, sizeof(Vector));
}

void
sampler_2d(const bool jitter, const size_t usteps, const size_t vsteps, bool (*constraint_fn)(const double *), Sampler s)
{
    (void)constraint_fn;
    s->jittered = jitter;
    s->dimensions = 2;
    s->steps_by_dimension = (size_t *)malloc(2 * sizeof(size_t));
    s->steps_by_dimension[0] = usteps;
    s->steps_by_dimension[1] = vsteps;
    size_t len = usteps * vsteps;
    s->arr = len > 0 ? (double *)malloc(2 * len * sizeof(double)) : NULL;
    sampler_reset_2d(s);
}

void
sampler_get_point_2d(Sampler s, const size_t *index, double *result)
{
    const double *p = s->arr + 2 * (index[1] * s->steps_by_dimension[0] + index[0]);
    result[0] = p[0];
    result[1] = p[1];
}

void
sampler_free(Sampler s)
{
    if (s) {
        free(s->steps_by_dimension);
        free(s->arr);
        s->steps_by_dimension = NULL;
        s->arr = NULL;
    }
}

bool
sampler_default_constraint(const double *x)
{
    (void)x;
    return true;
}

/* orthonormal frame around n (reference sampler.c:73-92) */
static void
frame(const Vector n, Vector nt, Vector nb)
{
    Vector tmp;
    nt[3] = nb[3] = 0;
    if (fabs(n[0]) > fabs(n[1])) {
        tmp[0] = n[2];
        tmp[1] = 0;
        tmp[2] = -n[0];
        vector_scale(tmp, sqrt(n[0] * n[0] + n[2] * n[2]));
    } else {
        tmp[0] = 0;
        tmp[1] = -n[2];
        tmp[2] = n[1];
        vector_scale(tmp, sqrt(n[1] * n[1] + n[2] * n[2]));
    }
    tmp[3] = 0;
    vector_normalize(tmp, nt);
    vector_scale(nt, -1.0);
    vector_cross((double *)n, nt, nb);
}

void
sampler_hemisphere(Sampler s, Vector normalv, bool cosine_weighted, size_t *index, double *rands, Vector res)
{
    if (s->needs_hemi_coords) {
        s->needs_hemi_coords = false;
        frame(normalv, s->nt, s->nb);
    }
    sampler_get_point_2d(s, index, rands);
    Vector v, local;
    if (cosine_weighted) {
        double r = sqrt(rands[1]);
        double theta = 2 * M_PI * rands[0];
        v[0] = r * cos(theta);
        v[2] = r * sin(theta);
        v[1] = sqrt(fmax(0.0, 1.0 - rands[1]));
    } else {
        double sin_theta = sqrt(1 - rands[0] * rands[0]);
        double phi = 2 * M_PI * rands[1];
        v[0] = sin_theta * cos(phi);
        v[1] = rands[0];
        v[2] = sin_theta * sin(phi);
    }
    v[3] = 0;
    vector_normalize(v, local);
    Vector w;
    w[0] = local[0] * s->nb[0] + local[1] * normalv[0] + local[2] * s->nt[0];
    w[1] = local[0] * s->nb[1] + local[1] * normalv[1] + local[2] * s->nt[1];
    w[2] = local[0] * s->nb[2] + local[1] * normalv[2] + local[2] * s->nt[2];
    w[3] = 0;
    vector_normalize(w, res);
}

void
sampler_circle(Sampler s, Vector normalv, double radius, size_t *index, double *rands, Point res)
{
    if (s->needs_hemi_coords) {
        s->needs_hemi_coords = false;
        frame(normalv, s->nt, s->nb);
    }
    sampler_get_point_2d(s, index, rands);
    double theta = rands[0] * 2.0 * M_PI;
    double r = sqrt(rands[1]) * radius;
    double x = r * cos(theta), z = r * sin(theta);
    res[0] = x * s->nb[0] + z * s->nt[0];
    res[1] = x * s->nb[1] + z * s->nt[1];
    res[2] = x * s->nb[2] + z * s->nt[2];
    res[3] = 1.0;
}
