/*
 * frt-mi355x host: camera and aperture construction.
 * Restates reference src/renderer/camera.c:84-241 (view transform, half-view
 * geometry, aperture shape parameters). Aperture sampling for the thin-lens
 * shapes draws from drand48 like the reference (camera.c:11-82); the point
 * aperture (the one every benchmark scene uses) is deterministic.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "src/renderer/camera.h"

static bool
aperture_accept(const struct aperture *ap, double x, double y)
{
    double u = 2 * x - 1, v = 2 * y - 1;
    switch (ap->type) {
    case CIRCULAR_APERTURE:
        return !(u * u + v * v > ap->u.circle.r1);
    case CROSS_APERTURE:
        return (u > ap->u.cross.x1 && u <= ap->u.cross.x2) || (v > ap->u.cross.y1 && v <= ap->u.cross.y2);
    case DIAMOND_APERTURE:
        if (u <= 0) {
            return (-u + ap->u.diamond.b1 <= v) && (v < u + ap->u.diamond.b2);
        }
        return (0 <= x) ? ((u + ap->u.diamond.b3 <= v) && (v < -u + ap->u.diamond.b4)) : false;
    case DOUGHNUT_APERTURE: {
        double mag = u * u + v * v;
        return !(mag > ap->u.doughnut.r1 || mag < ap->u.doughnut.r2);
    }
    default:
        return true;
    }
}

void
sample_aperture(double xy[2], size_t u, size_t v, const Aperture ap)
{
    (void)u;
    (void)v;
    double x, y;
    switch (ap->type) {
    case CIRCULAR_APERTURE:
    case CROSS_APERTURE:
    case DIAMOND_APERTURE:
    case DOUGHNUT_APERTURE:
        do {
            x = drand48();
            y = drand48();
        } while (!aperture_accept(ap, x, y));
        break;
    case SQUARE_APERTURE:
        x = drand48();
        y = drand48();
        break;
    default:
        x = 0.5;
        y = 0.5;
        break;
    }
    xy[0] = x - 0.5;
    xy[1] = y - 0.5;
}

void
camera_set_transform(Camera c, Matrix m)
{
    if (c) {
        matrix_copy(m, c->transform);
        matrix_inverse(m, c->transform_inverse);
    }
}

Camera
camera(size_t hsize, size_t vsize, double field_of_view, double canvas_distance, size_t usteps, size_t vsteps,
       Aperture ap, Matrix transform)
{
    Camera c = (Camera)malloc(sizeof(struct camera));
    c->hsize = hsize;
    c->vsize = vsize;
    c->field_of_view = field_of_view;
    c->canvas_distance = canvas_distance;
    c->aperture = *ap;
    c->usteps = usteps;
    c->vsteps = vsteps;
    camera_set_transform(c, transform);

    double half_view = canvas_distance * tan(field_of_view * 0.5);
    double aspect = (double)hsize / (double)vsize;
    if (aspect >= 1.0) {
        c->half_width = half_view;
        c->half_height = half_view / aspect;
    } else {
        c->half_width = half_view * aspect;
        c->half_height = half_view;
    }
    c->pixel_size = c->half_width * 2.0 / (double)hsize;
    return c;
}

void
view_transform(Point fr, Point to, Vector up, Matrix res)
{
    Vector v, forward, upn, left, true_up;
    Matrix orientation, m;
    vector_from_points(to, fr, v);
    vector_normalize(v, forward);
    vector_normalize(up, upn);
    vector_cross(forward, upn, left);
    vector_cross(left, forward, true_up);
    matrix(left[0], left[1], left[2], 0,
           true_up[0], true_up[1], true_up[2], 0,
           -forward[0], -forward[1], -forward[2], 0,
           0, 0, 0, 1,
           orientation);
    matrix_translate(-fr[0], -fr[1], -fr[2], m);
    matrix_multiply(orientation, m, res);
}

void
aperture(enum aperture_type type, double size, size_t usteps, size_t vsteps, bool jitter, Aperture res)
{
    res->type = type;
    res->size = size;
    res->jitter = jitter;
    /* the reference builds (and draws for) a per-aperture CMJ table here (camera.c:175) */
    sampler_2d(jitter, usteps, vsteps, sampler_default_constraint, &res->sampler);
    switch (type) {
    case CIRCULAR_APERTURE:
    case CROSS_APERTURE:
    case DIAMOND_APERTURE:
    case DOUGHNUT_APERTURE:
    case SQUARE_APERTURE:
        break;
    default:
        /* hexagonal / pentagonal / octagonal are unimplemented in the reference and fall back to a point */
        res->type = type == POINT_APERTURE ? POINT_APERTURE : type;
        break;
    }
}

void
circle_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct circle_aperture_args *args, Aperture res)
{
    aperture(CIRCULAR_APERTURE, size, usteps, vsteps, jitter, res);
    res->u.circle = *args;
}

void
cross_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct cross_aperture_args *args, Aperture res)
{
    aperture(CROSS_APERTURE, size, usteps, vsteps, jitter, res);
    res->u.cross = *args;
}

void
diamond_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct diamond_aperture_args *args, Aperture res)
{
    aperture(DIAMOND_APERTURE, size, usteps, vsteps, jitter, res);
    res->u.diamond = *args;
}

void
doughnut_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct doughnut_aperture_args *args, Aperture res)
{
    aperture(DOUGHNUT_APERTURE, size, usteps, vsteps, jitter, res);
    res->u.doughnut = *args;
}

void
square_aperture(double size, size_t usteps, size_t vsteps, bool jitter, Aperture res)
{
    aperture(SQUARE_APERTURE, size, usteps, vsteps, jitter, res);
}

void
point_aperture(Aperture res)
{
    aperture(POINT_APERTURE, 0, 1, 1, false, res);
}
