/*
 * frt-mi355x host: light construction and surface-point caches.
 *
 * Restates reference src/light/light.c:101-411. An area light stores its
 * edge vectors pre-divided by the step counts and pre-samples `cache_size`
 * rows of usteps*vsteps CMJ points (light.c:138-191); a circle light samples
 * a disc around its normal (light.c:101-136). Point and hemisphere lights
 * have a one-point cache. The CMJ tables draw from drand48 when jittered, in
 * the same order as the reference, so a scene built here has the same light
 * caches as the same scene built by the reference.
 */
#include <stdlib.h>
#include <string.h>

#include "src/light/light.h"
#include "src/libs/sampler/sampler.h"

Light
array_of_lights(size_t num)
{
    return (Light)calloc(num ? num : 1, sizeof(struct light));
}

const double *
frt_light_position(const struct light *l)
{
    /* point / hemisphere lights share the position slot at the start of the union */
    return l->type == HEMISPHERE_LIGHT ? l->u.hemi.position : l->u.point.position;
}

static Points
single_point_cache(const double *pos)
{
    Points pts = (Points)malloc(sizeof(struct pts));
    pts->points_num = 1;
    pts->points = (Point *)malloc(sizeof(Point));
    memcpy(pts->points[0], pos, sizeof(Point));
    return pts;
}

void
point_light(Point p, Color intensity, Light l)
{
    l->type = POINT_LIGHT;
    memcpy(l->intensity, intensity, 3 * sizeof(double));
    l->num_samples = 1;
    l->num_photons = 0;
    point_copy(l->u.point.position, p);
    l->surface_points_cache = single_point_cache(l->u.point.position);
    l->surface_points_cache_len = 1;
}

void
hemisphere_light(Point p, Point to, Color intensity, Light l)
{
    l->type = HEMISPHERE_LIGHT;
    memcpy(l->intensity, intensity, 3 * sizeof(double));
    l->num_samples = 1;
    l->num_photons = 0;
    point_copy(l->u.hemi.position, p);
    Vector n;
    vector_from_points(to, p, n);
    vector_normalize(n, l->u.hemi.normal);
    l->surface_points_cache = single_point_cache(l->u.hemi.position);
    l->surface_points_cache_len = 1;
}

void
area_light(Point corner, Vector full_uvec, size_t usteps, Vector full_vvec, size_t vsteps,
           bool jitter, size_t cache_size, Color intensity, Light l)
{
    l->type = AREA_LIGHT;
    point_copy(l->u.area.corner, corner);
    vector_copy(l->u.area.uvec, full_uvec);
    vector_scale(l->u.area.uvec, 1.0 / (double)usteps);
    l->u.area.usteps = usteps;
    vector_copy(l->u.area.vvec, full_vvec);
    vector_scale(l->u.area.vvec, 1.0 / (double)vsteps);
    l->u.area.vsteps = vsteps;
    l->u.area.jitter = jitter;
    memcpy(l->intensity, intensity, 3 * sizeof(double));
    l->num_samples = usteps * vsteps;
    l->num_photons = 0;

    Points rows = (Points)malloc(cache_size * sizeof(struct pts));
    struct sampler smp;
    sampler_2d(jitter, usteps, vsteps, sampler_default_constraint, &smp);
    for (size_t r = 0; r < cache_size; ++r) {
        rows[r].points_num = l->num_samples;
        rows[r].points = (Point *)malloc(l->num_samples * sizeof(Point));
        sampler_reset_2d(&smp);
        for (size_t v = 0; v < vsteps; ++v) {
            for (size_t u = 0; u < usteps; ++u) {
                size_t idx[2] = {u, v};
                double uv[2];
                sampler_get_point_2d(&smp, idx, uv);
                uv[0] *= (double)usteps;
                uv[1] *= (double)vsteps;
                /* corner + uvec*ju + vvec*jv (area_light_point_on_light, light.c:138-152) */
                double *pt = rows[r].points[v * usteps + u];
                double ux = l->u.area.uvec[0] * uv[0], uy = l->u.area.uvec[1] * uv[0], uz = l->u.area.uvec[2] * uv[0];
                double vx = l->u.area.vvec[0] * uv[1], vy = l->u.area.vvec[1] * uv[1], vz = l->u.area.vvec[2] * uv[1];
                pt[0] = corner[0] + ux + vx;
                pt[1] = corner[1] + uy + vy;
                pt[2] = corner[2] + uz + vz;
                pt[3] = 1.0;
            }
        }
    }
    sampler_free(&smp);
    l->surface_points_cache = rows;
    l->surface_points_cache_len = cache_size;
}

void
circle_light(Point origin, Point to, double radius, size_t usteps, size_t vsteps,
             bool jitter, size_t cache_size, Color intensity, Light l)
{
    l->type = CIRCLE_LIGHT;
    point_copy(l->u.circle.origin, origin);
    Vector n;
    vector_from_points(to, origin, n);
    vector_normalize(n, l->u.circle.normal);
    l->u.circle.radius = radius;
    l->u.circle.usteps = usteps;
    l->u.circle.vsteps = vsteps;
    l->u.circle.jitter = jitter;
    memcpy(l->intensity, intensity, 3 * sizeof(double));
    l->num_samples = usteps * vsteps;
    l->num_photons = 0;

    Points rows = (Points)malloc(cache_size * sizeof(struct pts));
    struct sampler smp;
    sampler_2d(jitter, usteps, vsteps, sampler_default_constraint, &smp);
    for (size_t r = 0; r < cache_size; ++r) {
        rows[r].points_num = l->num_samples;
        rows[r].points = (Point *)malloc(l->num_samples * sizeof(Point));
        sampler_reset_2d(&smp);
        for (size_t v = 0; v < vsteps; ++v) {
            for (size_t u = 0; u < usteps; ++u) {
                size_t idx[2] = {u, v};
                double rands[2];
                Point p;
                sampler_circle(&smp, l->u.circle.normal, radius, idx, rands, p);
                double *pt = rows[r].points[v * usteps + u];
                pt[0] = p[0] + origin[0];
                pt[1] = p[1] + origin[1];
                pt[2] = p[2] + origin[2];
                pt[3] = 1.0;
            }
        }
    }
    sampler_free(&smp);
    l->surface_points_cache = rows;
    l->surface_points_cache_len = cache_size;
}
