/*
 * frt-mi355x host API: light sources.
 * Field names / constructors follow reference src/light/light.h:17-105.
 * Area and circle lights pre-sample `cache_size` rows of usteps*vsteps points
 * at construction (CMJ, drand48 when jittered) exactly as the reference does
 * (light.c:101-191); the renderer picks a row per shading event.
 */
#ifndef FRT_LIGHT_H
#define FRT_LIGHT_H

#include <stdbool.h>
#include <stdlib.h>

#include "../libs/linalg/linalg.h"
#include "../color/color.h"

enum light_enum {
    AREA_LIGHT,
    CIRCLE_LIGHT,
    HEMISPHERE_LIGHT,
    POINT_LIGHT,
    SPOT_LIGHT
};

struct spot_light_fields { Point position; Vector normal; double outer_angle; double inner_angle; };
struct hemisphere_light_fields { Point position; Vector normal; };
struct point_light_fields { Point position; };
struct circle_light_fields { Point origin; Vector normal; double radius; size_t usteps; size_t vsteps; bool jitter; };
struct area_light_fields { Point corner; Vector uvec; size_t usteps; Vector vvec; size_t vsteps; bool jitter; };

typedef struct light {
    enum light_enum type;
    double intensity[3];
    size_t num_samples;
    size_t num_photons;
    union {
        struct area_light_fields area;
        struct circle_light_fields circle;
        struct hemisphere_light_fields hemi;
        struct point_light_fields point;
        struct spot_light_fields spot;
    } u;
    Points surface_points_cache;
    size_t surface_points_cache_len;
} *Light;

Light array_of_lights(size_t num);
void point_light(Point p, Color intensity, Light l);
void hemisphere_light(Point p, Point to, Color intensity, Light l);
void area_light(Point corner, Vector full_uvec, size_t usteps, Vector full_vvec, size_t vsteps,
                bool jitter, size_t cache_size, Color intensity, Light l);
void circle_light(Point origin, Point to, double radius, size_t usteps, size_t vsteps,
                  bool jitter, size_t cache_size, Color intensity, Light l);

/* the position a point / hemisphere light shades from (union alias as in light.c:202,245) */
const double *frt_light_position(const struct light *l);

#endif
