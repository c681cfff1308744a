/*
 * frt-mi355x host API: 2-D correlated multi-jitter (CMJ) sample tables.
 * Behaviour restated from reference src/libs/sampler/sampler.c:401-535
 * (sampler_2d / reset_canonical_2d / shuffle_2d / get_point_2d). Jittered
 * tables draw from glibc drand48() in the reference's call order.
 */
#ifndef FRT_SAMPLER_H
#define FRT_SAMPLER_H

#include <stdbool.h>
#include <stddef.h>
#include "../linalg/linalg.h"

typedef struct sampler {
    size_t dimensions;
    bool needs_hemi_coords;
    Vector nt, nb;
    size_t *steps_by_dimension;
    double *arr;
    bool jittered;
} *Sampler;

void sampler_2d(const bool jitter, const size_t usteps, const size_t vsteps, bool (*constraint_fn)(const double *), Sampler sampler);
void sampler_reset_2d(Sampler sampler);
void sampler_get_point_2d(Sampler sampler, const size_t *index, double *result);
void sampler_free(Sampler sampler);
bool sampler_default_constraint(const double *);

/* hemisphere / disc helpers (reference sampler.c:8-170) */
void sampler_hemisphere(Sampler sampler, Vector normalv, bool cosine_weighted, size_t *index, double *rands, Vector res);
void sampler_circle(Sampler sampler, Vector normalv, double radius, size_t *index, double *rands, Point res);

#endif
