/*
 * frt-mi355x host API: procedural and UV-mapped patterns.
 * Types, enums and constructor names follow reference src/pattern/pattern.h:8-181.
 * Patterns are data only on the host; evaluation happens on the GPU
 * (fast_ray_tracer_amd/csrc) and in the CPU oracle (oracle/frt_oracle.c).
 */
#ifndef FRT_PATTERN_H
#define FRT_PATTERN_H

#include <stdbool.h>
#include <stddef.h>

#include "../libs/canvas/canvas.h"
#include "../libs/linalg/linalg.h"
#include "../color/color.h"

enum pattern_type {
    CHECKER_PATTERN,
    GRADIENT_PATTERN,
    RADIAL_GRADIENT_PATTERN,
    RING_PATTERN,
    STRIPE_PATTERN,
    UV_ALIGN_CHECKER_PATTERN,
    UV_CHECKER_PATTERN,
    UV_GRADIENT_PATTERN,
    UV_RADIAL_GRADIENT_PATTERN,
    UV_TEXTURE_PATTERN,
    BLENDED_PATTERN,
    NESTED_PATTERN,
    PERTURBED_PATTERN,
    CUBE_MAP_PATTERN,
    CYLINDER_MAP_PATTERN,
    TEXTURE_MAP_PATTERN
};

enum uv_map_type {
    CUBE_UV_MAP,
    CYLINDER_UV_MAP,
    PLANE_UV_MAP,
    SPHERE_UV_MAP,
    TOROID_UV_MAP,
    TRIANGLE_UV_MAP
};

struct pattern;

struct concrete_pattern_fields { Color a; Color b; };
struct uv_align_check_fields { Color main; Color ul; Color ur; Color bl; Color br; };
struct uv_checker_fields { Color a; Color b; size_t width; size_t height; };
struct uv_texture_fields { Canvas canvas; };
struct blended_pattern_fields { struct pattern *pattern1; struct pattern *pattern2; };
struct nested_pattern_fields { struct pattern *pattern1; struct pattern *pattern2; struct pattern *pattern3; };
struct perturbed_pattern_fields {
    struct pattern *pattern1;
    double frequency;
    double scale_factor;
    double persistence;
    size_t octaves;
    int seed;
};
struct uv_map_pattern_fields { enum uv_map_type type; struct pattern *uv_faces; };

typedef struct pattern {
    Matrix transform;
    Matrix transform_inverse;
    bool transform_identity;
    enum pattern_type type;
    size_t ref_count;
    union {
        struct concrete_pattern_fields concrete;
        struct uv_align_check_fields uv_align_check;
        struct uv_checker_fields uv_check;
        struct uv_texture_fields uv_texture;
        struct blended_pattern_fields blended;
        struct nested_pattern_fields nested;
        struct perturbed_pattern_fields perturbed;
        struct uv_map_pattern_fields uv_map;
    } fields;
} *Pattern;

void checker_pattern(Color a, Color b, Pattern res);
void gradient_pattern(Color a, Color b, Pattern res);
void radial_gradient_pattern(Color a, Color b, Pattern res);
void ring_pattern(Color a, Color b, Pattern res);
void stripe_pattern(Color a, Color b, Pattern res);
void uv_align_check_pattern(Color main, Color ul, Color ur, Color bl, Color br, Pattern res);
void uv_check_pattern(Color a, Color b, size_t width, size_t height, Pattern res);
void uv_gradient_pattern(Color a, Color b, Pattern res);
void uv_radial_gradient_pattern(Color a, Color b, Pattern res);
void uv_texture_pattern(Canvas canvas, Pattern res);
void blended_pattern(Pattern p1, Pattern p2, Pattern res);
void nested_pattern(Pattern p1, Pattern p2, Pattern p3, Pattern res);
void perturbed_pattern(Pattern p1, double frequency, double scale_factor, double persistence, size_t octaves, int seed, Pattern res);
void texture_map_pattern(Pattern faces, enum uv_map_type type, Pattern res);

Pattern array_of_patterns(size_t num);
Pattern checker_pattern_alloc(Color a, Color b);
Pattern gradient_pattern_alloc(Color a, Color b);
Pattern radial_gradient_pattern_alloc(Color a, Color b);
Pattern ring_pattern_alloc(Color a, Color b);
Pattern stripe_pattern_alloc(Color a, Color b);
Pattern uv_align_check_pattern_alloc(Color main, Color ul, Color ur, Color bl, Color br);
Pattern uv_check_pattern_alloc(Color a, Color b, size_t width, size_t height);
Pattern uv_texture_pattern_alloc(Canvas canvas);
Pattern blended_pattern_alloc(Pattern p1, Pattern p2);
Pattern nested_pattern_alloc(Pattern p1, Pattern p2, Pattern p3);
Pattern perturbed_pattern_alloc(Pattern p1, double frequency, double scale_factor, double persistence, size_t octaves, int seed);
Pattern texture_map_pattern_alloc(Pattern faces, enum uv_map_type type);
void pattern_free(Pattern p);
void pattern_set_transform(Pattern pat, const Matrix transform);

/* number of uv faces a texture map of this kind owns (reference pattern.c:706-790) */
int frt_uv_map_face_count(enum uv_map_type type);

#endif
