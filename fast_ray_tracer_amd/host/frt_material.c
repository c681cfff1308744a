/*
 * frt-mi355x host: materials and pattern constructors.
 *
 * Material defaults restate reference src/material/material.c:7-31 (white
 * Ka/Kd/Ks, black Tf/Ke/refl, Ns 200, Ni 1, casts shadows). Patterns are plain
 * data here (type + colors + transform + child links); the evaluation
 * functions live on the device (csrc/frt_shade.hpp) and in the CPU oracle.
 * Reference-count semantics (pattern.c:633-700, material.c:102-125) are kept
 * so that generated main() code frees exactly what the reference frees.
 */
#include <stdlib.h>
#include <string.h>

#include "src/material/material.h"
#include "src/pattern/pattern.h"
#include "src/libs/linalg/linalg.h"

void
material(Material m)
{
    memset(m, 0, sizeof(*m));
    color_copy(m->Ka, WHITE);
    color_copy(m->Kd, WHITE);
    color_copy(m->Ks, WHITE);
    color_copy(m->Tf, BLACK);
    color_copy(m->Ke, BLACK);
    color_copy(m->refl, BLACK);
    m->Ns = 200.0;
    m->Ni = 1.0;
    m->Tr = 0.0;
    m->reflective = false;
    m->illum = 0;
    m->casts_shadow = true;
}

Material
material_alloc(void)
{
    Material m = (Material)malloc(sizeof(struct material));
    material(m);
    m->ref_count = 1;
    return m;
}

Material
array_of_materials(size_t num)
{
    return (Material)malloc(num * sizeof(struct material));
}

void
material_free(Material m)
{
    /*
     * Reference counts are kept (material.c:102-125) but storage is never
     * released: materials are shared by deep-copied shapes and live for the
     * whole process, and a miscounted free would turn into a use-after-free
     * during flattening.
     */
    if (m != NULL && m->ref_count > 0) {
        m->ref_count--;
    }
}

/* ---------------- patterns ---------------- */

int
frt_uv_map_face_count(enum uv_map_type type)
{
    switch (type) {
    case CUBE_UV_MAP:
        return 6;
    case CYLINDER_UV_MAP:
        return 3;
    case PLANE_UV_MAP:
    case SPHERE_UV_MAP:
    case TOROID_UV_MAP:
    case TRIANGLE_UV_MAP:
        return 1;
    default:
        return 0;
    }
}

void
pattern_set_transform(Pattern p, const Matrix m)
{
    if (p) {
        matrix_copy(m, p->transform);
        matrix_inverse(m, p->transform_inverse);
        p->transform_identity = frt_matrix_is_identity(m);
    }
}

static void
pattern_base(Pattern p, enum pattern_type type)
{
    memset(&p->fields, 0, sizeof(p->fields));
    p->ref_count = 0;
    p->type = type;
    pattern_set_transform(p, MATRIX_IDENTITY);
}

static void
two_color(Pattern p, enum pattern_type type, Color a, Color b)
{
    pattern_base(p, type);
    color_copy(p->fields.concrete.a, a);
    color_copy(p->fields.concrete.b, b);
}

void checker_pattern(Color a, Color b, Pattern res) { two_color(res, CHECKER_PATTERN, a, b); }
void gradient_pattern(Color a, Color b, Pattern res) { two_color(res, GRADIENT_PATTERN, a, b); }
void radial_gradient_pattern(Color a, Color b, Pattern res) { two_color(res, RADIAL_GRADIENT_PATTERN, a, b); }
void ring_pattern(Color a, Color b, Pattern res) { two_color(res, RING_PATTERN, a, b); }
void stripe_pattern(Color a, Color b, Pattern res) { two_color(res, STRIPE_PATTERN, a, b); }
void uv_gradient_pattern(Color a, Color b, Pattern res) { two_color(res, UV_GRADIENT_PATTERN, a, b); }
void uv_radial_gradient_pattern(Color a, Color b, Pattern res) { two_color(res, UV_RADIAL_GRADIENT_PATTERN, a, b); }

void
uv_align_check_pattern(Color main, Color ul, Color ur, Color bl, Color br, Pattern res)
{
    pattern_base(res, UV_ALIGN_CHECKER_PATTERN);
    color_copy(res->fields.uv_align_check.main, main);
    color_copy(res->fields.uv_align_check.ul, ul);
    color_copy(res->fields.uv_align_check.ur, ur);
    color_copy(res->fields.uv_align_check.bl, bl);
    color_copy(res->fields.uv_align_check.br, br);
}

void
uv_check_pattern(Color a, Color b, size_t width, size_t height, Pattern res)
{
    pattern_base(res, UV_CHECKER_PATTERN);
    color_copy(res->fields.uv_check.a, a);
    color_copy(res->fields.uv_check.b, b);
    res->fields.uv_check.width = width;
    res->fields.uv_check.height = height;
}

void
uv_texture_pattern(Canvas canvas, Pattern res)
{
    pattern_base(res, UV_TEXTURE_PATTERN);
    res->fields.uv_texture.canvas = canvas;
}

void
blended_pattern(Pattern p1, Pattern p2, Pattern res)
{
    pattern_base(res, BLENDED_PATTERN);
    res->fields.blended.pattern1 = p1;
    res->fields.blended.pattern2 = p2;
}

void
nested_pattern(Pattern p1, Pattern p2, Pattern p3, Pattern res)
{
    pattern_base(res, NESTED_PATTERN);
    res->fields.nested.pattern1 = p1;
    res->fields.nested.pattern2 = p2;
    res->fields.nested.pattern3 = p3;
}

void
perturbed_pattern(Pattern p1, double frequency, double scale_factor, double persistence, size_t octaves, int seed, Pattern res)
{
    pattern_base(res, PERTURBED_PATTERN);
    res->fields.perturbed.pattern1 = p1;
    res->fields.perturbed.frequency = frequency;
    res->fields.perturbed.scale_factor = scale_factor;
    res->fields.perturbed.persistence = persistence;
    res->fields.perturbed.octaves = octaves;
    res->fields.perturbed.seed = seed;
}

void
texture_map_pattern(Pattern faces, enum uv_map_type type, Pattern res)
{
    pattern_base(res, TEXTURE_MAP_PATTERN);
    res->fields.uv_map.type = type;
    res->fields.uv_map.uv_faces = faces;
    int n = frt_uv_map_face_count(type);
    for (int k = 0; k < n; ++k) {
        faces[k].ref_count += 1;
    }
}

Pattern
array_of_patterns(size_t num)
{
    return (Pattern)malloc(num * sizeof(struct pattern));
}

#define FRT_ALLOC2(name)                                 \
    Pattern name##_alloc(Color a, Color b)               \
    {                                                    \
        Pattern p = (Pattern)malloc(sizeof(struct pattern)); \
        name(a, b, p);                                   \
        return p;                                        \
    }
FRT_ALLOC2(checker_pattern)
FRT_ALLOC2(gradient_pattern)
FRT_ALLOC2(radial_gradient_pattern)
FRT_ALLOC2(ring_pattern)
FRT_ALLOC2(stripe_pattern)
#undef FRT_ALLOC2

Pattern
uv_align_check_pattern_alloc(Color main, Color ul, Color ur, Color bl, Color br)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    uv_align_check_pattern(main, ul, ur, bl, br, p);
    return p;
}

Pattern
uv_check_pattern_alloc(Color a, Color b, size_t width, size_t height)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    uv_check_pattern(a, b, width, height, p);
    return p;
}

Pattern
uv_texture_pattern_alloc(Canvas canvas)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    uv_texture_pattern(canvas, p);
    return p;
}

Pattern
blended_pattern_alloc(Pattern p1, Pattern p2)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    blended_pattern(p1, p2, p);
    return p;
}

Pattern
nested_pattern_alloc(Pattern p1, Pattern p2, Pattern p3)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    nested_pattern(p1, p2, p3, p);
    return p;
}

Pattern
perturbed_pattern_alloc(Pattern p1, double frequency, double scale_factor, double persistence, size_t octaves, int seed)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    perturbed_pattern(p1, frequency, scale_factor, persistence, octaves, seed, p);
    return p;
}

Pattern
texture_map_pattern_alloc(Pattern faces, enum uv_map_type type)
{
    Pattern p = (Pattern)malloc(sizeof(struct pattern));
    texture_map_pattern(faces, type, p);
    return p;
}

void
pattern_free(Pattern p)
{
    /*
     * The reference releases children before its own count
     * (pattern.c:633-700) and frees only heap blocks whose count reaches 0.
     * Generated code places UV faces inside array_of_patterns() blocks, so a
     * face is never free()d individually here; the whole scene is process
     * lifetime data and leaking it is exactly what the reference does.
     */
    if (p == NULL) {
        return;
    }
    if (p->ref_count > 0) {
        p->ref_count--;
    }
}
