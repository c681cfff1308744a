/*
 * frt-mi355x host API: the scene graph.
 *
 * A Shape is one node of the reference's object tree (reference
 * src/shapes/shapes.h:16-118): primitives, groups (BVH nodes) and CSG nodes,
 * each with its own transform / inverse and material. The field names the
 * codegen writes directly (fields.cylinder.minimum, fields.toroid.r1, ...) and
 * the ->divide hook that generated main() calls are kept; the per-shape
 * intersection scratch buffers and vtables of the reference are not needed
 * here because intersection runs on the GPU over a flattened copy
 * (fast_ray_tracer_amd/host/frt_flatten.c).
 */
#ifndef FRT_SHAPES_H
#define FRT_SHAPES_H

#include <stdbool.h>
#include <stddef.h>

#include "../libs/linalg/linalg.h"
#include "../libs/canvas/canvas.h"
#include "../renderer/ray.h"
#include "../intersection/intersection.h"
#include "../material/material.h"
#include "bounding_box.h"

enum shape_enum {
    SHAPE_CONE,
    SHAPE_CUBE,
    SHAPE_CYLINDER,
    SHAPE_PLANE,
    SHAPE_SMOOTH_TRIANGLE,
    SHAPE_SPHERE,
    SHAPE_TOROID,
    SHAPE_TRIANGLE,
    SHAPE_CSG,
    SHAPE_GROUP
};

enum csg_ops_enum {
    CSG_UNION,
    CSG_INTERSECT,
    CSG_DIFFERENCE
};

struct csg_fields {
    enum csg_ops_enum op;
    struct shape *left;
    struct shape *right;
};

struct group_fields {
    struct shape *children;
    size_t num_children;
    size_t size_children_array;
};

struct cone_cylinder_fields {
    double minimum;
    double maximum;
    bool closed;
};

struct toroid_fields {
    double r1;
    double r2;
};

struct triangle_fields {
    Point p1;
    Point p2;
    Point p3;
    Vector t1;
    Vector t2;
    Vector t3;
    Vector e1;
    Vector e2;
    bool use_textures;
    union {
        Vector normal;
        struct {
            Vector n1;
            Vector n2;
            Vector n3;
        } s_normals;
    } u_normals;
};

typedef struct shape {
    Matrix transform;
    Matrix transform_inverse;
    bool transform_identity;

    Material material;
    struct shape *parent;
    Bounding_box bbox;          /* own-space bounds (lazily computed) */
    Bounding_box bbox_inverse;  /* bounds in the parent's space (reference naming) */
    bool bbox_valid;

    enum shape_enum type;
    union {
        struct csg_fields csg;
        struct group_fields group;
        struct cone_cylinder_fields cone;
        struct cone_cylinder_fields cylinder;
        struct toroid_fields toroid;
        struct triangle_fields triangle;
    } fields;

    void (*divide)(struct shape *sh, size_t threshold);
} *Shape;

Shape array_of_shapes(size_t num);
Shape array_of_shapes_realloc(Shape ptr, size_t num);
void shape_free(Shape s);

void shape_set_transform(Shape obj, const Matrix transform);
void shape_set_material(Shape obj, Material m);
void shape_set_material_recursive(Shape obj, Material m);
void shape_copy(Shape s, Shape parent, Shape res);

/* bounds (reference shapes.c:193-224 and the per-type *_bounds) */
void shape_bounds(Shape sh, Bounding_box *res);
void shape_parent_space_bounds(Shape sh, Bounding_box *res);
void shape_divide(Shape sh, size_t threshold);
bool shape_includes(Shape a, Shape b);

void shape_recursive_parent_update(Shape sh, Shape parent);
void shape_recursive_invalidate_bounding_box(Shape sh);

#endif
