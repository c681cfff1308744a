/*
 * frt-mi355x host: scene-graph construction and BVH build.
 *
 * Restates the construction half of reference src/shapes/*.c: constructors
 * (sphere.c:49-72, plane.c:52-72, cube.c:99-119, cylinder.c:108-132,
 * cone.c:149-173, toroid.c:88-110, triangle.c:66-96/177-207, csg.c:162-191,
 * group.c:393-432), deep copy (world.c:36-90), lazily cached bounds
 * (shapes.c:193-224 and the per-type *_bounds) and the midpoint-split BVH
 * builder group_divide (group.c:184-370) including its in-place swap
 * partition, because the reference's shadow-ray semantics depend on the exact
 * child order it produces.
 *
 * Intersection is not implemented here: render_multi flattens this graph
 * (frt_flatten.c) and the GPU traverses the flat copy.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "src/shapes/shapes.h"
#include "src/shapes/group.h"
#include "src/shapes/csg.h"
#include "src/shapes/sphere.h"
#include "src/shapes/plane.h"
#include "src/shapes/cube.h"
#include "src/shapes/cone.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/toroid.h"
#include "src/shapes/triangle.h"

#define GROUP_MIN_CAPACITY 16

static void group_divide(Shape g, size_t threshold);
static void csg_divide(Shape s, size_t threshold);

Shape
array_of_shapes(size_t num)
{
    return array_of_shapes_realloc(NULL, num);
}

Shape
array_of_shapes_realloc(Shape ptr, size_t num)
{
    return (Shape)realloc(ptr, num * sizeof(struct shape));
}

void
shape_divide(Shape sh, size_t threshold)
{
    (void)sh;
    (void)threshold;
}

bool
shape_includes(Shape a, Shape b)
{
    if (a == b) {
        return true;
    }
    if (a->type == SHAPE_GROUP) {
        for (size_t i = 0; i < a->fields.group.num_children; ++i) {
            if (shape_includes(a->fields.group.children + i, b)) {
                return true;
            }
        }
    } else if (a->type == SHAPE_CSG) {
        return shape_includes(a->fields.csg.left, b) || shape_includes(a->fields.csg.right, b);
    }
    return false;
}

void
shape_set_transform(Shape obj, const Matrix m)
{
    if (obj) {
        matrix_copy(m, obj->transform);
        matrix_inverse(m, obj->transform_inverse);
        obj->transform_identity = frt_matrix_is_identity(m);
    }
}

void
shape_set_material(Shape obj, Material m)
{
    if (obj == NULL || obj->material == m) {
        return;
    }
    if (obj->material) {
        material_free(obj->material);
    }
    obj->material = m;
    if (m) {
        m->ref_count++;
    }
}

void
shape_set_material_recursive(Shape obj, Material m)
{
    if (obj == NULL) {
        return;
    }
    shape_set_material(obj, m);
    if (obj->type == SHAPE_GROUP) {
        for (size_t i = 0; i < obj->fields.group.num_children; ++i) {
            shape_set_material_recursive(obj->fields.group.children + i, m);
        }
    }
}

static void
shape_init(Shape s, enum shape_enum type)
{
    shape_set_transform(s, MATRIX_IDENTITY);
    s->material = material_alloc();
    s->parent = NULL;
    s->type = type;
    bounding_box(&s->bbox);
    bounding_box(&s->bbox_inverse);
    s->bbox_valid = false;
    s->divide = shape_divide;
}

void sphere(Shape s) { shape_init(s, SHAPE_SPHERE); }
void plane(Shape s) { shape_init(s, SHAPE_PLANE); }
void cube(Shape s) { shape_init(s, SHAPE_CUBE); }

void
cylinder(Shape s)
{
    shape_init(s, SHAPE_CYLINDER);
    s->fields.cylinder.minimum = -INFINITY;
    s->fields.cylinder.maximum = INFINITY;
    s->fields.cylinder.closed = false;
}

void
cone(Shape s)
{
    shape_init(s, SHAPE_CONE);
    s->fields.cone.minimum = -DBL_MAX;
    s->fields.cone.maximum = DBL_MAX;
    s->fields.cone.closed = false;
}

void
toroid(Shape s)
{
    shape_init(s, SHAPE_TOROID);
    s->fields.toroid.r1 = 0.75;
    s->fields.toroid.r2 = 0.25;
}

static void
triangle_common(Shape s, enum shape_enum type, Point p1, Point p2, Point p3)
{
    shape_init(s, type);
    memset(&s->fields.triangle, 0, sizeof(s->fields.triangle));
    s->fields.triangle.use_textures = false;
    memcpy(s->fields.triangle.p1, p1, sizeof(Point));
    memcpy(s->fields.triangle.p2, p2, sizeof(Point));
    memcpy(s->fields.triangle.p3, p3, sizeof(Point));
    vector_from_points(p2, p1, s->fields.triangle.e1);
    vector_from_points(p3, p1, s->fields.triangle.e2);
}

void
triangle(Shape s, Point p1, Point p2, Point p3)
{
    triangle_common(s, SHAPE_TRIANGLE, p1, p2, p3);
    Vector cross;
    /* face normal = normalize(e2 x e1) (triangle.c:84-88) */
    vector_cross(s->fields.triangle.e2, s->fields.triangle.e1, cross);
    vector_normalize(cross, s->fields.triangle.u_normals.normal);
}

void
smooth_triangle(Shape s, Point p1, Point p2, Point p3, Vector n1, Vector n2, Vector n3)
{
    triangle_common(s, SHAPE_SMOOTH_TRIANGLE, p1, p2, p3);
    vector_copy(s->fields.triangle.u_normals.s_normals.n1, n1);
    vector_copy(s->fields.triangle.u_normals.s_normals.n2, n2);
    vector_copy(s->fields.triangle.u_normals.s_normals.n3, n3);
}

#define FRT_ALLOC0(name)                                 \
    Shape name##_alloc(void)                             \
    {                                                    \
        Shape s = (Shape)malloc(sizeof(struct shape));   \
        name(s);                                         \
        return s;                                        \
    }
FRT_ALLOC0(sphere)
FRT_ALLOC0(plane)
FRT_ALLOC0(cube)
FRT_ALLOC0(cone)
FRT_ALLOC0(cylinder)
FRT_ALLOC0(toroid)
#undef FRT_ALLOC0

Shape
triangle_array_alloc(Point p1, Point p2, Point p3)
{
    Shape s = (Shape)malloc(sizeof(struct shape));
    triangle(s, p1, p2, p3);
    return s;
}

Shape
triangle_point_alloc(Point p1, Point p2, Point p3)
{
    return triangle_array_alloc(p1, p2, p3);
}

Shape
smooth_triangle_alloc(Point p1, Point p2, Point p3, Vector n1, Vector n2, Vector n3)
{
    Shape s = (Shape)malloc(sizeof(struct shape));
    smooth_triangle(s, p1, p2, p3, n1, n2, n3);
    return s;
}

void
csg(Shape s, enum csg_ops_enum op, Shape left, Shape right)
{
    shape_init(s, SHAPE_CSG);
    s->fields.csg.op = op;
    s->fields.csg.left = left;
    s->fields.csg.right = right;
    left->parent = s;
    right->parent = s;
    s->divide = csg_divide;
}

Shape
csg_alloc(enum csg_ops_enum op, Shape left, Shape right)
{
    Shape s = (Shape)malloc(sizeof(struct shape));
    csg(s, op, left, right);
    return s;
}

/* ---------------- deep copy ---------------- */

void
shape_copy(Shape s, Shape parent, Shape res)
{
    if (s == res) {
        printf("Trying to copy a shape to itself.\n");
        return;
    }
    *res = *s;
    res->parent = parent;
    res->material = NULL;
    shape_set_material(res, s->material);
    if (s->type == SHAPE_CSG) {
        Shape lr = array_of_shapes(2);
        shape_copy(s->fields.csg.left, res, lr);
        shape_copy(s->fields.csg.right, res, lr + 1);
        res->fields.csg.left = lr;
        res->fields.csg.right = lr + 1;
    } else if (s->type == SHAPE_GROUP) {
        size_t n = s->fields.group.num_children;
        size_t cap = s->fields.group.size_children_array > n ? s->fields.group.size_children_array : n;
        res->fields.group.children = cap ? array_of_shapes(cap) : NULL;
        res->fields.group.size_children_array = cap;
        for (size_t i = 0; i < n; ++i) {
            shape_copy(s->fields.group.children + i, res, res->fields.group.children + i);
        }
    }
}

void
shape_free(Shape s)
{
    if (s == NULL) {
        return;
    }
    material_free(s->material);
    s->material = NULL;
    s->bbox_valid = false;
    if (s->type == SHAPE_GROUP) {
        group_free(s);
    }
}

void
group_free(Shape g)
{
    for (size_t i = 0; i < g->fields.group.num_children; ++i) {
        shape_free(g->fields.group.children + i);
    }
    free(g->fields.group.children);
    g->fields.group.children = NULL;
    g->fields.group.num_children = 0;
    g->fields.group.size_children_array = 0;
}

/* ---------------- parent links / bound invalidation ---------------- */

void
shape_recursive_parent_update(Shape sh, Shape parent)
{
    sh->parent = parent;
    if (sh->type == SHAPE_GROUP) {
        for (size_t i = 0; i < sh->fields.group.num_children; ++i) {
            shape_recursive_parent_update(sh->fields.group.children + i, sh);
        }
    } else if (sh->type == SHAPE_CSG) {
        shape_recursive_parent_update(sh->fields.csg.left, sh);
        shape_recursive_parent_update(sh->fields.csg.right, sh);
    }
}

void
shape_recursive_invalidate_bounding_box(Shape sh)
{
    sh->bbox_valid = false;
    bounding_box(&sh->bbox);
    if (sh->type == SHAPE_GROUP) {
        for (size_t i = 0; i < sh->fields.group.num_children; ++i) {
            shape_recursive_invalidate_bounding_box(sh->fields.group.children + i);
        }
    } else if (sh->type == SHAPE_CSG) {
        shape_recursive_invalidate_bounding_box(sh->fields.csg.left);
        shape_recursive_invalidate_bounding_box(sh->fields.csg.right);
    }
}

/* ---------------- bounds ---------------- */

static void
add_xyz(Bounding_box *b, double x, double y, double z)
{
    double p[4] = {x, y, z, 1.0};
    bounding_box_add_array(b, p);
}

void
shape_bounds(Shape sh, Bounding_box *res)
{
    if (!sh->bbox_valid) {
        sh->bbox_valid = true;
        Bounding_box *b = &sh->bbox;
        switch (sh->type) {
        case SHAPE_PLANE:
            add_xyz(b, -INFINITY, 0.0, -INFINITY);
            add_xyz(b, INFINITY, 0.0, INFINITY);
            break;
        case SHAPE_CYLINDER:
            add_xyz(b, -1.0, sh->fields.cylinder.minimum, -1.0);
            add_xyz(b, 1.0, sh->fields.cylinder.maximum, 1.0);
            break;
        case SHAPE_CONE: {
            double limit = fmax(fabs(sh->fields.cone.minimum), fabs(sh->fields.cone.maximum));
            add_xyz(b, -limit, sh->fields.cone.minimum, -limit);
            add_xyz(b, limit, sh->fields.cone.maximum, limit);
            break;
        }
        case SHAPE_TOROID: {
            double r1 = sh->fields.toroid.r1, r2 = sh->fields.toroid.r2;
            add_xyz(b, -r1 - r2, -r2, -r1 - r2);
            add_xyz(b, r1 + r2, r2, r1 + r2);
            break;
        }
        case SHAPE_TRIANGLE:
        case SHAPE_SMOOTH_TRIANGLE:
            bounding_box_add_array(b, sh->fields.triangle.p1);
            bounding_box_add_array(b, sh->fields.triangle.p2);
            bounding_box_add_array(b, sh->fields.triangle.p3);
            break;
        case SHAPE_CSG: {
            Bounding_box l, r;
            shape_parent_space_bounds(sh->fields.csg.left, &l);
            shape_parent_space_bounds(sh->fields.csg.right, &r);
            bounding_box_add_box(b, &l);
            bounding_box_add_box(b, &r);
            break;
        }
        case SHAPE_GROUP:
            for (size_t i = 0; i < sh->fields.group.num_children; ++i) {
                Bounding_box c;
                shape_parent_space_bounds(sh->fields.group.children + i, &c);
                bounding_box_add_box(b, &c);
            }
            break;
        default: /* sphere, cube: the unit box */
            add_xyz(b, -1.0, -1.0, -1.0);
            add_xyz(b, 1.0, 1.0, 1.0);
            break;
        }
        bounding_box_transform(&sh->bbox, sh->transform, &sh->bbox_inverse);
    }
    *res = sh->bbox;
}

void
shape_parent_space_bounds(Shape sh, Bounding_box *res)
{
    if (!sh->bbox_valid) {
        Bounding_box tmp;
        shape_bounds(sh, &tmp);
    }
    *res = sh->bbox_inverse;
}

/* ---------------- groups ---------------- */

void
group(Shape s, Shape children, size_t n)
{
    shape_init(s, SHAPE_GROUP);
    size_t cap = n > GROUP_MIN_CAPACITY ? n : GROUP_MIN_CAPACITY;
    s->fields.group.children = array_of_shapes(cap);
    for (size_t i = 0; i < n; ++i) {
        shape_copy(children + i, s, s->fields.group.children + i);
    }
    s->fields.group.num_children = n;
    s->fields.group.size_children_array = cap;
    shape_recursive_parent_update(s, s->parent);
    shape_recursive_invalidate_bounding_box(s);
    s->divide = group_divide;
}

Shape
group_alloc(Shape children, size_t n)
{
    Shape s = (Shape)malloc(sizeof(struct shape));
    group(s, children, n);
    return s;
}

void
group_add_children_stage(Shape g, Shape children, size_t n)
{
    for (size_t k = 0; k < n; ++k) {
        if (children + k == g) {
            continue; /* duplicates allowed, self reference not (group.c:59-79) */
        }
        if (g->fields.group.num_children + 1 >= g->fields.group.size_children_array) {
            size_t cap = g->fields.group.size_children_array ? 2 * g->fields.group.size_children_array : GROUP_MIN_CAPACITY;
            g->fields.group.children = array_of_shapes_realloc(g->fields.group.children, cap);
            g->fields.group.size_children_array = cap;
        }
        shape_copy(children + k, g, g->fields.group.children + g->fields.group.num_children);
        g->fields.group.num_children += 1;
    }
}

void
group_add_children_finish(Shape g)
{
    if (g) {
        shape_recursive_invalidate_bounding_box(g);
        shape_recursive_parent_update(g, g->parent);
    }
}

void
group_add_children(Shape g, Shape children, size_t n)
{
    group_add_children_stage(g, children, n);
    group_add_children_finish(g);
}

static void
swap_shapes(Shape a, Shape b)
{
    struct shape t = *a;
    *a = *b;
    *b = t;
}

static void
swap_flags(bool *m, size_t a, size_t b)
{
    bool t = m[a];
    m[a] = m[b];
    m[b] = t;
}

struct partition {
    size_t left_count, middle_count, right_count;
    long left_start, middle_start, right_start;
};

/*
 * Classify children against the two halves of the group's box and move them
 * in place into [left | middle | right] with the reference's two-pointer swap
 * passes (group.c:184-297). The passes are not stable; their exact swap
 * sequence fixes the child order of the built tree.
 */
static struct partition
partition_children(Shape g)
{
    Bounding_box box, lbox, rbox;
    shape_bounds(g, &box);
    bounding_box_split_bounds(&box, &lbox, &rbox);

    size_t n = g->fields.group.num_children;
    Shape ch = g->fields.group.children;
    bool *is_left = (bool *)calloc(n ? n : 1, sizeof(bool));
    bool *is_right = (bool *)calloc(n ? n : 1, sizeof(bool));
    struct partition p = {0, 0, 0, -1, -1, -1};

    for (size_t i = 0; i < n; ++i) {
        Bounding_box cb;
        shape_parent_space_bounds(ch + i, &cb);
        if (bounding_box_contains_box(&lbox, &cb)) {
            is_left[i] = true;
            p.left_count++;
        } else if (bounding_box_contains_box(&rbox, &cb)) {
            is_right[i] = true;
            p.right_count++;
        } else {
            p.middle_count++;
        }
    }

    size_t i = 0, j = 0;
    while (i < n && j < n) {
        if (is_left[i]) {
            if (p.left_start < 0) {
                p.left_start = (long)i;
            }
            i++;
            j++;
            continue;
        }
        while (j < n && !is_left[j]) {
            j++;
        }
        if (j < n) {
            swap_shapes(ch + i, ch + j);
            swap_flags(is_left, i, j);
            swap_flags(is_right, i, j);
        }
    }

    j = i;
    while (i < n && j < n) {
        if (!is_right[i]) {
            if (p.middle_start < 0) {
                p.middle_start = (long)i;
            }
            i++;
            j++;
            continue;
        }
        while (j < n && is_right[j]) {
            j++;
        }
        if (j < n) {
            swap_shapes(ch + i, ch + j);
            swap_flags(is_left, i, j);
            swap_flags(is_right, i, j);
        }
    }
    if (i < n) {
        p.right_start = (long)i;
    }

    free(is_left);
    free(is_right);
    return p;
}

static void
group_divide(Shape g, size_t threshold)
{
    size_t n = g->fields.group.num_children;
    if (threshold < n) {
        struct partition p = partition_children(g);
        if (p.middle_count != n) {
            size_t cap = p.middle_count + (p.left_count > 0) + (p.right_count > 0);
            if (cap < g->fields.group.size_children_array) {
                cap = g->fields.group.size_children_array;
            }
            Shape fresh = array_of_shapes(cap);
            Shape pos = fresh;
            Shape old = g->fields.group.children;
            /* new child order: left subgroup, right subgroup, then the straddlers (group.c:326-348) */
            if (p.left_count > 0) {
                group(pos, old + p.left_start, p.left_count);
                for (size_t k = 0; k < p.left_count; ++k) {
                    shape_free(old + p.left_start + k);
                }
                shape_recursive_parent_update(pos, g);
                pos++;
            }
            if (p.right_count > 0) {
                group(pos, old + p.right_start, p.right_count);
                for (size_t k = 0; k < p.right_count; ++k) {
                    shape_free(old + p.right_start + k);
                }
                shape_recursive_parent_update(pos, g);
                pos++;
            }
            if (p.middle_count > 0) {
                memcpy(pos, old + p.middle_start, p.middle_count * sizeof(struct shape));
            }
            free(old);
            g->fields.group.children = fresh;
            g->fields.group.num_children = p.middle_count + (p.left_count > 0) + (p.right_count > 0);
            g->fields.group.size_children_array = cap;
            shape_recursive_parent_update(g, g->parent);
        }
    }
    for (size_t k = 0; k < g->fields.group.num_children; ++k) {
        Shape c = g->fields.group.children + k;
        c->divide(c, threshold);
    }
}

static void
csg_divide(Shape s, size_t threshold)
{
    s->fields.csg.left->divide(s->fields.csg.left, threshold);
    s->fields.csg.right->divide(s->fields.csg.right, threshold);
}
