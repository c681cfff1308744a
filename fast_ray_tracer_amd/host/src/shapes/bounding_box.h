/*
 * frt-mi355x host API: axis-aligned bounding boxes, restated from reference
 * src/shapes/bounding_box.c:6-214 (empty box = +inf/-inf; transform = the 8
 * corners pushed through the matrix; slab test with the |d|<EPSILON rule).
 */
#ifndef FRT_BOUNDING_BOX_H
#define FRT_BOUNDING_BOX_H

#include <stdbool.h>
#include "../libs/linalg/linalg.h"

struct ray;

typedef struct bbox {
    Point min;
    Point max;
} Bounding_box;

void bounding_box(Bounding_box *res);
void bounding_box_add_array(Bounding_box *box, double point[4]);
void bounding_box_add_box(Bounding_box *box, Bounding_box *other);
bool bounding_box_contains_array(Bounding_box *box, double point[4]);
bool bounding_box_contains_box(Bounding_box *box, Bounding_box *other);
void bounding_box_transform(Bounding_box *box, const Matrix m, Bounding_box *res);
bool bounding_box_intersects(Bounding_box *box, struct ray *r);
void bounding_box_split_bounds(Bounding_box *box, Bounding_box *left_res, Bounding_box *right_res);

#endif
