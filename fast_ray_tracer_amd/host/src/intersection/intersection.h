/* frt-mi355x host API: intersection records (reference src/intersection/intersection.h:9-20). */
#ifndef FRT_INTERSECTION_H
#define FRT_INTERSECTION_H

#include <stdbool.h>
#include <stddef.h>

struct shape;
typedef struct shape *Shape;

typedef struct intersection {
    double t;
    double u;
    double v;
    Shape object;
} *Intersection;

typedef struct intersections {
    Intersection xs;
    size_t array_len;
    size_t num;
} *Intersections;

#endif
