/* frt-mi355x host API: rays (reference src/renderer/ray.h). */
#ifndef FRT_RAY_H
#define FRT_RAY_H

#include "../libs/linalg/linalg.h"

typedef struct ray {
    Point origin;
    Vector direction;
} *Ray;

void ray_array(Point origin, Vector direction, Ray ray);
void ray_transform(Ray original, Matrix m, Ray res);
void ray_position(Ray ray, double t, Point position);

#endif
