/* frt-mi355x host API: sphere constructor (reference src/shapes/sphere.h). */
#ifndef FRT_SPHERE_H
#define FRT_SPHERE_H
#include "shapes.h"
Shape sphere_alloc(void);
void sphere(Shape s);
#endif
