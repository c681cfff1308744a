/* frt-mi355x host API: plane constructor (reference src/shapes/plane.h). */
#ifndef FRT_PLANE_H
#define FRT_PLANE_H
#include "shapes.h"
Shape plane_alloc(void);
void plane(Shape s);
#endif
