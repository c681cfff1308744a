/* frt-mi355x host API: cylinder constructor (reference src/shapes/cylinder.h). */
#ifndef FRT_CYLINDER_H
#define FRT_CYLINDER_H
#include "shapes.h"
Shape cylinder_alloc(void);
void cylinder(Shape s);
#endif
