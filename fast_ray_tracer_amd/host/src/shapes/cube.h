/* frt-mi355x host API: cube constructor (reference src/shapes/cube.h). */
#ifndef FRT_CUBE_H
#define FRT_CUBE_H
#include "shapes.h"
Shape cube_alloc(void);
void cube(Shape s);
#endif
