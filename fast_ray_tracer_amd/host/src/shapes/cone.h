/* frt-mi355x host API: cone constructor (reference src/shapes/cone.h). */
#ifndef FRT_CONE_H
#define FRT_CONE_H
#include "shapes.h"
Shape cone_alloc(void);
void cone(Shape s);
#endif
