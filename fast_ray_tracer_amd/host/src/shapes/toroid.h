/* frt-mi355x host API: toroid constructor (reference src/shapes/toroid.h). */
#ifndef FRT_TOROID_H
#define FRT_TOROID_H
#include "shapes.h"
Shape toroid_alloc(void);
void toroid(Shape s);
#endif
