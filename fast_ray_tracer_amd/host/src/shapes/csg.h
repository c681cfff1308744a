/* frt-mi355x host API: constructive solid geometry node (reference src/shapes/csg.h). */
#ifndef FRT_CSG_H
#define FRT_CSG_H
#include "shapes.h"
Shape csg_alloc(enum csg_ops_enum op, Shape left_child, Shape right_child);
void csg(Shape s, enum csg_ops_enum op, Shape left_child, Shape right_child);
#endif
