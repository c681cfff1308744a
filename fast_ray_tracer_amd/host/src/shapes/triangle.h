/* frt-mi355x host API: flat and smooth triangles (reference src/shapes/triangle.h). */
#ifndef FRT_TRIANGLE_H
#define FRT_TRIANGLE_H
#include "../libs/linalg/linalg.h"
#include "shapes.h"
Shape triangle_point_alloc(Point p1, Point p2, Point p3);
Shape triangle_array_alloc(Point p1, Point p2, Point p3);
Shape smooth_triangle_alloc(Point p1, Point p2, Point p3, Vector n1, Vector n2, Vector n3);
void triangle(Shape s, Point p1, Point p2, Point p3);
void smooth_triangle(Shape s, Point p1, Point p2, Point p3, Vector n1, Vector n2, Vector n3);
#endif
