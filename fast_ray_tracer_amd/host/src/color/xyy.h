/* frt-mi355x host API: xyY (identity in the reference, src/color/xyy.c). */
#ifndef FRT_XYY_H
#define FRT_XYY_H
#include "color.h"
void xyy_to_rgb(const Color xyy, Color rgb);
#endif
