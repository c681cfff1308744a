/* frt-mi355x host API: HSL (an empty stub in the reference, src/color/hsl.c:4-6). */
#ifndef FRT_HSL_H
#define FRT_HSL_H
#include "color.h"
void hsl_to_rgb(const Color hsl, Color rgb);
#endif
