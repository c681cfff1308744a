/* frt-mi355x host API: sRGB conversions (reference src/color/srgb.c:16-24). */
#ifndef FRT_SRGB_H
#define FRT_SRGB_H
#include "color.h"
void srgb_to_rgb(const Color srgb, Color rgb);
void srgb_to_xyz(const Color srgb, Color xyz);
#endif
