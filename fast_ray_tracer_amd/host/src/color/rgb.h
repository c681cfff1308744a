/* frt-mi355x host API: linear-RGB conversions (reference src/color/rgb.h). */
#ifndef FRT_RGB_H
#define FRT_RGB_H
#include "color.h"
void rgb_to_rgb(const Color from, Color to);
void rgb_to_hsl(const Color rgb, Color hsl);
void rgb_to_xyz(const Color rgb, Color xyz);
void rgb_to_lab(const Color rgb, Color lab);
void rgb_to_srgb(const Color rgb, Color srgb);
#endif
