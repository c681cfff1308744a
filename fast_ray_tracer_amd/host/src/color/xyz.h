/* frt-mi355x host API: CIE XYZ conversions (reference src/color/xyz.h). */
#ifndef FRT_XYZ_H
#define FRT_XYZ_H
#include "color.h"
void xyz_to_rgb(const Color xyz, Color rgb);
void xyz_to_srgb(const Color xyz, Color srgb);
void xyz_to_lab(const Color xyz, Color lab);
#endif
