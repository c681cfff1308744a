/* frt-mi355x host API: CIE Lab, D65 2-degree white (reference src/color/lab.h:13-19). */
#ifndef FRT_LAB_H
#define FRT_LAB_H
#include "color.h"
void lab_to_xyz(const Color lab, Color xyz);
void lab_to_rgb(const Color lab, Color rgb);
#endif
