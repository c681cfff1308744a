/*
 * frt-mi355x host: color arithmetic and color-space conversions.
 * Formulas restated from reference src/color/{color,rgb,srgb,xyz,lab,xyy,hsl}.c
 * (same constants, same pow/branch structure) so the values the codegen feeds
 * into materials and patterns are bit-identical to the reference's.
 */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "src/color/color.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"
#include "src/color/lab.h"
#include "src/color/hsl.h"
#include "src/libs/linalg/linalg.h"

/* D65, 2-degree observer (reference src/color/lab.h:13-19) */
static const double D65_WHITE[3] = {0.95047, 1.00000, 1.08883};

/* linear sRGB primaries <-> XYZ (reference src/color/xyz.h:28-38) */
static const double RGB2XYZ[9] = {
    0.412453, 0.357580, 0.180423,
    0.212671, 0.715160, 0.072169,
    0.019334, 0.119193, 0.950227};
static const double XYZ2RGB[9] = {
    3.240479, -1.537150, -0.498535,
    -0.969256, 1.875992, 0.041556,
    0.055648, -0.204043, 1.057311};

void
color_accumulate(Color acc, const Color other)
{
    acc[0] += other[0];
    acc[1] += other[1];
    acc[2] += other[2];
}

void
color_scale(Color acc, const double s)
{
    acc[0] *= s;
    acc[1] *= s;
    acc[2] *= s;
}

void color_copy(Color to, const Color from) { memcpy(to, from, sizeof(Color)); }
void color_triple_copy(ColorTriple to, const ColorTriple from) { memcpy(to, from, sizeof(ColorTriple)); }

void
print_color(const Color c)
{
    printf("Color: [%f %f %f]\n", c[0], c[1], c[2]);
}

void
print_color_triple(const ColorTriple c)
{
    print_color(c);
    print_color(c + 4);
    print_color(c + 8);
    printf("\n");
}

void
color_average(Color c1, Color c2, Color res)
{
    for (int k = 0; k < 3; ++k) {
        res[k] = (c1[k] + c2[k]) / 2.0;
    }
}

void
color_triple_average(Color c1, Color c2, Color res)
{
    for (int part = 0; part < 12; part += 4) {
        color_average(c1 + part, c2 + part, res + part);
    }
}

static void
mat3_apply(const double *m, const Color in, Color out)
{
    double r[3];
    for (int k = 0; k < 3; ++k) {
        r[k] = m[3 * k + 0] * in[0] + m[3 * k + 1] * in[1] + m[3 * k + 2] * in[2];
    }
    out[0] = r[0];
    out[1] = r[1];
    out[2] = r[2];
}

void rgb_to_rgb(const Color from, Color to) { color_copy(to, from); }
void xyy_to_rgb(const Color xyy, Color rgb) { color_copy(rgb, xyy); }

void
hsl_to_rgb(const Color hsl, Color rgb)
{
    /* The reference leaves this conversion empty (src/color/hsl.c:4-6): the
     * output color is left untouched. Kept identical for drop-in parity. */
    (void)hsl;
    (void)rgb;
}

void rgb_to_xyz(const Color rgb, Color xyz) { mat3_apply(RGB2XYZ, rgb, xyz); }
void xyz_to_rgb(const Color xyz, Color rgb) { mat3_apply(XYZ2RGB, xyz, rgb); }

void
rgb_to_srgb(const Color rgb, Color srgb)
{
    for (int k = 0; k < 3; ++k) {
        double x = rgb[k];
        srgb[k] = x < 0.0031308 ? x * 12.92 : (1.055 * pow(x, 1.0 / 2.4) - 0.055);
    }
}

void
srgb_to_rgb(const Color srgb, Color rgb)
{
    for (int k = 0; k < 3; ++k) {
        double x = srgb[k];
        rgb[k] = x <= 0.04045 ? x / 12.92 : pow((x + 0.055) / 1.055, 2.4);
    }
}

void
srgb_to_xyz(const Color srgb, Color xyz)
{
    Color lin;
    srgb_to_rgb(srgb, lin);
    rgb_to_xyz(lin, xyz);
}

void
xyz_to_srgb(const Color xyz, Color srgb)
{
    Color lin;
    xyz_to_rgb(xyz, lin);
    rgb_to_srgb(lin, srgb);
}

static double
lab_f(double t)
{
    return t > 0.008856 ? pow(t, 1.0 / 3.0) : 7.787 * t + 16.0 / 116.0;
}

void
xyz_to_lab(const Color xyz, Color lab)
{
    double x = xyz[0] / D65_WHITE[0];
    double y = xyz[1] / D65_WHITE[1];
    double z = xyz[2] / D65_WHITE[2];
    double fx = lab_f(x), fy = lab_f(y), fz = lab_f(z);
    lab[0] = y > 0.008856 ? 116.0 * pow(y, 1.0 / 3.0) - 16.0 : 903.3 * y;
    lab[1] = 500.0 * (fx - fy);
    lab[2] = 200.0 * (fy - fz);
}

void
lab_to_xyz(const Color lab, Color xyz)
{
    double p = (lab[0] + 16.0) / 116.0;
    xyz[0] = D65_WHITE[0] * pow(p + lab[1] / 500.0, 3.0);
    xyz[1] = D65_WHITE[1] * pow(p, 3.0);
    xyz[2] = D65_WHITE[2] * pow(p - lab[2] / 200.0, 3.0);
}

void
lab_to_rgb(const Color lab, Color rgb)
{
    Color xyz;
    lab_to_xyz(lab, xyz);
    xyz_to_rgb(xyz, rgb);
}

void
rgb_to_lab(const Color rgb, Color lab)
{
    Color xyz;
    rgb_to_xyz(rgb, xyz);
    xyz_to_lab(xyz, lab);
}

void
rgb_to_hsl(const Color rgb, Color hsl)
{
    double r = rgb[0], g = rgb[1], b = rgb[2];
    double hi = fmax(fmax(r, g), b);
    double lo = fmin(fmin(r, g), b);
    hsl[2] = (hi + lo) / 2.0;
    hsl[1] = hsl[2] < 0.5 ? (hi - lo) / (hi + lo) : (hi - lo) / (2.0 - hi - lo);
    if (equal(hi, r)) {
        hsl[0] = (g - b) / (hi - lo);
    } else if (equal(hi, g)) {
        hsl[0] = 2.0 + (b - r) / (hi - lo);
    } else {
        hsl[0] = 4.0 + (r - g) / (hi - lo);
    }
    hsl[0] *= 60;
    if (hsl[0] < 0) {
        hsl[0] += 360.0;
    }
}

static int
cmp_diff(double l, double r)
{
    return (l - r < 0) ? -1 : ((l - r > 0) ? 1 : 0);
}

int lab_compare_l(const Color l, const Color r) { return cmp_diff(l[0], r[0]); }
int lab_compare_a(const Color l, const Color r) { return cmp_diff(l[1], r[1]); }
int lab_compare_b(const Color l, const Color r) { return cmp_diff(l[2], r[2]); }
