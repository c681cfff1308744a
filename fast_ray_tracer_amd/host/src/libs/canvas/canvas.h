/*
 * frt-mi355x host API: framebuffer / texture canvas.
 * Field and function names follow reference src/libs/canvas/canvas.h:10-38.
 * A Canvas is hsize*vsize Color (double[4]) in row-major order, row 0 = top.
 */
#ifndef FRT_CANVAS_H
#define FRT_CANVAS_H

#include <stddef.h>
#include <stdbool.h>

#include "../../color/color.h"

typedef struct canvas {
    Color *arr;
    size_t width;
    size_t height;
    bool super_sample;
    void (*color_space_fn)(const Color, Color);
} *Canvas;

typedef struct ppm_struct {
    unsigned char *arr;
    size_t len;
} *Ppm;

Canvas canvas_alloc(size_t width, size_t height, bool super_sample, void (*color_space_fn)(const Color, Color));
Ppm ppm_alloc(size_t len);
void canvas_free(Canvas c);
void ppm_free(Ppm p);

/* (frt: render_multi's canvas, its array in page-locked memory that the device writes by DMA; canvas_free hands the
 * array to a one-entry pool the next such canvas of the same size reuses. frt_canvas_pool_release frees the pooled
 * array: frt_render_multi_release calls it) */
Canvas frt_canvas_alloc_pinned(size_t width, size_t height, bool super_sample, void (*color_space_fn)(const Color, Color));
void frt_canvas_pool_release(void);

void canvas_write_pixels(Canvas c, int col, int row, Color *colors, size_t num);
void canvas_write_pixel(Canvas c, int col, int row, Color color);
void canvas_pixel_at(Canvas c, int col, int row, Color res);

Ppm construct_ppm(Canvas c, bool use_scaling);
int write_ppm_file(Canvas c, const bool use_scaling, const char *file_name);
int write_png(Canvas c, const char *file_name);

void construct_canvas_from_ppm_file(Canvas *c, const char *file_path, bool super_sample, void (*color_space_fn)(const Color, Color));
int read_png(Canvas *c, const char *filename, bool super_sample, void (*color_space_fn)(const Color, Color));

#endif
