/*
 * frt-mi355x host: canvas storage and image I/O.
 *
 * The output contract of the drop-in boundary is the reference's: a Color
 * (double[4]) canvas, row 0 at the top, written as a 16-bit big-endian P6 PPM
 * with the reference's normalisation (reference src/libs/canvas/canvas.c:150-327)
 * and as a 16-bit sRGB PNG through libpng (canvas.c:376-510). Texture readers
 * (PNG, ASCII PPM) follow canvas.c:330-672. The encode runs on the host after
 * the device canvas has been copied back.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <png.h>

#include "src/libs/canvas/canvas.h"
#include "src/color/rgb.h"
#include "src/libs/linalg/linalg.h"
#include "frt_device.h"

#define FRT_SQRT3 1.7320508075688772

/*
 * A canvas with a word of our own behind the reference's struct: the byte size of its array when that array is
 * page-locked (frt_canvas_alloc_pinned), 0 when malloc'd. render_multi's canvas is page-locked so that the device's
 * copy of the frame is one DMA into it (into malloc'd memory the runtime stages it through its own buffers, and a
 * fresh 66 MB array at 1920x1080 first takes ~16 000 page faults); canvas_free hands such an array to a one-entry
 * pool that the next render_multi of the same size takes again.
 */
typedef struct {
    struct canvas c;
    size_t pinned_bytes;
} canvas_box;

static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;
static void *g_pool_arr;     /* an idle page-locked array */
static size_t g_pool_bytes;

static Canvas
canvas_new(size_t width, size_t height, bool super_sample, void (*color_space_fn)(const Color, Color))
{
    canvas_box *b = (canvas_box *)malloc(sizeof(canvas_box));
    if (b == NULL) {
        return NULL;
    }
    b->pinned_bytes = 0;
    b->c.arr = NULL;
    b->c.width = width;
    b->c.height = height;
    b->c.super_sample = super_sample;
    b->c.color_space_fn = color_space_fn;
    return &b->c;
}

Canvas
canvas_alloc(size_t width, size_t height, bool super_sample, void (*color_space_fn)(const Color, Color))
{
    Canvas c = canvas_new(width, height, super_sample, color_space_fn);
    if (c != NULL) {
        c->arr = (Color *)malloc(width * height * sizeof(Color));
    }
    return c;
}

Canvas
frt_canvas_alloc_pinned(size_t width, size_t height, bool super_sample, void (*color_space_fn)(const Color, Color))
{
    Canvas c = canvas_new(width, height, super_sample, color_space_fn);
    if (c == NULL) {
        return NULL;
    }
    const size_t bytes = width * height * sizeof(Color);
    void *stale = NULL;
    pthread_mutex_lock(&g_pool_lock);
    if (g_pool_arr != NULL && g_pool_bytes == bytes) {
        c->arr = (Color *)g_pool_arr;
        g_pool_arr = NULL;
    } else {
        stale = g_pool_arr;  /* (another size: freed, outside the lock) */
        g_pool_arr = NULL;
    }
    pthread_mutex_unlock(&g_pool_lock);
    frt_host_pinned_free(stale);
    if (c->arr == NULL) {
        c->arr = (Color *)frt_host_pinned_alloc(bytes);
    }
    if (c->arr != NULL) {
        ((canvas_box *)c)->pinned_bytes = bytes;
    } else {
        c->arr = (Color *)malloc(bytes);  /* (no page-locked memory: an ordinary array) */
    }
    return c;
}

void
frt_canvas_pool_release(void)
{
    pthread_mutex_lock(&g_pool_lock);
    void *p = g_pool_arr;
    g_pool_arr = NULL;
    g_pool_bytes = 0;
    pthread_mutex_unlock(&g_pool_lock);
    frt_host_pinned_free(p);
}

Ppm
ppm_alloc(size_t len)
{
    Ppm p = (Ppm)malloc(sizeof(struct ppm_struct));
    p->arr = (unsigned char *)malloc(len);
    p->len = len;
    return p;
}

void
canvas_free(Canvas c)
{
    if (c == NULL) {
        return;
    }
    canvas_box *b = (canvas_box *)c;
    if (b->pinned_bytes > 0) {
        void *spill = c->arr;
        pthread_mutex_lock(&g_pool_lock);
        if (g_pool_arr == NULL) {
            g_pool_arr = c->arr;
            g_pool_bytes = b->pinned_bytes;
            spill = NULL;
        }
        pthread_mutex_unlock(&g_pool_lock);
        frt_host_pinned_free(spill);
    } else {
        free(c->arr);
    }
    free(b);
}

void
ppm_free(Ppm p)
{
    if (p) {
        free(p->arr);
        free(p);
    }
}

void
canvas_write_pixels(Canvas c, int col, int row, Color *colors, size_t num)
{
    memcpy(c->arr + (size_t)row * c->width + col, colors, num * sizeof(Color));
}

void
canvas_write_pixel(Canvas c, int col, int row, Color color)
{
    memcpy(c->arr[(size_t)row * c->width + col], color, sizeof(Color));
}

void
canvas_pixel_at(Canvas c, int col, int row, Color res)
{
    /* reference canvas.c:115-148: optional 3x3 wrap-around box filter, then
     * the canvas's color-space function per fetch */
    if (!c->super_sample) {
        c->color_space_fn(c->arr[(size_t)row * c->width + col], res);
        return;
    }
    Color acc = {0.0, 0.0, 0.0, 0.0};
    int w = (int)c->width, h = (int)c->height;
    int cc = col - 1;
    for (int j = 0; j < 3; ++j, ++cc) {
        if (cc < 0) cc += w;
        if (cc == w) cc = 0;
        int rr = row - 1;
        for (int i = 0; i < 3; ++i, ++rr) {
            if (rr < 0) rr += h;
            if (rr == h) rr = 0;
            color_accumulate(acc, c->arr[(size_t)rr * c->width + cc]);
        }
    }
    color_scale(acc, 1.0 / 9.0);
    c->color_space_fn(acc, res);
}

static uint16_t
quantize(double srgb, double srgb_max, double inverse)
{
    if (srgb > srgb_max) {
        return 65535;
    }
    if (srgb < 0) {
        return 0;
    }
    return (uint16_t)floor(srgb * inverse);
}

Ppm
construct_ppm(Canvas c, bool use_scaling)
{
    char header[32];
    int n = snprintf(header, sizeof(header), "P6\n%zu %zu\n65535\n", c->width, c->height);
    size_t npx = c->width * c->height;
    Ppm ppm = ppm_alloc(npx * 6 + (size_t)n + 1);
    unsigned char *out = ppm->arr;
    memcpy(out, header, (size_t)n);
    out += n;

    /* pass 1: per-channel linear maximum (starts at 0) */
    Color rgb_max = {0.0, 0.0, 0.0, 0.0};
    for (size_t i = 0; i < npx; ++i) {
        for (int k = 0; k < 3; ++k) {
            if (c->arr[i][k] > rgb_max[k]) {
                rgb_max[k] = c->arr[i][k];
            }
        }
    }
    print_color(rgb_max);

    /* pass 2: maximum of sRGB(pixel / rgb_max) */
    Color srgb_max = {0.0, 0.0, 0.0, 0.0};
    for (size_t i = 0; i < npx; ++i) {
        Color t, s;
        memcpy(t, c->arr[i], sizeof(Color));
        t[0] /= rgb_max[0];
        t[1] /= rgb_max[1];
        t[2] /= rgb_max[2];
        rgb_to_srgb(t, s);
        for (int k = 0; k < 3; ++k) {
            if (s[k] > srgb_max[k]) {
                srgb_max[k] = s[k];
            }
        }
    }
    print_color(srgb_max);

    double inv[3] = {65535.0 / srgb_max[0], 65535.0 / srgb_max[1], 65535.0 / srgb_max[2]};

    for (size_t i = 0; i < npx; ++i) {
        Color t, s;
        memcpy(t, c->arr[i], sizeof(Color));
        if (use_scaling) {
            double len = t[0] + t[1] + t[2];
            if (len > FRT_SQRT3) {
                color_scale(t, 1.0 / len);
                color_scale(t, FRT_SQRT3);
            }
        } else {
            for (int k = 0; k < 3; ++k) {
                if (t[k] > 1.0) {
                    t[k] = 1.0;
                } else if (t[k] < 0) {
                    t[k] = 0.0;
                }
            }
        }
        rgb_to_srgb(t, s);
        for (int k = 0; k < 3; ++k) {
            uint16_t q = quantize(s[k], srgb_max[k], inv[k]);
            *out++ = (unsigned char)(q >> 8);
            *out++ = (unsigned char)(q & 0xFF);
        }
    }
    *out = '\n';
    return ppm;
}

static char *
with_suffix(const char *path, const char *suffix)
{
    size_t a = strlen(path), b = strlen(suffix);
    char *s = (char *)malloc(a + b + 1);
    memcpy(s, path, a);
    memcpy(s + a, suffix, b + 1);
    return s;
}

int
write_ppm_file(Canvas c, const bool use_scaling, const char *file_path)
{
    char *full = with_suffix(file_path, ".ppm");
    Ppm ppm = construct_ppm(c, use_scaling);
    FILE *f = fopen(full, "wb");
    int rc = 0;
    if (f == NULL) {
        fprintf(stderr, "frt: cannot open %s for writing\n", full);
        rc = 1;
    } else {
        fwrite(ppm->arr, 1, ppm->len, f);
        fclose(f);
    }
    ppm_free(ppm);
    free(full);
    return rc;
}

int
write_png(Canvas c, const char *file_name)
{
    /* 48-bit RGB, sRGB intent absolute, empty Title text, clamped linear -> sRGB
     * -> floor(x*65535) (reference canvas.c:376-510) */
    int code = 0;
    char *full = with_suffix(file_name, ".png");
    uint16_t *buffer = NULL;
    png_structp png = NULL;
    png_infop info = NULL;
    FILE *fp = fopen(full, "wb");
    if (fp == NULL) {
        code = 1;
        goto done;
    }
    png = png_create_write_struct(PNG_LIBPNG_VER_STRING, NULL, NULL, NULL);
    if (png == NULL) {
        code = 2;
        goto done;
    }
    info = png_create_info_struct(png);
    if (info == NULL) {
        code = 2;
        goto done;
    }
    if (setjmp(png_jmpbuf(png))) {
        code = 2;
        goto done;
    }
    png_init_io(png, fp);
    png_set_IHDR(png, info, (png_uint_32)c->width, (png_uint_32)c->height, 16, PNG_COLOR_TYPE_RGB,
                 PNG_INTERLACE_NONE, PNG_COMPRESSION_TYPE_BASE, PNG_FILTER_TYPE_BASE);
    png_set_sRGB(png, info, PNG_sRGB_INTENT_ABSOLUTE);
    png_text title;
    memset(&title, 0, sizeof(title));
    title.compression = PNG_TEXT_COMPRESSION_NONE;
    title.key = (png_charp) "Title";
    title.text = NULL;
    title.text_length = 0;
    png_set_text(png, info, &title, 1);
    png_write_info(png, info);

    size_t npx = c->width * c->height;
    buffer = (uint16_t *)malloc(npx * 3 * sizeof(uint16_t));
    unsigned char *out = (unsigned char *)buffer;
    for (size_t i = 0; i < npx; ++i) {
        Color t, s;
        memcpy(t, c->arr[i], sizeof(Color));
        for (int k = 0; k < 3; ++k) {
            if (t[k] > 1.0) {
                t[k] = 1.0;
            } else if (t[k] < 0) {
                t[k] = 0.0;
            }
        }
        rgb_to_srgb(t, s);
        for (int k = 0; k < 3; ++k) {
            uint16_t q = quantize(s[k], 1.0, 65535.0);
            *out++ = (unsigned char)(q >> 8);
            *out++ = (unsigned char)(q & 0xFF);
        }
    }
    for (size_t row = 0; row < c->height; ++row) {
        png_write_row(png, (png_bytep)buffer + 3 * sizeof(uint16_t) * row * c->width);
    }
    png_write_end(png, NULL);

done:
    if (fp) fclose(fp);
    if (info) png_free_data(png, info, PNG_FREE_ALL, -1);
    if (png) png_destroy_write_struct(&png, &info);
    free(buffer);
    free(full);
    return code;
}

void
construct_canvas_from_ppm_file(Canvas *c, const char *file_path, bool super_sample, void (*color_space_fn)(const Color, Color))
{
    /* ASCII sample values after a "P6"-style header (reference canvas.c:330-365) */
    char magic[32];
    size_t w, h, maxv;
    FILE *f = fopen(file_path, "r");
    if (f == NULL) {
        printf("Error opening file %s", file_path);
        return;
    }
    if (fscanf(f, "%31s %zu %zu %zu", magic, &w, &h, &maxv) != 4) {
        fclose(f);
        return;
    }
    *c = canvas_alloc(w, h, super_sample, color_space_fn);
    for (size_t i = 0; i < w * h; ++i) {
        unsigned int v[3] = {0, 0, 0};
        for (int k = 0; k < 3; ++k) {
            if (fscanf(f, "%u", &v[k]) != 1) {
                v[k] = 0;
            }
            (*c)->arr[i][k] = (double)v[k] / (double)maxv;
        }
        (*c)->arr[i][3] = 0.0;
    }
    fclose(f);
}

int
read_png(Canvas *c, const char *filename, bool super_sample, void (*color_space_fn)(const Color, Color))
{
    int code = 0;
    png_structp png = NULL;
    png_infop info = NULL;
    png_bytep *rows = NULL;
    unsigned char *buffer = NULL;
    FILE *fp = fopen(filename, "rb");
    if (fp == NULL) {
        code = 1;
        goto done;
    }
    png = png_create_read_struct(PNG_LIBPNG_VER_STRING, NULL, NULL, NULL);
    if (png == NULL) {
        code = 2;
        goto done;
    }
    info = png_create_info_struct(png);
    if (info == NULL) {
        code = 2;
        goto done;
    }
    if (setjmp(png_jmpbuf(png))) {
        code = 2;
        goto done;
    }
    png_init_io(png, fp);
    png_read_info(png, info);
    png_byte color_type = png_get_color_type(png, info);
    png_byte depth = png_get_bit_depth(png, info);
    size_t w = png_get_image_width(png, info);
    size_t h = png_get_image_height(png, info);
    if (color_type == PNG_COLOR_TYPE_PALETTE) png_set_palette_to_rgb(png);
    if (color_type == PNG_COLOR_TYPE_GRAY && depth < 8) png_set_expand_gray_1_2_4_to_8(png);
    if (color_type == PNG_COLOR_TYPE_GRAY || color_type == PNG_COLOR_TYPE_GRAY_ALPHA) png_set_gray_to_rgb(png);
    if (color_type & PNG_COLOR_MASK_ALPHA) png_set_strip_alpha(png);
    png_read_update_info(png, info);

    size_t bytes_per_sample = depth == 16 ? 2 : 1;
    rows = (png_bytep *)malloc(h * sizeof(png_bytep));
    buffer = (unsigned char *)malloc(w * h * 3 * bytes_per_sample);
    for (size_t i = 0; i < h; ++i) {
        rows[i] = buffer + 3 * i * w * bytes_per_sample;
    }
    png_read_image(png, rows);

    *c = canvas_alloc(w, h, super_sample, color_space_fn);
    const unsigned char *p = buffer;
    for (size_t i = 0; i < w * h; ++i) {
        Color *o = (*c)->arr + i;
        (*o)[3] = 0.0;
        if (depth == 16) {
            for (int k = 0; k < 3; ++k) {
                uint16_t v = (uint16_t)(((p[2 * k] & 0xff) << 8) | (p[2 * k + 1] & 0xff));
                (*o)[k] = (double)v / 65535.0;
            }
            p += 6;
        } else {
            for (int k = 0; k < 3; ++k) {
                (*o)[k] = (double)p[k] / 255.0;
            }
            p += 3;
        }
    }

done:
    if (fp) fclose(fp);
    if (info) png_free_data(png, info, PNG_FREE_ALL, -1);
    if (png) png_destroy_read_struct(&png, &info, NULL);
    free(rows);
    free(buffer);
    return code;
}

/* Encode a raw rgba canvas (width*height*4 doubles) exactly as write_ppm_file
 * would; used by tests and bench.py to compare PPM bytes without touching the
 * file system. Returns the byte count, writes into out when it is large enough. */
size_t
frt_encode_ppm(const double *rgba, size_t width, size_t height, int use_scaling, unsigned char *out, size_t cap)
{
    struct canvas c;
    c.arr = (Color *)rgba;
    c.width = width;
    c.height = height;
    c.super_sample = false;
    c.color_space_fn = NULL;
    Ppm p = construct_ppm(&c, use_scaling != 0);
    size_t n = p->len;
    if (out != NULL && cap >= n) {
        memcpy(out, p->arr, n);
    }
    ppm_free(p);
    return n;
}
