/*
 * frt-mi355x host API: pinhole / aperture camera.
 * Names follow reference src/renderer/camera.h:9-89 (the codegen writes
 * ap.u.circle.r1 etc. and reads cam->usteps / cam->aperture.jitter).
 */
#ifndef FRT_CAMERA_H
#define FRT_CAMERA_H

#include <stdbool.h>

#include "../libs/linalg/linalg.h"
#include "../libs/sampler/sampler.h"

enum aperture_type {
    CIRCULAR_APERTURE,
    CROSS_APERTURE,
    DIAMOND_APERTURE,
    DOUGHNUT_APERTURE,
    HEXAGONAL_APERTURE,
    PENTAGONAL_APERTURE,
    POINT_APERTURE,
    SQUARE_APERTURE,
    OCTAGONAL_APERTURE,
};

struct circle_aperture_args { double r1; };
struct cross_aperture_args { double x1, x2, y1, y2; };
struct diamond_aperture_args { double b1, b2, b3, b4; };
struct doughnut_aperture_args { double r1, r2; };

typedef struct aperture {
    enum aperture_type type;
    double size;
    bool jitter;
    struct sampler sampler;
    union {
        struct circle_aperture_args circle;
        struct cross_aperture_args cross;
        struct diamond_aperture_args diamond;
        struct doughnut_aperture_args doughnut;
    } u;
} *Aperture;

typedef struct camera {
    size_t hsize;
    size_t vsize;
    size_t usteps;
    size_t vsteps;
    double field_of_view;
    double canvas_distance;
    struct aperture aperture;
    double half_width;
    double half_height;
    double pixel_size;
    Matrix transform;
    Matrix transform_inverse;
} *Camera;

Camera camera(size_t hsize, size_t vsize, double field_of_view, double canvas_distance, size_t usteps, size_t vsteps, Aperture aperture, Matrix transform);
void view_transform(Point fr, Point to, Vector up, Matrix res);
void camera_set_transform(Camera c, Matrix m);
void aperture(enum aperture_type type, double size, size_t usteps, size_t vsteps, bool jitter, Aperture res);
/* aperture sample in [-0.5,0.5)^2 before scaling by size (reference camera.c:85-90) */
void sample_aperture(double xy[2], size_t u, size_t v, const Aperture aperture);

void circle_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct circle_aperture_args *args, Aperture res);
void cross_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct cross_aperture_args *args, Aperture res);
void diamond_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct diamond_aperture_args *args, Aperture res);
void doughnut_aperture(double size, size_t usteps, size_t vsteps, bool jitter, struct doughnut_aperture_args *args, Aperture res);
void square_aperture(double size, size_t usteps, size_t vsteps, bool jitter, Aperture res);
void point_aperture(Aperture res);

#endif
