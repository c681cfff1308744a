/*
 * frt-mi355x host API: render entry points.
 *
 * render_multi() is the drop-in boundary (reference src/renderer/renderer.h:46-47,
 * called by generated main() at yaml_parser/yaml_parser.py:218). It flattens
 * the scene and renders on MI355X through the device C-ABI declared in
 * include/frt_device.h; there is no CPU fallback.
 */
#ifndef FRT_RENDERER_H
#define FRT_RENDERER_H

#include <stdbool.h>
#include <stdlib.h>

#include "../libs/linalg/linalg.h"
#include "../libs/canvas/canvas.h"
#include "../color/color.h"
#include "../light/light.h"
#include "../shapes/shapes.h"
#include "../intersection/intersection.h"
#include "world.h"
#include "camera.h"
#include "ray.h"

Canvas render(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter);
Canvas render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter);

/* frt extensions (no reference counterpart; main.c does not call them): the reason the last render_multi
 * failed ("" after a successful call), and the release of the device handles render_multi keeps between calls
 * for a repeat of the same scene (host/frt_render.c) */
const char *frt_render_multi_error(void);
void frt_render_multi_release(void);

#endif
