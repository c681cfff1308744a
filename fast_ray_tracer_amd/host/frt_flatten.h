/*
 * frt-mi355x host: flattening of the pointer-linked scene graph into the
 * device layout declared in include/frt_device.h.
 */
#ifndef FRT_FLATTEN_H
#define FRT_FLATTEN_H

#include "frt_device.h"
#include "src/renderer/renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Build a host-memory frt_scene for (cam, w). Returns 0 on success; on failure
 * writes a message into err (size errlen). Free with frt_flat_scene_free. */
int frt_flatten_scene(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter,
                      frt_scene *out, char *err, size_t errlen);
void frt_flat_scene_free(frt_scene *s);

#ifdef __cplusplus
}
#endif

#endif
