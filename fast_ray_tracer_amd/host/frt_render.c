/*
 * frt-mi355x host: the drop-in render entry points.
 *
 * render_multi / render keep the reference's signature and ownership
 * contract (reference src/renderer/renderer.h:46-47, renderer.c:244-317): they
 * return a freshly allocated Canvas of hsize x vsize Colors that the caller
 * writes and frees. Instead of a pthread pool over deep world copies, the
 * scene is flattened once (frt_flatten.c) and rendered on an MI355X through
 * the device C ABI (include/frt_device.h). There is no CPU fallback: if the
 * device path cannot run, the process stops with a message.
 *
 * Environment knobs (main.c stays unchanged):
 *   FRT_DEVICE=<n>         HIP device to render on (default 0)
 *   FRT_SEED=<u64>         counter-RNG seed for multi-row area-light caches
 *   FRT_STATS_OUT=<file>   write a JSON line of frame statistics
 *
 * The frt_capture_* functions let a harness compile an unmodified generated
 * main.c with -Drender_multi=frt_capture_render_multi to obtain the built
 * Camera / World without rendering (used by the Python bindings, tests and
 * bench.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "frt_device.h"
#include "frt_flatten.h"
#include "src/renderer/renderer.h"

static char g_host_error[512];

const char *
frt_host_last_error(void)
{
    return g_host_error;
}

static int
unsupported_config(World w, Camera cam, char *err, size_t n)
{
    const struct illumination_config *ic = &w->global_config->illumination;
    if ((ic->include_global || ic->debug_visualize_photon_map) &&
        (w->photon_maps == NULL || !w->frt_photons_requested || ic->gi.photon_count == 0)) {
        /* the reference dereferences the missing maps (renderer.c:874 -> pm.c:101) */
        snprintf(err, n, "global illumination requested without traced photon maps is not supported "
                         "(the reference would read a NULL photon map)");
        return 1;
    }
    (void)cam;
    return 0;
}

frt_scene_handle *
frt_host_prepare(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter, int device)
{
    g_host_error[0] = '\0';
    if (w == NULL || cam == NULL || w->global_config == NULL) {
        snprintf(g_host_error, sizeof(g_host_error), "null camera / world / global_config");
        return NULL;
    }
    if (unsupported_config(w, cam, g_host_error, sizeof(g_host_error))) {
        return NULL;
    }
    frt_scene fs;
    if (frt_flatten_scene(cam, w, usteps, vsteps, jitter, &fs, g_host_error, sizeof(g_host_error))) {
        return NULL;
    }
    frt_scene_handle *h = NULL;
    int rc = frt_scene_upload(&fs, device, &h);
    frt_flat_scene_free(&fs);
    if (rc) {
        snprintf(g_host_error, sizeof(g_host_error), "%s", frt_last_error());
        return NULL;
    }
    return h;
}

static void
write_stats(const char *path, const frt_frame_stats *st, Camera cam, size_t usteps, size_t vsteps)
{
    FILE *f = fopen(path, "w");
    if (f == NULL) {
        return;
    }
    fprintf(f,
            "{\"width\": %zu, \"height\": %zu, \"usteps\": %zu, \"vsteps\": %zu, \"render_ms\": %.6f, "
            "\"primary_rays\": %llu, \"secondary_rays\": %llu, \"shadow_rays\": %llu, "
            "\"pruned_secondary\": %llu, \"errors\": %llu}\n",
            cam->hsize, cam->vsize, usteps, vsteps, st->render_ms, (unsigned long long)st->primary_rays,
            (unsigned long long)st->secondary_rays, (unsigned long long)st->shadow_rays,
            (unsigned long long)st->pruned_secondary, (unsigned long long)st->errors);
    fclose(f);
}

Canvas
render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    const char *dev_env = getenv("FRT_DEVICE");
    int device = dev_env ? atoi(dev_env) : 0;
    frt_scene_handle *h = frt_host_prepare(cam, w, usteps, vsteps, jitter, device);
    if (h == NULL) {
        fprintf(stderr, "frt: render_multi cannot run on the GPU: %s\n", g_host_error);
        exit(2);
    }
    Canvas c = canvas_alloc(cam->hsize, cam->vsize, false, NULL);
    frt_frame_params p;
    memset(&p, 0, sizeof(p));
    p.row_begin = 0;
    p.row_end = (int64_t)cam->vsize;
    p.row_stride = 1;
    const char *seed_env = getenv("FRT_SEED");
    p.seed = seed_env ? strtoull(seed_env, NULL, 10) : 0x5eedULL;
    frt_frame_stats st;
    const char *stats_path = getenv("FRT_STATS_OUT");
    if (frt_render_rows(h, &p, (double *)c->arr, stats_path ? &st : NULL)) {
        fprintf(stderr, "frt: render failed: %s\n", frt_last_error());
        exit(3);
    }
    if (stats_path) {
        write_stats(stats_path, &st, cam, usteps, vsteps);
    }
    frt_scene_release(h);
    return c;
}

Canvas
render(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    /* the reference's single-threaded variant has the same contract (renderer.c:284-317) */
    return render_multi(cam, w, usteps, vsteps, jitter);
}

/* ---------------- capture hooks for harnesses ---------------- */

static struct {
    Camera cam;
    World w;
    size_t usteps, vsteps;
    bool jitter;
    int captured;
    unsigned short drand48_state[3];
} g_capture;

Canvas
frt_capture_render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    /* generated main() keeps global_config on its stack: keep a copy that outlives main() */
    if (w != NULL && w->global_config != NULL) {
        Global_config kept = (Global_config)malloc(sizeof(struct global_config));
        *kept = *w->global_config;
        w->global_config = kept;
    }
    g_capture.cam = cam;
    g_capture.w = w;
    g_capture.usteps = usteps;
    g_capture.vsteps = vsteps;
    g_capture.jitter = jitter;
    g_capture.captured = 1;
    {
        /* snapshot drand48's state at the render_multi call (the reference's
         * jitter / aperture draws start from here); seed48 returns the old state */
        unsigned short probe[3] = {0, 0, 0};
        unsigned short *old = seed48(probe);
        memcpy(g_capture.drand48_state, old, sizeof(g_capture.drand48_state));
        seed48(g_capture.drand48_state);
    }
    Canvas c = canvas_alloc(1, 1, false, NULL);
    memset(c->arr, 0, sizeof(Color));
    return c;
}

int
frt_capture_write_ppm(Canvas c, const bool use_scaling, const char *path)
{
    (void)c;
    (void)use_scaling;
    (void)path;
    return 0;
}

int
frt_capture_write_png(Canvas c, const char *path)
{
    (void)c;
    (void)path;
    return 0;
}

int frt_captured(void) { return g_capture.captured; }
Camera frt_captured_camera(void) { return g_capture.cam; }
World frt_captured_world(void) { return g_capture.w; }
size_t frt_captured_usteps(void) { return g_capture.usteps; }
size_t frt_captured_vsteps(void) { return g_capture.vsteps; }
int frt_captured_jitter(void) { return g_capture.jitter ? 1 : 0; }
void frt_captured_drand48(unsigned short out[3]) { memcpy(out, g_capture.drand48_state, sizeof(g_capture.drand48_state)); }
void frt_set_drand48(const unsigned short in[3]) { seed48((unsigned short *)in); }
size_t frt_camera_hsize(Camera c) { return c->hsize; }
size_t frt_camera_vsize(Camera c) { return c->vsize; }

/* Put glibc's drand48() / rand() streams back into their fresh-process state
 * (drand48 state 0 with the default multiplier, rand() seeded with 1), so a
 * scene built inside a long-lived process draws the same jittered light
 * caches as the reference's one-shot executable does. */
void
frt_reset_libc_rng(void)
{
    unsigned short zero[3] = {0, 0, 0};
    seed48(zero);
    srand(1);
}
