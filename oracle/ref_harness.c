/*
 * TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/bin/* (the reference
 * build), never into the product. The scene's main.c is compiled with
 * -Drender_multi=frt_ref_render_multi; this wrapper calls the reference's own
 * render_multi (reference src/renderer/renderer.c:244), times it, and dumps
 * the raw canvas (width*height*4 doubles, row-major, row 0 = top).
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "src/renderer/renderer.h"

#include "src/renderer/photon_tracer.h"

static int g_traced_photons = 0;

static void
reseed_from_env(unsigned long long salt)
{
    const char *seed_env = getenv("FRT_REF_DRAND_SEED");
    if (seed_env != NULL) {
        unsigned long long sd = strtoull(seed_env, NULL, 10) ^ salt;
        unsigned short s48[3] = {(unsigned short)(sd & 0xffff), (unsigned short)((sd >> 16) & 0xffff),
                                 (unsigned short)((sd >> 32) & 0xffff)};
        seed48(s48);
        srand((unsigned)(sd & 0x7fffffff));  /* area-light cache rows / photon emission points: rand() */
    }
}

/* main.c's trace_photons call (compiled with -Dtrace_photons=frt_ref_trace_photons):
 * independent statistical runs re-seed drand48 / rand() before the photons are
 * traced, so every run has its own photon maps (reference photon_tracer.c:203) */
void
frt_ref_trace_photons(const World w, size_t num_maps, bool populate_caustic_map, bool populate_global_map)
{
    reseed_from_env(0);
    g_traced_photons = 1;
    trace_photons(w, num_maps, populate_caustic_map, populate_global_map);
}

Canvas
frt_ref_render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    /* statistical goldens: a second, independent reference run re-seeds drand48
     * (pixel jitter, aperture samples) after the scene is built; after a photon
     * pass with a salted seed, so the render does not replay the photon stream */
    reseed_from_env(g_traced_photons ? 0x5bd1e995ULL : 0);
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    Canvas c = render_multi(cam, w, usteps, vsteps, jitter);
    clock_gettime(CLOCK_MONOTONIC, &b);
    double secs = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);

    const char *canvas_path = getenv("FRT_REF_CANVAS");
    if (canvas_path != NULL) {
        FILE *f = fopen(canvas_path, "wb");
        if (f != NULL) {
            fwrite(c->arr, sizeof(Color), c->width * c->height, f);
            fclose(f);
        }
    }
    const char *stats_path = getenv("FRT_REF_STATS");
    if (stats_path != NULL) {
        FILE *f = fopen(stats_path, "w");
        if (f != NULL) {
            fprintf(f, "{\"render_multi_seconds\": %.9f, \"width\": %zu, \"height\": %zu, "
                       "\"usteps\": %zu, \"vsteps\": %zu, \"threads\": %zu}\n",
                    secs, c->width, c->height, usteps, vsteps, w->global_config->threading.num_threads);
            fclose(f);
        }
    }
    return c;
}
