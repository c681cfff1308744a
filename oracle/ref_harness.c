/*
 * TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/bin/* (the reference
 * build), never into the product. The scene's main.c is compiled with
 * -Drender_multi=frt_ref_render_multi; this wrapper calls the reference's own
 * render_multi (reference src/renderer/renderer.c:244), times it, and dumps
 * the raw canvas (width*height*4 doubles, row-major, row 0 = top).
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <time.h>

#include "src/renderer/renderer.h"

#include "src/renderer/photon_tracer.h"
#include "src/libs/photon_map/pm.h"

static int g_traced_photons = 0;

/* ---- photon-map fixtures (FRT_REF_PM_DUMP=<prefix>) ----
 * The build links with -Wl,--wrap=pm_balance, so trace_photons' pm_balance calls (reference
 * photon_tracer.c:254-256, pm.c:329) come here: map m's photons are written before balancing
 * (<prefix>_<m>_stored.bin: the stored order) and after (<prefix>_<m>_kd.bin: the balanced kd-tree,
 * heap index 1..n). Record per photon: pos[3], power[3] (doubles), theta, phi, plane (int32 each).
 * FRT_REF_PM_QUERIES=<file> (int32 count, then per query: int32 map, double pos[3], double normal[3])
 * and FRT_REF_PM_OUT=<file>: after trace_photons, pm_irradiance_estimate (pm.c:91) of every query with
 * the scene's radius / photon count / cone-filter k; per query: double irrad[3], int64 found. */
void __real_pm_balance(PhotonMap *pm);
static int g_balance_calls = 0;

static void
dump_photons(const PhotonMap *pm, const char *prefix, int m, const char *what)
{
    char path[1024];
    snprintf(path, sizeof(path), "%s_%d_%s.bin", prefix, m, what);
    FILE *f = fopen(path, "wb");
    if (f == NULL)
        return;
    long n = pm->stored_photons;
    fwrite(&n, sizeof(n), 1, f);
    for (long i = 1; i <= n; ++i) {
        const Photon *p = pm->photons + i;
        int32_t b[3] = {p->theta, p->phi, p->plane};
        fwrite(p->pos, sizeof(double), 3, f);
        fwrite(p->power, sizeof(double), 3, f);
        fwrite(b, sizeof(int32_t), 3, f);
    }
    fclose(f);
}

void
__wrap_pm_balance(PhotonMap *pm)
{
    const char *prefix = getenv("FRT_REF_PM_DUMP");
    const int m = g_balance_calls++;
    if (prefix != NULL)
        dump_photons(pm, prefix, m, "stored");
    __real_pm_balance(pm);
    if (prefix != NULL)
        dump_photons(pm, prefix, m, "kd");
}

static void
run_queries(const World w)
{
    const char *qpath = getenv("FRT_REF_PM_QUERIES"), *opath = getenv("FRT_REF_PM_OUT");
    if (qpath == NULL || opath == NULL)
        return;
    FILE *q = fopen(qpath, "rb"), *o = fopen(opath, "wb");
    if (q == NULL || o == NULL)
        return;
    int32_t n = 0;
    if (fread(&n, sizeof(n), 1, q) != 1)
        n = 0;
    const double radius = w->global_config->illumination.gi.irradiance_estimate_radius;
    const int num = (int)w->global_config->illumination.gi.irradiance_estimate_num;
    const double cone = w->global_config->illumination.gi.irradiance_estimate_cone_filter_k;
    for (int32_t i = 0; i < n; ++i) {
        int32_t m;
        double pos[3], nrm[3], irrad[3];
        if (fread(&m, sizeof(m), 1, q) != 1 || fread(pos, sizeof(double), 3, q) != 3 || fread(nrm, sizeof(double), 3, q) != 3)
            break;
        int64_t found = pm_irradiance_estimate(w->photon_maps + m, irrad, pos, nrm, radius, num, cone);
        fwrite(irrad, sizeof(double), 3, o);
        fwrite(&found, sizeof(found), 1, o);
    }
    fclose(q);
    fclose(o);
}

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
    run_queries(w);
}

Canvas
frt_ref_render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    /* statistical goldens: a second, independent reference run re-seeds drand48
     * (pixel jitter, aperture samples) after the scene is built; after a photon
     * pass with a salted seed, so the render does not replay the photon stream */
    reseed_from_env(g_traced_photons ? 0x5bd1e995ULL : 0);
    /* FRT_REF_THREADS: the pool size of the reference's render_multi (renderer.c:244-281 sizes its pthread
     * pool by threading.num_threads), e.g. the CPU share of the machine it is timed on */
    const char *thr = getenv("FRT_REF_THREADS");
    if (thr != NULL && atoi(thr) > 0)
        w->global_config->threading.num_threads = (size_t)atoi(thr);
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
