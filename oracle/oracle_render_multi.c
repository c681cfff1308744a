/*
 * TEST INFRASTRUCTURE ONLY — a render_multi built on the CPU oracle, for
 * building a generated main.c as a CPU "port" executable
 * (-Drender_multi=frt_oracle_render_multi). Threads: FRT_ORACLE_THREADS, else
 * the scene's thread-count (the reference's pool size, renderer.c:249).
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "frt_oracle.h"

Canvas
frt_oracle_render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    const char *env = getenv("FRT_ORACLE_THREADS");
    int threads = env ? atoi(env) : (int)w->global_config->threading.num_threads;
    Canvas c = canvas_alloc(cam->hsize, cam->vsize, false, NULL);
    frt_oracle_stats st;
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    if (frt_oracle_render_rows(cam, w, usteps, vsteps, jitter, 0, cam->vsize, threads, (double *)c->arr, &st)) {
        fprintf(stderr, "frt oracle: render failed\n");
        exit(2);
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    const char *stats_path = getenv("FRT_ORACLE_STATS");
    if (stats_path) {
        FILE *f = fopen(stats_path, "w");
        if (f) {
            double secs = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
            fprintf(f, "{\"render_seconds\": %.9f, \"threads\": %d, \"primary_rays\": %llu, \"secondary_rays\": %llu, "
                       "\"shadow_rays\": %llu, \"zero_weight_secondary\": %llu}\n",
                    secs, threads, (unsigned long long)st.primary_rays, (unsigned long long)st.secondary_rays,
                    (unsigned long long)st.shadow_rays, (unsigned long long)st.zero_weight_secondary);
            fclose(f);
        }
    }
    return c;
}
