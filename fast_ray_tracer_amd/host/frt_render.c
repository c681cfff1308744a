/*
 * frt-mi355x host: the drop-in render entry points.
 *
 * render_multi / render keep the reference's signature and ownership
 * contract (reference src/renderer/renderer.h:46-47, renderer.c:244-317): they
 * return a freshly allocated Canvas of hsize x vsize Colors that the caller
 * writes and frees. Instead of a pthread pool over deep world copies, the
 * scene is flattened once (frt_flatten.c) and rendered on an MI355X through
 * the device C ABI (include/frt_device.h). There is no CPU fallback: if the
 * device path cannot run, render_multi logs the reason and returns a zeroed
 * canvas (the reference has no error return).
 *
 * Environment knobs (main.c stays unchanged):
 *   FRT_DEVICES=<i,j,..>   devices to split the rows over (default: every visible GPU, or the
 *                          launcher's LOCAL_RANK alone; precedence below, render_devices)
 *   FRT_GPUS=<n>           devices 0..n-1;  FRT_DEVICE=<n>: that one device
 *   FRT_SEED=<u64>         counter-RNG seed for multi-row area-light caches
 *   FRT_STATS_OUT=<file>   write a JSON line of frame statistics
 *
 * The frt_capture_* functions let a harness compile an unmodified generated
 * main.c with -Drender_multi=frt_capture_render_multi to obtain the built
 * Camera / World without rendering (used by the Python bindings, tests and
 * bench.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "frt_device.h"
#include "frt_flatten.h"
#include "src/renderer/renderer.h"

static char g_host_error[512];
/* the last render_multi's failure ("" after a successful one): the canvas alone cannot say, a scene
 * may render black */
static char g_render_error[512];

const char *
frt_host_last_error(void)
{
    return g_host_error;
}

const char *
frt_render_multi_error(void)
{
    return g_render_error;
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

/* flatten + check: the device-independent half of frt_host_prepare */
static int
host_flatten(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter, frt_scene *fs)
{
    g_host_error[0] = '\0';
    if (w == NULL || cam == NULL || w->global_config == NULL) {
        snprintf(g_host_error, sizeof(g_host_error), "null camera / world / global_config");
        return -1;
    }
    if (unsupported_config(w, cam, g_host_error, sizeof(g_host_error))) {
        return -1;
    }
    if (frt_flatten_scene(cam, w, usteps, vsteps, jitter, fs, g_host_error, sizeof(g_host_error))) {
        return -1;
    }
    return 0;
}

frt_scene_handle *
frt_host_prepare(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter, int device)
{
    frt_scene fs;
    if (host_flatten(cam, w, usteps, vsteps, jitter, &fs)) {
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
write_stats(const char *path, const frt_frame_stats *st, Camera cam, size_t usteps, size_t vsteps, int ndev)
{
    FILE *f = fopen(path, "w");
    if (f == NULL) {
        return;
    }
    fprintf(f,
            "{\"width\": %zu, \"height\": %zu, \"usteps\": %zu, \"vsteps\": %zu, \"devices\": %d, \"render_ms\": %.6f, "
            "\"primary_rays\": %llu, \"secondary_rays\": %llu, \"shadow_rays\": %llu, "
            "\"pruned_secondary\": %llu, \"errors\": %llu}\n",
            cam->hsize, cam->vsize, usteps, vsteps, ndev, st->render_ms, (unsigned long long)st->primary_rays,
            (unsigned long long)st->secondary_rays, (unsigned long long)st->shadow_rays,
            (unsigned long long)st->pruned_secondary, (unsigned long long)st->errors);
    fclose(f);
}

/*
 * Devices render_multi uses: the first of these that is set decides (the later ones are ignored)
 *   FRT_DEVICES=<i,j,...>  explicit list (a device may repeat: several handles on one GPU)
 *   FRT_GPUS=<n>           devices 0 .. n-1
 *   FRT_DEVICE=<n>         that one device
 *   LOCAL_RANK=<r>         (set by torchrun-style launchers: one process per GPU) device r mod visible
 *                          alone, so processes sharing a node do not all take every GPU
 *   otherwise              every visible device (the reference's pool is sized by
 *                          threading.num_threads; here the unit of parallelism is a GPU)
 */
#define FRT_MAX_RENDER_DEVICES 64

static int
render_devices(int *dev, int cap, char *err, size_t errlen)
{
    const int visible = frt_device_count();
    int n = 0;
    const char *list = getenv("FRT_DEVICES");
    const char *count = getenv("FRT_GPUS");
    const char *one = getenv("FRT_DEVICE");
    if (list != NULL && *list) {
        const char *q = list;
        while (*q && n < cap) {
            char *end = NULL;
            long v = strtol(q, &end, 10);
            if (end == q) {
                break;
            }
            dev[n++] = (int)v;
            q = (*end == ',') ? end + 1 : end;
        }
    } else if (count != NULL && *count) {
        int k = atoi(count);
        for (int i = 0; i < k && n < cap; ++i) {
            dev[n++] = i;
        }
    } else if (one != NULL && *one) {
        dev[n++] = atoi(one);
    } else if (getenv("LOCAL_RANK") != NULL && *getenv("LOCAL_RANK") && visible > 0) {
        dev[n++] = atoi(getenv("LOCAL_RANK")) % visible;
    } else {
        for (int i = 0; i < visible && n < cap; ++i) {
            dev[n++] = i;
        }
    }
    if (visible <= 0) {
        snprintf(err, errlen, "no HIP device visible (the GPU path has no CPU fallback)");
        return -1;
    }
    if (n == 0) {
        snprintf(err, errlen, "no render device selected (FRT_DEVICES / FRT_GPUS)");
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        if (dev[i] < 0 || dev[i] >= visible) {
            snprintf(err, errlen, "render device %d out of range (%d visible)", dev[i], visible);
            return -1;
        }
    }
    return n;
}

static double
now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return 1e3 * (double)ts.tv_sec + 1e-6 * (double)ts.tv_nsec;
}

/* one device's share of the frame: upload, render rows k, k+N, k+2N, ..., release */
typedef struct {
    const frt_scene *fs;
    frt_scene_handle *h;      /* in: a kept handle of the same scene and device (NULL: upload); out: the handle */
    int keep;                 /* keep the handle for the next render_multi instead of releasing it */
    int device, k, n;
    int64_t height, width;
    uint64_t seed;
    double *rows;             /* rows_of(k) x width x 4 */
    int want_stats;
    frt_frame_stats st;
    int rc;
    char err[512];
    double upload_ms, upload_phases[8], render_ms, release_ms;
} device_job;

static void *
device_worker(void *arg)
{
    device_job *j = (device_job *)arg;
    frt_scene_handle *h = j->h;
    const double t0 = now_ms();
    if (h == NULL) {
        j->rc = frt_scene_upload(j->fs, j->device, &h);
        j->upload_ms = now_ms() - t0;
        frt_upload_phases(j->upload_phases, 8);
        if (j->rc) {
            snprintf(j->err, sizeof(j->err), "device %d: upload: %s", j->device, frt_last_error());
            return NULL;
        }
    }
    const double t1 = now_ms();
    frt_frame_params p;
    memset(&p, 0, sizeof(p));
    p.row_begin = j->k;
    p.row_end = j->height;
    p.row_stride = j->n;
    p.seed = j->seed;
    j->rc = frt_render_rows(h, &p, j->rows, j->want_stats ? &j->st : NULL);
    j->render_ms = now_ms() - t1;
    if (j->rc) {
        snprintf(j->err, sizeof(j->err), "device %d: render: %s", j->device, frt_last_error());
    }
    const double t2 = now_ms();
    if (j->keep) {
        j->h = h;  /* (render_multi keeps it, or releases it once when the call fails) */
    } else {
        frt_scene_release(h);
        j->h = NULL;
    }
    j->release_ms = now_ms() - t2;
    return NULL;
}

/*
 * The handles of the last render_multi stay alive (FRT_RM_KEEP=0: released at once, as before): a later call
 * with the same flattened scene on the same devices renders on them without uploading the scene, compiling or
 * loading its kernels or allocating the level state again, and the one call a generated main() makes does not
 * wait for the release (the process's exit frees the device memory, as it frees the reference's per-thread
 * world copies). A call with another scene or device list releases them first.
 */
static struct {
    int n;
    int dev[64];
    frt_scene_handle *h[64];
    frt_scene fs;  /* the flattened scene they were uploaded from (owned) */
    char *knobs;   /* the FRT_* environment at their upload (knob_signature; owned) */
} g_kept;

/* render_multi's process-wide state (g_kept, g_warmed, g_rm_phases, g_render_error) is used under this lock: two
 * threads calling render_multi at once render one after the other instead of racing on the kept handles */
static pthread_mutex_t g_rm_lock = PTHREAD_MUTEX_INITIALIZER;

extern char **environ;

/*
 * The FRT_* environment, sorted, as one string: the engine reads its knobs (FRT_JIT, FRT_JIT_BEAM, FRT_MESH,
 * FRT_SHADE_SORT, FRT_JIT_NODE_BEAM, FRT_EYE_CAM, the stage sizes, ...) when a scene is uploaded, so kept handles
 * are reused only under the same knobs. The per-call variables (the device list, seed, stats path, this switch)
 * are left out. Returns a malloc'd string (NULL when out of memory: then nothing is reused).
 */
static int
cmp_str(const void *a, const void *b)
{
    return strcmp(*(const char *const *)a, *(const char *const *)b);
}

static char *
knob_signature(void)
{
    static const char *const per_call[] = {"FRT_DEVICES=", "FRT_GPUS=", "FRT_DEVICE=", "FRT_SEED=", "FRT_STATS_OUT=",
                                           "FRT_RM_KEEP="};
    size_t n = 0, len = 1;
    for (char **e = environ; e != NULL && *e != NULL; ++e) {
        n += strncmp(*e, "FRT_", 4) == 0;
    }
    const char **v = (const char **)malloc((n ? n : 1) * sizeof(char *));
    if (v == NULL) {
        return NULL;
    }
    size_t m = 0;
    for (char **e = environ; e != NULL && *e != NULL; ++e) {
        if (strncmp(*e, "FRT_", 4) != 0) {
            continue;
        }
        int skip = 0;
        for (size_t q = 0; q < sizeof(per_call) / sizeof(per_call[0]); ++q) {
            skip = skip || strncmp(*e, per_call[q], strlen(per_call[q])) == 0;
        }
        if (!skip && m < n) {
            v[m++] = *e;
            len += strlen(*e) + 1;
        }
    }
    qsort(v, m, sizeof(char *), cmp_str);
    char *out = (char *)malloc(len);
    if (out != NULL) {
        out[0] = '\0';
        for (size_t q = 0; q < m; ++q) {
            strcat(out, v[q]);
            strcat(out, "\n");
        }
    }
    free(v);
    return out;
}

static int
same_bytes(const void *a, const void *b, size_t n)
{
    return n == 0 || (a != NULL && b != NULL && memcmp(a, b, n) == 0);
}

/* the same flattened scene, byte for byte (padding included: a difference there only costs a fresh upload) */
static int
scenes_equal(const frt_scene *a, const frt_scene *b)
{
    if (a->num_nodes != b->num_nodes || a->num_roots != b->num_roots || a->num_xforms != b->num_xforms ||
        a->prim_len != b->prim_len || a->num_materials != b->num_materials || a->num_patterns != b->num_patterns ||
        a->num_textures != b->num_textures || a->texel_len != b->texel_len || a->num_lights != b->num_lights ||
        a->light_point_len != b->light_point_len || memcmp(&a->camera, &b->camera, sizeof(a->camera)) != 0 ||
        memcmp(&a->config, &b->config, sizeof(a->config)) != 0) {
        return 0;
    }
    const size_t nst = 2 * (size_t)a->camera.usteps * (size_t)a->camera.vsteps;
    return same_bytes(a->nodes, b->nodes, sizeof(frt_node) * (size_t)a->num_nodes) &&
           same_bytes(a->roots, b->roots, sizeof(int32_t) * (size_t)a->num_roots) &&
           same_bytes(a->xforms, b->xforms, sizeof(double) * 16 * (size_t)a->num_xforms) &&
           same_bytes(a->prim_data, b->prim_data, sizeof(double) * (size_t)a->prim_len) &&
           same_bytes(a->materials, b->materials, sizeof(frt_material) * (size_t)a->num_materials) &&
           same_bytes(a->patterns, b->patterns, sizeof(frt_pattern) * (size_t)a->num_patterns) &&
           same_bytes(a->textures, b->textures, sizeof(frt_texture) * (size_t)a->num_textures) &&
           same_bytes(a->texels, b->texels, sizeof(double) * (size_t)a->texel_len) &&
           same_bytes(a->lights, b->lights, sizeof(frt_light) * (size_t)a->num_lights) &&
           same_bytes(a->light_points, b->light_points, sizeof(double) * (size_t)a->light_point_len) &&
           same_bytes(a->sample_table, b->sample_table, sizeof(double) * nst);
}

static void
release_kept(void)
{
    for (int k = 0; k < g_kept.n; ++k) {
        if (g_kept.h[k] != NULL) {
            frt_scene_release(g_kept.h[k]);
        }
    }
    if (g_kept.n > 0) {
        frt_flat_scene_free(&g_kept.fs);
    }
    free(g_kept.knobs);
    g_kept.knobs = NULL;
    g_kept.n = 0;
}

/*
 * Release the handles render_multi keeps between calls (their device memory: the scene, the compiled kernels and
 * the level state; a GI scene's gather buffers are GBs). The next render_multi uploads afresh. Safe to call at any
 * time, also with nothing kept; the Python runtime calls it at exit and before it opens handles of its own.
 */
void
frt_render_multi_release(void)
{
    pthread_mutex_lock(&g_rm_lock);
    release_kept();
    pthread_mutex_unlock(&g_rm_lock);
    frt_canvas_pool_release();
}

/* the phases of the last render_multi on this process, in ms (frt_render_multi_phases) */
static double g_rm_phases[16];

/*
 * Diagnostics: the phases of the last render_multi, in ms: out[0] flatten, [1] upload (the slowest device),
 * [2..9] that device's frt_upload_phases, [10] render of its rows incl. the copy to host memory (the slowest
 * device), [11] placing the rows into the canvas, [12] release, [13] total, [14] the devices' runtime
 * initialisation (frt_device_warmup, on threads beside the flatten, once per device and process), [15] the wait
 * for it after the flatten. Writes min(n, 16); returns 16.
 */
int
frt_render_multi_phases(double *out, int n)
{
    for (int i = 0; i < n && i < 16; ++i) {
        out[i] = g_rm_phases[i];
    }
    return 16;
}

typedef struct {
    int device;
    double ms;
} warmup_job;

static int g_warmed[64];  /* devices frt_device_warmup ran on in this process (render_multi's thread only) */

static void *
warmup_worker(void *arg)
{
    warmup_job *j = (warmup_job *)arg;
    const double t0 = now_ms();
    frt_device_warmup(j->device);
    j->ms = now_ms() - t0;
    return NULL;
}


/*
 * The drop-in entry point (reference renderer.c:244-281). Rows are interleaved
 * over the selected devices (row r on device r mod N), each device rendering
 * from its own copy of the flattened scene on its own host thread and stream;
 * the rows are then placed into the caller's canvas — a placement, not a
 * reduction, so the canvas is bit-identical for any device count. The
 * reference has no error return: on failure this logs the reason to stderr
 * and returns the (zeroed) canvas, as SURVEY.md 8(b) asks of a replacement.
 */
static Canvas
render_multi_locked(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    const double rm0 = now_ms();
    memset(g_rm_phases, 0, sizeof(g_rm_phases));
    const size_t width = cam != NULL ? cam->hsize : 1, height = cam != NULL ? cam->vsize : 1;
    int dev[FRT_MAX_RENDER_DEVICES];
    char err[512];
    frt_scene fs;
    g_render_error[0] = '\0';
    const int n = render_devices(dev, FRT_MAX_RENDER_DEVICES, err, sizeof(err));
    /* (the canvas is zeroed only where a failure leaves it unwritten: a successful render writes every pixel; with
     * devices its array is page-locked, so one device's frame lands in it by DMA) */
    Canvas c = n > 0 ? frt_canvas_alloc_pinned(width, height, false, NULL) : canvas_alloc(width, height, false, NULL);
    if (n < 0) {
        fprintf(stderr, "frt: render_multi cannot run on the GPU: %s\n", err);
        snprintf(g_render_error, sizeof(g_render_error), "%s", err);
        memset(c->arr, 0, width * height * sizeof(Color));
        return c;
    }
    /* the devices' HIP contexts are created on threads of their own while this thread flattens the scene (a
     * process's first context costs more than the flatten; frt_device_warmup) */
    warmup_job wj[FRT_MAX_RENDER_DEVICES];
    pthread_t wt[FRT_MAX_RENDER_DEVICES];
    int nw = 0;
    for (int k = 0; k < n; ++k) {
        int seen = dev[k] < 64 && g_warmed[dev[k]];  /* (once per device and process) */
        for (int q = 0; q < nw; ++q) {
            seen = seen || wj[q].device == dev[k];
        }
        if (seen) {
            continue;
        }
        if (dev[k] < 64) {
            g_warmed[dev[k]] = 1;
        }
        wj[nw].device = dev[k];
        wj[nw].ms = 0.0;
        if (pthread_create(&wt[nw], NULL, warmup_worker, &wj[nw]) == 0) {
            ++nw;
        }
    }
    const double fl0 = now_ms();
    const int flat_rc = host_flatten(cam, w, usteps, vsteps, jitter, &fs);
    g_rm_phases[0] = now_ms() - fl0;
    const double wj0 = now_ms();
    for (int q = 0; q < nw; ++q) {
        pthread_join(wt[q], NULL);
        g_rm_phases[14] = wj[q].ms > g_rm_phases[14] ? wj[q].ms : g_rm_phases[14];
    }
    g_rm_phases[15] = now_ms() - wj0;
    if (flat_rc) {
        fprintf(stderr, "frt: render_multi cannot run on the GPU: %s\n", g_host_error);
        snprintf(g_render_error, sizeof(g_render_error), "%s", g_host_error);
        memset(c->arr, 0, width * height * sizeof(Color));
        return c;
    }
    const char *keep_env = getenv("FRT_RM_KEEP");
    const int keep = !(keep_env != NULL && atoi(keep_env) == 0) && n <= 64;
    int reuse = keep && g_kept.n == n;
    for (int k = 0; reuse && k < n; ++k) {
        reuse = g_kept.dev[k] == dev[k] && g_kept.h[k] != NULL;
    }
    char *knobs = knob_signature();
    reuse = reuse && knobs != NULL && g_kept.knobs != NULL && strcmp(knobs, g_kept.knobs) == 0 &&
            scenes_equal(&fs, &g_kept.fs);
    if (!reuse) {
        release_kept();
    }
    const char *seed_env = getenv("FRT_SEED");
    const uint64_t seed = seed_env ? strtoull(seed_env, NULL, 10) : 0x5eedULL;
    const char *stats_path = getenv("FRT_STATS_OUT");
    device_job *jobs = (device_job *)calloc((size_t)n, sizeof(device_job));
    pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    int failed = jobs == NULL || th == NULL;
    for (int k = 0; !failed && k < n; ++k) {
        device_job *j = &jobs[k];
        const int64_t nrows = ((int64_t)height - k + n - 1) / n;
        j->fs = &fs;
        j->h = reuse ? g_kept.h[k] : NULL;
        j->keep = keep;
        j->device = dev[k];
        j->k = k;
        j->n = n;
        j->height = (int64_t)height;
        j->width = (int64_t)width;
        j->seed = seed;
        j->want_stats = stats_path != NULL;
        /* one device renders every row in order: straight into the canvas (a Color is 4 doubles) */
        j->rows = n == 1 ? (double *)c->arr : (double *)malloc((size_t)(nrows > 0 ? nrows : 1) * width * 4 * sizeof(double));
        if (j->rows == NULL) {
            failed = 1;
            snprintf(err, sizeof(err), "out of host memory");
        }
    }
    int started = 0;
    if (!failed) {
        if (n == 1) {
            device_worker(&jobs[0]);  /* no extra thread for the common single-device case */
            started = 0;
        } else {
            for (; started < n; ++started) {
                if (pthread_create(&th[started], NULL, device_worker, &jobs[started])) {
                    break;
                }
            }
            for (int k = 0; k < started; ++k) {
                pthread_join(th[k], NULL);
            }
            if (started < n) {
                failed = 1;
                snprintf(err, sizeof(err), "pthread_create failed");
            }
        }
    }
    frt_frame_stats total;
    memset(&total, 0, sizeof(total));
    for (int k = 0; !failed && k < n; ++k) {
        if (jobs[k].rc) {
            failed = 1;
            snprintf(err, sizeof(err), "%s", jobs[k].err);
        }
    }
    if (!failed) {
        int slow = 0;
        for (int k = 0; k < n; ++k) {
            if (jobs[k].upload_ms > jobs[slow].upload_ms) {
                slow = k;
            }
            g_rm_phases[10] = jobs[k].render_ms > g_rm_phases[10] ? jobs[k].render_ms : g_rm_phases[10];
            g_rm_phases[12] = jobs[k].release_ms > g_rm_phases[12] ? jobs[k].release_ms : g_rm_phases[12];
        }
        g_rm_phases[1] = jobs[slow].upload_ms;
        memcpy(g_rm_phases + 2, jobs[slow].upload_phases, 8 * sizeof(double));
    }
    const double place0 = now_ms();
    if (!failed) {
        for (int k = 0; k < n; ++k) {
            const device_job *j = &jobs[k];
            int64_t i = 0;
            for (int64_t r = k; n > 1 && r < (int64_t)height; r += n, ++i) {
                memcpy(c->arr + (size_t)r * width, j->rows + (size_t)i * width * 4, width * sizeof(Color));
            }
            total.primary_rays += j->st.primary_rays;
            total.secondary_rays += j->st.secondary_rays;
            total.shadow_rays += j->st.shadow_rays;
            total.pruned_secondary += j->st.pruned_secondary;
            total.errors |= j->st.errors;
            if (j->st.render_ms > total.render_ms) {
                total.render_ms = j->st.render_ms;
            }
        }
        g_rm_phases[11] = now_ms() - place0;
        if (stats_path) {
            write_stats(stats_path, &total, cam, usteps, vsteps, n);
        }
    } else {
        fprintf(stderr, "frt: render_multi failed: %s\n", err);
        snprintf(g_render_error, sizeof(g_render_error), "%s", err[0] ? err : "failed");
        memset(c->arr, 0, width * height * sizeof(Color));
    }
    for (int k = 0; jobs != NULL && n > 1 && k < n; ++k) {
        free(jobs[k].rows);
    }
    int kept_all = keep && !failed && jobs != NULL;
    for (int k = 0; kept_all && k < n; ++k) {
        kept_all = jobs[k].h != NULL;
    }
    if (kept_all) {
        if (!reuse) {  /* (the new scene's handles and flattened scene) */
            g_kept.n = n;
            for (int k = 0; k < n; ++k) {
                g_kept.dev[k] = dev[k];
                g_kept.h[k] = jobs[k].h;
            }
            g_kept.fs = fs;
            memset(&fs, 0, sizeof(fs));
            g_kept.knobs = knobs;
            knobs = NULL;
        }
    } else if (reuse) {
        /* (a failed call keeps nothing. Reused: the jobs hold the kept handles or nothing (a job that was never
         * set up), so every kept handle is released once through g_kept, whatever the jobs got to) */
        release_kept();
    } else {
        for (int k = 0; jobs != NULL && k < n; ++k) {
            if (jobs[k].h != NULL) {
                frt_scene_release(jobs[k].h);
            }
        }
    }
    free(knobs);
    free(jobs);
    free(th);
    frt_flat_scene_free(&fs);
    g_rm_phases[13] = now_ms() - rm0;
    return c;
}

Canvas
render_multi(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter)
{
    pthread_mutex_lock(&g_rm_lock);
    Canvas c = render_multi_locked(cam, w, usteps, vsteps, jitter);
    pthread_mutex_unlock(&g_rm_lock);
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
double *frt_canvas_data(Canvas c) { return (double *)c->arr; }

/* test hook: set the captured world's direct-illumination path length, returning the old one */
int
frt_world_path_length(World w, int v)
{
    const int old = (int)w->global_config->illumination.di.path_length;
    w->global_config->illumination.di.path_length = (size_t)v;
    return old;
}
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
