/*
 * frt_device.h — C ABI of the MI355X (gfx950) render engine.
 *
 * This is the thin boundary between the C11 host library (the drop-in
 * scene API under fast_ray_tracer_amd/host/src/...) and the hand-written HIP
 * kernels in fast_ray_tracer_amd/csrc. Plain structs, pointers and sizes only.
 *
 * What it replaces in the reference:
 *   frt_render_rows / frt_render_rows_device  -> the body of
 *       Canvas render_multi(Camera, World, size_t, size_t, bool)
 *       (reference src/renderer/renderer.h:47, renderer.c:244-281): the
 *       row-per-job pthread pool over per-thread deep world copies, and the
 *       per-sample recursion color_at -> intersect_world -> shade_hit
 *       (renderer.c:74-979, world.c:163-197).
 *   frt_scene                                 -> the pointer-linked object
 *       tree (struct shape, shapes.h:85-118), materials (material.h:196-220),
 *       patterns (pattern.h:119-142), lights (light.h:57-76), camera
 *       (camera.h:60-73) and config (config.h:56-62), flattened by
 *       fast_ray_tracer_amd/host/frt_flatten.c.
 *
 * How the reference's render_multi binds to it: see INTEGRATION.md.
 * All scene arithmetic is IEEE binary64, matching the reference.
 */
#ifndef FRT_DEVICE_H
#define FRT_DEVICE_H

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define FRT_ABI_VERSION 3u  /* 3: frt_frame_stats grew the beam-stage counters (round 4) */

/* node kinds: same numbering as the reference's enum shape_enum (shapes.h:16-27) */
enum frt_node_type {
    FRT_CONE = 0,
    FRT_CUBE = 1,
    FRT_CYLINDER = 2,
    FRT_PLANE = 3,
    FRT_SMOOTH_TRIANGLE = 4,
    FRT_SPHERE = 5,
    FRT_TOROID = 6,
    FRT_TRIANGLE = 7,
    FRT_CSG = 8,
    FRT_GROUP = 9
};

/*
 * One node of the object tree in depth-first pre-order (the reference's child
 * order, which its shadow-ray semantics depend on). A subtree occupies
 * [index, skip). For a CSG node the left operand starts at index+1 and the
 * right operand at right.
 */
typedef struct frt_node {
    int32_t type;      /* enum frt_node_type */
    int32_t skip;      /* first pre-order index after this subtree */
    int32_t parent;    /* parent node, -1 for a world shape */
    int32_t tparent;   /* nearest strict ancestor with a transform, -1 if none */
    int32_t xform;     /* index into frt_scene.xforms (16 doubles, the inverse), -1 = identity */
    int32_t material;  /* index into frt_scene.materials (leaves) */
    int32_t prim;      /* offset into frt_scene.prim_data (leaves), CSG: operation (enum csg_ops_enum) */
    int32_t right;     /* CSG: pre-order index of the right operand */
    double bbox[6];    /* groups and CSG: own-space bounds min xyz, max xyz */
} frt_node;

/* per-leaf parameters in prim_data (doubles), by type:
 *   cylinder / cone : minimum, maximum, closed
 *   toroid          : r1, r2
 *   triangle        : p1[3] e1[3] e2[3] normal[3] t1[2] t2[2] t3[2] use_textures
 *   smooth triangle : p1[3] e1[3] e2[3] n1[3] n2[3] n3[3] t1[2] t2[2] t3[2] use_textures */
#define FRT_TRI_P1 0
#define FRT_TRI_E1 3
#define FRT_TRI_E2 6
#define FRT_TRI_N 9
#define FRT_TRI_N2 12
#define FRT_TRI_N3 15
#define FRT_TRI_UV_FLAT 12
#define FRT_TRI_UV_SMOOTH 18

typedef struct frt_material {
    double Ka[3], Kd[3], Ks[3], Tf[3], refl[3];
    double Ns, Ni, Tr;
    int32_t reflective;
    int32_t casts_shadow;
    /* pattern indices (frt_scene.patterns) or -1 */
    int32_t map_Ka, map_Kd, map_Ks, map_Ns, map_d, map_bump, map_refl;
    int32_t pad;
} frt_material;

/* pattern kinds: same numbering as the reference's enum pattern_type (pattern.h:23-41) */
typedef struct frt_pattern {
    int32_t type;
    int32_t transform_identity;
    int32_t uv_map;        /* texture map: enum uv_map_type */
    int32_t faces;         /* texture map: index of the first face pattern */
    int32_t child[3];      /* blended / nested / perturbed operands */
    int32_t texture;       /* uv texture: index into frt_scene.textures */
    int32_t width, height; /* uv checker */
    int32_t octaves, seed; /* perturbed */
    double inv[16];        /* inverse pattern transform */
    double color[5][3];    /* a,b (concrete / uv check); main,ul,ur,bl,br (align check) */
    double frequency, scale_factor, persistence;
} frt_pattern;

/* texture: texel (col,row) = canvas_pixel_at(canvas, col, row) pre-evaluated on the host
 * (color-space function and optional 3x3 super-sampling applied), 3 doubles per texel */
typedef struct frt_texture {
    int64_t offset; /* into frt_scene.texels, in doubles */
    int32_t width, height;
} frt_texture;

enum frt_light_type { FRT_AREA_LIGHT = 0, FRT_CIRCLE_LIGHT = 1, FRT_HEMISPHERE_LIGHT = 2, FRT_POINT_LIGHT = 3 };

typedef struct frt_light {
    int32_t type;
    int32_t num_samples; /* points per cache row */
    int32_t rows;        /* cache rows (reference cache_size), 1 for point lights */
    int32_t pad;
    int64_t points;      /* offset into frt_scene.light_points (3 doubles per point, row-major) */
    double intensity[3];
    /* photon emission (reference light.c:14-99, photon_tracer.c:195-233) */
    double normal[3];    /* emission hemisphere axis: area normalize(uvec x vvec), circle / hemisphere normal */
    double position[3];  /* point / hemisphere light position */
    int64_t num_photons; /* photons apportioned to this light by CIE L* (trace_photons) */
} frt_light;

typedef struct frt_camera {
    int64_t hsize, vsize, usteps, vsteps;
    double half_width, half_height, pixel_size, canvas_distance;
    double inv[16];          /* camera transform inverse */
    double aperture_size;
    int32_t aperture_type;   /* enum aperture_type (camera.h:9-19) */
    int32_t jitter;          /* jittered CMJ sub-pixel tables */
    double aperture_args[4];
} frt_camera;

typedef struct frt_config {
    int32_t include_direct, include_ambient, include_diffuse, include_spec_highlight, include_specular;
    int32_t path_length;
    int32_t all_ni_one;      /* every material has Ni == 1.0: n1 = n2 = 1 without the container walk */
    int32_t pad;
    /* global illumination (reference renderer.c:52-71, photon_tracer.c, pm.c) */
    int32_t use_gi;                 /* include_global || debug_visualize_photon_map */
    int32_t visualize_photon_map;
    int32_t include_caustics;       /* gi.include_caustics */
    int32_t include_final_gather;   /* gi.include_final_gather */
    int32_t gi_usteps, gi_vsteps;   /* final-gather hemisphere grid */
    int32_t irradiance_num;         /* k of the k-nearest-photon estimate */
    int32_t gi_path_length;         /* photon bounces */
    int32_t trace_caustic_map;      /* trace_photons(populate_caustic_map, ...) */
    int32_t trace_global_map;       /* trace_photons(..., populate_global_map) */
    int64_t photon_count;           /* photons per map (gi.photon_count); 0: no maps */
    double irradiance_radius;
    double cone_filter_k;
} frt_config;

typedef struct frt_scene {
    uint32_t abi_version;
    int32_t num_nodes;
    const frt_node *nodes;
    int32_t num_roots;       /* world shapes (generated main() has one: the divided world group) */
    int32_t pad0;
    const int32_t *roots;    /* pre-order index of each world shape */
    int32_t num_xforms;
    int32_t pad1;
    const double *xforms;    /* 16 doubles per transform (the inverse matrix, row-major) */
    int64_t prim_len;
    const double *prim_data;
    int32_t num_materials;
    int32_t num_patterns;
    const frt_material *materials;
    const frt_pattern *patterns;
    int32_t num_textures;
    int32_t pad2;
    const frt_texture *textures;
    int64_t texel_len;       /* doubles */
    const double *texels;
    int32_t num_lights;
    int32_t pad3;
    const frt_light *lights;
    int64_t light_point_len; /* doubles */
    const double *light_points;
    frt_camera camera;
    const double *sample_table; /* usteps*vsteps*2: the non-jittered CMJ table (sampler.c:401-510) */
    frt_config config;
} frt_scene;

typedef struct frt_scene_handle frt_scene_handle;

typedef struct frt_frame_params {
    int64_t row_begin, row_end; /* rows of the frame to render */
    int64_t row_stride;         /* render rows row_begin, row_begin+stride, ... (1 = contiguous) */
    uint64_t seed;              /* counter-RNG seed for stochastic rows (area-light cache rows, jitter) */
    int64_t batch_samples;      /* camera samples per wavefront batch (0 = engine default) */
    int32_t count_reference_rays; /* 1: also count the rays the reference would cast (slower) */
    int32_t pad;
} frt_frame_params;

typedef struct frt_frame_stats {
    uint64_t primary_rays;
    uint64_t secondary_rays;      /* reflection / refraction rays actually traced */
    uint64_t shadow_rays;         /* shadow rays actually traced */
    uint64_t pruned_secondary;    /* zero-weight secondary rays not traced */
    uint64_t hits;                /* path nodes shaded */
    uint64_t errors;              /* capacity / depth overflows (non-zero = result invalid) */
    double render_ms;             /* wall time of the device work (events) */
    double kernel_ms[8];          /* per-kernel accumulated time: trace, shadow, shade, combine, resolve, trace (level 0), prepare, gi */
    uint64_t kernel_launches[8];
    double shadow_kernel_bytes;   /* algorithmic bytes moved by the shadow kernel (DESIGN.md byte model) */
    uint64_t gather_rays;         /* final-gather rays traced (global illumination) */
    uint64_t photons[2];          /* photons in the caustic / global map used by this frame */
    double photon_ms;             /* photon tracing + map build of this frame (0 when the maps were reused) */
    int32_t shadow_jit;           /* 1: the scene-specialised shadow kernel ran (frt_jit.hip), 0: the generic walk */
    int32_t photon_pass;          /* 1: this frame traced its photon maps (a new seed), 0: maps reused / no GI */
    /* kernels inside the slots above (HIP events around each launch on the engine stream):
       0 frt_jit_beam / frt_jit_beam_list (node pair kernel), 1 frt_jit_shadow (per-ray kernel), 2 k_gather_est,
       3 k_gather_hit, 4 frt_jit_tile (tile pair kernel), 5 frt_jit_sub (sub-part pair kernel), 6 frt_jit_subtile
       (sub-tile pair kernel), 7 k_shade_lit (the shading of the path nodes some light reaches), 8 k_lit_scan +
       k_lit_scatter (the lit list in light-row order, multi-row lights); 9-15 unused */
    double sub_ms[16];
    uint64_t sub_launches[16];
    uint64_t shadow_rays_walked;  /* shadow rays walked one by one; the rest of shadow_rays were resolved
                                     (exactly, for every ray) per (node, light part) by frt_jit_beam */
    /* the scene-specialised pair kernels' work this frame (0 without them) */
    uint64_t shadow_tile_pairs;   /* (tile of consecutive path nodes, light part) beams frt_jit_tile tested */
    uint64_t shadow_tile_mixed;   /* of those, the ones it could not decide (their nodes go to frt_jit_beam_list) */
    uint64_t shadow_pairs;        /* (path node, light part) beams tested by frt_jit_beam / frt_jit_beam_list */
    uint64_t shadow_pairs_mixed;  /* of those, the ones left mixed */
    uint64_t shadow_sub_pairs;    /* (tile, light sub-part) beams of the mixed tile pairs tested by frt_jit_sub */
    uint64_t shadow_sub_mixed;    /* of those, the ones left mixed */
    uint64_t shadow_subtile_pairs; /* (sub-tile, light sub-part) beams of those tested by frt_jit_subtile */
    uint64_t shadow_subtile_mixed; /* of those, the ones whose nodes frt_jit_beam_list tested */
    uint64_t lit_nodes;           /* path nodes some light sample reaches (k_shade_lit's lanes); counted per frame
                                     when stats are asked for */
} frt_frame_stats;

/* number of HIP devices visible (0 when no GPU) */
int frt_device_count(void);

/* create the HIP runtime's context on `device` ahead of use (render_multi runs it on a thread of its own per device
 * while it flattens the scene); returns 0, or -1 when the device cannot be set */
int frt_device_warmup(int device);

/* page-locked host memory (hipHostMalloc) for render_multi's canvas array, which the device then writes by DMA
 * instead of through the runtime's staging copies into pageable memory (the reference's canvas_alloc mallocs it,
 * src/libs/canvas/canvas.c:21-24; canvas_free hands it back, canvas.c:54); NULL when it cannot be allocated.
 * frt_host_pinned_free releases it (NULL: nothing) */
void *frt_host_pinned_alloc(size_t bytes);
void frt_host_pinned_free(void *p);

/* sizeof(frt_frame_stats) as this library was built: a caller's mirror of the struct (runtime.py FrameStats)
 * checks its size against it before passing one in (no device needed) */
size_t frt_frame_stats_size(void);

/* message of the last failing call on this thread */
const char *frt_last_error(void);

/* copy a flattened scene into HBM on `device`; the host scene may be freed afterwards */
int frt_scene_upload(const frt_scene *scene, int device, frt_scene_handle **out);

/* render rows into a host buffer (rows x hsize x 4 doubles, rows in the order rendered) */
int frt_render_rows(frt_scene_handle *h, const frt_frame_params *params, double *host_rgba,
                    frt_frame_stats *stats);

/* same, writing into device memory on the handle's device (e.g. a torch tensor's storage) */
int frt_render_rows_device(frt_scene_handle *h, const frt_frame_params *params, double *device_rgba,
                           frt_frame_stats *stats);

void frt_scene_release(frt_scene_handle *h);

/* Diagnostics (no device needed): generate the scene-specialised shadow kernel of a flattened
 * scene and compile it for gfx950 with hiprtc, as frt_scene_upload does. Returns 0 compiled,
 * 1 scene not eligible (the generic walk runs), -1 compile error. `log` receives the reason or
 * the compiler log, `src` (may be NULL) the generated HIP source. */
int frt_jit_check(const frt_scene *scene, char *log, size_t log_cap, char *src, size_t src_cap);

/* Diagnostics (no device needed): the meshes frt_scene_upload would search per lane (group subtrees of
 * groups and triangles only, scenes over 512 nodes) and their BVHs, checked: every triangle of a mesh
 * in exactly one leaf, every box containing its triangles' vertices and its children's boxes, every
 * child's smallest pre-order index right. out[0] meshes, out[1] their triangles, out[2] BVH nodes,
 * out[3] deepest level (min(n, 4) written). Returns 0 when sound, else the number of violations. */
int frt_mesh_check(const frt_scene *scene, int64_t *out, int n);

/* Diagnostics (current device): the engine's binary64 sqrt / reciprocal core sequences and normalize
 * (frt_math.hpp) against the compiler's sqrt and division (bit for bit), and the shading's Newton-refined
 * estimates against their 2^-46 relative bound, on n lanes of random vectors; returns the number of
 * failed checks (0: all hold), or -1 on a HIP error. */
int64_t frt_math_selftest(int64_t n, uint64_t seed);

/* Counters of the scene-specialised kernels' code-object cache since the library was loaded (no device
 * needed): out[0] hiprtc compiles, out[1] code objects read from the on-disk cache, out[2] code objects
 * written to it, out[3] modules loaded (one per device and scene source), out[4] uploads that found
 * their device's module loaded already. A scene's kernels are compiled once per process (every device
 * and handle shares the code object) and, through the on-disk cache (FRT_JIT_CACHE_DIR, default
 * $XDG_CACHE_HOME/frt_jit or ~/.cache/frt_jit; FRT_JIT_CACHE=0 turns it off), once per machine.
 * Writes min(n, 5) counters; returns 5. */
int frt_jit_cache_stats(int64_t *out, int n);

/* Diagnostics: the phases of this thread's last frt_scene_upload, in ms: out[0] device selection (the
 * process's first HIP call initialises the runtime here), [1] scene buffers to HBM, [2] walk records and
 * mesh BVHs, [3] the scene-specialised kernels' source, [4] their code object (0 when this process had it;
 * an on-disk cache read or a hiprtc compile otherwise), [5] its load into the device's module, [6] the
 * rest (light tables, work buffers, stream), [7] total. Writes min(n, 8); returns 8. */
int frt_upload_phases(double *out, int n);

/* Counters of the photon passes since the library was loaded: out[0] photon passes traced, out[1] passes a
 * handle took from another device's trace of the same scene and seed (render_multi over N devices traces
 * and balances once per process). Writes min(n, 2); returns 2. */
int frt_photon_pass_stats(int64_t *out, int n);

/* Photon map entry points (parity tests; no scene needed).
 * frt_pm_balance replaces pm_balance (reference src/libs/photon_map/pm.c:329-494): the balanced
 * kd-tree of n photons given in the reference's storage order (pos: 3 doubles each); heap_of[i] = the
 * heap index (1..n) of photon i, plane[h] (n + 1 entries) = the split axis of heap node h. Host only.
 * frt_pm_estimate replaces pm_irradiance_estimate (pm.c:91-156, with pm_locate_photons pm.c:163-252)
 * over one map balanced as above: nq queries (pos[3], normal[3] each) on `device`; irrad receives 3
 * doubles per query (before lighting_gi's scaling), found the photons used. pos / power: 3 doubles per
 * photon in storage order, power already scaled (pm_scale_photon_power); theta_phi: the photon's stored
 * direction bytes (Photon.theta, Photon.phi, pm.c:288-300; decoded as pm_photon_dir does). */
int frt_pm_balance(const double *pos, int64_t n, int32_t *heap_of, int8_t *plane);
int frt_pm_estimate(int device, const double *pos, const double *power, const uint8_t *theta_phi, int64_t n,
                    const double *queries, int64_t nq, double radius, int32_t k, double cone_k,
                    double *irrad, int64_t *found);

#ifdef __cplusplus
}
#endif

#endif
