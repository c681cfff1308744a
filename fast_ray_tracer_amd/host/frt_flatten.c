/*
 * frt-mi355x host: scene flattening for the GPU.
 *
 * Walks the world's object tree in the reference's child order and emits the
 * pre-order node array of include/frt_device.h: every group / CSG keeps its
 * own-space bounds (computed with the reference's lazily cached bounds,
 * shapes.c:193-224), every non-identity node its inverse transform, every
 * leaf its primitive parameters and a deduplicated material. Patterns are
 * flattened recursively (texture-map faces kept contiguous), textures are
 * pre-evaluated through canvas_pixel_at so the device reads exactly the
 * color the reference's per-fetch color-space call would produce
 * (canvas.c:115-148), and light caches are copied row by row.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "frt_flatten.h"
#include "src/libs/sampler/sampler.h"

typedef struct growbuf {
    void *data;
    size_t count, cap, elem;
} growbuf;

static void *
gb_push(growbuf *b, size_t n)
{
    if (b->count + n > b->cap) {
        size_t cap = b->cap ? b->cap : 64;
        while (cap < b->count + n) cap *= 2;
        b->data = realloc(b->data, cap * b->elem);
        b->cap = cap;
    }
    void *p = (char *)b->data + b->count * b->elem;
    memset(p, 0, n * b->elem);
    b->count += n;
    return p;
}

/* pointer -> index map (open addressing) */
typedef struct ptrmap {
    const void **keys;
    int32_t *vals;
    size_t cap, count;
} ptrmap;

static size_t
ptr_hash(const void *p)
{
    uintptr_t x = (uintptr_t)p;
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    return (size_t)x;
}

static void pm_put(ptrmap *m, const void *k, int32_t v);

static void
pm_grow(ptrmap *m)
{
    ptrmap n = {0};
    n.cap = m->cap ? 2 * m->cap : 256;
    n.keys = (const void **)calloc(n.cap, sizeof(void *));
    n.vals = (int32_t *)calloc(n.cap, sizeof(int32_t));
    for (size_t i = 0; i < m->cap; ++i) {
        if (m->keys[i]) pm_put(&n, m->keys[i], m->vals[i]);
    }
    free(m->keys);
    free(m->vals);
    *m = n;
}

static void
pm_put(ptrmap *m, const void *k, int32_t v)
{
    if (2 * (m->count + 1) > m->cap) pm_grow(m);
    size_t i = ptr_hash(k) & (m->cap - 1);
    while (m->keys[i] && m->keys[i] != k) i = (i + 1) & (m->cap - 1);
    if (!m->keys[i]) m->count++;
    m->keys[i] = k;
    m->vals[i] = v;
}

static int
pm_get(const ptrmap *m, const void *k, int32_t *v)
{
    if (m->cap == 0) return 0;
    size_t i = ptr_hash(k) & (m->cap - 1);
    while (m->keys[i]) {
        if (m->keys[i] == k) {
            *v = m->vals[i];
            return 1;
        }
        i = (i + 1) & (m->cap - 1);
    }
    return 0;
}

static void
pm_free(ptrmap *m)
{
    free(m->keys);
    free(m->vals);
}

typedef struct flat_ctx {
    growbuf nodes, xforms, prims, materials, patterns, textures, texels, roots;
    ptrmap mat_map, pat_map, tex_map;
    int all_ni_one;
    int depth_error;
    char *err;
    size_t errlen;
} flat_ctx;

static int32_t
add_xform(flat_ctx *c, const double *inv)
{
    double *x = (double *)gb_push(&c->xforms, 16);
    memcpy(x, inv, 16 * sizeof(double));
    return (int32_t)(c->xforms.count / 16 - 1);
}

static int32_t add_pattern(flat_ctx *c, Pattern p);

static int32_t
add_texture(flat_ctx *c, Canvas cv)
{
    int32_t idx;
    if (pm_get(&c->tex_map, cv, &idx)) return idx;
    frt_texture *t = (frt_texture *)gb_push(&c->textures, 1);
    idx = (int32_t)(c->textures.count - 1);
    t->width = (int32_t)cv->width;
    t->height = (int32_t)cv->height;
    t->offset = (int64_t)c->texels.count;
    double *tx = (double *)gb_push(&c->texels, 3 * cv->width * cv->height);
    for (size_t row = 0; row < cv->height; ++row) {
        for (size_t col = 0; col < cv->width; ++col) {
            Color px;
            canvas_pixel_at(cv, (int)col, (int)row, px);
            double *o = tx + 3 * (row * cv->width + col);
            o[0] = px[0];
            o[1] = px[1];
            o[2] = px[2];
        }
    }
    /* gb_push may have moved the texture array */
    pm_put(&c->tex_map, cv, idx);
    return idx;
}

static void
fill_pattern(flat_ctx *c, int32_t slot, Pattern p)
{
    frt_pattern fp;
    memset(&fp, 0, sizeof(fp));
    fp.type = (int32_t)p->type;
    fp.transform_identity = p->transform_identity ? 1 : 0;
    memcpy(fp.inv, p->transform_inverse, sizeof(fp.inv));
    fp.child[0] = fp.child[1] = fp.child[2] = -1;
    fp.faces = -1;
    fp.texture = -1;
    switch (p->type) {
    case CHECKER_PATTERN:
    case GRADIENT_PATTERN:
    case RADIAL_GRADIENT_PATTERN:
    case RING_PATTERN:
    case STRIPE_PATTERN:
    case UV_GRADIENT_PATTERN:
    case UV_RADIAL_GRADIENT_PATTERN:
        memcpy(fp.color[0], p->fields.concrete.a, 3 * sizeof(double));
        memcpy(fp.color[1], p->fields.concrete.b, 3 * sizeof(double));
        break;
    case UV_CHECKER_PATTERN:
        memcpy(fp.color[0], p->fields.uv_check.a, 3 * sizeof(double));
        memcpy(fp.color[1], p->fields.uv_check.b, 3 * sizeof(double));
        fp.width = (int32_t)p->fields.uv_check.width;
        fp.height = (int32_t)p->fields.uv_check.height;
        break;
    case UV_ALIGN_CHECKER_PATTERN:
        memcpy(fp.color[0], p->fields.uv_align_check.main, 3 * sizeof(double));
        memcpy(fp.color[1], p->fields.uv_align_check.ul, 3 * sizeof(double));
        memcpy(fp.color[2], p->fields.uv_align_check.ur, 3 * sizeof(double));
        memcpy(fp.color[3], p->fields.uv_align_check.bl, 3 * sizeof(double));
        memcpy(fp.color[4], p->fields.uv_align_check.br, 3 * sizeof(double));
        break;
    case UV_TEXTURE_PATTERN:
        fp.texture = add_texture(c, p->fields.uv_texture.canvas);
        break;
    case BLENDED_PATTERN:
        fp.child[0] = add_pattern(c, p->fields.blended.pattern1);
        fp.child[1] = add_pattern(c, p->fields.blended.pattern2);
        break;
    case NESTED_PATTERN:
        fp.child[0] = add_pattern(c, p->fields.nested.pattern1);
        fp.child[1] = add_pattern(c, p->fields.nested.pattern2);
        fp.child[2] = add_pattern(c, p->fields.nested.pattern3);
        break;
    case PERTURBED_PATTERN:
        fp.child[0] = add_pattern(c, p->fields.perturbed.pattern1);
        fp.frequency = p->fields.perturbed.frequency;
        fp.scale_factor = p->fields.perturbed.scale_factor;
        fp.persistence = p->fields.perturbed.persistence;
        fp.octaves = (int32_t)p->fields.perturbed.octaves;
        fp.seed = p->fields.perturbed.seed;
        break;
    case TEXTURE_MAP_PATTERN: {
        int nf = frt_uv_map_face_count(p->fields.uv_map.type);
        fp.uv_map = (int32_t)p->fields.uv_map.type;
        /* faces must be contiguous: reserve the block first, then fill it */
        size_t first = c->patterns.count;
        gb_push(&c->patterns, (size_t)nf);
        fp.faces = (int32_t)first;
        for (int k = 0; k < nf; ++k) {
            fill_pattern(c, (int32_t)first + k, p->fields.uv_map.uv_faces + k);
        }
        break;
    }
    default:
        break;
    }
    ((frt_pattern *)c->patterns.data)[slot] = fp;
}

static int32_t
add_pattern(flat_ctx *c, Pattern p)
{
    if (p == NULL) return -1;
    int32_t idx;
    if (pm_get(&c->pat_map, p, &idx)) return idx;
    gb_push(&c->patterns, 1);
    idx = (int32_t)(c->patterns.count - 1);
    pm_put(&c->pat_map, p, idx);
    fill_pattern(c, idx, p);
    return idx;
}

static int32_t
add_material(flat_ctx *c, Material m)
{
    int32_t idx;
    if (pm_get(&c->mat_map, m, &idx)) return idx;
    frt_material fm;
    memset(&fm, 0, sizeof(fm));
    memcpy(fm.Ka, m->Ka, 3 * sizeof(double));
    memcpy(fm.Kd, m->Kd, 3 * sizeof(double));
    memcpy(fm.Ks, m->Ks, 3 * sizeof(double));
    memcpy(fm.Tf, m->Tf, 3 * sizeof(double));
    memcpy(fm.refl, m->refl, 3 * sizeof(double));
    fm.Ns = m->Ns;
    fm.Ni = m->Ni;
    fm.Tr = m->Tr;
    fm.reflective = m->reflective ? 1 : 0;
    fm.casts_shadow = m->casts_shadow ? 1 : 0;
    if (m->Ni != 1.0) c->all_ni_one = 0;
    fm.map_Ka = add_pattern(c, m->map_Ka);
    fm.map_Kd = add_pattern(c, m->map_Kd);
    fm.map_Ks = add_pattern(c, m->map_Ks);
    fm.map_Ns = add_pattern(c, m->map_Ns);
    fm.map_d = add_pattern(c, m->map_d);
    fm.map_bump = add_pattern(c, m->map_bump);
    fm.map_refl = add_pattern(c, m->map_refl);
    frt_material *slot = (frt_material *)gb_push(&c->materials, 1);
    *slot = fm;
    idx = (int32_t)(c->materials.count - 1);
    pm_put(&c->mat_map, m, idx);
    return idx;
}

static void
add_prim(flat_ctx *c, Shape s, frt_node *nd)
{
    nd->prim = (int32_t)c->prims.count;
    switch (s->type) {
    case SHAPE_CYLINDER:
    case SHAPE_CONE: {
        double *p = (double *)gb_push(&c->prims, 3);
        p[0] = s->fields.cylinder.minimum;
        p[1] = s->fields.cylinder.maximum;
        p[2] = s->fields.cylinder.closed ? 1.0 : 0.0;
        break;
    }
    case SHAPE_TOROID: {
        double *p = (double *)gb_push(&c->prims, 2);
        p[0] = s->fields.toroid.r1;
        p[1] = s->fields.toroid.r2;
        break;
    }
    case SHAPE_TRIANGLE:
    case SHAPE_SMOOTH_TRIANGLE: {
        const struct triangle_fields *t = &s->fields.triangle;
        int smooth = s->type == SHAPE_SMOOTH_TRIANGLE;
        size_t uvo = smooth ? FRT_TRI_UV_SMOOTH : FRT_TRI_UV_FLAT;
        double *p = (double *)gb_push(&c->prims, uvo + 7);
        memcpy(p + FRT_TRI_P1, t->p1, 3 * sizeof(double));
        memcpy(p + FRT_TRI_E1, t->e1, 3 * sizeof(double));
        memcpy(p + FRT_TRI_E2, t->e2, 3 * sizeof(double));
        if (smooth) {
            memcpy(p + FRT_TRI_N, t->u_normals.s_normals.n1, 3 * sizeof(double));
            memcpy(p + FRT_TRI_N2, t->u_normals.s_normals.n2, 3 * sizeof(double));
            memcpy(p + FRT_TRI_N3, t->u_normals.s_normals.n3, 3 * sizeof(double));
        } else {
            memcpy(p + FRT_TRI_N, t->u_normals.normal, 3 * sizeof(double));
        }
        p[uvo + 0] = t->t1[0];
        p[uvo + 1] = t->t1[1];
        p[uvo + 2] = t->t2[0];
        p[uvo + 3] = t->t2[1];
        p[uvo + 4] = t->t3[0];
        p[uvo + 5] = t->t3[1];
        p[uvo + 6] = t->use_textures ? 1.0 : 0.0;
        break;
    }
    default:
        nd->prim = -1;
        break;
    }
}

static int32_t
emit(flat_ctx *c, Shape s, int32_t parent, int32_t tparent, int depth)
{
    if (depth > 4096) {
        c->depth_error = 1;
        return -1;
    }
    int32_t idx = (int32_t)c->nodes.count;
    gb_push(&c->nodes, 1);
    frt_node nd;
    memset(&nd, 0, sizeof(nd));
    nd.type = (int32_t)s->type;
    nd.parent = parent;
    nd.tparent = tparent;
    nd.xform = s->transform_identity ? -1 : add_xform(c, s->transform_inverse);
    nd.material = s->material ? add_material(c, s->material) : -1;
    nd.prim = -1;
    nd.right = -1;
    int32_t child_tparent = nd.xform >= 0 ? idx : tparent;
    if (s->type == SHAPE_GROUP || s->type == SHAPE_CSG) {
        Bounding_box b;
        shape_bounds(s, &b);
        memcpy(nd.bbox, b.min, 3 * sizeof(double));
        memcpy(nd.bbox + 3, b.max, 3 * sizeof(double));
    }
    if (s->type == SHAPE_GROUP) {
        for (size_t i = 0; i < s->fields.group.num_children; ++i) {
            emit(c, s->fields.group.children + i, idx, child_tparent, depth + 1);
        }
    } else if (s->type == SHAPE_CSG) {
        nd.prim = (int32_t)s->fields.csg.op;
        emit(c, s->fields.csg.left, idx, child_tparent, depth + 1);
        nd.right = (int32_t)c->nodes.count;
        emit(c, s->fields.csg.right, idx, child_tparent, depth + 1);
    } else {
        add_prim(c, s, &nd);
    }
    nd.skip = (int32_t)c->nodes.count;
    ((frt_node *)c->nodes.data)[idx] = nd;
    return idx;
}

static void
warm_bounds(Shape s)
{
    Bounding_box b;
    shape_bounds(s, &b);
    if (s->type == SHAPE_GROUP) {
        for (size_t i = 0; i < s->fields.group.num_children; ++i) warm_bounds(s->fields.group.children + i);
    } else if (s->type == SHAPE_CSG) {
        warm_bounds(s->fields.csg.left);
        warm_bounds(s->fields.csg.right);
    }
}

int
frt_flatten_scene(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter, frt_scene *out,
                  char *err, size_t errlen)
{
    flat_ctx c;
    memset(&c, 0, sizeof(c));
    c.nodes.elem = sizeof(frt_node);
    c.xforms.elem = sizeof(double);
    c.prims.elem = sizeof(double);
    c.materials.elem = sizeof(frt_material);
    c.patterns.elem = sizeof(frt_pattern);
    c.textures.elem = sizeof(frt_texture);
    c.texels.elem = sizeof(double);
    c.roots.elem = sizeof(int32_t);
    c.all_ni_one = 1;
    c.err = err;
    c.errlen = errlen;

    if (w->global_config == NULL) {
        snprintf(err, errlen, "world has no global_config");
        return -1;
    }
    for (size_t i = 0; i < w->shapes_num; ++i) warm_bounds(w->shapes + i);
    for (size_t i = 0; i < w->shapes_num; ++i) {
        int32_t r = emit(&c, w->shapes + i, -1, -1, 0);
        *(int32_t *)gb_push(&c.roots, 1) = r;
    }
    if (c.depth_error) {
        snprintf(err, errlen, "scene tree deeper than 4096 levels");
        return -1;
    }

    memset(out, 0, sizeof(*out));
    out->abi_version = FRT_ABI_VERSION;
    out->num_nodes = (int32_t)c.nodes.count;
    out->nodes = (const frt_node *)c.nodes.data;
    out->num_roots = (int32_t)c.roots.count;
    out->roots = (const int32_t *)c.roots.data;
    out->num_xforms = (int32_t)(c.xforms.count / 16);
    out->xforms = (const double *)c.xforms.data;
    out->prim_len = (int64_t)c.prims.count;
    out->prim_data = (const double *)c.prims.data;
    out->num_materials = (int32_t)c.materials.count;
    out->materials = (const frt_material *)c.materials.data;
    out->num_patterns = (int32_t)c.patterns.count;
    out->patterns = (const frt_pattern *)c.patterns.data;
    out->num_textures = (int32_t)c.textures.count;
    out->textures = (const frt_texture *)c.textures.data;
    out->texel_len = (int64_t)c.texels.count;
    out->texels = (const double *)c.texels.data;

    /* lights: cache rows copied point by point */
    frt_light *lights = (frt_light *)calloc(w->lights_num ? w->lights_num : 1, sizeof(frt_light));
    size_t total_pts = 0;
    for (size_t i = 0; i < w->lights_num; ++i) {
        const struct light *l = w->lights + i;
        total_pts += l->surface_points_cache_len * l->num_samples;
    }
    double *pts = (double *)malloc((total_pts ? total_pts : 1) * 3 * sizeof(double));
    size_t at = 0;
    for (size_t i = 0; i < w->lights_num; ++i) {
        const struct light *l = w->lights + i;
        frt_light *fl = lights + i;
        switch (l->type) {
        case AREA_LIGHT: fl->type = FRT_AREA_LIGHT; break;
        case CIRCLE_LIGHT: fl->type = FRT_CIRCLE_LIGHT; break;
        case HEMISPHERE_LIGHT: fl->type = FRT_HEMISPHERE_LIGHT; break;
        default: fl->type = FRT_POINT_LIGHT; break;
        }
        fl->num_samples = (int32_t)l->num_samples;
        fl->rows = (int32_t)l->surface_points_cache_len;
        /* photon emission data (light.c:14-99) */
        if (l->type == AREA_LIGHT) {
            Vector tmp;
            vector_cross((double *)l->u.area.uvec, (double *)l->u.area.vvec, tmp);
            Vector nrm;
            vector_normalize(tmp, nrm);
            memcpy(fl->normal, nrm, 3 * sizeof(double));
        } else if (l->type == CIRCLE_LIGHT) {
            memcpy(fl->normal, l->u.circle.normal, 3 * sizeof(double));
        } else if (l->type == HEMISPHERE_LIGHT) {
            memcpy(fl->normal, l->u.hemi.normal, 3 * sizeof(double));
            memcpy(fl->position, l->u.hemi.position, 3 * sizeof(double));
        } else {
            memcpy(fl->position, frt_light_position(l), 3 * sizeof(double));
        }
        fl->points = (int64_t)(3 * at);
        memcpy(fl->intensity, l->intensity, 3 * sizeof(double));
        for (size_t r = 0; r < l->surface_points_cache_len; ++r) {
            for (size_t k = 0; k < l->num_samples; ++k) {
                const double *src = (l->type == AREA_LIGHT || l->type == CIRCLE_LIGHT)
                                        ? l->surface_points_cache[r].points[k]
                                        : frt_light_position(l);
                memcpy(pts + 3 * at, src, 3 * sizeof(double));
                at++;
            }
        }
    }
    out->num_lights = (int32_t)w->lights_num;
    out->lights = lights;
    out->light_point_len = (int64_t)(3 * at);
    out->light_points = pts;

    frt_camera *fc = &out->camera;
    fc->hsize = (int64_t)cam->hsize;
    fc->vsize = (int64_t)cam->vsize;
    fc->usteps = (int64_t)usteps;
    fc->vsteps = (int64_t)vsteps;
    fc->half_width = cam->half_width;
    fc->half_height = cam->half_height;
    fc->pixel_size = cam->pixel_size;
    fc->canvas_distance = cam->canvas_distance;
    memcpy(fc->inv, cam->transform_inverse, sizeof(fc->inv));
    fc->aperture_size = cam->aperture.size;
    fc->aperture_type = (int32_t)cam->aperture.type;
    fc->jitter = jitter ? 1 : 0;
    fc->aperture_args[0] = cam->aperture.u.cross.x1;
    fc->aperture_args[1] = cam->aperture.u.cross.x2;
    fc->aperture_args[2] = cam->aperture.u.cross.y1;
    fc->aperture_args[3] = cam->aperture.u.cross.y2;

    /* the non-jittered CMJ sub-pixel table every pixel uses (renderer.c:145-151) */
    struct sampler smp;
    sampler_2d(false, usteps, vsteps, sampler_default_constraint, &smp);
    double *table = (double *)malloc(2 * usteps * vsteps * sizeof(double));
    for (size_t v = 0; v < vsteps; ++v) {
        for (size_t u = 0; u < usteps; ++u) {
            size_t idx[2] = {u, v};
            sampler_get_point_2d(&smp, idx, table + 2 * (v * usteps + u));
        }
    }
    sampler_free(&smp);
    out->sample_table = table;

    const struct illumination_config *ic = &w->global_config->illumination;
    out->config.include_direct = ic->include_direct;
    out->config.include_ambient = ic->di.include_ambient;
    out->config.include_diffuse = ic->di.include_diffuse;
    out->config.include_spec_highlight = ic->di.include_specular_highlight;
    out->config.include_specular = ic->di.include_specular;
    out->config.path_length = (int32_t)ic->di.path_length;
    out->config.all_ni_one = c.all_ni_one;
    /* global illumination (renderer.c:52-71: use_gi = include_global || visualize_photon_map) */
    out->config.use_gi = (ic->include_global || ic->debug_visualize_photon_map) ? 1 : 0;
    out->config.visualize_photon_map = ic->debug_visualize_photon_map ? 1 : 0;
    out->config.include_caustics = ic->gi.include_caustics ? 1 : 0;
    out->config.include_final_gather = ic->gi.include_final_gather ? 1 : 0;
    out->config.gi_usteps = (int32_t)ic->gi.usteps;
    out->config.gi_vsteps = (int32_t)ic->gi.vsteps;
    out->config.irradiance_num = (int32_t)ic->gi.irradiance_estimate_num;
    out->config.gi_path_length = (int32_t)ic->gi.path_length;
    out->config.irradiance_radius = ic->gi.irradiance_estimate_radius;
    out->config.cone_filter_k = ic->gi.irradiance_estimate_cone_filter_k;
    if (w->photon_maps != NULL && w->frt_photons_requested) {
        out->config.photon_count = (int64_t)w->photon_maps->max_photons;
        out->config.trace_caustic_map = w->frt_trace_caustic;
        out->config.trace_global_map = w->frt_trace_global;
    }
    /* apportion the photons by CIE L* of each light's intensity (photon_tracer.c:202-215) */
    if (out->config.photon_count > 0 && w->lights_num > 0) {
        double total_lightness = 0.0;
        Color lab;
        for (size_t i = 0; i < w->lights_num; ++i) {
            rgb_to_lab(w->lights[i].intensity, lab);
            total_lightness += lab[0];
        }
        for (size_t i = 0; i < w->lights_num; ++i) {
            rgb_to_lab(w->lights[i].intensity, lab);
            lights[i].num_photons = (int64_t)(size_t)((double)(size_t)out->config.photon_count * lab[0] / total_lightness);
        }
    }

    pm_free(&c.mat_map);
    pm_free(&c.pat_map);
    pm_free(&c.tex_map);
    return 0;
}

void
frt_flat_scene_free(frt_scene *s)
{
    free((void *)s->nodes);
    free((void *)s->roots);
    free((void *)s->xforms);
    free((void *)s->prim_data);
    free((void *)s->materials);
    free((void *)s->patterns);
    free((void *)s->textures);
    free((void *)s->texels);
    free((void *)s->lights);
    free((void *)s->light_points);
    free((void *)s->sample_table);
    memset(s, 0, sizeof(*s));
}
