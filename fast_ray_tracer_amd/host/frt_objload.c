/*
 * frt-mi355x host: Wavefront OBJ / MTL loader.
 *
 * Restates reference src/libs/obj_loader/obj_loader.c:18-546 so that a mesh
 * loads into the same group structure, child order, triangle kinds and
 * materials as in the reference: faces are fan-triangulated in line order
 * into the current named group ("##default_group" first), smooth triangles
 * when the first vertex of a face carries a normal, and the named groups that
 * received faces become children of the result group in creation order.
 * MTL keywords are matched by prefix in the reference's order (so any line
 * starting with 'd' sets dissolve). Texture maps become TRIANGLE_UV_MAP
 * texture patterns.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "src/libs/obj_loader/obj_loader.h"
#include "src/shapes/group.h"
#include "src/shapes/triangle.h"
#include "src/color/rgb.h"

#define NAME_MAX_LEN 256

struct named_material {
    char name[NAME_MAX_LEN];
    Material material;
};

struct material_table {
    struct named_material *items;
    size_t count, cap;
};

static void
table_add(struct material_table *t, const char *name, Material m)
{
    if (t->count == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 16;
        t->items = (struct named_material *)realloc(t->items, t->cap * sizeof(*t->items));
    }
    snprintf(t->items[t->count].name, NAME_MAX_LEN, "%s", name);
    t->items[t->count].material = m;
    t->count++;
}

static Material
table_find(const struct material_table *t, const char *name)
{
    /* newest first, as a hash-table insert at the chain head would return */
    for (size_t k = t->count; k-- > 0;) {
        if (strcmp(t->items[k].name, name) == 0) {
            return t->items[k].material;
        }
    }
    return NULL;
}

static void
finalize_material_flags(Material m)
{
    /* obj_loader.c:41-56 */
    if (m == NULL) {
        return;
    }
    m->reflective = m->refl[0] > 0 || m->refl[1] > 0 || m->refl[2] > 0 || m->map_refl != NULL;
    if (m->Tr > 0 && (equal(m->Tf[0], 0) && equal(m->Tf[1], 0) && equal(m->Tf[1], 0))) {
        m->Tf[0] = m->Tf[1] = m->Tf[2] = m->Tr;
    } else if (equal(m->Tr, 0) && (m->Tf[0] > 0 || m->Tf[1] > 0 || m->Tf[2] > 0)) {
        m->Tr = (m->Tf[0] + m->Tf[1] + m->Tf[2]) / 3.0;
    }
}

static Pattern
load_texture_map(const char *line, void (*color_space_fn)(const Color, Color))
{
    char file[NAME_MAX_LEN] = {0};
    double scale = 1.0;
    int rv = sscanf(line, "%*s -bm %lf %255s", &scale, file);
    if (rv == 0) {
        sscanf(line, "%*s %255s", file);
    }
    size_t len = strlen(file);
    Pattern pats = array_of_patterns(2);
    if (access(file, F_OK) == -1) {
        printf("file '%s' does not exist.", file);
        return NULL;
    }
    Canvas image = NULL;
    if (len >= 3 && strcmp(file + len - 3, "ppm") == 0) {
        construct_canvas_from_ppm_file(&image, file, false, color_space_fn);
    } else if (len >= 3 && strcmp(file + len - 3, "png") == 0) {
        read_png(&image, file, false, color_space_fn);
    } else {
        printf("unrecognized file format for file %s\n", file);
        return NULL;
    }
    uv_texture_pattern(image, pats + 1);
    texture_map_pattern(pats + 1, TRIANGLE_UV_MAP, pats);
    return pats;
}

static void
read3(const char *line, double *out)
{
    sscanf(line, "%*s %lf %lf %lf", out, out + 1, out + 2);
}

static void
parse_mtl(FILE *f, struct material_table *table, void (*color_space_fn)(const Color, Color))
{
    char line[1024];
    char pending_name[NAME_MAX_LEN] = {0};
    Material cur = NULL;
    bool have_pending = false;
    Color tmp;

    while (fgets(line, sizeof(line), f)) {
        const char *p = line;
        while (*p == ' ' || *p == '\t') p++;
        if (*p == '#' || *p == '\r' || *p == '\n' || *p == '\0') {
            continue;
        }
        if (strncmp(p, "newmtl", 6) == 0) {
            finalize_material_flags(cur);
            if (have_pending) {
                table_add(table, pending_name, cur);
            }
            pending_name[0] = '\0';
            sscanf(p, "%*s %255s", pending_name);
            cur = material_alloc();
            have_pending = true;
        } else if (cur == NULL) {
            continue;
        } else if (strncmp(p, "illum", 5) == 0) {
            sscanf(p, "%*s %zu", &cur->illum);
        } else if (strncmp(p, "d", 1) == 0) {
            sscanf(p, "%*s %lf", &cur->Tr);
            cur->Tr = 1.0 - cur->Tr;
        } else if (strncmp(p, "Tr", 2) == 0) {
            sscanf(p, "%*s %lf", &cur->Tr);
        } else if (strncmp(p, "Ni", 2) == 0) {
            sscanf(p, "%*s %lf", &cur->Ni);
        } else if (strncmp(p, "Ns", 2) == 0) {
            sscanf(p, "%*s %lf", &cur->Ns);
        } else if (strncmp(p, "Ka", 2) == 0) {
            read3(p, tmp);
            color_space_fn(tmp, cur->Ka);
        } else if (strncmp(p, "Kd", 2) == 0) {
            read3(p, tmp);
            color_space_fn(tmp, cur->Kd);
        } else if (strncmp(p, "Ks", 2) == 0) {
            read3(p, cur->Ks);
        } else if (strncmp(p, "Tf", 2) == 0) {
            read3(p, cur->Tf);
            for (int k = 0; k < 3; ++k) {
                cur->Tf[k] = 1.0 - cur->Tf[k];
            }
        } else if (strncmp(p, "Ke", 2) == 0) {
            read3(p, cur->Ke);
        } else if (strncmp(p, "noshadow", 8) == 0) {
            cur->casts_shadow = false;
        } else if (strncmp(p, "map_Ka", 6) == 0) {
            Pattern pat = load_texture_map(p, color_space_fn);
            material_set_pattern(cur, map_Ka, pat);
        } else if (strncmp(p, "map_Kd", 6) == 0) {
            Pattern pat = load_texture_map(p, color_space_fn);
            material_set_pattern(cur, map_Kd, pat);
        } else if (strncmp(p, "map_bump", 8) == 0) {
            Pattern pat = load_texture_map(p, rgb_to_rgb);
            material_set_pattern(cur, map_bump, pat);
        } else {
            printf("Line \"%s\" not recognized while parsing .mtl file\n", line);
        }
    }
    finalize_material_flags(cur);
    if (have_pending) {
        table_add(table, pending_name, cur);
    }
}

struct vertex_array {
    double *v; /* 4 doubles per entry */
    size_t count, cap;
};

static double *
va_slot(struct vertex_array *a, double w)
{
    if (a->count == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 32768;
        a->v = (double *)realloc(a->v, 4 * a->cap * sizeof(double));
    }
    double *s = a->v + 4 * a->count++;
    s[0] = s[1] = s[2] = 0.0;
    s[3] = w;
    return s;
}

/* one face corner: v, v/t, v//n or v/t/n (1-based indices) */
static int
parse_corner(const char *tok, size_t *v, size_t *t, size_t *n)
{
    *v = *t = *n = 0;
    const char *slash = strchr(tok, '/');
    if (slash == NULL) {
        sscanf(tok, "%zu", v);
        return 1;
    }
    if (slash[1] == '/') {
        sscanf(tok, "%zu//%zu", v, n);
        return -1; /* normals, no textures */
    }
    return sscanf(tok, "%zu/%zu/%zu", v, t, n);
}

struct named_group {
    char *name;
    Shape group;
};

static void
add_face(char *line, struct vertex_array *verts, struct vertex_array *texs, struct vertex_array *norms,
         Material cur_material, Shape target, bool *started)
{
    size_t v0, t0, n0;
    char *tok = strtok(line, " \t");
    if (tok == NULL) {
        return;
    }
    int kind = parse_corner(tok, &v0, &t0, &n0);
    bool use_normals = kind == -1 || kind == 3;
    bool use_textures = kind == 2 || kind == 3;

    char *b = strtok(NULL, " \t");
    char *c = strtok(NULL, " \t");
    size_t produced = 0;
    while (b != NULL && c != NULL && *c != '\n') {
        size_t v1, t1, n1, v2, t2, n2;
        parse_corner(b, &v1, &t1, &n1);
        parse_corner(c, &v2, &t2, &n2);
        struct shape tri;
        if (use_normals) {
            smooth_triangle(&tri, verts->v + 4 * (v0 - 1), verts->v + 4 * (v1 - 1), verts->v + 4 * (v2 - 1),
                            norms->v + 4 * (n0 - 1), norms->v + 4 * (n1 - 1), norms->v + 4 * (n2 - 1));
        } else {
            triangle(&tri, verts->v + 4 * (v0 - 1), verts->v + 4 * (v1 - 1), verts->v + 4 * (v2 - 1));
        }
        if (use_textures) {
            vector_copy(tri.fields.triangle.t1, texs->v + 4 * (t0 - 1));
            vector_copy(tri.fields.triangle.t2, texs->v + 4 * (t1 - 1));
            vector_copy(tri.fields.triangle.t3, texs->v + 4 * (t2 - 1));
            tri.fields.triangle.use_textures = true;
        }
        if (cur_material != NULL) {
            shape_set_material(&tri, cur_material);
        }
        group_add_children_stage(target, &tri, 1);
        shape_free(&tri);
        produced++;
        b = c;
        c = strtok(NULL, " \t");
    }
    if (produced > 0) {
        *started = true;
    }
}

void
construct_group_from_obj_file(const char *file_path, void (*color_space_fn)(const Color, Color), Shape result)
{
    FILE *f = fopen(file_path, "r");
    if (f == NULL) {
        printf("Error opening file %s", file_path);
        return;
    }
    struct vertex_array verts = {0}, texs = {0}, norms = {0};
    struct material_table materials = {0};
    size_t ngroups = 1, gcap = 64, current = 0;
    struct named_group *groups = (struct named_group *)malloc(gcap * sizeof(*groups));
    groups[0].name = strdup("##default_group");
    groups[0].group = array_of_shapes(1);
    group(groups[0].group, NULL, 0);
    Material cur_material = NULL;
    bool started = false;
    char line[1024];

    while (fgets(line, sizeof(line), f)) {
        if (strncmp(line, "v ", 2) == 0) {
            read3(line, va_slot(&verts, 1.0));
        } else if (strncmp(line, "vt ", 3) == 0) {
            read3(line, va_slot(&texs, 0.0));
        } else if (strncmp(line, "vn ", 3) == 0) {
            read3(line, va_slot(&norms, 0.0));
        } else if (strncmp(line, "f ", 2) == 0) {
            add_face(line + 2, &verts, &texs, &norms, cur_material, groups[current].group, &started);
        } else if (strncmp(line, "g ", 2) == 0) {
            char name[NAME_MAX_LEN] = {0};
            sscanf(line, "%*s %255s", name);
            size_t i = 0;
            while (i < ngroups && strcmp(name, groups[i].name) != 0) {
                i++;
            }
            started = false;
            if (i == ngroups) {
                if (ngroups == gcap) {
                    gcap *= 2;
                    groups = (struct named_group *)realloc(groups, gcap * sizeof(*groups));
                }
                groups[ngroups].name = strdup(name);
                groups[ngroups].group = array_of_shapes(1);
                group(groups[ngroups].group, NULL, 0);
                current = ngroups++;
            } else {
                current = i;
            }
        } else if (strncmp(line, "usemtl", 6) == 0) {
            char name[NAME_MAX_LEN] = {0};
            sscanf(line, "%*s %255s", name);
            Material m = table_find(&materials, name);
            if (m != NULL) {
                cur_material = m;
            } else {
                printf("Material %s not found.\n", name);
            }
        } else if (strncmp(line, "mtllib", 6) == 0) {
            char name[NAME_MAX_LEN] = {0};
            sscanf(line, "%*s %255s", name);
            FILE *mf = access(name, F_OK) < 0 ? NULL : fopen(name, "r");
            if (mf == NULL) {
                printf("file %s not found.\n", name);
            } else {
                parse_mtl(mf, &materials, color_space_fn);
                fclose(mf);
            }
        }
    }
    fclose(f);

    for (size_t i = 0; i < ngroups; ++i) {
        group_add_children_finish(groups[i].group);
    }
    group(result, NULL, 0);
    for (size_t i = 0; i < ngroups; ++i) {
        if (groups[i].group->fields.group.num_children > 0) {
            group_add_children(result, groups[i].group, 1);
        }
    }
    for (size_t i = 0; i < ngroups; ++i) {
        free(groups[i].name);
        shape_free(groups[i].group);
        free(groups[i].group);
    }
    free(groups);
    free(verts.v);
    free(texs.v);
    free(norms.v);
    free(materials.items);
}
