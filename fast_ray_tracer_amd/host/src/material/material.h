/*
 * frt-mi355x host API: MTL-style materials.
 * Field names and the material_set_pattern macro follow reference
 * src/material/material.h:196-257 (the codegen writes these fields directly).
 */
#ifndef FRT_MATERIAL_H
#define FRT_MATERIAL_H

#include <stdbool.h>
#include <stdlib.h>

#include "../color/color.h"
#include "../pattern/pattern.h"

typedef struct material {
    Color Ka;
    Color Kd;
    Color Ks;
    Color Tf;
    Color Ke;
    Color refl;
    double Ns;
    double Ni;
    double Tr;
    size_t illum;
    bool casts_shadow;
    bool reflective;
    Pattern map_Ka;
    Pattern map_Kd;
    Pattern map_Ks;
    Pattern map_Ns;
    Pattern map_d;
    Pattern map_bump;
    Pattern map_disp;
    Pattern map_refl;
    size_t ref_count;
} *Material;

void material(Material m);
Material material_alloc(void);
Material array_of_materials(size_t num);
void material_free(Material m);

#define material_set_pattern(m, field, p) \
if (m != NULL) {\
    if (m->field != NULL) {\
        pattern_free(m->field);\
    }\
    m->field = (p);\
    if ((p) != NULL) {\
        p->ref_count++;\
    }\
}

#endif
