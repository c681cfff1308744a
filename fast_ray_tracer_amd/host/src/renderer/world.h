/*
 * frt-mi355x host API: the world container (reference src/renderer/world.h:25-34).
 * Generated main() fills lights / shapes / photon_maps / global_config directly.
 */
#ifndef FRT_WORLD_H
#define FRT_WORLD_H

#include <stdlib.h>

#include "../libs/photon_map/pm.h"
#include "../light/light.h"
#include "../shapes/shapes.h"
#include "config.h"

typedef struct world {
    Light lights;
    Shape shapes;
    size_t lights_num;
    size_t shapes_num;
    PhotonMap *photon_maps;
    Global_config global_config;
    /* frt: trace_photons() records its request here; the photons are traced on the GPU by render_multi */
    int frt_photons_requested;
    int frt_trace_caustic, frt_trace_global;
} *World;

World world(void);

#endif
