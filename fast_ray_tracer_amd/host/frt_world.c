/*
 * frt-mi355x host: world container and photon-map storage.
 *
 * world() mirrors reference src/renderer/world.c:14-28. The photon-map
 * storage API (pm.h) keeps the reference's struct so generated main() can
 * allocate maps; trace_photons() records the request and render_multi traces
 * the photons on the GPU (frt_gi.hpp).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "src/renderer/world.h"
#include "src/renderer/photon_tracer.h"
#include "src/libs/photon_map/pm.h"

World
world(void)
{
    World w = (World)calloc(1, sizeof(struct world));
    return w;
}

PhotonMap *
array_of_photon_maps(size_t num)
{
    return (PhotonMap *)calloc(num ? num : 1, sizeof(PhotonMap));
}

void
init_Photon_map(long max_phot, PhotonMap *pm)
{
    /* reference pm.c:11-47: 1-based heap storage and 256-entry direction tables */
    memset(pm, 0, sizeof(*pm));
    pm->stored_photons = 0;
    pm->prev_scale = 1;
    pm->max_photons = max_phot;
    pm->photons = (Photon *)malloc((size_t)(max_phot + 1) * sizeof(Photon));
    for (int k = 0; k < 3; ++k) {
        pm->bbox_min[k] = 1e8f;
        pm->bbox_max[k] = -1e8f;
    }
    for (int i = 0; i < 256; ++i) {
        double angle = (double)i * (1.0 / 256.0) * M_PI;
        pm->costheta[i] = cos(angle);
        pm->sintheta[i] = sin(angle);
        pm->cosphi[i] = cos(2.0 * angle);
        pm->sinphi[i] = sin(2.0 * angle);
    }
}

void
delete_Photon_map(PhotonMap *pm)
{
    free(pm->photons);
    pm->photons = NULL;
}

void
pm_store(PhotonMap *pm, double power[3], double pos[3], double dir[3])
{
    if (pm->stored_photons >= pm->max_photons) {
        return;
    }
    pm->stored_photons++;
    Photon *p = &pm->photons[pm->stored_photons];
    for (int k = 0; k < 3; ++k) {
        p->pos[k] = pos[k];
        if (pos[k] < pm->bbox_min[k]) pm->bbox_min[k] = pos[k];
        if (pos[k] > pm->bbox_max[k]) pm->bbox_max[k] = pos[k];
        p->power[k] = power[k];
    }
    int theta = (int)(acos(dir[2]) * (256.0 / M_PI));
    p->theta = (unsigned char)(theta > 255 ? 255 : theta);
    int phi = (int)(atan2(dir[1], dir[0]) * (256.0 / (2.0 * M_PI)));
    if (phi > 255) {
        p->phi = 255;
    } else if (phi < 0) {
        p->phi = (unsigned char)(phi + 256);
    } else {
        p->phi = (unsigned char)phi;
    }
}

void
pm_scale_photon_power(PhotonMap *pm, double scale)
{
    for (long i = pm->prev_scale; i <= pm->stored_photons; ++i) {
        for (int k = 0; k < 3; ++k) {
            pm->photons[i].power[k] *= scale;
        }
    }
    pm->prev_scale = pm->stored_photons;
}

void
pm_balance(PhotonMap *pm)
{
    (void)pm;
}

void
trace_photons(const World w, const size_t num_photons, bool include_caustics, bool include_final_gather)
{
    /* Reference photon_tracer.c:195-245 traces here, on the CPU. frt records the
     * request; render_multi traces the photons on the GPU after the scene upload
     * (fast_ray_tracer_amd/csrc/frt_gi.hpp), then balances the maps on the host. */
    (void)num_photons;
    if (w == NULL) {
        return;
    }
    w->frt_photons_requested = 1;
    w->frt_trace_caustic = include_caustics ? 1 : 0;
    w->frt_trace_global = include_final_gather ? 1 : 0;
}
