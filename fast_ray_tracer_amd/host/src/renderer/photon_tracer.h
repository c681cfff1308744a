/* frt-mi355x host API: photon tracing pre-pass (reference src/renderer/photon_tracer.h). */
#ifndef FRT_PHOTON_TRACER_H
#define FRT_PHOTON_TRACER_H

#include <stdbool.h>
#include <stddef.h>
#include "../libs/photon_map/pm.h"
#include "world.h"

void trace_photons(const World w, const size_t num_photons, bool include_caustics, bool include_final_gather);
PhotonMap *array_of_photon_maps(size_t num);

#endif
