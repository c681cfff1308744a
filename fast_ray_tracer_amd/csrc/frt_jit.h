// frt-mi355x scene-specialised shadow kernel (frt_jit.hip): host interface used by the engine.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace frt {
struct WalkNode;
}
struct frt_light;

// the pair kernel (frt_jit_beam) decides a light's samples in parts of this many consecutive samples
// (FRT_JIT_PART overrides the default, for A/B runs)
int frt_jit_part_size();
// the parts (frt_jit.hip): spatially compact groups of the light's samples; returns the part count
int frt_jit_light_parts(const frt_light& L, const double* light_points, int PS, std::vector<int32_t>& order);

// HIP source of the shadow kernel for this tree and these lights ("" and `why` set when the scene
// is not eligible: too many nodes, or a CSG unit with a leaf whose list is unsorted)
std::string frt_jit_shadow_source(const frt::WalkNode* wn, int num_nodes, const int32_t* roots, int num_roots,
                                  const frt_light* lights, int num_lights, std::string& why);

// compile with hiprtc for `device` (cached per device and source); 0 on success, *fn = the per-ray
// kernel frt_jit_shadow, *fn_beam = the pair kernel frt_jit_beam (hipFunction_t)
int frt_jit_compile(const std::string& src, int device, void** fn, void** fn_beam, std::string& log);

// compile only (no device needed): 0 on success
int frt_jit_compile_only(const std::string& src, const std::string& arch, std::string& log);
