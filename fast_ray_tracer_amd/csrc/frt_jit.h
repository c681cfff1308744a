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
// the tile pair kernel (frt_jit_tile) decides runs of this many consecutive path nodes at once (a power of two
// up to 64; 0: off; FRT_JIT_TILE overrides the default 64)
int frt_jit_tile_size();
// the sub-tile kernel (frt_jit_subtile, after the sub-part pass) re-decides the tile sub-pairs left mixed for runs of
// this many of the tile's nodes (a power of two below the tile size; 0: off; FRT_JIT_SUBTILE overrides the default)
int frt_jit_subtile_size();
// the sub-part pass (frt_jit_sub, after the tile kernel) splits the parts of the tile pairs left mixed into this many
// sub-parts (2 ... 32; 0: off; FRT_JIT_SUB overrides the default 16); their sizes, the largest (PS2), and the
// sub-parts' samples
int frt_jit_sub_count();
std::vector<int> frt_jit_sub_sizes(int c, int Q);
int frt_jit_sub_ps(int PS, int Q);
int frt_jit_light_subparts(const frt_light& L, const double* light_points, const std::vector<int32_t>& order, int PS,
                           int Q, std::vector<int32_t>& order2);
// the parts (frt_jit.hip): spatially compact groups of the light's samples; returns the part count
int frt_jit_light_parts(const frt_light& L, const double* light_points, int PS, std::vector<int32_t>& order);

// HIP source of the shadow kernel for this tree and these lights ("" and `why` set when the scene
// is not eligible: too many nodes, or a CSG unit with a leaf whose list is unsorted)
std::string frt_jit_shadow_source(const frt::WalkNode* wn, int num_nodes, const int32_t* roots, int num_roots,
                                  const frt_light* lights, int num_lights, std::string& why);

// the kernels of a scene's module (hipFunction_t; tile / list are null when the source has none)
struct FrtJitFns {
    void* shadow = nullptr;  // frt_jit_shadow: per ray
    void* beam = nullptr;    // frt_jit_beam: every (node, part) pair
    void* tile = nullptr;    // frt_jit_tile: every (tile, part) pair
    void* list = nullptr;    // frt_jit_beam_list: the nodes of the listed tile pairs
    void* sub = nullptr;     // frt_jit_sub: the sub-parts of the tile pairs left mixed
    void* subtile = nullptr; // frt_jit_subtile: the sub-tiles of the tile sub-pairs left mixed
    void* trace = nullptr;   // frt_jit_trace: closest hit per ray (null where the scene has none)
};
// compile with hiprtc for `device` (cached per device and source); 0 on success
int frt_jit_compile(const std::string& src, int device, FrtJitFns& fns, std::string& log);

// this thread's last frt_jit_compile: ms to obtain the code object (0 when the process had it; a disk
// read or a hiprtc compile otherwise) and to load it into the device's module
void frt_jit_last_phases(double* obtain_ms, double* load_ms);

// compile only (no device needed): 0 on success
int frt_jit_compile_only(const std::string& src, const std::string& arch, std::string& log);
