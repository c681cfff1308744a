/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the frt-mi355x hot path.
 *
 * A plain-C restatement of the reference's per-sample recursion
 * (reference src/renderer/renderer.c:74-979, src/renderer/world.c:163-197,
 * src/intersection/intersection.c:42-145, src/shapes/*_local_intersect,
 * src/pattern/pattern.c, src/libs/quartic/Roots3And4.c) that walks the host
 * scene graph the drop-in API builds. It is the checker the GPU path is
 * compared against (tests/, __graft_entry__.smoke, bench.py's cpu_baseline);
 * the product never links or calls it. It is itself pinned against the real
 * reference (oracle/build_ref.sh -> oracle/_ref) through tests/golden.
 */
#ifndef FRT_ORACLE_H
#define FRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "src/renderer/renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct frt_oracle_stats {
    uint64_t primary_rays;    /* camera samples */
    uint64_t secondary_rays;  /* reflect + refract color_at calls (zero-weight ones included) */
    uint64_t shadow_rays;     /* is_shadowed calls */
    uint64_t zero_weight_secondary; /* refraction rays whose filter Tf*d is exactly 0 */
} frt_oracle_stats;

/*
 * Render rows [row_begin, row_end) of the frame into out (row-major, 4 doubles
 * per pixel, rows relative to row_begin) with nthreads pthreads, one row per
 * job as the reference's pool does (renderer.c:244-281). Area-light rows and
 * jittered sub-pixel tables draw from glibc rand()/drand48() as the reference
 * does, so with nthreads = 1 a stochastic scene reproduces a reference run
 * with thread-count 1 (same process state assumed).
 */
int frt_oracle_render_rows(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter,
                           size_t row_begin, size_t row_end, int nthreads, double *out,
                           frt_oracle_stats *stats);
/* rows row_begin, row_begin + row_stride, ... below row_end (one row job each; out: one row after another) */
int frt_oracle_render_rows_strided(Camera cam, World w, size_t usteps, size_t vsteps, bool jitter,
                                   size_t row_begin, size_t row_end, size_t row_stride, int nthreads, double *out,
                                   frt_oracle_stats *stats);

#ifdef __cplusplus
}
#endif

#endif
