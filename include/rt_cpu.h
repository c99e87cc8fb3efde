/* rt_cpu.h — the CPU backend of the path tracer (librtx_cpu.so).
 *
 * The reference renders on the host when its CLI is given -p without -g
 * (input/CLI.cpp:4-92 -> StaticCamera::render_cpu, StaticCamera.cpp:32-134:
 * rows of the frame on a ThreadPool).  rtx_render --backend cpu --threads N
 * takes that role here: the GPU kernel's own per-path source (csrc/rt_path.h:
 * camera ray, closest hit, media, materials, textures, light sampling) compiled
 * for the host by g++ and run one path at a time, image rows handed to N host
 * threads as they free up.  It draws the same counter-based samples as the GPU
 * library (the Philox stream keyed by seed, pixel and stratum), so its frame
 * equals rt_render's to fp64 summation order (a pixel's strata are added in
 * stratum order here, in completion order on the GPU).
 *
 * This is an explicit second backend chosen by the caller, never a fallback:
 * librtx_hip.so does not load it, and the Python package (rtx/) never does.
 * It is not the measured hot path; bench.py times the reference's own CPU
 * path as its baseline.
 */
#ifndef RT_CPU_H
#define RT_CPU_H
#include "rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_CPU_ABI_VERSION 2

int rt_cpu_abi_version(void);
const char *rt_cpu_last_error(void); /* thread-local; valid until the next call */

/* Render rows [row_begin,row_end) x strata [sample_begin, +sample_count) of
   `frame` (from rt_camera_setup) on `threads` host threads (<= 0:
   rt_cpu_default_threads()) into host_rgb, RT_OUT_SCALED or RT_OUT_SUM, in
   the GPU library's output layouts (rt_render_params): RT_LAYOUT_FRAME,
   row-major, 3 doubles per pixel, index (j-row_begin)*W+i; RT_LAYOUT_TILES,
   the tiles tile_first + k*tile_stride of the band at [k][64][3], or with
   strata_chunks > 1 each chunk's partial sums at [k][chunk][64][3].  The
   params are validated as rt_render validates them (the same messages);
   accumulate must be 0 and RT_CHUNKS_AUTO is refused (a GPU work-unit
   plan).  A pixel's strata are added in stratum order, so any thread count
   gives the same bytes.  Synchronous. */
int rt_cpu_render(const rt_scene_desc *desc, const rt_frame *frame, const rt_render_params *params,
                  int32_t threads, double *host_rgb);

/* The default thread count: the CPUs this process may run on (its affinity
   mask, capped by a cgroup v2 cpu.max quota) -- not
   std::thread::hardware_concurrency(), which counts the whole machine. */
int rt_cpu_default_threads(void);

#ifdef __cplusplus
}
#endif
#endif
