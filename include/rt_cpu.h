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

#define RT_CPU_ABI_VERSION 1

int rt_cpu_abi_version(void);
const char *rt_cpu_last_error(void); /* thread-local; valid until the next call */

/* Render rows [row_begin,row_end) x strata [sample_begin, +sample_count) of
   `frame` (from rt_camera_setup) on `threads` host threads (<= 0: one per
   hardware thread) into host_rgb: row-major, 3 doubles per pixel, index
   (j-row_begin)*W+i, RT_OUT_SCALED or RT_OUT_SUM.  Only whole-frame launches
   (tile_first 0, tile_stride 0/1, RT_LAYOUT_FRAME, accumulate 0); tile
   layouts are the GPU library's.  Synchronous. */
int rt_cpu_render(const rt_scene_desc *desc, const rt_frame *frame, const rt_render_params *params,
                  int32_t threads, double *host_rgb);

#ifdef __cplusplus
}
#endif
#endif
