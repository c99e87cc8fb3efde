// rtx_cpu.cpp — librtx_cpu.so, the CPU backend (include/rt_cpu.h).
//
// The reference's CPU path (StaticCamera::render_cpu, StaticCamera.cpp:32-134)
// renders rows on its ThreadPool; here the GPU kernel's per-path source
// (csrc/rt_path.h) is compiled for the host and each host thread takes the next
// unrendered row (an atomic counter: expensive rows do not hold up a static
// share), tracing a pixel's strata one path at a time in stratum order.  The
// scene is compiled by the same scene compiler as the GPU library
// (csrc/rt_scene.cpp), the world BVH built by its host SAH builder, and the
// path code instance chosen by the same feature bits (rtx::scene_features),
// binary walk only.
#include "../../include/rt_cpu.h"
#include "../csrc/rt_path.h"
#include "../csrc/rt_scene.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <string>
#include <thread>
#include <utility>
#include <vector>

using namespace rtp;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

// One pixel's strata [s0, s1), each path to its end (rt_path.h segment), added
// in stratum order.
template <unsigned F>
void render_pixel(const DScene &S, const DCamera &C, uint64_t seed, int i, int j, int s0, int s1,
                  int *stack, const DNode *lnodes, double acc[3]) {
  Counters cnt{};
  for (int k = s0; k < s1; ++k) {
    Key key{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)(j * C.W + i), (uint32_t)k};
    PathState ps;
    ps.ray = camera_ray(C, key, i, j, k);
    ps.T = v3(1.0, 1.0, 1.0);
    ps.bounce = 0;
    ps.active = C.max_depth > 0;
    while (ps.active) {
      if (!segment<false, F>(S, C, ps, key, stack, lnodes, cnt)) {
        acc[0] += ps.T.x;
        acc[1] += ps.T.y;
        acc[2] += ps.T.z;
        ps.active = false;
      }
    }
  }
}

typedef void (*PixelFn)(const DScene &, const DCamera &, uint64_t, int, int, int, int, int *,
                        const DNode *, double *);
template <unsigned... Fs>
constexpr std::array<PixelFn, sizeof...(Fs)> pixel_fns(std::integer_sequence<unsigned, Fs...>) {
  return {render_pixel<Fs>...};
}
// the binary-walk instances: MEDIA | XFORM | LIGHTS | NOISE | FLAT
constexpr auto kPixelFns = pixel_fns(std::make_integer_sequence<unsigned, F_FLAT * 2>{});

// Default worker count: the CPUs this process may run on -- the affinity
// mask, capped by a cgroup v2 cpu.max quota -- not hardware_concurrency(),
// which on a quota-limited box (the GPU box: 16 of 256) oversubscribes the
// quota many times over (README: the reference's pool collapsing there).
int usable_cpus() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  if (FILE *fp = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long per = 0;
    if (std::fscanf(fp, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
      const long long quota = std::atoll(q);
      if (quota > 0) n = std::min<int>(n, (int)std::max<long long>(1, quota / per));
    }
    std::fclose(fp);
  }
  return std::max(1, n);
}

} // namespace

extern "C" {

int rt_cpu_abi_version(void) { return RT_CPU_ABI_VERSION; }

const char *rt_cpu_last_error(void) { return g_err.c_str(); }

int rt_cpu_default_threads(void) { return usable_cpus(); }

int rt_cpu_render(const rt_scene_desc *desc, const rt_frame *f, const rt_render_params *p,
                  int32_t threads, double *host_rgb) {
  if (!desc || !host_rgb) return fail(RT_ERR_INVALID, "null argument");
  // the GPU library's validation (rt_scene.cpp launch_geometry), so both
  // backends accept and refuse the same launches
  DCamera C;
  DLaunch L;
  std::string err;
  int rc = rtx::device_camera(f, C, err);
  if (rc == RT_OK) rc = rtx::launch_geometry(f, p, L, err);
  if (rc != RT_OK) return fail(rc, err);
  if (L.accumulate) return fail(RT_ERR_INVALID, "rt_cpu_render writes its output (accumulate 0)");

  rtx::HostScene H;
  rc = rtx::compile_scene(desc, H, err);
  if (rc != RT_OK) return fail(rc, err);
  if (H.device_bvh) rtx::build_world_bvh_host(H); // the device builders are the GPU library's
  const int stack_depth = std::max(1, H.bvh_depth + 1);
  if (stack_depth > RT_STACK_DEPTH)
    return fail(RT_ERR_UNSUPPORTED, "world BVH deeper than the traversal stack (" +
                                        std::to_string(H.bvh_depth) + " levels)");
  DScene S{};
  S.nodes = H.nodes.data();
  S.items = H.items.data();
  S.bitems = H.bitems.data();
  S.mitems = H.mitems.data();
  S.mbox = H.mbox.data();
  S.n_mitems = (int32_t)H.mitems.size();
  S.xforms = H.xforms.data();
  S.spheres = H.spheres.data();
  S.quads = H.quads.data();
  S.media = H.media.data();
  S.mats = H.mats.data();
  S.texs = H.texs.data();
  S.perlin = H.perlin.data();
  S.lights = H.lights.data();
  S.n_lights = (int32_t)H.lights.size();
  S.n_nodes = (int32_t)H.nodes.size();
  S.root_is_leaf = H.root_is_leaf;
  S.n_root_items = H.n_root_items;
  S.features = rtx::scene_features(H) | (H.root_is_leaf ? F_FLAT : 0);
  S.static_spheres = rtx::all_spheres_static(H);
  S.stack_depth = stack_depth;
  S.n_lds_nodes = S.n_nodes; // the walk reads every node from `lnodes`, in the staged form
  std::vector<DNodeL> lnodes_l;
  const DNode *lnodes = S.nodes;
  {
    lnodes_l.reserve(H.nodes.size());
    for (const DNode &nd : H.nodes) lnodes_l.push_back(lds_node(nd, true));
    lnodes = (const DNode *)(const void *)lnodes_l.data();
  }
  const PixelFn fn = kPixelFns[S.features & (F_FLAT * 2 - 1)];
  const bool scaled = L.output == RT_OUT_SCALED;
  const uint64_t seed = p->seed;
  const int s0 = L.sample_begin, s1 = L.sample_begin + L.sample_count;

  // Work items: frame layout -- rows of the band, pixels (j - row_begin) * W + i;
  // tile layout -- the launch's tiles t = tile_first + k * tile_stride (8x8,
  // row-major over the band), tile k's pixel s = (j - y0) * 8 + (i - x0) at
  // [k][s] (one chunk) or each chunk's partial sums at [k][c][s], chunk c the
  // strata [s0 + c * chunk_strata, +chunk_strata) -- the GPU library's
  // RT_LAYOUT_TILES output; pixels past the frame's edge are 0.
  const int n_items = L.compact ? L.n_local_tiles : L.row_end - L.row_begin;
  int nt = threads > 0 ? threads : usable_cpus();
  nt = std::max(1, std::min(nt, std::max(1, n_items)));
  std::atomic<int> next{0};
  std::atomic<int> status{RT_OK};
  auto work = [&]() {
    try {
      std::vector<int> stack((size_t)RT_STACK_DEPTH * 64);
      for (int k; status.load(std::memory_order_relaxed) == RT_OK && (k = next.fetch_add(1)) < n_items;) {
        if (!L.compact) {
          const int j = L.row_begin + k;
          for (int i = 0; i < C.W; ++i) {
            double acc[3] = {0.0, 0.0, 0.0};
            fn(S, C, seed, i, j, s0, s1, stack.data(), lnodes, acc);
            double *o = host_rgb + 3 * ((size_t)k * C.W + i);
            for (int c = 0; c < 3; ++c) o[c] = scaled ? C.scale * acc[c] : acc[c];
          }
          continue;
        }
        const int64_t t = L.tile_first + (int64_t)k * L.tile_stride;
        const int x0 = (int)(t % L.tiles_x) * 8, y0 = L.row_begin + (int)(t / L.tiles_x) * 8;
        for (int c = 0; c < L.n_chunks; ++c) {
          const int c0 = std::min(s1, s0 + c * L.chunk_strata), c1 = std::min(s1, c0 + L.chunk_strata);
          double *o = host_rgb + ((size_t)k * L.n_chunks + c) * 64 * 3;
          for (int sp = 0; sp < 64; ++sp) {
            const int i = x0 + (sp & 7), j = y0 + (sp >> 3);
            double acc[3] = {0.0, 0.0, 0.0};
            if (i < C.W && j < L.row_end) fn(S, C, seed, i, j, c0, c1, stack.data(), lnodes, acc);
            for (int ch = 0; ch < 3; ++ch) o[3 * sp + ch] = scaled ? C.scale * acc[ch] : acc[ch];
          }
        }
      }
    } catch (const std::bad_alloc &) {
      int ok = RT_OK;
      status.compare_exchange_strong(ok, RT_ERR_OOM);
    } catch (...) {
      int ok = RT_OK;
      status.compare_exchange_strong(ok, RT_ERR_INVALID);
    }
  };
  std::vector<std::thread> pool;
  try {
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  } catch (const std::exception &ex) { // fewer threads than asked: the rest still run
    (void)ex;
  }
  work();
  for (auto &t : pool) t.join();
  const int st = status.load();
  if (st == RT_ERR_OOM) return fail(st, "out of host memory in a render thread");
  if (st != RT_OK) return fail(st, "a render thread threw");
  return RT_OK;
}

} // extern "C"
