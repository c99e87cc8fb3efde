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

DCamera host_camera(const rt_frame &f) {
  DCamera C{};
  auto cp = [](double *d, const rt_vec3 &v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
  };
  cp(C.center, f.center);
  cp(C.p00, f.pixel00_loc);
  cp(C.du, f.pixel_delta_u);
  cp(C.dv, f.pixel_delta_v);
  cp(C.disk_u, f.defocus_disk_u);
  cp(C.disk_v, f.defocus_disk_v);
  cp(C.bg, f.background);
  C.defocus_angle = f.defocus_angle;
  C.scale = f.pixel_samples_scale;
  C.W = f.image_width;
  C.H = f.image_height;
  C.sqrt_spp = f.sqrt_spp;
  C.rs = 1.0 / f.sqrt_spp;
  C.max_depth = f.max_depth;
  return C;
}

} // namespace

extern "C" {

int rt_cpu_abi_version(void) { return RT_CPU_ABI_VERSION; }

const char *rt_cpu_last_error(void) { return g_err.c_str(); }

int rt_cpu_render(const rt_scene_desc *desc, const rt_frame *f, const rt_render_params *p,
                  int32_t threads, double *host_rgb) {
  if (!desc || !f || !p || !host_rgb) return fail(RT_ERR_INVALID, "null argument");
  if (f->image_width <= 0 || f->image_height <= 0 || f->sqrt_spp <= 0)
    return fail(RT_ERR_INVALID, "frame not set up (rt_camera_setup)");
  if (p->tile_first != 0 || p->tile_stride > 1 || p->layout != RT_LAYOUT_FRAME || p->accumulate)
    return fail(RT_ERR_INVALID, "rt_cpu_render takes whole-frame launches (RT_LAYOUT_FRAME, "
                                "tile_first 0, tile_stride 0/1, accumulate 0)");
  if (p->output != RT_OUT_SCALED && p->output != RT_OUT_SUM) return fail(RT_ERR_INVALID, "unknown output mode");
  int r0 = p->row_begin, r1 = p->row_end;
  if (r0 == 0 && r1 == 0) r1 = f->image_height;
  if (r0 < 0 || r1 > f->image_height || r0 > r1) return fail(RT_ERR_INVALID, "row range outside the image");
  const int n = f->sqrt_spp * f->sqrt_spp;
  const int s0 = p->sample_begin, s1 = p->sample_count < 0 ? n : s0 + p->sample_count;
  if (s0 < 0 || s1 < s0 || s1 > n) return fail(RT_ERR_INVALID, "sample range outside [0, sqrt_spp^2)");

  rtx::HostScene H;
  std::string err;
  int rc = rtx::compile_scene(desc, H, err);
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
  if (RT_LDS_TRIPLE) {
    lnodes_l.reserve(H.nodes.size());
    for (const DNode &nd : H.nodes) lnodes_l.push_back(lds_node(nd, RT_SLAB_FMA && RT_SLAB_SIGN));
    lnodes = (const DNode *)(const void *)lnodes_l.data();
  }
  const DCamera C = host_camera(*f);
  const PixelFn fn = kPixelFns[S.features & (F_FLAT * 2 - 1)];
  const bool scaled = p->output == RT_OUT_SCALED;
  const uint64_t seed = p->seed;

  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, std::max(1, r1 - r0)));
  std::atomic<int> next_row{r0};
  auto work = [&]() {
    std::vector<int> stack((size_t)RT_STACK_DEPTH * 64);
    for (int j; (j = next_row.fetch_add(1)) < r1;)
      for (int i = 0; i < C.W; ++i) {
        double acc[3] = {0.0, 0.0, 0.0};
        fn(S, C, seed, i, j, s0, s1, stack.data(), lnodes, acc);
        double *o = host_rgb + 3 * ((size_t)(j - r0) * C.W + i);
        for (int c = 0; c < 3; ++c) o[c] = scaled ? C.scale * acc[c] : acc[c];
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
  return RT_OK;
}

} // extern "C"
