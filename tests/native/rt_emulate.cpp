// tests/native/rt_emulate.cpp — TEST INFRASTRUCTURE ONLY.
//
// Runs the HIP kernel's own per-path source (real-time-ray-tracing-engine_amd/
// csrc/rt_path.h: camera_ray, trace, segment, lights, media, textures) on the
// host, one path at a time, over the scene the library's own scene compiler
// builds (csrc/rt_scene.cpp).  Comparing it with the oracle separates logic
// errors in the kernel source from gfx950 code-generation problems: the
// emulator is compiled by g++, the kernel by hipcc for gfx950.
// Not part of the product: the library never calls this, and it is built under
// tests/native/build only.
#include "../../real-time-ray-tracing-engine_amd/csrc/rt_path.h"
#include "../../real-time-ray-tracing-engine_amd/csrc/rt_scene.h"

#include <algorithm>
#include <array>
#include <utility>
#include <string>
#include <vector>

using namespace rtp;

namespace {

template <unsigned F>
void trace_pixel(const DScene &S, const DCamera &C, const rt_render_params &p, int i, int j,
                 int s0, int s1, int *stk, const DNode *ln, double acc[3]) {
  Counters cnt{};
  for (int k = s0; k < s1; ++k) {
    Key key{(uint32_t)p.seed, (uint32_t)(p.seed >> 32), (uint32_t)(j * C.W + i), (uint32_t)k};
    PathState ps;
    ps.ray = camera_ray(C, key, i, j, k);
    ps.T = v3(1.0, 1.0, 1.0);
    ps.bounce = 0;
    ps.active = C.max_depth > 0;
    while (ps.active) {
      bool cont = segment<false, F>(S, C, ps, key, stk, ln, cnt);
      if (!cont) {
        acc[0] += ps.T.x;
        acc[1] += ps.T.y;
        acc[2] += ps.T.z;
        ps.active = false;
      }
    }
  }
}

typedef void (*PixelFn)(const DScene &, const DCamera &, const rt_render_params &, int, int, int,
                        int, int *, const DNode *, double *);
template <unsigned... Fs>
constexpr std::array<PixelFn, sizeof...(Fs)> pixel_fns(std::integer_sequence<unsigned, Fs...>) {
  return {trace_pixel<Fs>...};
}
// one per kernel instance (rt_kernel.hip render_table)
constexpr auto kFns = pixel_fns(std::make_integer_sequence<unsigned, F_ALL + 1>{});

} // namespace

extern "C" int emu_render(const rt_scene_desc *desc, const rt_frame *f, const rt_render_params *p,
                          int features, double *out) {
  rtx::HostScene H;
  std::string err;
  if (rtx::compile_scene(desc, H, err) != RT_OK) return -1;
  if (H.device_bvh) rtx::build_world_bvh_host(H); // the device builder needs a GPU
  // features bit 5 (F_BVH4): walk the 4-wide collapse of the same tree, as the
  // library does for large scenes (rt_api.cpp)
  const bool bvh4 = (features & F_BVH4) && !H.root_is_leaf && !H.nodes.empty();
  int depth4 = 0;
  if (bvh4) depth4 = rtx::collapse_bvh4(H.nodes, H.nodes4);
  DScene S;
  S.nodes = bvh4 ? (const DNode *)(const void *)H.nodes4.data() : H.nodes.data();
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
  S.n_nodes = (int32_t)(bvh4 ? H.nodes4.size() : H.nodes.size());
  S.root_is_leaf = H.root_is_leaf;
  S.n_root_items = H.n_root_items;
  S.features = features;
  S.static_spheres = rtx::all_spheres_static(H);
  // rt_scene_create's rule: the walk pushes with no overflow check, so a tree
  // deeper than the stack is refused, not clamped
  S.stack_depth = bvh4 ? rtx::bvh4_stack_depth(depth4) : std::max(1, H.bvh_depth + 1);
  if (S.stack_depth > (bvh4 ? RT_STACK_DEPTH4 : RT_STACK_DEPTH)) return -2;
  S.n_lds_nodes = S.n_nodes; // host: the whole tree is the "LDS" copy
  // in the form the kernel stages it: DNode4 as is, binary nodes as DNodeL
  std::vector<DNodeL> lnodes_l;
  const DNode *ln = S.nodes;
  if (!bvh4) {
    for (const DNode &nd : H.nodes) lnodes_l.push_back(lds_node(nd, true));
    ln = (const DNode *)(const void *)lnodes_l.data();
  }
  DCamera C;
  auto cp = [](double *d, const rt_vec3 &v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
  };
  cp(C.center, f->center);
  cp(C.p00, f->pixel00_loc);
  cp(C.du, f->pixel_delta_u);
  cp(C.dv, f->pixel_delta_v);
  cp(C.disk_u, f->defocus_disk_u);
  cp(C.disk_v, f->defocus_disk_v);
  cp(C.bg, f->background);
  C.defocus_angle = f->defocus_angle;
  C.scale = f->pixel_samples_scale;
  C.W = f->image_width;
  C.H = f->image_height;
  C.sqrt_spp = f->sqrt_spp;
  C.rs = 1.0 / C.sqrt_spp;
  C.max_depth = f->max_depth;
  int r0 = p->row_begin, r1 = p->row_end;
  if (r0 == 0 && r1 == 0) r1 = f->image_height;
  int n = f->sqrt_spp * f->sqrt_spp;
  int s0 = p->sample_begin, s1 = p->sample_count < 0 ? n : s0 + p->sample_count;
  std::vector<int> stack(std::max(RT_STACK_DEPTH, RT_STACK_DEPTH4) * 64);
  // the instance the library would pick: the caller's feature bits plus F_FLAT
  // for a flat world, F_BVH4 for a collapsed tree (rt_api.cpp)
  PixelFn fn = kFns[(features & 15) | (H.root_is_leaf ? F_FLAT : 0u) | (bvh4 ? F_BVH4 : 0u)];
  for (int j = r0; j < r1; ++j)
    for (int i = 0; i < C.W; ++i) {
      double acc[3] = {0, 0, 0};
      fn(S, C, *p, i, j, s0, s1, stack.data(), ln, acc);
      double sc = (p->output == RT_OUT_SCALED) ? C.scale : 1.0;
      double *o = out + 3 * ((size_t)(j - r0) * C.W + i);
      o[0] = (p->output == RT_OUT_SCALED) ? sc * acc[0] : acc[0];
      o[1] = (p->output == RT_OUT_SCALED) ? sc * acc[1] : acc[1];
      o[2] = (p->output == RT_OUT_SCALED) ? sc * acc[2] : acc[2];
    }
  return 0;
}

// The 4-wide collapse of the world BVH of `desc` (tests/test_emulator.py):
// info = {binary nodes, 4-wide nodes, binary depth, 4-wide levels, leaf entries
// of the binary tree, leaf entries of the 4-wide tree, 1 if the two leaf-entry
// lists are equal in order, inner children with a box different from the binary
// node they came from, empty slots, 1 if every inner entry points forward (BFS)}
extern "C" int emu_bvh4_info(const rt_scene_desc *desc, long long *info) {
  rtx::HostScene H;
  std::string err;
  if (rtx::compile_scene(desc, H, err) != RT_OK) return -1;
  if (H.device_bvh) rtx::build_world_bvh_host(H);
  if (H.root_is_leaf || H.nodes.empty()) return -2;
  const int d4 = rtx::collapse_bvh4(H.nodes, H.nodes4);
  // leaf entries in depth-first child order, both trees
  std::vector<int> lb, l4;
  std::vector<int> st{0};
  auto walk2 = [&](auto &&self, int n) -> void {
    for (int k = 0; k < 2; ++k) {
      const int e = H.nodes[n].entry[k];
      if (e >= 0) self(self, e);
      else lb.push_back(e);
    }
  };
  walk2(walk2, 0);
  long long empty = 0, forward = 1;
  auto walk4 = [&](auto &&self, int n) -> void {
    for (int k = 0; k < 4; ++k) {
      const int e = H.nodes4[n].entry[k];
      if (e == -1) ++empty;
      else if (e >= 0) {
        if (e <= n) forward = 0;
        self(self, e);
      } else l4.push_back(e);
    }
  };
  walk4(walk4, 0);
  // every child box of a 4-wide node is a child box of some binary node
  std::vector<std::array<float, 6>> bb;
  for (const DNode &n : H.nodes) {
    bb.push_back({n.lo[0][0], n.lo[1][0], n.lo[2][0], n.hi[0][0], n.hi[1][0], n.hi[2][0]});
    bb.push_back({n.lo[0][1], n.lo[1][1], n.lo[2][1], n.hi[0][1], n.hi[1][1], n.hi[2][1]});
  }
  std::sort(bb.begin(), bb.end());
  long long foreign = 0;
  for (const DNode4 &q : H.nodes4)
    for (int k = 0; k < 4; ++k)
      if (q.entry[k] != -1) {
        std::array<float, 6> b{q.lo[0][k], q.lo[1][k], q.lo[2][k], q.hi[0][k], q.hi[1][k], q.hi[2][k]};
        foreign += !std::binary_search(bb.begin(), bb.end(), b);
      }
  info[0] = (long long)H.nodes.size();
  info[1] = (long long)H.nodes4.size();
  info[2] = H.bvh_depth;
  info[3] = d4;
  info[4] = (long long)lb.size();
  info[5] = (long long)l4.size();
  info[6] = lb == l4;
  info[7] = foreign;
  info[8] = empty;
  info[9] = forward;
  return 0;
}

// sincos_2pi over n uniforms (its accuracy test, tests/test_emulator.py)
extern "C" void emu_sincos_2pi(const double *u, int n, double *s, double *c) {
  for (int k = 0; k < n; ++k) rtp::sincos_2pi(u[k], s[k], c[k]);
}

// sin_n (the noise texture's sin) over n arguments (its accuracy test,
// tests/test_emulator.py)
extern "C" void emu_sin_n(const double *x, int n, double *s) {
  for (int k = 0; k < n; ++k) s[k] = rtp::sin_n(x[k]);
}

// div_mk (Markstein quotient from a shared reciprocal) over n operand pairs
// (its bit-exactness test, tests/test_emulator.py)
extern "C" void emu_div_mk(const double *x, const double *b, int n, double *q) {
  for (int k = 0; k < n; ++k) q[k] = rtp::div_mk(x[k], b[k], 1.0 / b[k]);
}

// Conservativeness of the kernel's fp32 slab tests (tests/test_emulator.py):
// for n rays (o, d: 3 doubles each) against n boxes (lo, hi: 3 floats each) and
// windows [tmin, tmax] (floats), out[k] = 1 if the subtract-form test passes,
// | 2 if the FMA-form test passes.
extern "C" void emu_slab(const double *o, const double *d, const float *lo, const float *hi,
                         const float *tmin, const float *tmax, int n, int *out) {
  for (int k = 0; k < n; ++k) {
    rtp::Ray r;
    r.o = rtp::v3(o[3 * k], o[3 * k + 1], o[3 * k + 2]);
    r.d = rtp::v3(d[3 * k], d[3 * k + 1], d[3 * k + 2]);
    r.tm = 0.0;
    const rtp::RayF<false> qs = rtp::ray_f32<false>(r);
    const rtp::RayF<true> qf = rtp::ray_f32<true>(r);
    const float inf = __builtin_huge_valf();
    int v = 0;
    if (rtp::slab<false>(qs, lo + 3 * k, hi + 3 * k, tmin[k], tmax[k]) != inf) v |= 1;
    if (rtp::slab<true>(qf, lo + 3 * k, hi + 3 * k, tmin[k], tmax[k]) != inf) v |= 2;
    out[k] = v;
  }
}

// The axis-aligned quad formulas against the full Plane::hit formulas
// (tests/test_emulator.py): the world's quads of `desc` (compiled by the
// library's scene compiler, which sets DQuad::aa) against n rays (o, d: 3
// doubles each) on [tmin, tmax]; out[4k..4k+3] = (hit, t) of quad_t on the quad
// as compiled and (hit, t) with aa cleared, for quad k % n_quads.
extern "C" int emu_quad_forms(const rt_scene_desc *desc, const double *o, const double *d,
                              double tmin, double tmax, int n, double *out, int *n_aa) {
  rtx::HostScene H;
  std::string err;
  if (rtx::compile_scene(desc, H, err) != RT_OK || H.quads.empty()) return -1;
  *n_aa = 0;
  for (const DQuad &q : H.quads) *n_aa += q.aa >= 0;
  for (int k = 0; k < n; ++k) {
    const DQuad &q = H.quads[k % H.quads.size()];
    DQuad g = q;
    g.aa = -1;
    rtp::Ray r;
    r.o = rtp::v3(o[3 * k], o[3 * k + 1], o[3 * k + 2]);
    r.d = rtp::v3(d[3 * k], d[3 * k + 1], d[3 * k + 2]);
    r.tm = 0.0;
    double t0 = 0, t1 = 0;
    const bool h0 = rtp::quad_t(q, r, tmin, tmax, t0);
    const bool h1 = rtp::quad_t(g, r, tmin, tmax, t1);
    out[4 * k] = h0;
    out[4 * k + 1] = h0 ? t0 : 0.0;
    out[4 * k + 2] = h1;
    out[4 * k + 3] = h1 ? t1 : 0.0;
  }
  return 0;
}

// Both boundary queries of ConstantMedium::hit for medium m (index into the
// compiled media, in scene order) on n medium-frame rays (x, y, z, dx, dy, dz,
// time), through the kernel source's box_span (make_box boundaries) and its
// general boundary_span.  out per ray: box_span's code (1 span, 0 none, -1
// deferred, -2 not a box), its t1, t2, then boundary_span's result (1 / 0), t1, t2.
extern "C" int emu_medium_spans(const rt_scene_desc *desc, int m, const double *rays, int n,
                                double *out) {
  rtx::HostScene H;
  std::string err;
  if (rtx::compile_scene(desc, H, err) != RT_OK) return -1;
  if (m < 0 || m >= (int)H.media.size()) return -2;
  DScene S{};
  S.bitems = H.bitems.data();
  S.xforms = H.xforms.data();
  S.spheres = H.spheres.data();
  S.quads = H.quads.data();
  S.media = H.media.data();
  const DMedium &M = H.media[m];
  for (int k = 0; k < n; ++k) {
    const double *q = rays + 7 * k;
    Ray r{v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), q[6]};
    double *o = out + 6 * k;
    double a1 = 0, a2 = 0, g1 = 0, g2 = 0;
    const int rc = M.box ? box_span(S, M, r, a1, a2) : -2;
    const bool g = boundary_span(S, M, r, g1, g2);
    o[0] = rc;
    o[1] = rc == 1 ? a1 : 0.0;
    o[2] = rc == 1 ? a2 : 0.0;
    o[3] = g ? 1.0 : 0.0;
    o[4] = g ? g1 : 0.0;
    o[5] = g ? g2 : 0.0;
  }
  return 0;
}
