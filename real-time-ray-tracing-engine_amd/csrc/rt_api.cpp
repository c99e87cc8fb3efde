// rt_api.cpp — implementation of include/rt_api.h on the HIP runtime.
//
// Ownership model (replaces the reference's singleton CudaSceneContext with its
// __device__ d_scene_context symbol, CudaSceneContext.cuh:25-181 / .cu:9-38):
// every rt_scene owns one device allocation holding all of its tables, a HIP
// stream, two timing events and a lazily grown output buffer.  Nothing is global,
// so several scenes (and several devices) coexist.  Errors never exit() or throw
// across the ABI: they return a negative code and set a thread-local message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_layout.h"
#include "rt_scene.h"

extern "C" hipError_t rtk_launch_render(const DScene *S, const DCamera *C, const DLaunch *P,
                                        double *out, unsigned long long *stats,
                                        hipStream_t stream);
extern "C" hipError_t rtk_lds_plan(int features, int stack_depth, int lds_cap, RtkLdsPlan *plan);
extern "C" hipError_t rtk_lds_plan_pc(int features, int stack_depth, int force_waves, int *pcw,
                                      int64_t *free_bytes,
                                      int *blocks_per_cu);
extern "C" int rtk_lds_prims_enabled(void);
extern "C" int rtk_lds_perlin_enabled(void);
extern "C" size_t rtk_lbvh_temp_bytes(int n);
extern "C" size_t rtk_sah_temp_bytes(int n);
extern "C" hipError_t rtk_build_sah(const double *boxes, const DItem *items_in, int n,
                                    DNode *nodes, DItem *items_out, void *temp,
                                    size_t temp_bytes, int stack_budget, int *n_nodes,
                                    int *depth, int *root_leaf, hipStream_t st);
extern "C" hipError_t rtk_build_lbvh(const double *boxes, const DItem *items_in, int n,
                                     const double *scene_lo, const double *scene_hi,
                                     DNode *nodes, DItem *items_out, int *depth_dev, void *temp,
                                     size_t temp_bytes, hipStream_t st);
extern "C" hipError_t rtk_launch_render_chunked(const DScene *S, const DCamera *C,
                                                const DLaunch *P, int n_head, int head_chunks,
                                                int n_chunks, double *out, double *scratch,
                                                hipStream_t stream);
extern "C" hipError_t rtk_launch_to_bytes(const double *rgb, int64_t n, double scale,
                                          uint8_t *bytes, hipStream_t stream);
extern "C" hipError_t rtk_launch_tiles_sum(const double *parts, int64_t n_tiles, int chunks, double *out,
                                           hipStream_t stream);
extern "C" int rtk_cost_f(int features);
extern "C" hipError_t rtk_launch_tile_order(const uint32_t *cost, int n, int n_head, int32_t *order,
                                            hipStream_t stream);
extern "C" hipError_t rtk_launch_shard_finish(const double *parts, int n_local, int n_head, int head_chunks,
                                              int n_chunks, const int32_t *order, double *out,
                                              hipStream_t stream);
extern "C" hipError_t rtk_launch_tiles_to_frame(const double *tiles, int n_shards, int64_t shard_stride,
                                                int W, int row_begin, int row_end, double scale, int scaled,
                                                int accumulate, double *out, hipStream_t stream);

struct rt_scene {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  char *block = nullptr; // all scene tables
  size_t block_bytes = 0;
  DScene ds;
  rt_scene_info info;
  double *out_buf = nullptr; // rt_render staging
  size_t out_bytes = 0;
  unsigned long long *stats = nullptr;
  int32_t *unit_ctr = nullptr; // work-unit counter of persistent launches (scene block)
  double *scratch = nullptr; // chunk partials of chunked frame launches
  size_t scratch_bytes = 0;
  double *probe_buf = nullptr; // output of the tile-order probe (tile_order_probe)
  size_t probe_bytes = 0;
  int wave_slots = 0;        // resident waves of the render instance on this device
  int pc_grid = 0;           // resident blocks of the persistent instance on this device
  double binary_cost = -1.0; // SAH cost of the binary tree when the device holds the 4-wide one
  rt_tuning tune{};          // explicit tuning (rt_scene_create_tuned; zero: the default plan)
  // cost-ordered dispatch ("tile order", launch()): per-tile unit costs
  // measured by the shape's probe launch (or, in the launches that measure
  // their own, by the last launch) and two order buffers: the one a launch
  // reads, the one the sort after a measuring launch writes for the next
  // ... one slot per launch shape (signature), least recently used replaced:
  // a scene that alternates tile subsets (several ranks' shares on one
  // device) keeps an order for each instead of probing one slot again
  struct OrderSlot {
    uint32_t *tile_cost = nullptr;
    int32_t *tile_order[2] = {nullptr, nullptr};
    int cap = 0, cur = 0;
    bool ready = false;
    int32_t sig[10] = {};
    uint64_t used = 0; // launch counter at the slot's last use
  };
  static constexpr int kOrderSlots = 4;
  OrderSlot order[kOrderSlots];
  uint64_t order_clock = 0;
  // The scene's launches form one chain across streams: `last` is recorded
  // after each call's last kernel on its stream, and a launch on another
  // stream first waits for it (order_after_last) -- the launches share the
  // work-unit counter, the scratch and the order slots, so two of them must
  // never overlap, whichever streams the caller passes.  The last launch's
  // completion therefore implies all earlier ones': destroy and buffer growth
  // wait for `last` and the scene's own stream -- not for the whole device.
  hipEvent_t last = nullptr;
  hipStream_t last_st = nullptr;
  bool has_last = false;
};

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &m) {
  g_err = m;
  return code;
}

int hip_err(hipError_t e, const char *what) {
  return set_err(RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard { // restore the caller's current device
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Scene memory is stream-ordered: hipMallocFromPoolAsync / hipFreeAsync on the
// scene's own stream.  A plain hipFree -- and hipFreeAsync of hipMalloc'd memory --
// waits for every stream of the device (tools/free_probe.hip on gfx950: 300 ms
// behind another stream's 300 ms kernel); hipFreeAsync of pool memory returns
// at once.  So destroying or growing one scene waits only for that scene's own
// work (wait_scene), never for other scenes or threads on the device.
// The allocations come from the library's own pool on the scene's device,
// which keeps freed memory reserved for the next scene or buffer (release
// threshold UINT64_MAX): with the device's default pool (threshold 0) the
// synchronisation after the frees handed the memory back to the system and
// waited for the whole device to do so (tests/test_scene_lifetime.py: a
// destroy waited out another scene's 300 ms render that way).
hipMemPool_t scene_pool(int device) {
  static std::mutex mu;
  static std::vector<hipMemPool_t> pools;
  std::lock_guard<std::mutex> lock(mu);
  if ((int)pools.size() <= device) pools.resize(device + 1, nullptr);
  if (!pools[device]) {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) return nullptr;
    uint64_t keep = ~0ull;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    pools[device] = pool;
  }
  return pools[device];
}
// A destroyed scene's buffers, idle (the destroy waited for the scene's last
// launch) but not yet freed: destroy enqueues nothing on any stream, since a
// HIP stream may share one of the device's few hardware queues
// (GPU_MAX_HW_QUEUES) with another scene's busy stream, and anything queued
// behind that stream's kernel -- a free, a synchronisation -- waits for it
// (tests/test_scene_lifetime.py measured exactly that).  The next allocation
// on the device frees them on its own stream, stream-ordered, before it
// allocates; what no later allocation reaps is released at process exit.
struct Graveyard {
  std::mutex mu;
  std::vector<std::pair<int, void *>> ptrs; // (device, pool allocation)
};
Graveyard &graveyard() {
  static Graveyard *g = new Graveyard(); // never destroyed: usable from any static destructor
  return *g;
}
template <class T>
void bury(rt_scene *s, T *&p) {
  if (p) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> lock(g.mu);
    g.ptrs.emplace_back(s->device, (void *)p);
  }
  p = nullptr;
}
void reap(rt_scene *s) {
  Graveyard &g = graveyard();
  std::lock_guard<std::mutex> lock(g.mu);
  auto keep = g.ptrs.begin();
  for (auto &e : g.ptrs) {
    if (e.first == s->device) (void)hipFreeAsync(e.second, s->stream);
    else *keep++ = e;
  }
  g.ptrs.erase(keep, g.ptrs.end());
}
hipError_t scene_alloc(rt_scene *s, void **p, size_t bytes) {
  *p = nullptr;
  reap(s); // earlier scenes' idle buffers back into the pool first
  hipMemPool_t pool = scene_pool(s->device);
  if (!pool) return hipErrorOutOfMemory;
  hipError_t e = hipMallocFromPoolAsync(p, std::max<size_t>(bytes, 1), pool, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream); // usable from any stream from here on
  if (e != hipSuccess) *p = nullptr;
  return e;
}
template <class T>
void scene_free(rt_scene *s, T *&p) { // after wait_scene: nothing still reads p
  if (p) (void)hipFreeAsync((void *)p, s->stream);
  p = nullptr;
}
hipError_t upload(rt_scene *s, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s->stream);
  return e == hipSuccess ? hipStreamSynchronize(s->stream) : e;
}
// everything this scene has launched has completed: its own stream, and its
// last launch (which every earlier launch precedes: order_after_last)
void wait_scene(rt_scene *s) {
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->has_last) (void)hipEventSynchronize(s->last);
}
// before a call's first kernel on st: after the scene's previous launch
int order_after_last(rt_scene *s, hipStream_t st) {
  if (!s->has_last || s->last_st == st) return RT_OK;
  hipError_t e = hipStreamWaitEvent(st, s->last, 0);
  return e == hipSuccess ? RT_OK : hip_err(e, "hipStreamWaitEvent");
}
// after a call's last kernel on st
int mark_last(rt_scene *s, hipStream_t st) {
  hipError_t e = hipEventRecord(s->last, st);
  if (e != hipSuccess) return hip_err(e, "hipEventRecord");
  s->last_st = st;
  s->has_last = true;
  return RT_OK;
}

// the shared launch validation (rt_scene.cpp; the CPU backend applies the same)
int to_device_camera(const rt_frame *f, DCamera &c) {
  std::string err;
  int rc = rtx::device_camera(f, c, err);
  return rc ? set_err(rc, err) : RT_OK;
}

int to_launch(const rt_frame *f, const rt_render_params *p, DLaunch &L) {
  std::string err;
  int rc = rtx::launch_geometry(f, p, L, err);
  return rc ? set_err(rc, err) : RT_OK;
}

// doubles an output of this launch covers
size_t out_doubles(const rt_frame *f, const DLaunch &L) {
  if (L.compact) return (size_t)L.n_local_tiles * L.n_chunks * 64 * 3;
  return (size_t)f->image_width * (L.row_end - L.row_begin) * 3;
}

} // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char *rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(int32_t *count) {
  if (!count) return set_err(RT_ERR_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return hip_err(e, "hipGetDeviceCount");
  }
  *count = n;
  return RT_OK;
}

int rt_camera_setup(const rt_camera_desc *camera, rt_frame *frame) {
  std::string err;
  int rc = rtx::camera_setup(camera, frame, err);
  if (rc != RT_OK) return set_err(rc, err);
  return RT_OK;
}

// Builds the world BVH on the device over the scene's world items (uploaded in
// scene order at `items`): the binned-SAH builder (rt_bvh_sah.hip) or the linear
// BVH (rt_bvh_build.hip); writes the nodes and the items in leaf order in place.
// Depth at which the device SAH builder switches to balanced splits (the host
// builder's force_median bound); rt_tuning.sah_stack_budget lowers it in tests.
static int sah_stack_budget(const rt_tuning &t) {
  int b = RT_STACK_DEPTH - 2;
  if (t.sah_stack_budget > 0) b = std::max(1, std::min(b, (int)t.sah_stack_budget));
  return b;
}
struct DeviceTree {
  int n_nodes = 0, depth = -1, root_leaf = 0;
};
static hipError_t device_bvh_build(rt_scene *s, const rtx::HostScene &H, DNode *nodes,
                                   DItem *items, DeviceTree &tree) {
  const int n = (int)H.items.size();
  const bool sah = H.device_bvh == RT_BVH_DEVICE_SAH;
  const size_t a_box = (6 * sizeof(double) * n + 255) & ~size_t(255);
  const size_t a_items = (sizeof(DItem) * n + 255) & ~size_t(255);
  const size_t lb = sah ? rtk_sah_temp_bytes(n) : rtk_lbvh_temp_bytes(n);
  const size_t total = a_box + a_items + 256 + lb;
  char *tmp = nullptr;
  hipError_t e = scene_alloc(s, (void **)&tmp, total);
  if (e != hipSuccess) return e;
  double *d_box = (double *)tmp;
  DItem *d_sorted = (DItem *)(tmp + a_box);
  int *d_depth = (int *)(tmp + a_box + a_items);
  void *d_lb = tmp + a_box + a_items + 256;
  e = hipMemcpyAsync(d_box, H.item_boxes.data(), 6 * sizeof(double) * n, hipMemcpyHostToDevice,
                     s->stream);
  if (sah) {
    if (e == hipSuccess)
      e = rtk_build_sah(d_box, items, n, nodes, d_sorted, d_lb, lb, sah_stack_budget(s->tune),
                        &tree.n_nodes, &tree.depth, &tree.root_leaf, s->stream);
  } else {
    tree.n_nodes = n - 1;
    if (e == hipSuccess)
      e = rtk_build_lbvh(d_box, items, n, H.scene_lo, H.scene_hi, nodes, d_sorted, d_depth, d_lb,
                         lb, s->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(&tree.depth, d_depth, sizeof(int), hipMemcpyDeviceToHost, s->stream);
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(items, d_sorted, sizeof(DItem) * n, hipMemcpyDeviceToDevice, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) (void)hipStreamSynchronize(s->stream); // nothing may still use tmp
  scene_free(s, tmp);
  return e;
}

int rt_scene_create(const rt_scene_desc *desc, int32_t device, rt_scene **out) {
  return rt_scene_create_tuned(desc, device, nullptr, out);
}

int rt_scene_create_tuned(const rt_scene_desc *desc, int32_t device, const rt_tuning *tuning,
                          rt_scene **out) {
  if (!out) return set_err(RT_ERR_INVALID, "null output pointer");
  *out = nullptr;
  rt_tuning tune{};
  if (tuning) tune = *tuning;
  rtx::HostScene H;
  H.sah_leaf_max = tune.sah_leaf_max;
  H.sah_leaf_split = tune.sah_leaf_split;
  H.sah_trav_x4 = tune.sah_trav_x4;
  H.sah_bins = tune.sah_bins;
  std::string err;
  int rc = rtx::compile_scene(desc, H, err);
  if (rc != RT_OK) return set_err(rc, err);
  // the compacted leaf tests pack (item << 6 | lane) into an int (rt_path.h leaf_share)
  if (H.items.size() >= ((size_t)1 << 25))
    return set_err(RT_ERR_UNSUPPORTED, "more than 2^25 - 1 world primitives");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_err(e, "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return set_err(RT_ERR_INVALID, "device index out of range");
  DeviceGuard g(device);

  // one allocation, 256-B aligned sub-ranges
  struct Part {
    const void *src;
    size_t bytes;
    size_t off;
  };
  std::vector<Part> parts;
  size_t off = 0;
  auto add = [&](const void *src, size_t bytes, size_t reserve = 0) {
    parts.push_back(Part{src, bytes, off});
    reserve = std::max(reserve, bytes);
    off += align256(reserve ? reserve : 1);
    return parts.size() - 1;
  };
  // 4-wide world BVH (RT_FEAT_BVH4): asked for, or automatic from kBvh4Min
  // primitives; collapsed from the binary tree once that exists (host or device
  // build) into the node range, which is sized for it (<= one 4-wide node per
  // binary node)
  const int arity_req = desc->bvh_arity;
  const bool want4 = arity_req == 4 || (arity_req == 0 && H.items.size() >= (size_t)rtx::kBvh4Min);
  size_t iN = add(H.device_bvh ? nullptr : H.nodes.data(),
                  H.device_bvh ? 0 : H.nodes.size() * sizeof(DNode),
                  H.nodes.size() * (want4 ? sizeof(DNode4) : sizeof(DNode)));
  size_t iI = add(H.items.data(), H.items.size() * sizeof(DItem));
  size_t iB = add(H.bitems.data(), H.bitems.size() * sizeof(DItem));
  size_t iMI = add(H.mitems.data(), H.mitems.size() * sizeof(DItem));
  size_t iMB = add(H.mbox.data(), H.mbox.size() * sizeof(float));
  size_t iX = add(H.xforms.data(), H.xforms.size() * sizeof(DXform));
  size_t iS = add(H.spheres.data(), H.spheres.size() * sizeof(DSphere));
  size_t iQ = add(H.quads.data(), H.quads.size() * sizeof(DQuad));
  size_t iM = add(H.media.data(), H.media.size() * sizeof(DMedium));
  size_t iMa = add(H.mats.data(), H.mats.size() * sizeof(DMat));
  size_t iTx = add(H.texs.data(), H.texs.size() * sizeof(DTex));
  size_t iP = add(H.perlin.data(), H.perlin.size() * sizeof(DPerlin));
  size_t iLi = add(H.lights.data(), H.lights.size() * sizeof(DLight));
  size_t iSt = add(nullptr, RT_N_STATS * sizeof(unsigned long long));
  size_t iUc = add(nullptr, sizeof(int32_t));

  rt_scene *s = new rt_scene();
  s->device = device;
  s->tune = tune;
  s->block_bytes = off;
  if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreate(&s->ev0)) != hipSuccess || (e = hipEventCreate(&s->ev1)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&s->last, hipEventDisableTiming)) != hipSuccess) {
    rt_scene_destroy(s);
    return hip_err(e, "stream/event create");
  }
  e = scene_alloc(s, (void **)&s->block, off);
  if (e != hipSuccess) {
    rt_scene_destroy(s);
    return set_err(RT_ERR_OOM, std::string("hipMallocFromPoolAsync scene: ") + hipGetErrorString(e));
  }
  for (const Part &p : parts)
    if (p.src && p.bytes) {
      e = upload(s, s->block + p.off, p.src, p.bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        rt_scene_destroy(s);
        return hip_err(e, "upload scene");
      }
    }
  auto P = [&](size_t i) { return (const void *)(s->block + parts[i].off); };
  // with H.nodes holding the final binary tree: collapse and upload the 4-wide
  // one -- kept binary when its stack would not fit RT_STACK_DEPTH4, or when
  // its traversal stacks (three entries per 4-wide level, so a deep or lopsided
  // collapse costs more LDS than the binary walk's one per level) would not fit
  // the 4-wide instance's per-block LDS share at its occupancy target: LDS must
  // never lower occupancy
  auto collapse4 = [&](int features) -> hipError_t {
    if (!want4 || H.root_is_leaf || H.nodes.empty()) return hipSuccess;
    const int d4 = rtx::collapse_bvh4(H.nodes, H.nodes4);
    RtkLdsPlan plan4{};
    hipError_t fe = rtk_lds_plan(features | RT_FEAT_BVH4, rtx::bvh4_stack_depth(d4), tune.lds_cap, &plan4);
    if (fe != hipSuccess) return fe;
    if (rtx::bvh4_stack_depth(d4) > RT_STACK_DEPTH4 || !plan4.stack_fits) {
      H.nodes4.clear();
      return hipSuccess;
    }
    s->binary_cost = rtx::bvh_sah_cost(H.nodes);
    H.bvh_arity = 4;
    H.bvh_depth4 = d4;
    return upload(s, (void *)P(iN), H.nodes4.data(), H.nodes4.size() * sizeof(DNode4),
                  hipMemcpyHostToDevice);
  };
  DScene &d = s->ds;
  d.nodes = (const DNode *)P(iN);
  d.items = (const DItem *)P(iI);
  d.bitems = (const DItem *)P(iB);
  d.mitems = (const DItem *)P(iMI);
  d.mbox = (const float *)P(iMB);
  d.n_mitems = (int32_t)H.mitems.size();
  d.xforms = (const DXform *)P(iX);
  d.spheres = (const DSphere *)P(iS);
  d.quads = (const DQuad *)P(iQ);
  d.media = (const DMedium *)P(iM);
  d.mats = (const DMat *)P(iMa);
  d.texs = (const DTex *)P(iTx);
  d.perlin = (const DPerlin *)P(iP);
  d.lights = (const DLight *)P(iLi);
  d.n_lights = (int32_t)H.lights.size();
  d.n_nodes = (int32_t)H.nodes.size();
  d.root_is_leaf = H.root_is_leaf;
  d.n_root_items = H.n_root_items;
  d.static_spheres = rtx::all_spheres_static(H);
  d.features = rtx::scene_features(H);
  d.features |= tune.extra_features & 15; // debug: widen the instance
  // device-built world BVH (rt_bvh_build.hip), host SAH fallback if the linear
  // tree is deeper than the traversal stack
  int builder = RT_BVH_HOST;
  if (H.device_bvh) {
    DeviceTree tree;
    hipError_t be = device_bvh_build(s, H, (DNode *)P(iN), (DItem *)P(iI), tree);
    if (be != hipSuccess) {
      rt_scene_destroy(s);
      return hip_err(be, "device BVH build");
    }
    const int max_depth = tune.lbvh_max_depth > 0 ? (int)tune.lbvh_max_depth : RT_STACK_DEPTH - 1;
    if (tree.depth >= 0 && tree.depth <= max_depth) {
      H.bvh_depth = tree.depth;
      H.nodes.resize(tree.n_nodes); // the device arrays hold the tree; sizes only
      H.root_is_leaf = tree.root_leaf > 0;
      H.n_root_items = tree.root_leaf;
      builder = H.device_bvh;
      if (want4 && !H.root_is_leaf) { // the collapse runs on the host copy
        hipError_t ce = upload(s, H.nodes.data(), P(iN), H.nodes.size() * sizeof(DNode),
                               hipMemcpyDeviceToHost);
        if (ce != hipSuccess) {
          rt_scene_destroy(s);
          return hip_err(ce, "BVH download");
        }
      }
    } else { // too deep for the per-lane stack: rebuild on the host (depth-capped SAH)
      rtx::build_world_bvh_host(H);
      hipError_t ue = upload(s, (void *)P(iN), H.nodes.data(), H.nodes.size() * sizeof(DNode),
                             hipMemcpyHostToDevice);
      if (ue == hipSuccess)
        ue = upload(s, (void *)P(iI), H.items.data(), H.items.size() * sizeof(DItem),
                    hipMemcpyHostToDevice);
      if (ue != hipSuccess) {
        rt_scene_destroy(s);
        return hip_err(ue, "BVH upload");
      }
    }
    d.n_nodes = (int32_t)H.nodes.size();
    d.root_is_leaf = H.root_is_leaf;
    d.n_root_items = H.n_root_items;
  }
  if ((e = collapse4(d.features)) != hipSuccess) {
    rt_scene_destroy(s);
    return hip_err(e, "4-wide BVH upload");
  }
  if (d.root_is_leaf) d.features |= RT_FEAT_FLAT;
  // traversal stack: one entry per BVH level suffices (a pushed entry is the
  // sibling of a node on the current root path; three per level for 4-wide
  // nodes); LDS prefix of the BFS-ordered nodes sized to what the instance's
  // occupancy leaves free
  // the walk pushes without an overflow check (rt_path.h trace): the depth the
  // host sizes the stack from must be the tree's, never clamped below it
  if (H.bvh_depth + 1 > RT_STACK_DEPTH) {
    rt_scene_destroy(s);
    return set_err(RT_ERR_UNSUPPORTED, "world BVH deeper than the traversal stack (" +
                                           std::to_string(H.bvh_depth) + " levels)");
  }
  d.stack_depth = std::max(1, H.bvh_depth + 1);
  if (H.bvh_arity == 4) {
    d.features |= RT_FEAT_BVH4;
    d.n_nodes = (int32_t)H.nodes4.size();
    d.stack_depth = rtx::bvh4_stack_depth(H.bvh_depth4);
  }
  RtkLdsPlan plan{};
  {
    int cus = 0;
    hipError_t be = rtk_lds_plan(d.features, d.stack_depth, tune.lds_cap, &plan);
    if (be == hipSuccess) be = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (be != hipSuccess) {
      rt_scene_destroy(s);
      return set_err(RT_ERR_DEVICE, std::string("hipFuncGetAttributes: ") + hipGetErrorString(be));
    }
    s->wave_slots = cus * 4 * plan.waves_per_simd;
    int budget = plan.n_nodes;
    if (!plan.stack_fits) {
      // the traversal stacks and static LDS exceed the block's share at the
      // occupancy target (a compiler or register change can move that share):
      // stage no nodes and accept fewer resident blocks per CU, as long as
      // one block still fits the 64 KB a block may use without opt-in
      if (plan.fixed_bytes > 64 * 1024) {
        rt_scene_destroy(s);
        return set_err(RT_ERR_UNSUPPORTED, "BVH traversal stacks exceed the per-block LDS limit");
      }
      std::fprintf(stderr,
                   "rtx: traversal stacks need %d B of LDS per block, above the %d B share at %d "
                   "waves/SIMD: no BVH nodes staged, lower occupancy\n",
                   (int)plan.fixed_bytes, (int)plan.block_budget, (int)plan.waves_per_simd);
      budget = 0;
      s->wave_slots = cus * plan.resident_waves_per_cu;
    }
    if (tune.lds_nodes != 0) // A/B experiments, within the plan (< 0: none)
      budget = std::max(0, std::min((int)tune.lds_nodes, plan.n_nodes));
    d.n_lds_nodes = std::max(0, std::min(budget, d.n_nodes));
    // the persistent instance: its node prefix, then -- if the whole tree is
    // staged and room is left -- the world items and spheres (-1: no
    // persistent launches)
    int64_t pc_free = -1;
    int pcw = 0;
    int pc_bpc = 0;
    be = rtk_lds_plan_pc(d.features, d.stack_depth, tune.pc_waves, &pcw, &pc_free, &pc_bpc);
    d.pc_waves = pcw;
    s->pc_grid = cus * pc_bpc;
    if (be != hipSuccess) {
      rt_scene_destroy(s);
      return set_err(RT_ERR_DEVICE, std::string("hipFuncGetAttributes: ") + hipGetErrorString(be));
    }
    const int64_t node_b = RT_LDS_NODE_BYTES(d.features);
    d.n_lds_nodes_pc = pc_free < 0 ? -1 : (int32_t)std::min<int64_t>(pc_free / node_b, d.n_nodes);
    if (tune.lds_nodes_pc != 0 && d.n_lds_nodes_pc >= 0) // A/B experiments, within what the plan leaves free
      d.n_lds_nodes_pc = (int32_t)std::max<int64_t>(
          0, std::min<int64_t>({(int64_t)tune.lds_nodes_pc, d.n_nodes, pc_free / node_b}));
    d.lds_items_pc = d.lds_spheres_pc = 0;
    const int64_t prim_b = (int64_t)(H.items.size() * sizeof(DItem) + H.spheres.size() * sizeof(DSphere));
    if (rtk_lds_prims_enabled() && !tune.no_lds_prims && pc_free >= 0 &&
        d.n_lds_nodes_pc == d.n_nodes && pc_free - (int64_t)d.n_nodes * node_b >= prim_b &&
        !H.items.empty()) {
      d.lds_items_pc = (int32_t)H.items.size();
      d.lds_spheres_pc = (int32_t)H.spheres.size();
    }
  }
  // the one Perlin table of a noise scene in LDS (tune.no_lds_perlin: from
  // HBM, A/B runs and the bit-identity test); several tables stay in HBM
  d.lds_perlin = (d.features & RT_FEAT_NOISE) && H.perlin.size() == 1 && rtk_lds_perlin_enabled() &&
                 !tune.no_lds_perlin;
  s->stats = (unsigned long long *)(s->block + parts[iSt].off);
  s->unit_ctr = (int32_t *)(s->block + parts[iUc].off);

  rt_scene_info &in = s->info;
  std::memset(&in, 0, sizeof in);
  in.n_nodes = d.n_nodes;
  in.n_leaf_refs = (int32_t)H.items.size(); // leaves are item ranges
  in.n_spheres = (int32_t)H.spheres.size();
  in.n_quads = (int32_t)H.quads.size();
  in.n_objects = (int32_t)(H.items.size() + H.mitems.size());
  in.n_light_leaves = (int32_t)H.lights.size();
  in.bvh_depth = H.bvh_depth;
  in.node_bytes = (int32_t)(H.bvh_arity == 4 ? sizeof(DNode4) : sizeof(DNode));
  in.sphere_bytes = (int32_t)sizeof(DSphere);
  in.quad_bytes = (int32_t)sizeof(DQuad);
  in.device_bytes = (int64_t)off;
  in.features = d.features;
  in.lds_nodes = d.n_lds_nodes;
  in.bvh_builder = builder;
  in.bvh_arity = H.bvh_arity;
  in.stack_depth = d.stack_depth;
  in.lds_fixed_bytes = plan.fixed_bytes;
  in.lds_block_budget = plan.block_budget;
  in.waves_per_simd = plan.waves_per_simd;
  in.lds_nodes_persistent = d.n_lds_nodes_pc;
  in.lds_prims_persistent = d.lds_items_pc > 0;
  in.persistent_block_waves = d.pc_waves;
  in.lds_perlin = d.lds_perlin;
  in.lds_node_bytes = RT_LDS_NODE_BYTES(d.features);
  *out = s;
  return RT_OK;
}

int rt_scene_info_get(const rt_scene *s, rt_scene_info *info) {
  if (!s || !info) return set_err(RT_ERR_INVALID, "null argument");
  *info = s->info;
  return RT_OK;
}

int rt_scene_destroy(rt_scene *s) {
  if (!s) return RT_OK;
  DeviceGuard g(s->device);
  // launches on caller streams (rt_render_device) may still read the scene's
  // tables and use its scratch / tile-order buffers: wait for this scene's
  // work -- its stream and its last launch on each caller stream -- and no
  // other (stream-ordered frees, scene_alloc)
  wait_scene(s);
  // ... then hand its buffers to the graveyard (no stream operation here:
  // see Graveyard)
  bury(s, s->out_buf);
  bury(s, s->scratch);
  bury(s, s->probe_buf);
  for (auto &o : s->order) {
    bury(s, o.tile_cost);
    bury(s, o.tile_order[0]);
    bury(s, o.tile_order[1]);
  }
  bury(s, s->block);
  if (s->last) (void)hipEventDestroy(s->last);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
  return RT_OK;
}

// Work units of a frame-layout launch over every tile (SplitPlan): the waves
// should end together, so the launch must end on short units, while every
// unit pays a refill drain at its end (its last paths finish while lanes
// idle) and long units pay it less often.
//  * Frames of more than 4 tiles per resident wave (1080p: 7.9 on 4,096 wave
//    slots) whose head plan keeps the partials within 4 frames: head tiles
//    whole (up to 64 strata: written straight into the frame, C2) or in
//    chunks of 128 strata (C3: 2 per tile), and the last `slots` x
//    rt_tuning.tail_tiles (default 0.25) tiles in 8x finer chunks, the units the
//    waves take last (dispatch / counter order), so the launch ends on a
//    short unit (C2 +3.9 %, C3 +1.2 % over the uniform split;
//    profiles/r03f_ab.log).  Whole 256-strata tiles as C3's head: -9 %
//    (r03e_ab.log, r04b_head_strata_ab.log); chunks of 128 strata measure the
//    same as 64 with half the partial writes (r04b).
//  * Otherwise every tile split, ~RTX_CHUNK_TARGET (default 32) units per
//    wave slot (the round-1 rule), the last tiles again in finer chunks.
// rt_tuning.chunk_target < 0: whole tiles only (tests).
struct SplitPlan {
  int n_head, head_chunks, chunks; // head tiles, their chunks; the tail tiles' chunks
};
static size_t plan_parts(const SplitPlan &sp, int n_local) { // chunk partial records
  return (size_t)(sp.head_chunks > 1 ? (int64_t)sp.n_head * sp.head_chunks : 0) +
         (size_t)(n_local - sp.n_head) * (sp.n_head < n_local ? sp.chunks : 0);
}
static SplitPlan frame_plan(const rt_scene *s, const DLaunch &L) {
  SplitPlan sp{L.n_local_tiles, 1, 1};
  if (L.compact || L.tile_stride != 1 || L.tile_first != 0 || L.sample_count < 2) return sp;
  const rt_tuning &tu = s->tune;
  const int target = tu.chunk_target == 0 ? 32 : tu.chunk_target;
  if (target <= 0 || s->wave_slots <= 0) return sp;
  // wave slots of the instance that runs the launch (the persistent one's own
  // residency for the feature sets that have one)
  const int64_t tiles = (int64_t)L.n_local_tiles,
                slots = s->pc_grid > 0 && s->ds.pc_waves > 0 ? (int64_t)s->pc_grid * s->ds.pc_waves : s->wave_slots;
  auto no_empty = [&](int64_t c) { // chunk count with no empty chunks
    c = std::max<int64_t>(1, std::min<int64_t>(c, L.sample_count));
    const int64_t cs = (L.sample_count + c - 1) / c;
    return (int)((L.sample_count + cs - 1) / cs);
  };
  // tail tiles per wave slot: a quarter for the head/tail plan since the head
  // tiles are taken most expensive first (tile order; C2 +0.9 %, C3 +0.2 %,
  // profiles/r05x_ab.log), a half after the uniform split (C4 -1.6 % at a
  // quarter)
  const double tail_ht = tu.tail_tiles == 0.0 ? 0.25 : std::max(0.0, tu.tail_tiles);
  const double tail = tu.tail_tiles == 0.0 ? 0.5 : std::max(0.0, tu.tail_tiles);
  // head units: whole tiles up to 64 strata (C2); beyond, chunks of 128
  // strata (C3: 2 per tile -- as fast as 4 chunks of 64, half the partial
  // writes; whole 256-strata tiles -9 %, profiles/r04b_head_strata_ab.log)
  const int head_max = tu.head_strata > 0 ? (int)tu.head_strata : L.sample_count <= 64 ? 64 : 128;
  const int64_t head_chunks = (L.sample_count + head_max - 1) / head_max;
  const int split = tu.tail_split > 0 ? (int)tu.tail_split : 8; // tail chunks per head chunk
  // partial records of a head/tail plan: bounded by 4 frames (a tail of
  // chunked tiles + head chunks); otherwise the uniform split
  const bool bounded = head_chunks == 1 || head_chunks * tiles <= 4 * tiles;
  if (tiles > 4 * slots && tail > 0 && bounded) {
    const int64_t n_tail = std::min<int64_t>(tiles, std::max<int64_t>(1, (int64_t)(tail_ht * slots)));
    sp.head_chunks = no_empty((L.sample_count + head_max - 1) / head_max);
    sp.chunks = no_empty(split * (int64_t)sp.head_chunks);
    sp.n_head = (int)(tiles - n_tail);
    if (sp.chunks <= 1) sp = SplitPlan{L.n_local_tiles, 1, 1};
    return sp;
  }
  const int64_t c = ((int64_t)target * slots + tiles - 1) / std::max<int64_t>(1, tiles);
  sp.chunks = no_empty(c);
  if (sp.chunks > 1) sp.n_head = 0;
  // ... with the last `slots` x rt_tuning.tail_tiles (default 0.5 here) tiles in `split` times finer
  // chunks when the frame has a tile per wave slot (C4, C5: the uniform
  // units last 15 / 84 ms: C4 +1.7 %, C5 +0.9 %, profiles/r03ae_ab.log;
  // rt_tuning.no_uniform_tail: off, A/B runs)
  if (!tu.no_uniform_tail && sp.chunks > 1 && tiles > slots && tail > 0) {
    const int64_t n_tail = std::min<int64_t>(tiles, std::max<int64_t>(1, (int64_t)(tail * slots)));
    const int tc = no_empty(split * (int64_t)sp.chunks);
    if (tc > sp.chunks && n_tail < tiles) {
      sp.head_chunks = sp.chunks;
      sp.chunks = tc;
      sp.n_head = (int)(tiles - n_tail);
    }
  }
  return sp;
}

// Work units of a tile-subset launch that returns its tiles' sums
// (strata_chunks = RT_CHUNKS_AUTO: one rank's share of a tile-sharded frame).
// A share of more than 4 tiles per wave slot takes the frame plan.  A smaller
// one (an 8-way rank of a 1080p frame: 4,050 tiles on 4,096 slots) cannot
// hand whole tiles to the waves -- the slowest tile would be the launch -- so
// every tile is split into head units of `sub_head_strata` strata, and the
// last sub_tail_permille / 1000 x slots tiles into `sub_tail_split` times
// finer chunks, which the waves take last (dispatch / counter order) so the
// launch ends on short units.  Long units drain less often (a unit ends with
// its last paths finishing while lanes idle), short ones balance the end.
// Defaults from 8-way sweeps on one GPU (profiles/r05n_*, r05o_*): head units
// of 16 x sqrt(strata / 64) strata (C2 16, C3 32, C4 64), a tail of an eighth
// of the slots' tiles in halves of those: against every tile in the rank's
// uniform chunks, C2's share -3 to -8 %, C3's -1.5 %, C4's -0.8 % (a quarter
// then; an eighth since tile order, C2 -3.4 %: profiles/r05x_sim_C2.log).
constexpr int kSubTailSplit = 2, kSubTailPermille = 125;
static SplitPlan subset_plan(const rt_scene *s, const DLaunch &L) {
  SplitPlan sp{L.n_local_tiles, 1, 1};
  if (L.sample_count < 2 || L.n_local_tiles < 1 || s->wave_slots <= 0) return sp;
  const rt_tuning &tu = s->tune;
  const int64_t tiles = (int64_t)L.n_local_tiles,
                slots = s->pc_grid > 0 && s->ds.pc_waves > 0 ? (int64_t)s->pc_grid * s->ds.pc_waves : s->wave_slots;
  if (tiles > 4 * slots) {
    DLaunch F = L;
    F.compact = 0;
    F.tile_first = 0;
    F.tile_stride = 1;
    return frame_plan(s, F);
  }
  auto no_empty = [&](int64_t c) { // chunk count with no empty chunks
    c = std::max<int64_t>(1, std::min<int64_t>(c, L.sample_count));
    const int64_t cs = (L.sample_count + c - 1) / c;
    return (int)((L.sample_count + cs - 1) / cs);
  };
  const int head = tu.sub_head_strata > 0
                       ? tu.sub_head_strata
                       : std::max(1, (int)std::lround(16.0 * std::sqrt(L.sample_count / 64.0)));
  const int split = tu.sub_tail_split > 0 ? tu.sub_tail_split : kSubTailSplit;
  const int permille = tu.sub_tail_permille != 0 ? tu.sub_tail_permille : kSubTailPermille;
  sp.head_chunks = no_empty((L.sample_count + head - 1) / head);
  sp.chunks = sp.head_chunks;
  sp.n_head = (int)tiles;
  if (permille > 0) {
    const int64_t n_tail = std::min<int64_t>(tiles, std::max<int64_t>(1, slots * permille / 1000));
    const int tc = no_empty((int64_t)split * sp.head_chunks);
    if (tc > sp.head_chunks) {
      sp.chunks = tc;
      sp.n_head = (int)(tiles - n_tail);
    }
  }
  if (sp.n_head == 0) sp.head_chunks = 1; // every tile a tail tile
  return sp;
}

static int ensure_scratch(rt_scene *s, size_t bytes) {
  if (s->scratch_bytes >= bytes) return RT_OK;
  if (s->scratch) {
    wait_scene(s); // this scene's launches on any stream may still read it
    scene_free(s, s->scratch);
    s->scratch_bytes = 0;
  }
  hipError_t e = scene_alloc(s, (void **)&s->scratch, bytes);
  if (e != hipSuccess) return set_err(RT_ERR_OOM, std::string("hipMallocFromPoolAsync scratch: ") + hipGetErrorString(e));
  s->scratch_bytes = bytes;
  return RT_OK;
}

// Cost-ordered dispatch ("tile order"): a launch's work units are taken in
// plan order (head units, then the finer tail chunks -- unit index order is
// the dispatcher's and the persistent counter's order), so the launch ends on
// whatever tiles come last.  Tiles differ several-fold in cost (sky vs glass,
// r05t: C2's units 0.2-2.5 ms at one device), and a costly tile met last
// keeps its wave slot busy while the others idle: the one-device C2 frame
// spent 7.7 % of its slot-time idle, an 8-way rank's share 14.5 %.  So the
// first launch of a shape is preceded by a probe that measures its tiles'
// costs (tile_order_probe) and a one-block sort that orders the tiles most
// expensive first (longest processing time first); every launch of the shape
// takes that order: the plan's k-th tile is tile_order[k].  The head tiles are ordered among themselves and
// the tail tiles among themselves (the tail still last), so every tile keeps
// its own split into units -- whole, head chunks or tail chunks -- and so its
// summation grouping: only the schedule moves, and the frames are
// bit-identical with and without it (rt_tuning.no_tile_order,
// tests/test_tile_order.py).  (Ordering across the split, so the cheapest
// tiles became the tail, regrouped those tiles' sums: not bit-identical.)
// The slot of a launch shape: the one holding its signature, else the least
// recently used (its order reset), with room for n tiles.
static int order_slot(rt_scene *s, const int32_t sig[10], int n, rt_scene::OrderSlot *&slot) {
  slot = nullptr;
  for (auto &o : s->order)
    if (o.ready && std::equal(sig, sig + 10, o.sig)) slot = &o;
  if (!slot) {
    slot = &s->order[0];
    for (auto &o : s->order)
      if (o.used < slot->used) slot = &o;
    slot->ready = false;
    std::copy(sig, sig + 10, slot->sig);
  }
  slot->used = ++s->order_clock;
  if (slot->cap >= n) return RT_OK;
  if (slot->tile_cost) wait_scene(s); // this scene's launches on any stream may still use them
  scene_free(s, slot->tile_cost);
  scene_free(s, slot->tile_order[0]);
  scene_free(s, slot->tile_order[1]);
  slot->cap = 0;
  slot->ready = false;
  hipError_t e = scene_alloc(s, (void **)&slot->tile_cost, (size_t)n * sizeof(uint32_t));
  if (e == hipSuccess) e = scene_alloc(s, (void **)&slot->tile_order[0], (size_t)n * sizeof(int32_t));
  if (e == hipSuccess) e = scene_alloc(s, (void **)&slot->tile_order[1], (size_t)n * sizeof(int32_t));
  if (e != hipSuccess) return set_err(RT_ERR_OOM, std::string("hipMallocFromPoolAsync tile order: ") + hipGetErrorString(e));
  slot->cap = n;
  return RT_OK;
}

// The order of a launch shape: one launch of the STATS instance over the same
// tiles -- whole tiles of at most kProbeStrata strata each (rt_tuning
// probe_strata), into a scratch buffer -- adds each tile's duration to the
// slot's cost counters, and the sort orders the plan's head and tail tiles by
// them.  Once per launch shape (order slot); the launches of the shape then
// take the order.  The render instances measure nothing themselves: the cost
// bookkeeping compiled into them cost C4 12.5 % (r05u_ab.log) and C2 / C3 / C5
// 0.9 % (r06y_ab_C*.log), while a once-per-shape order ranks the tiles as well
// as one re-measured after every launch (r06x / r06y).
static int tile_order_probe(rt_scene *s, const DCamera &C, const DLaunch &L, const SplitPlan &sp,
                            rt_scene::OrderSlot *os, hipStream_t st) {
  // 16 strata: C4 +0.2 % over 4 (r06u), C2 +0.6 % / C3 +0.9 % over 4 and 1 (r06aa)
  constexpr int kProbeStrata = 16;
  const size_t bytes = std::max<size_t>(1, (size_t)L.n_local_tiles * 64 * 3) * sizeof(double);
  if (s->probe_bytes < bytes) {
    if (s->probe_buf) wait_scene(s);
    scene_free(s, s->probe_buf);
    s->probe_bytes = 0;
    hipError_t ae = scene_alloc(s, (void **)&s->probe_buf, bytes);
    if (ae != hipSuccess) return set_err(RT_ERR_OOM, std::string("hipMallocFromPoolAsync probe: ") + hipGetErrorString(ae));
    s->probe_bytes = bytes;
  }
  DLaunch Q = L;
  Q.sample_count = std::min(L.sample_count, s->tune.probe_strata > 0 ? s->tune.probe_strata : kProbeStrata);
  Q.output = RT_OUT_SUM;
  Q.accumulate = 0;
  Q.compact = 1;
  Q.n_head = L.n_local_tiles;
  Q.head_chunks = 1;
  Q.n_chunks = 1;
  Q.chunk_strata = Q.sample_count;
  Q.parts = nullptr;
  Q.parts_final = 0;
  Q.unit_ctr = nullptr;
  Q.grid_cap = 0;
  Q.tile_order = nullptr;
  Q.tile_cost = os->tile_cost;
  hipError_t e = hipMemsetAsync(os->tile_cost, 0, (size_t)L.n_local_tiles * sizeof(uint32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(s->stats, 0, RT_N_STATS * sizeof(unsigned long long), st);
  if (e == hipSuccess) e = rtk_launch_render(&s->ds, &C, &Q, s->probe_buf, s->stats, st);
  if (e == hipSuccess)
    e = rtk_launch_tile_order(os->tile_cost, L.n_local_tiles, std::min(sp.n_head, L.n_local_tiles),
                              os->tile_order[os->cur], st);
  if (e != hipSuccess) return hip_err(e, "tile order probe");
  os->ready = true;
  return RT_OK;
}

// forced: the split plan of a tile-layout launch whose whole tiles go to
// dev_out (compact) and split tiles' raw partials to the scene's scratch
// (rt_multi_render's shards, reproducing the one-device frame's units).
// *order_used: the dispatch order the launch used (null: plan order) -- what a
// finish kernel run after it must map the plan's tiles with.
static int launch(rt_scene *s, const DCamera &C, const DLaunch &L, double *dev_out,
                  unsigned long long *stats, hipStream_t st, const SplitPlan *forced = nullptr,
                  const int32_t **order_used = nullptr) {
  if (order_used) *order_used = nullptr;
  const SplitPlan sp = forced ? *forced : stats ? SplitPlan{L.n_local_tiles, 1, 1} : frame_plan(s, L);
  const size_t n_parts = plan_parts(sp, L.n_local_tiles);
  const bool split = !L.compact && n_parts > 0;
  if (split || forced) {
    int rc = ensure_scratch(s, std::max<size_t>(1, n_parts * 64 * 3) * sizeof(double));
    if (rc) return rc;
  }
  // persistent waves pulling work units (rt_tuning.no_persistent: one unit
  // per wave, for A/B runs)
  const bool persistent = !s->tune.no_persistent;
  DLaunch Lp = L;
  if (persistent && s->wave_slots > 0) {
    Lp.unit_ctr = s->unit_ctr;
    Lp.grid_cap = s->pc_grid > 0 ? s->pc_grid // resident persistent blocks
                                 : std::max(1, s->wave_slots / std::max(1, s->ds.pc_waves));
    // rt_tuning.grid_cap: fewer resident blocks (tests: many units per wave)
    if (s->tune.grid_cap > 0) Lp.grid_cap = s->tune.grid_cap;
  }
  // cost-ordered dispatch: frame launches and forced / library plans, not the
  // STATS instance nor a caller's explicit chunk layout (its partials are the
  // output, by plan tile).  Progressive frames too (one stratum per pixel:
  // C4 0.90 -> 0.81 ms per frame, C2 0.222 -> 0.212, r06aa_ab_progressive.log),
  // now that the costs are measured once per shape, not by every launch.
  const bool ordered = !s->tune.no_tile_order && stats == nullptr && (forced || !L.parts_final) &&
                       L.n_local_tiles > 1;
  const int32_t sig[10] = {L.n_local_tiles, L.tile_first, L.tile_stride, L.tiles_x, L.row_begin,
                           L.row_end,       L.sample_count, sp.n_head,   sp.head_chunks, sp.chunks};
  // after the scene's previous launch, whichever stream it ran on
  if (int rc = order_after_last(s, st)) return rc;
  rt_scene::OrderSlot *os = nullptr;
  // The first tile-subset launch of a shape (a multi-GPU rank's share) in the
  // flat world runs in plan order in the COST instance (rt_kernel.hip), which
  // measures its own units, and the sort after it gives the order every later
  // launch of the shape takes in the plain instance: an 8-way C2 share 0.81 ms
  // against 0.85 with the probe's order or with costs re-measured after every
  // launch (r06ag: an order measured under cost order itself ranks worse).
  // Every other shape takes its probe's order.
  // (Frame launches ordered this way measured the same as with the probe:
  // r06ah_first_measure_frames_ab_C2.log.)
  bool kernel_costs = ordered && forced != nullptr && rtk_cost_f(s->ds.features);
  if (ordered) {
    int rc = order_slot(s, sig, L.n_local_tiles, os);
    if (rc) return rc;
    if (os->ready) kernel_costs = false;
    if (!kernel_costs && !os->ready && (rc = tile_order_probe(s, C, L, sp, os, st))) return rc;
    Lp.tile_order = os->ready ? os->tile_order[os->cur] : nullptr;
  } else {
    Lp.tile_order = nullptr;
  }
  Lp.tile_cost = nullptr;
  if (kernel_costs) {
    hipError_t me = hipMemsetAsync(os->tile_cost, 0, (size_t)L.n_local_tiles * sizeof(uint32_t), st);
    if (me != hipSuccess) return hip_err(me, "hipMemsetAsync tile cost");
    Lp.tile_cost = os->tile_cost;
  }
  hipError_t e = hipEventRecord(s->ev0, st);
  if (e != hipSuccess) return hip_err(e, "hipEventRecord");
  if (forced) {
    Lp.n_head = sp.n_head;
    Lp.head_chunks = sp.head_chunks;
    Lp.n_chunks = sp.chunks;
    Lp.chunk_strata = (L.sample_count + sp.chunks - 1) / sp.chunks;
    Lp.parts = s->scratch;
    Lp.parts_final = 0;
  } else if (L.parts_final) {
    Lp.parts = dev_out; // tile layout, strata_chunks > 1: the chunk partials are the output
  }
  e = split ? rtk_launch_render_chunked(&s->ds, &C, &Lp, sp.n_head, sp.head_chunks, sp.chunks, dev_out,
                                        s->scratch, st)
            : rtk_launch_render(&s->ds, &C, &Lp, dev_out, stats, st);
  if (e != hipSuccess) return hip_err(e, "render kernel launch");
  e = hipEventRecord(s->ev1, st);
  if (e != hipSuccess) return hip_err(e, "hipEventRecord");
  s->timed = true;
  if (order_used) *order_used = Lp.tile_order;
  if (kernel_costs) { // the next launch's order, into the buffer this one did not read
    const int next = os->cur ^ 1;
    e = rtk_launch_tile_order(os->tile_cost, L.n_local_tiles, std::min(sp.n_head, L.n_local_tiles),
                              os->tile_order[next], st);
    if (e != hipSuccess) return hip_err(e, "tile order");
    os->cur = next;
    os->ready = true;
  }
  return mark_last(s, st);
}

static int ensure_out(rt_scene *s, size_t bytes) {
  if (s->out_bytes >= bytes) return RT_OK;
  if (s->out_buf) {
    (void)hipStreamSynchronize(s->stream); // only the scene's own stream writes it
    scene_free(s, s->out_buf);
    s->out_bytes = 0;
  }
  hipError_t e = scene_alloc(s, (void **)&s->out_buf, bytes);
  if (e != hipSuccess) return set_err(RT_ERR_OOM, std::string("hipMallocFromPoolAsync output: ") + hipGetErrorString(e));
  s->out_bytes = bytes;
  return RT_OK;
}

int rt_render(rt_scene *s, const rt_frame *f, const rt_render_params *p, double *host_rgb) {
  if (!s || !host_rgb) return set_err(RT_ERR_INVALID, "null argument");
  DCamera C;
  DLaunch L;
  int rc = to_device_camera(f, C);
  if (rc) return rc;
  if ((rc = to_launch(f, p, L))) return rc;
  DeviceGuard g(s->device);
  rt_render_params q = *p;
  q.accumulate = 0;
  L.accumulate = 0;
  size_t n = out_doubles(f, L);
  if ((rc = ensure_out(s, n * sizeof(double)))) return rc;
  if ((rc = launch(s, C, L, s->out_buf, nullptr, s->stream))) return rc;
  hipError_t e = hipMemcpyAsync(host_rgb, s->out_buf, n * sizeof(double), hipMemcpyDeviceToHost,
                                s->stream);
  if (e != hipSuccess) return hip_err(e, "hipMemcpyAsync D2H");
  e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return hip_err(e, "render kernel");
  return RT_OK;
}

int rt_render_device(rt_scene *s, const rt_frame *f, const rt_render_params *p, double *dev_rgb,
                     void *hip_stream) {
  if (!s || !dev_rgb || !p) return set_err(RT_ERR_INVALID, "null argument");
  DCamera C;
  DLaunch L;
  const bool auto_units = p->strata_chunks == RT_CHUNKS_AUTO;
  if (auto_units && (p->layout != RT_LAYOUT_TILES || p->output != RT_OUT_SUM || p->accumulate))
    return set_err(RT_ERR_INVALID, "RT_CHUNKS_AUTO returns raw tile sums: RT_LAYOUT_TILES, "
                                   "RT_OUT_SUM, accumulate 0");
  rt_render_params q = *p;
  if (auto_units) q.strata_chunks = 0;
  int rc = to_device_camera(f, C);
  if (rc) return rc;
  if ((rc = to_launch(f, &q, L))) return rc;
  DeviceGuard g(s->device);
  hipStream_t st = (hipStream_t)hip_stream; // NULL = the HIP null stream (HIP convention)
  if (!auto_units) return launch(s, C, L, dev_rgb, nullptr, st);
  // the subset's own units: whole head tiles straight into dev_rgb, chunk
  // partials into the scratch, added in chunk order into dev_rgb (the
  // rt_multi shards' finish), all on `st`
  const SplitPlan sp = subset_plan(s, L);
  const int32_t *order = nullptr;
  if ((rc = launch(s, C, L, dev_rgb, nullptr, st, &sp, &order))) return rc;
  hipError_t e = rtk_launch_shard_finish(s->scratch, L.n_local_tiles, sp.n_head, sp.head_chunks, sp.chunks,
                                         order, dev_rgb, st);
  if (e != hipSuccess) return hip_err(e, "tile chunk sum");
  return mark_last(s, st); // the chunk sum reads the scratch: the chain ends after it
}

int rt_render_stats(rt_scene *s, const rt_frame *f, const rt_render_params *p,
                    rt_path_stats *stats) {
  if (!s || !stats || !p) return set_err(RT_ERR_INVALID, "null argument");
  DCamera C;
  DLaunch L;
  // RT_CHUNKS_AUTO: the counters of the subset plan's own units
  const bool auto_units = p->strata_chunks == RT_CHUNKS_AUTO && p->layout == RT_LAYOUT_TILES;
  rt_render_params q = *p;
  if (auto_units) q.strata_chunks = 0;
  int rc = to_device_camera(f, C);
  if (rc) return rc;
  if ((rc = to_launch(f, &q, L))) return rc;
  DeviceGuard g(s->device);
  L.accumulate = 0;
  size_t n = out_doubles(f, L);
  if ((rc = ensure_out(s, n * sizeof(double)))) return rc;
  hipError_t e = hipMemsetAsync(s->stats, 0, RT_N_STATS * sizeof(unsigned long long), s->stream);
  if (e != hipSuccess) return hip_err(e, "hipMemsetAsync stats");
  SplitPlan sp{};
  if (auto_units) sp = subset_plan(s, L);
  if ((rc = launch(s, C, L, s->out_buf, s->stats, s->stream, auto_units ? &sp : nullptr))) return rc;
  unsigned long long h[RT_N_STATS];
  e = hipMemcpyAsync(h, s->stats, sizeof h, hipMemcpyDeviceToHost, s->stream);
  if (e != hipSuccess) return hip_err(e, "hipMemcpyAsync stats");
  e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return hip_err(e, "stats kernel");
  stats->samples = h[0];
  stats->segments = h[1];
  stats->node_visits = h[2];
  stats->sphere_tests = h[3];
  stats->quad_tests = h[4];
  stats->other_tests = h[5];
  stats->light_tests = h[6];
  stats->shade_events = h[7];
  stats->wave_trips = h[8];
  stats->wave_node_iters = h[9];
  stats->wave_leaf_iters = h[10];
  stats->wave_shade_iters = h[11];
  stats->cyc_loop = h[12];
  stats->cyc_regen = h[13];
  stats->cyc_trace = h[14];
  stats->cyc_media = h[15];
  stats->cyc_shade = h[16];
  stats->cyc_lights = h[17];
  stats->model_trace_max = h[18];
  stats->model_trace_pair_max = h[19];
  stats->noise_evals = h[20];
  stats->wave_noise_iters = h[21];
  stats->medium_box_tests = h[22];
  stats->medium_box_deferred = h[23];
  return RT_OK;
}

int rt_scene_bvh_cost(const rt_scene *s, double *cost) {
  if (!s || !cost) return set_err(RT_ERR_INVALID, "null argument");
  *cost = 0.0;
  if (s->binary_cost >= 0.0) { // the device holds the 4-wide collapse
    *cost = s->binary_cost;
    return RT_OK;
  }
  const int n = s->ds.n_nodes;
  if (s->ds.root_is_leaf || n <= 0) return RT_OK;
  std::vector<DNode> nodes(n);
  DeviceGuard g(s->device);
  hipError_t e = hipMemcpy(nodes.data(), s->ds.nodes, sizeof(DNode) * n, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_err(e, "hipMemcpy nodes");
  *cost = rtx::bvh_sah_cost(nodes);
  return RT_OK;
}

int rt_last_kernel_ms(rt_scene *s, double *ms) {
  if (!s || !ms) return set_err(RT_ERR_INVALID, "null argument");
  if (!s->timed) return set_err(RT_ERR_INVALID, "no kernel launched yet");
  DeviceGuard g(s->device);
  hipError_t e = hipEventSynchronize(s->ev1);
  if (e != hipSuccess) return hip_err(e, "hipEventSynchronize");
  float t = 0;
  e = hipEventElapsedTime(&t, s->ev0, s->ev1);
  if (e != hipSuccess) return hip_err(e, "hipEventElapsedTime");
  *ms = t;
  return RT_OK;
}

int rt_to_bytes_device(const double *rgb, int64_t n, double scale, uint8_t *bytes,
                       void *hip_stream) {
  if (!rgb || !bytes || n < 0) return set_err(RT_ERR_INVALID, "invalid argument");
  hipError_t e = rtk_launch_to_bytes(rgb, n, scale, bytes, (hipStream_t)hip_stream);
  if (e != hipSuccess) return hip_err(e, "to_bytes launch");
  return RT_OK;
}

// ---------------------------------------------------------------- tile exchange
int rt_tiles_sum_device(const double *parts, int64_t n_tiles, int32_t chunks, double *device_tiles,
                        void *hip_stream) {
  if (!parts || !device_tiles || n_tiles < 0 || chunks < 1) return set_err(RT_ERR_INVALID, "invalid argument");
  if (parts == device_tiles && chunks > 1) return set_err(RT_ERR_INVALID, "parts and tiles must not alias");
  hipError_t e = rtk_launch_tiles_sum(parts, n_tiles, chunks, device_tiles, (hipStream_t)hip_stream);
  if (e != hipSuccess) return hip_err(e, "tiles_sum launch");
  return RT_OK;
}

int rt_tiles_to_frame_device(const double *device_tiles, int32_t n_shards, int64_t shard_stride,
                             const rt_frame *f, const rt_render_params *p, double *device_rgb,
                             void *hip_stream) {
  if (!device_tiles || !device_rgb || !f || !p || n_shards < 1)
    return set_err(RT_ERR_INVALID, "invalid argument");
  DLaunch L;
  int rc = to_launch(f, p, L);
  if (rc) return rc;
  const int64_t n_tiles = (int64_t)L.tiles_x * L.tiles_y;
  if (shard_stride < (n_tiles + n_shards - 1) / n_shards)
    return set_err(RT_ERR_INVALID, "shard_stride below the tiles of one shard");
  hipError_t e = rtk_launch_tiles_to_frame(device_tiles, n_shards, shard_stride, f->image_width, L.row_begin,
                                           L.row_end, f->pixel_samples_scale, p->output == RT_OUT_SCALED,
                                           p->accumulate, device_rgb, (hipStream_t)hip_stream);
  if (e != hipSuccess) return hip_err(e, "tiles_to_frame launch");
  return RT_OK;
}

// ---------------------------------------------------------------- multi-device
// One rt_scene per shard, one host thread per shard (StaticCamera::render_gpu's
// single-device loop, StaticCamera.cpp:136-313, spread over N devices).  Shard
// k renders tiles k, k+N, k+2N, ... in the compact tile layout and finishes
// them on its own device (shard_finish_kernel: chunk partials added in chunk
// order -- split_sum_kernel's order); the compact tiles travel device to
// device (xGMI peer copies) into a staging buffer on shard 0's device, where
// tiles_to_frame_kernel reorders them into the frame, copied to the host once.
// With the frame launch's chunk split the frame is bit-identical to rt_render
// on one device.
struct rt_multi {
  std::vector<rt_scene *> scenes; // one per shard; scenes[0]'s device is the root
  std::vector<double> ms;
  double gather_ms = 0.0;
  double *stage = nullptr; // root device: [shard][stride tiles][64][3]
  size_t stage_bytes = 0;
  double *frame = nullptr; // root device: the assembled rows
  size_t frame_bytes = 0;
};

int rt_multi_destroy(rt_multi *m) {
  if (!m) return RT_OK;
  if (!m->scenes.empty() && m->scenes[0]) {
    DeviceGuard g(m->scenes[0]->device);
    for (rt_scene *s : m->scenes)
      if (s) {
        DeviceGuard gs(s->device);
        (void)hipStreamSynchronize(s->stream);
      }
    bury(m->scenes[0], m->stage); // idle: every shard stream was synchronised above
    bury(m->scenes[0], m->frame);
  }
  for (rt_scene *s : m->scenes) rt_scene_destroy(s);
  delete m;
  return RT_OK;
}

int rt_multi_create(const rt_scene_desc *desc, const int32_t *devices, int32_t n_devices,
                    int32_t n_shards, rt_multi **out) {
  return rt_multi_create_tuned(desc, devices, n_devices, n_shards, nullptr, out);
}

int rt_multi_create_tuned(const rt_scene_desc *desc, const int32_t *devices, int32_t n_devices,
                          int32_t n_shards, const rt_tuning *tuning, rt_multi **out) {
  if (!out || !desc || !devices) return set_err(RT_ERR_INVALID, "null argument");
  *out = nullptr;
  if (n_devices < 1 || n_shards < n_devices)
    return set_err(RT_ERR_INVALID, "need n_devices >= 1 and n_shards >= n_devices");
  if (n_shards > RT_MULTI_MAX_SHARDS) // each shard holds a device scene copy and a host thread
    return set_err(RT_ERR_INVALID, "n_shards exceeds RT_MULTI_MAX_SHARDS");
  rt_multi *m = new (std::nothrow) rt_multi();
  if (!m) return set_err(RT_ERR_OOM, "host allocation");
  std::vector<int> rc(n_shards, RT_OK);
  std::vector<std::string> err(n_shards);
  try {
    m->scenes.assign(n_shards, nullptr);
    m->ms.assign(n_shards, 0.0);
    std::vector<std::thread> th;
    try {
      for (int k = 0; k < n_shards; ++k)
        th.emplace_back([&, k]() {
          rc[k] = rt_scene_create_tuned(desc, devices[k % n_devices], tuning, &m->scenes[k]);
          if (rc[k] != RT_OK) err[k] = g_err; // thread-local message of this worker
        });
    } catch (const std::exception &ex) { // thread creation failed: join the started ones
      for (auto &t : th) t.join();
      rt_multi_destroy(m);
      return set_err(RT_ERR_DEVICE, std::string("shard thread: ") + ex.what());
    }
    for (auto &t : th) t.join();
  } catch (const std::exception &ex) { // host allocation inside the containers
    rt_multi_destroy(m);
    return set_err(RT_ERR_OOM, std::string("rt_multi_create: ") + ex.what());
  }
  for (int k = 0; k < n_shards; ++k)
    if (rc[k] != RT_OK) {
      rt_multi_destroy(m);
      return set_err(rc[k], "shard " + std::to_string(k) + ": " + err[k]);
    }
  // direct xGMI access from every shard device to the root's memory (where
  // the peer copies land); without it hipMemcpyPeerAsync stages through the host
  const int root = devices[0];
  for (int d = 1; d < n_devices && d < n_shards; ++d) {
    if (devices[d] == root) continue;
    int can = 0;
    const hipError_t ce = hipDeviceCanAccessPeer(&can, devices[d], root);
    if (ce != hipSuccess) (void)hipGetLastError();
    if (ce == hipSuccess && can) {
      DeviceGuard g(devices[d]);
      const hipError_t e = hipDeviceEnablePeerAccess(root, 0);
      // any failure (already enabled or not) leaves no direct peer access to
      // rely on: the peer copies then stage through the host.  Clear the
      // thread's last error so the first multi frame's launch checks do not
      // report it.
      if (e != hipSuccess) {
        (void)hipGetLastError();
        if (e != hipErrorPeerAccessAlreadyEnabled)
          fprintf(stderr, "rt_multi_create: no peer access from device %d to %d (%s); "
                          "peer copies stage through the host\n",
                  devices[d], root, hipGetErrorString(e));
      }
    }
  }
  *out = m;
  return RT_OK;
}

// One shard of rt_multi_render: the tiles t = first + k * stride in the tile
// layout with the one-device frame's split plan -- tiles below plan.n_head
// (global index) as head units, the rest as tail chunks -- raw sums, finished
// on the shard's device into its compact tiles [k][64][3] (whole head tiles
// by their own units, chunked tiles by shard_finish_kernel), then copied into
// the root's staging slot `dst`.  *t_done: host clock (ms) when the render and
// finish kernels had completed.
static int render_shard(rt_scene *s, const rt_frame *f, const rt_render_params *p, int first, int stride,
                        const SplitPlan &plan, double *dst, int root_dev, double *t_done) {
  DCamera C;
  DLaunch L;
  rt_render_params q = *p;
  q.tile_first = first;
  q.tile_stride = stride;
  q.layout = RT_LAYOUT_TILES;
  q.strata_chunks = 0;
  q.output = RT_OUT_SUM;
  q.accumulate = 0;
  int rc = to_device_camera(f, C);
  if (rc) return rc;
  if ((rc = to_launch(f, &q, L))) return rc;
  SplitPlan sp = plan;
  sp.n_head = plan.n_head > first ? std::min(L.n_local_tiles, (plan.n_head - first + stride - 1) / stride) : 0;
  DeviceGuard g(s->device);
  const size_t nt = (size_t)L.n_local_tiles * 64 * 3;
  if ((rc = ensure_out(s, std::max<size_t>(nt, 1) * sizeof(double)))) return rc;
  const int32_t *order = nullptr;
  if ((rc = launch(s, C, L, s->out_buf, nullptr, s->stream, &sp, &order))) return rc;
  hipError_t e = rtk_launch_shard_finish(s->scratch, L.n_local_tiles, sp.n_head, sp.head_chunks, sp.chunks,
                                         order, s->out_buf, s->stream);
  if (e == hipSuccess && (rc = mark_last(s, s->stream))) return rc;
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return hip_err(e, "shard render");
  *t_done = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  if (nt) {
    e = s->device == root_dev
            ? hipMemcpyAsync(dst, s->out_buf, nt * sizeof(double), hipMemcpyDeviceToDevice, s->stream)
            : hipMemcpyPeerAsync(dst, root_dev, s->out_buf, s->device, nt * sizeof(double), s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) return hip_err(e, "shard tiles to the root device");
  }
  return RT_OK;
}

int rt_multi_render(rt_multi *m, const rt_frame *f, const rt_render_params *p, double *host_rgb) {
  if (!m || !host_rgb || !p) return set_err(RT_ERR_INVALID, "null argument");
  if (p->tile_first != 0 || p->tile_stride > 1 || p->layout != RT_LAYOUT_FRAME)
    return set_err(RT_ERR_INVALID, "rt_multi_render takes a whole-frame launch "
                                   "(tile_first 0, tile_stride 0/1, RT_LAYOUT_FRAME)");
  DLaunch L;
  rt_render_params full = *p;
  full.strata_chunks = 0;
  full.accumulate = 0;
  int rc = to_launch(f, &full, L);
  if (rc) return rc;
  const int n = (int)m->scenes.size();
  rt_scene *root = m->scenes[0];
  // the one-device frame launch's units (so the frame is bit-identical to
  // rt_render on one device), or every tile in strata_chunks chunks if asked
  SplitPlan plan = frame_plan(root, L);
  if (p->strata_chunks > 0)
    plan = SplitPlan{0, 1, std::max(1, std::min(p->strata_chunks, std::max(1, L.sample_count)))};
  const int64_t n_tiles = (int64_t)L.tiles_x * L.tiles_y;
  const int64_t stride = (n_tiles + n - 1) / n; // staging slot per shard, in tiles
  const size_t frame_d = (size_t)(L.row_end - L.row_begin) * f->image_width * 3;
  {
    DeviceGuard g(root->device);
    auto grow = [&](double *&buf, size_t &have, size_t bytes, const char *what) -> int {
      if (have >= bytes) return RT_OK;
      // the last rt_multi_render synchronised every shard's stream and the
      // root's before it returned: nothing still uses buf
      scene_free(root, buf);
      have = 0;
      hipError_t e = scene_alloc(root, (void **)&buf, bytes);
      if (e != hipSuccess) return set_err(RT_ERR_OOM, std::string("hipMalloc ") + what + ": " + hipGetErrorString(e));
      have = bytes;
      return RT_OK;
    };
    if ((rc = grow(m->stage, m->stage_bytes, std::max<size_t>(1, (size_t)n * stride * 64 * 3) * sizeof(double),
                   "multi staging")))
      return rc;
    if ((rc = grow(m->frame, m->frame_bytes, std::max<size_t>(1, frame_d) * sizeof(double), "multi frame")))
      return rc;
  }
  std::vector<int> src(n, RT_OK);
  std::vector<double> t_done(n, 0.0);
  std::vector<std::string> err(n);
  std::vector<std::thread> th;
  try {
    for (int k = 0; k < n; ++k) {
      m->ms[k] = 0.0;
      if (k >= n_tiles) continue; // more shards than tiles
      th.emplace_back([&, k]() {
        src[k] = render_shard(m->scenes[k], f, p, k, n, plan, m->stage + (size_t)k * stride * 64 * 3,
                              root->device, &t_done[k]);
        if (src[k] == RT_OK) src[k] = rt_last_kernel_ms(m->scenes[k], &m->ms[k]);
        if (src[k] != RT_OK) err[k] = g_err;
      });
    }
  } catch (const std::exception &ex) { // thread creation failed: join the started ones
    for (auto &t : th) t.join();
    return set_err(RT_ERR_DEVICE, std::string("shard thread: ") + ex.what());
  }
  for (auto &t : th) t.join();
  for (int k = 0; k < n; ++k)
    if (src[k] != RT_OK) return set_err(src[k], "shard " + std::to_string(k) + ": " + err[k]);
  DeviceGuard g(root->device);
  hipError_t e = rtk_launch_tiles_to_frame(m->stage, n, stride, f->image_width, L.row_begin, L.row_end,
                                           f->pixel_samples_scale, p->output == RT_OUT_SCALED, 0, m->frame,
                                           root->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(root->stream);
  if (e != hipSuccess) return hip_err(e, "tiles_to_frame");
  const double t_frame =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  m->gather_ms = t_frame - *std::max_element(t_done.begin(), t_done.end());
  e = hipMemcpyAsync(host_rgb, m->frame, frame_d * sizeof(double), hipMemcpyDeviceToHost, root->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(root->stream);
  if (e != hipSuccess) return hip_err(e, "frame D2H");
  return RT_OK;
}

int rt_multi_shard_ms(rt_multi *m, double *ms) {
  if (!m || !ms) return set_err(RT_ERR_INVALID, "null argument");
  for (size_t k = 0; k < m->ms.size(); ++k) ms[k] = m->ms[k];
  return RT_OK;
}

int rt_multi_gather_ms(rt_multi *m, double *ms) {
  if (!m || !ms) return set_err(RT_ERR_INVALID, "null argument");
  *ms = m->gather_ms;
  return RT_OK;
}

} // extern "C"
