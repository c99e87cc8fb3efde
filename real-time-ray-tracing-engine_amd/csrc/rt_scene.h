// rt_scene.h — host scene compiler: rt_scene_desc -> flat device layout.
#ifndef RT_SCENE_H
#define RT_SCENE_H
#include "../../include/rt_api.h"
#include "rt_layout.h"

#include <string>
#include <vector>

namespace rtx {

struct HostScene {
  std::vector<DNode> nodes;
  std::vector<DNode4> nodes4; // the world BVH collapsed to 4-wide nodes (bvh_arity 4)
  std::vector<DItem> items;
  std::vector<DItem> mitems; // media (not in the BVH)
  std::vector<float> mbox;   // 6 per medium
  std::vector<DItem> bitems;
  std::vector<DXform> xforms;
  std::vector<DSphere> spheres;
  std::vector<DQuad> quads;
  std::vector<DMedium> media;
  std::vector<DMat> mats;
  std::vector<DTex> texs;
  std::vector<DPerlin> perlin;
  std::vector<DLight> lights;
  int32_t root_is_leaf = 0;
  int32_t n_root_items = 0;
  int32_t bvh_depth = 0;
  int32_t bvh_arity = 2;  // 4: nodes4 is the tree the kernel walks
  int32_t bvh_depth4 = 0; // levels of 4-wide nodes
  // device-built world BVH (0: built on the host; RT_BVH_DEVICE: linear BVH,
  // rt_bvh_build.hip; RT_BVH_DEVICE_SAH: binned SAH, rt_bvh_sah.hip): items still
  // in scene order, their boxes (lo xyz, hi xyz) and the centroid bounds; nodes
  // sized, not filled
  int32_t device_bvh = 0;
  // host SAH builder overrides (rt_tuning sah_*; 0: the builder's defaults),
  // set by the caller before compile_scene
  int32_t sah_leaf_max = 0, sah_leaf_split = 0, sah_trav_x4 = 0, sah_bins = 0;
  std::vector<double> item_boxes;
  double scene_lo[3] = {0, 0, 0}, scene_hi[3] = {0, 0, 0};
};

// 1 when no sphere moves (DScene::static_spheres): the kernel then skips the
// center.at(time) arithmetic, whose result is c0 exactly for these spheres.
inline int32_t all_spheres_static(const HostScene &H) {
  for (const DSphere &s : H.spheres)
    if (s.dir[0] != 0.0 || s.dir[1] != 0.0 || s.dir[2] != 0.0) return 0;
  return 1;
}

// The feature bits of the path-tracer instance a compiled scene needs
// (RT_FEAT_MEDIA / XFORM / LIGHTS / NOISE; RT_FEAT_FLAT and RT_FEAT_BVH4 follow
// from the world tree once it is built): the GPU library's choice and the CPU
// backend's (host/rtx_cpu.cpp) alike.
inline int32_t scene_features(const HostScene &H) {
  int32_t f = 0;
  if (!H.mitems.empty()) f |= RT_FEAT_MEDIA;
  for (const DItem &it : H.items)
    if (it.xf_count) f |= RT_FEAT_XFORM;
  for (const DItem &it : H.mitems)
    if (it.xf_count) f |= RT_FEAT_XFORM;
  for (const DLight &L : H.lights)
    if (L.xf_count) f |= RT_FEAT_XFORM;
  if (!H.lights.empty()) f |= RT_FEAT_LIGHTS;
  for (const DTex &t : H.texs)
    if (t.kind == RT_TEX_NOISE) f |= RT_FEAT_NOISE;
  return f;
}

// Scenes with at least this many world primitives build their BVH on the
// device when rt_scene_desc.bvh_builder is RT_BVH_AUTO.
constexpr int kDeviceBuildMin = 65536;

// Host SAH build from HostScene::item_boxes (fallback of the device build).
void build_world_bvh_host(HostScene &H);

// Scenes with at least this many world primitives walk a 4-wide BVH when
// rt_scene_desc.bvh_arity is 0 (auto).
constexpr int kBvh4Min = 4096;

// Collapses the binary BFS-ordered tree `bin` (root 0) into 4-wide nodes, BFS
// order, root 0: each 4-wide node starts from one binary node's two children
// and repeatedly replaces its largest-area inner child by that child's two
// children until it holds four (or only leaves).  Leaf entries keep their
// encoding, so the leaf item ranges are shared with the binary tree.  Returns
// the number of 4-wide levels.
int collapse_bvh4(const std::vector<DNode> &bin, std::vector<DNode4> &out);

// SAH cost of a binary tree (rt_scene_bvh_cost): 1 + sum over child boxes of
// (1 for an inner child, its item count for a leaf) x area / root area.
double bvh_sah_cost(const std::vector<DNode> &nodes);

// The traversal stack a 4-wide walk of depth4 levels needs: at most three
// pushed siblings per level on the current root path.
inline int bvh4_stack_depth(int depth4) { return 3 * depth4 + 1; }

// Returns RT_OK or an error code with `err` filled.
int compile_scene(const rt_scene_desc *desc, HostScene &out, std::string &err);

// Camera::initialize (Camera.cpp:31-73), same operation order.
int camera_setup(const rt_camera_desc *cam, rt_frame *frame, std::string &err);

// The validation both backends apply to a launch (librtx_hip.so's rt_render*
// and librtx_cpu.so's rt_cpu_render): a set-up frame -> the kernel's camera
// values, and the params' row band, stratum range, output, layout, tile subset
// and chunk count -> the launch geometry (one work unit per tile, or every
// tile in strata_chunks chunks).  strata_chunks < 0 is refused here:
// RT_CHUNKS_AUTO is resolved by the callers that accept it.
int device_camera(const rt_frame *frame, DCamera &c, std::string &err);
int launch_geometry(const rt_frame *frame, const rt_render_params *p, DLaunch &L, std::string &err);

} // namespace rtx
#endif
