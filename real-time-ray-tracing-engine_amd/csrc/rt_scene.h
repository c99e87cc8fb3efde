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
};

// Returns RT_OK or an error code with `err` filled.
int compile_scene(const rt_scene_desc *desc, HostScene &out, std::string &err);

// Camera::initialize (Camera.cpp:31-73), same operation order.
int camera_setup(const rt_camera_desc *cam, rt_frame *frame, std::string &err);

} // namespace rtx
#endif
