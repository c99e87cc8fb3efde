/* oracle/ref_binding.hpp — the reference-side binding of INTEGRATION.md,
 * compiled against the reference's own headers and classes.
 *
 * TEST INFRASTRUCTURE: it is included by oracle/ref_bridge.cpp, which is built
 * into oracle/_ref/libref.so from /root/reference/src (oracle/Makefile `ref`).
 * It is not part of the product.  tests/test_binding.py builds scenes as
 * reference objects, converts them back to rt_scene_desc here, and checks that
 * the tables and the GPU images match the original descriptions.  That shows
 * the binding a reference maintainer would add works against the real classes.
 *
 * This is the same walk as INTEGRATION.md, with two differences:
 *   - RotateY goes through get_angle() (RotateY.hpp:23-25).  The reference
 *     stores only sin/cos, and a maintainer would add the two getters to use
 *     RT_STORED_FORM instead.  atan2(sin, cos) * 180/pi is within an ulp or so
 *     of the constructor angle.
 *   - The world and light lists are converted before any BVHNode wrap, and
 *     use_bvh is passed through unchanged.
 */
#ifndef RT_REF_BINDING_HPP
#define RT_REF_BINDING_HPP

#include "../include/rt_api.h"

#include "core/HittableList.hpp"
#include "core/Ray.hpp"
#include "optimization/BVHNode.hpp"
#include "scene/materials/DielectricMaterial.hpp"
#include "scene/materials/DiffuseLightMaterial.hpp"
#include "scene/materials/IsotropicMaterial.hpp"
#include "scene/materials/LambertianMaterial.hpp"
#include "scene/materials/MetalMaterial.hpp"
#include "scene/mediums/ConstantMedium.hpp"
#include "scene/objects/Plane.hpp"
#include "scene/objects/RotateY.hpp"
#include "scene/objects/Sphere.hpp"
#include "scene/objects/Translate.hpp"
#include "scene/textures/CheckerTexture.hpp"
#include "scene/textures/NoiseTexture.hpp"
#include "scene/textures/SolidColorTexture.hpp"

#include <unordered_map>
#include <vector>

class RtSceneBuilder {
public:
  std::vector<rt_texture_desc> tex;
  std::vector<rt_perlin_desc> perlin;
  std::vector<rt_material_desc> mat;
  std::vector<rt_object_desc> obj;
  std::vector<int32_t> kids;

  static rt_vec3 v(const Vec3 &a) { return rt_vec3{a.x(), a.y(), a.z()}; }

  int texture(const TexturePtr &t) {
    auto it = tex_ids.find(t.get());
    if (it != tex_ids.end()) return it->second;
    rt_texture_desc d{};
    d.even = d.odd = d.perlin = -1;
    if (auto s = dynamic_cast<const SolidColorTexture *>(t.get())) {
      d.kind = RT_TEX_SOLID;
      d.color = v(s->get_albedo());
    } else if (auto c = dynamic_cast<const CheckerTexture *>(t.get())) {
      d.kind = RT_TEX_CHECKER;
      d.scale = c->get_scale();
      d.even = texture(c->get_even_texture());
      d.odd = texture(c->get_odd_texture());
    } else if (auto n = dynamic_cast<const NoiseTexture *>(t.get())) {
      d.kind = RT_TEX_NOISE;
      d.scale = n->get_scale();
      const PerlinNoise &p = n->get_perlin();
      rt_perlin_desc pd;
      for (int k = 0; k < RT_PERLIN_POINTS; ++k) {
        pd.rand_vec[k] = v(p.rand_vec()[k]);
        pd.perm_x[k] = p.perm_x()[k];
        pd.perm_y[k] = p.perm_y()[k];
        pd.perm_z[k] = p.perm_z()[k];
      }
      d.perlin = (int32_t)perlin.size();
      perlin.push_back(pd);
    }
    tex.push_back(d);
    return tex_ids[t.get()] = (int)tex.size() - 1;
  }

  int material(const MaterialPtr &m) {
    if (!m) return -1;
    auto it = mat_ids.find(m.get());
    if (it != mat_ids.end()) return it->second;
    rt_material_desc d{};
    d.texture = -1;
    d.refraction_index = 1.0;
    if (auto l = dynamic_cast<const LambertianMaterial *>(m.get())) {
      d.kind = RT_MAT_LAMBERTIAN;
      d.texture = texture(l->get_texture());
    } else if (auto me = dynamic_cast<const MetalMaterial *>(m.get())) {
      d.kind = RT_MAT_METAL;
      d.albedo = v(me->get_albedo());
      d.fuzz = me->get_fuzz();
    } else if (auto di = dynamic_cast<const DielectricMaterial *>(m.get())) {
      d.kind = RT_MAT_DIELECTRIC;
      d.refraction_index = di->get_refraction_index();
    } else if (auto e = dynamic_cast<const DiffuseLightMaterial *>(m.get())) {
      d.kind = RT_MAT_DIFFUSE_LIGHT;
      d.texture = texture(e->get_texture());
    } else if (auto is = dynamic_cast<const IsotropicMaterial *>(m.get())) {
      d.kind = RT_MAT_ISOTROPIC;
      d.texture = texture(is->get_texture());
    }
    mat.push_back(d);
    return mat_ids[m.get()] = (int)mat.size() - 1;
  }

  int list(const std::vector<int32_t> &ids) {
    rt_object_desc d{};
    d.kind = RT_OBJ_LIST;
    d.material = d.phase = -1;
    d.child = (int32_t)kids.size();
    d.count = (int32_t)ids.size();
    kids.insert(kids.end(), ids.begin(), ids.end());
    obj.push_back(d);
    return (int)obj.size() - 1;
  }

  int object(const HittablePtr &h) {
    rt_object_desc d{};
    d.material = d.child = d.phase = -1;
    if (auto s = dynamic_cast<const Sphere *>(h.get())) {
      d.kind = RT_OBJ_SPHERE;
      d.material = material(s->get_material());
      Ray c = s->get_center();
      d.a = v(c.origin());
      d.b = v(c.direction()); // c1 - c0 as stored (zero for static spheres)
      d.moving = RT_STORED_FORM;
      d.s = s->get_radius();
    } else if (auto p = dynamic_cast<const Plane *>(h.get())) {
      d.kind = RT_OBJ_QUAD;
      d.material = material(p->get_material());
      d.a = v(p->get_corner());
      d.b = v(p->get_u_side());
      d.c = v(p->get_v_side());
    } else if (auto r = dynamic_cast<const RotateY *>(h.get())) {
      d.kind = RT_OBJ_ROTATE_Y;
      d.child = object(r->get_object());
      d.s = r->get_angle(); // see the header note: stored sin/cos need two getters
    } else if (auto t = dynamic_cast<const Translate *>(h.get())) {
      d.kind = RT_OBJ_TRANSLATE;
      d.child = object(t->get_object());
      d.a = v(t->get_offset());
    } else if (auto m = dynamic_cast<const ConstantMedium *>(h.get())) {
      d.kind = RT_OBJ_MEDIUM;
      d.child = object(m->get_boundary());
      d.s = m->get_density();
      d.phase = material(m->get_phase_function());
    } else if (auto l = dynamic_cast<const HittableList *>(h.get())) {
      std::vector<int32_t> ids;
      for (const HittablePtr &k : l->get_objects()) ids.push_back(object(k));
      return list(ids);
    } else if (auto b = dynamic_cast<const BVHNode *>(h.get())) {
      return list({object(b->get_left()), object(b->get_right())});
    }
    obj.push_back(d);
    return (int)obj.size() - 1;
  }

  rt_scene_desc finish(const HittableList &world, const HittableList &lights, bool use_bvh) {
    std::vector<int32_t> w, l;
    for (const HittablePtr &k : world.get_objects()) w.push_back(object(k));
    world_id = list(w);
    for (const HittablePtr &k : lights.get_objects()) l.push_back(object(k));
    lights_id = l.empty() ? -1 : list(l);
    rt_scene_desc d{};
    d.textures = tex.data();
    d.n_textures = (int32_t)tex.size();
    d.perlin = perlin.data();
    d.n_perlin = (int32_t)perlin.size();
    d.materials = mat.data();
    d.n_materials = (int32_t)mat.size();
    d.objects = obj.data();
    d.n_objects = (int32_t)obj.size();
    d.children = kids.data();
    d.n_children = (int32_t)kids.size();
    d.world = world_id;
    d.lights = lights_id;
    d.use_bvh = use_bvh ? 1 : 0;
    return d;
  }

private:
  std::unordered_map<const void *, int> tex_ids, mat_ids;
  int world_id = -1, lights_id = -1;
};

#endif
