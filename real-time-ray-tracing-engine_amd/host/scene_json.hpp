// scene_json.hpp — JSON scene file -> rt_scene_desc / rt_camera_desc (C++ host).
//
// The C++ twin of rtx/scene.py: same schema, same error cases, and the SAME table
// index assignment (textures/materials are created on first reference, objects
// children-first, the world list then the light list), so both hosts hand the
// library identical descriptions (tests/test_cli.py compares them field by field).
// Object types map one to one onto the reference classes: sphere (Sphere.cpp:8-23),
// quad (Plane.cpp:6-21), box (make_box, PlaneUtility.hpp:11-39), list
// (HittableList), rotate_y (RotateY.cpp:5-35), translate (Translate.cpp:7-10),
// constant_medium (ConstantMedium.cpp:7-21).
#pragma once

#include "../../include/rt_api.h"
#include "json_min.hpp"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace rtxhost {

struct SceneError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct LoadedScene {
  std::vector<rt_texture_desc> textures;
  std::vector<rt_perlin_desc> perlin;
  std::vector<rt_material_desc> materials;
  std::vector<rt_object_desc> objects;
  std::vector<int32_t> children;
  int32_t world = -1, lights = -1, use_bvh = 0;
  rt_camera_desc camera{};

  rt_scene_desc desc() const {
    rt_scene_desc d{};
    d.textures = textures.data();
    d.n_textures = (int32_t)textures.size();
    d.perlin = perlin.data();
    d.n_perlin = (int32_t)perlin.size();
    d.materials = materials.data();
    d.n_materials = (int32_t)materials.size();
    d.objects = objects.data();
    d.n_objects = (int32_t)objects.size();
    d.children = children.data();
    d.n_children = (int32_t)children.size();
    d.world = world;
    d.lights = lights;
    d.use_bvh = use_bvh;
    return d;
  }
};

namespace detail {

using jsonmin::Value;

inline rt_vec3 v3(const Value &v, const char *what) {
  if (!v.is_array() || v.arr.size() != 3) throw SceneError(std::string(what) + " must be a 3-element list");
  return rt_vec3{v.arr[0].number(), v.arr[1].number(), v.arr[2].number()};
}

class Loader {
public:
  explicit Loader(const Value &doc) : doc_(doc) {}

  LoadedScene run() {
    camera();
    if (const Value *b = doc_.find("use_bvh")) S.use_bvh = b->number() != 0 ? 1 : 0;
    if (const Value *p = doc_.find("perlin"))
      for (const auto &kv : p->obj) {
        S.perlin.push_back(perlin(kv.second));
        named_perlin_[kv.first] = (int)S.perlin.size() - 1;
      }
    tex_specs_ = doc_.find("textures");
    mat_specs_ = doc_.find("materials");
    std::vector<int32_t> ids;
    if (const Value *w = doc_.find("world"))
      for (const Value &o : w->arr) ids.push_back(object(o, true));
    S.world = add_list(ids);
    const Value *l = doc_.find("lights");
    if (l && l->kind != Value::Null) {
      std::vector<int32_t> lids;
      for (const Value &o : l->arr) lids.push_back(object(o, false));
      S.lights = add_list(lids);
    }
    return S;
  }

private:
  const Value &doc_;
  LoadedScene S;
  const Value *tex_specs_ = nullptr, *mat_specs_ = nullptr;
  std::map<std::string, int> named_tex_, named_mat_, named_perlin_;

  void camera() { // CameraConfig.hpp:12-35 defaults
    rt_camera_desc &c = S.camera;
    c = rt_camera_desc{};
    c.image_width = 600;
    c.samples_per_pixel = 10;
    c.max_depth = 10;
    c.aspect_ratio = 1.0;
    c.vfov = 90.0;
    c.defocus_angle = 0.0;
    c.focus_dist = 10.0;
    c.lookfrom = rt_vec3{0, 0, 0};
    c.lookat = rt_vec3{0, 0, -1};
    c.vup = rt_vec3{0, 1, 0};
    c.background = rt_vec3{0, 0, 0};
    const Value *cv = doc_.find("camera");
    if (!cv) return;
    for (const auto &kv : cv->obj) {
      const std::string &k = kv.first;
      const Value &v = kv.second;
      if (k == "image_width") c.image_width = (int32_t)v.number();
      else if (k == "samples_per_pixel") c.samples_per_pixel = (int32_t)v.number();
      else if (k == "max_depth") c.max_depth = (int32_t)v.number();
      else if (k == "aspect_ratio") c.aspect_ratio = v.number();
      else if (k == "vfov") c.vfov = v.number();
      else if (k == "defocus_angle") c.defocus_angle = v.number();
      else if (k == "focus_dist") c.focus_dist = v.number();
      else if (k == "lookfrom") c.lookfrom = v3(v, "lookfrom");
      else if (k == "lookat") c.lookat = v3(v, "lookat");
      else if (k == "vup") c.vup = v3(v, "vup");
      else if (k == "background") c.background = v3(v, "background");
    }
    if (c.image_width < 1 || c.samples_per_pixel < 1 || c.max_depth < 0)
      throw SceneError("camera: image_width/samples_per_pixel must be >= 1");
  }

  rt_perlin_desc perlin(const Value &p) {
    rt_perlin_desc d{};
    const Value &rv = p.at("rand_vec");
    if (rv.arr.size() != 256) throw SceneError("perlin.rand_vec needs 256 vectors");
    for (int k = 0; k < 256; ++k) d.rand_vec[k] = v3(rv.arr[k], "perlin.rand_vec");
    const char *names[3] = {"perm_x", "perm_y", "perm_z"};
    int32_t *dst[3] = {d.perm_x, d.perm_y, d.perm_z};
    for (int a = 0; a < 3; ++a) {
      const Value &arr = p.at(names[a]);
      if (arr.arr.size() != 256) throw SceneError(std::string("perlin.") + names[a] + " must have 256 entries");
      std::vector<int> seen(256, 0);
      for (int k = 0; k < 256; ++k) {
        int x = (int)arr.arr[k].number();
        if (x < 0 || x > 255 || seen[x]++) throw SceneError(std::string("perlin.") + names[a] + " must be a permutation of 0..255");
        dst[a][k] = x;
      }
    }
    return d;
  }

  int add_texture(int32_t kind, rt_vec3 color, double scale, int even, int odd, int perl) {
    rt_texture_desc t{};
    t.kind = kind;
    t.even = even;
    t.odd = odd;
    t.perlin = perl;
    t.scale = scale;
    t.color = color;
    S.textures.push_back(t);
    return (int)S.textures.size() - 1;
  }
  int solid(rt_vec3 c) { return add_texture(RT_TEX_SOLID, c, 0.0, -1, -1, -1); }

  int tex(const Value &ref) {
    if (ref.is_array()) return solid(v3(ref, "color"));
    if (ref.is_object()) return tex_spec(ref);
    if (!ref.is_string()) throw SceneError("bad texture reference");
    auto it = named_tex_.find(ref.str);
    if (it == named_tex_.end()) {
      const Value *spec = tex_specs_ ? tex_specs_->find(ref.str) : nullptr;
      if (!spec) throw SceneError("unknown texture '" + ref.str + "'");
      named_tex_[ref.str] = -2; // cycle guard
      int id = tex_spec(*spec);
      named_tex_[ref.str] = id;
      return id;
    }
    if (it->second == -2) throw SceneError("texture cycle at '" + ref.str + "'");
    return it->second;
  }
  int tex_spec(const Value &t) {
    std::string ty = t.find("type") ? t.at("type").str : "";
    if (ty == "solid") return solid(v3(t.at("color"), "color"));
    if (ty == "checker") {
      int even = tex(t.at("even"));
      int odd = tex(t.at("odd"));
      return add_texture(RT_TEX_CHECKER, rt_vec3{0, 0, 0}, t.at("scale").number(), even, odd, -1);
    }
    if (ty == "noise") {
      auto p = named_perlin_.find(t.at("perlin").str);
      if (p == named_perlin_.end()) throw SceneError("unknown perlin table");
      return add_texture(RT_TEX_NOISE, rt_vec3{0, 0, 0}, t.at("scale").number(), -1, -1, p->second);
    }
    throw SceneError("unknown texture type '" + ty + "'");
  }

  int add_material(int32_t kind, int texture, rt_vec3 albedo, double fuzz, double ri) {
    rt_material_desc m{};
    m.kind = kind;
    m.texture = texture;
    m.albedo = albedo;
    m.fuzz = fuzz;
    m.refraction_index = ri;
    S.materials.push_back(m);
    return (int)S.materials.size() - 1;
  }
  int tex_or_color(const Value &m, const char *key) {
    if (m.has("texture")) return tex(m.at("texture"));
    return solid(v3(m.at(key), key));
  }
  int mat(const Value *ref) {
    if (!ref || ref->kind == Value::Null) return -1;
    if (ref->is_object()) return mat_spec(*ref);
    auto it = named_mat_.find(ref->str);
    if (it != named_mat_.end()) return it->second;
    const Value *spec = mat_specs_ ? mat_specs_->find(ref->str) : nullptr;
    if (!spec) throw SceneError("unknown material '" + ref->str + "'");
    int id = mat_spec(*spec);
    named_mat_[ref->str] = id;
    return id;
  }
  int mat_spec(const Value &m) {
    std::string ty = m.find("type") ? m.at("type").str : "";
    const rt_vec3 z{0, 0, 0};
    if (ty == "lambertian") {
      int t = tex_or_color(m, "albedo");
      return add_material(RT_MAT_LAMBERTIAN, t, z, 0.0, 1.0);
    }
    if (ty == "metal")
      return add_material(RT_MAT_METAL, -1, v3(m.at("albedo"), "albedo"),
                          m.has("fuzz") ? m.at("fuzz").number() : 0.0, 1.0);
    if (ty == "dielectric")
      return add_material(RT_MAT_DIELECTRIC, -1, z, 0.0, m.at("refraction_index").number());
    if (ty == "diffuse_light") {
      int t = tex_or_color(m, "emit");
      return add_material(RT_MAT_DIFFUSE_LIGHT, t, z, 0.0, 1.0);
    }
    if (ty == "isotropic") {
      int t = tex_or_color(m, "albedo");
      return add_material(RT_MAT_ISOTROPIC, t, z, 0.0, 1.0);
    }
    throw SceneError("unknown material type '" + ty + "'");
  }

  int add_object(int32_t kind, int material, int child, int count, rt_vec3 a, rt_vec3 b,
                 rt_vec3 c, double s, int moving, int phase) {
    rt_object_desc o{};
    o.kind = kind;
    o.material = material;
    o.child = child;
    o.count = count;
    o.a = a;
    o.b = b;
    o.c = c;
    o.s = s;
    o.moving = moving;
    o.phase = phase;
    S.objects.push_back(o);
    return (int)S.objects.size() - 1;
  }
  int add_list(const std::vector<int32_t> &ids) {
    int first = (int)S.children.size();
    S.children.insert(S.children.end(), ids.begin(), ids.end());
    return add_object(RT_OBJ_LIST, -1, first, (int)ids.size(), {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
                      0.0, 0, -1);
  }

  int object(const Value &o, bool need_material) {
    std::string ty = o.find("type") ? o.at("type").str : "";
    const Value *mref = o.find("material");
    bool no_mat = !mref || mref->kind == Value::Null;
    const rt_vec3 z{0, 0, 0};
    if (ty == "sphere") {
      if (need_material && no_mat) throw SceneError("world sphere without material");
      int m = mat(mref);
      if (o.has("displacement")) // stored form: Sphere's m_center direction (c1 - c0)
        return add_object(RT_OBJ_SPHERE, m, -1, 0, v3(o.at("center"), "center"),
                          v3(o.at("displacement"), "displacement"), z, o.at("radius").number(),
                          RT_STORED_FORM, -1);
      if (o.has("center2"))
        return add_object(RT_OBJ_SPHERE, m, -1, 0, v3(o.at("center"), "center"),
                          v3(o.at("center2"), "center2"), z, o.at("radius").number(), 1, -1);
      return add_object(RT_OBJ_SPHERE, m, -1, 0, v3(o.at("center"), "center"), z, z,
                        o.at("radius").number(), 0, -1);
    }
    if (ty == "quad") {
      if (need_material && no_mat) throw SceneError("world quad without material");
      int m = mat(mref);
      return add_object(RT_OBJ_QUAD, m, -1, 0, v3(o.at("Q"), "Q"), v3(o.at("u"), "u"),
                        v3(o.at("v"), "v"), 0.0, 0, -1);
    }
    if (ty == "box") { // make_box, PlaneUtility.hpp:11-39
      if (need_material && no_mat) throw SceneError("world box without material");
      int m = mat(mref);
      rt_vec3 a = v3(o.at("a"), "a"), b = v3(o.at("b"), "b");
      rt_vec3 mn{std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)};
      rt_vec3 mx{std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)};
      rt_vec3 dx{mx.x - mn.x, 0.0, 0.0}, dy{0.0, mx.y - mn.y, 0.0}, dz{0.0, 0.0, mx.z - mn.z};
      rt_vec3 ndx{-dx.x, -dx.y, -dx.z}, ndz{-dz.x, -dz.y, -dz.z};
      rt_vec3 Qs[6] = {{mn.x, mn.y, mx.z}, {mx.x, mn.y, mx.z}, {mx.x, mn.y, mn.z},
                       {mn.x, mn.y, mn.z}, {mn.x, mx.y, mx.z}, {mn.x, mn.y, mn.z}};
      rt_vec3 Us[6] = {dx, ndz, ndx, dz, dx, dx};
      rt_vec3 Vs[6] = {dy, dy, dy, dy, ndz, dz};
      std::vector<int32_t> ids;
      for (int k = 0; k < 6; ++k)
        ids.push_back(add_object(RT_OBJ_QUAD, m, -1, 0, Qs[k], Us[k], Vs[k], 0.0, 0, -1));
      return add_list(ids);
    }
    if (ty == "list") {
      std::vector<int32_t> ids;
      for (const Value &k : o.at("objects").arr) ids.push_back(object(k, need_material));
      return add_list(ids);
    }
    if (ty == "rotate_y") {
      int ch = object(o.at("object"), need_material);
      if (o.has("sin_cos")) { // stored form: RotateY's (sin, cos)
        const Value &sc = o.at("sin_cos");
        if (!sc.is_array() || sc.arr.size() != 2) throw SceneError("rotate_y.sin_cos must be [sin, cos]");
        return add_object(RT_OBJ_ROTATE_Y, -1, ch, 0, rt_vec3{sc.arr[0].number(), sc.arr[1].number(), 0.0},
                          z, z, 0.0, RT_STORED_FORM, -1);
      }
      return add_object(RT_OBJ_ROTATE_Y, -1, ch, 0, z, z, z, o.at("angle").number(), 0, -1);
    }
    if (ty == "translate") {
      int ch = object(o.at("object"), need_material);
      return add_object(RT_OBJ_TRANSLATE, -1, ch, 0, v3(o.at("offset"), "offset"), z, z, 0.0, 0, -1);
    }
    if (ty == "constant_medium") {
      int ch = object(o.at("boundary"), false);
      int ph;
      if (o.has("phase")) {
        ph = mat(o.find("phase"));
      } else {
        int t = tex_or_color(o, "albedo");
        ph = add_material(RT_MAT_ISOTROPIC, t, z, 0.0, 1.0);
      }
      double dens = o.at("density").number();
      if (!(dens > 0)) throw SceneError("constant_medium density must be > 0");
      return add_object(RT_OBJ_MEDIUM, -1, ch, 0, z, z, z, dens, 0, ph);
    }
    throw SceneError("unknown object type '" + ty + "'");
  }
};

} // namespace detail

inline LoadedScene load_scene_text(const std::string &text) {
  jsonmin::Value doc = jsonmin::parse(text);
  if (!doc.is_object()) throw SceneError("scene file must hold a JSON object");
  return detail::Loader(doc).run();
}

inline LoadedScene load_scene_file(const std::string &path) {
  std::ifstream f(path);
  if (!f) throw SceneError("cannot open scene file " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return load_scene_text(ss.str());
}

} // namespace rtxhost
