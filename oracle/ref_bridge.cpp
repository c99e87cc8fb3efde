/* oracle/ref_bridge.cpp — TEST INFRASTRUCTURE: drives the REAL reference code.
 *
 * Compiled (by oracle/Makefile, target `ref`) together with the reference's own
 * CPU sources where they lie under /root/reference/src (every .cpp except
 * main.cpp and core/camera/DynamicCamera.cpp, which pull in SDL3 — the only
 * SDL dependency, DynamicCamera.hpp:5-6, and neither is on the hot path).  The
 * output goes to oracle/_ref/ (git-ignored).  Nothing here is shipped: it is the
 * source of the golden fixtures in tests/golden/ and, optionally, the timed
 * "reference" CPU baseline.
 *
 * It rebuilds the reference object graph from an rt_scene_desc and calls the
 * reference's own Camera::initialize / get_ray / ray_color in the serial order of
 * StaticCamera::render_cpu (StaticCamera.cpp:102-131), after seeding the main
 * thread's engine (Utility.hpp:16-19 returns it by reference).
 */
#include "../include/rt_api.h"

#include "core/HitRecord.hpp"
#include "core/Hittable.hpp"
#include "core/HittableList.hpp"
#include "core/Ray.hpp"
#include "core/camera/Camera.hpp"
#include "core/camera/StaticCamera.hpp"
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
#include "utils/ColorUtility.hpp"
#include "utils/concurrency/ThreadPool.hpp"
#include "ref_binding.hpp"
#include "scene/Scene.hpp"
#include "utils/math/Utility.hpp"
#include "utils/math/Vec3Utility.hpp"

#include <atomic>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

namespace {

Vec3 V3(const rt_vec3 &v) { return Vec3(v.x, v.y, v.z); }

struct Graph {
  std::vector<TexturePtr> tex;
  std::vector<MaterialPtr> mat;
  std::vector<HittablePtr> obj;
  std::vector<PerlinNoise> perlin;
  const rt_scene_desc *D = nullptr;

  TexturePtr texture(int i) {
    if (tex[i]) return tex[i];
    const rt_texture_desc &t = D->textures[i];
    if (t.kind == RT_TEX_SOLID) {
      tex[i] = std::make_shared<SolidColorTexture>(V3(t.color));
    } else if (t.kind == RT_TEX_CHECKER) {
      tex[i] = std::make_shared<CheckerTexture>(t.scale, texture(t.even), texture(t.odd));
    } else {
      tex[i] = std::make_shared<NoiseTexture>(t.scale, perlin[t.perlin]);
    }
    return tex[i];
  }
  MaterialPtr material(int i) {
    if (i < 0) return MaterialPtr();
    if (mat[i]) return mat[i];
    const rt_material_desc &m = D->materials[i];
    switch (m.kind) {
    case RT_MAT_LAMBERTIAN:
      mat[i] = std::make_shared<LambertianMaterial>(texture(m.texture));
      break;
    case RT_MAT_METAL:
      mat[i] = std::make_shared<MetalMaterial>(V3(m.albedo), m.fuzz);
      break;
    case RT_MAT_DIELECTRIC:
      mat[i] = std::make_shared<DielectricMaterial>(m.refraction_index);
      break;
    case RT_MAT_DIFFUSE_LIGHT:
      mat[i] = std::make_shared<DiffuseLightMaterial>(texture(m.texture));
      break;
    default:
      mat[i] = std::make_shared<IsotropicMaterial>(texture(m.texture));
    }
    return mat[i];
  }
  HittablePtr object(int i) {
    if (obj[i]) return obj[i];
    const rt_object_desc &o = D->objects[i];
    HittablePtr h;
    switch (o.kind) {
    case RT_OBJ_SPHERE:
      if (o.moving)
        h = std::make_shared<Sphere>(V3(o.a), V3(o.b), o.s, material(o.material));
      else
        h = std::make_shared<Sphere>(V3(o.a), o.s, material(o.material));
      break;
    case RT_OBJ_QUAD:
      h = std::make_shared<Plane>(V3(o.a), V3(o.b), V3(o.c), material(o.material));
      break;
    case RT_OBJ_LIST: {
      auto l = std::make_shared<HittableList>();
      for (int k = 0; k < o.count; ++k) l->add(object(D->children[o.child + k]));
      h = l;
      break;
    }
    case RT_OBJ_ROTATE_Y:
      h = std::make_shared<RotateY>(object(o.child), o.s);
      break;
    case RT_OBJ_TRANSLATE:
      h = std::make_shared<Translate>(object(o.child), V3(o.a));
      break;
    default:
      h = std::make_shared<ConstantMedium>(object(o.child), o.s, material(o.phase));
    }
    obj[i] = h;
    return h;
  }
  void load(const rt_scene_desc *d) {
    D = d;
    for (int p = 0; p < d->n_perlin; ++p) {
      Vec3 rv[256];
      int px[256], py[256], pz[256];
      for (int k = 0; k < 256; ++k) {
        rv[k] = V3(d->perlin[p].rand_vec[k]);
        px[k] = d->perlin[p].perm_x[k];
        py[k] = d->perlin[p].perm_y[k];
        pz[k] = d->perlin[p].perm_z[k];
      }
      perlin.emplace_back(rv, px, py, pz);
    }
    tex.assign(d->n_textures, nullptr);
    mat.assign(d->n_materials, nullptr);
    obj.assign(d->n_objects, nullptr);
  }
};

CameraConfig make_config(const rt_camera_desc *c, bool bvh, bool par) {
  CameraConfig cfg;
  cfg.image_width = c->image_width;
  cfg.samples_per_pixel = c->samples_per_pixel;
  cfg.max_depth = c->max_depth;
  cfg.aspect_ratio = c->aspect_ratio;
  cfg.vfov = c->vfov;
  cfg.defocus_angle = c->defocus_angle;
  cfg.focus_dist = c->focus_dist;
  cfg.lookfrom = V3(c->lookfrom);
  cfg.lookat = V3(c->lookat);
  cfg.vup = V3(c->vup);
  cfg.background = V3(c->background);
  cfg.use_parallelism = par;
  cfg.use_bvh = bvh;
  cfg.use_gpu = false;
  cfg.use_debug = false;
  return cfg;
}

// Exposes the protected hot-path members of the reference Camera.
struct GoldenCamera : public Camera {
  explicit GoldenCamera(const CameraConfig &c) : Camera(c) {}
  void render(HittableList &, HittableList &) override {}
  void setup() { initialize(); }
  void frame(rt_frame *f) const {
    auto cv = [](const Vec3 &v) { return rt_vec3{v.x(), v.y(), v.z()}; };
    f->image_width = m_image_width;
    f->image_height = m_image_height;
    f->sqrt_spp = int(std::sqrt(m_samples_per_pixel));
    f->max_depth = m_max_depth;
    f->center = cv(m_center);
    f->pixel00_loc = cv(m_pixel00_loc);
    f->pixel_delta_u = cv(m_pixel_delta_u);
    f->pixel_delta_v = cv(m_pixel_delta_v);
    f->u = cv(m_u);
    f->v = cv(m_v);
    f->w = cv(m_w);
    f->defocus_disk_u = cv(m_defocus_disk_u);
    f->defocus_disk_v = cv(m_defocus_disk_v);
    f->defocus_angle = m_defocus_angle;
    f->pixel_samples_scale = m_pixel_samples_scale;
    f->background = cv(m_background);
  }
  // StaticCamera::render_cpu serial branch (StaticCamera.cpp:102-131), but keeping
  // the scaled float radiance instead of quantising it.
  void trace(HittableList &world, HittableList &lights, double *out) {
    int sq = static_cast<int>(std::sqrt(m_samples_per_pixel));
    for (int j = 0; j < m_image_height; ++j)
      for (int i = 0; i < m_image_width; ++i) {
        Color pc(0, 0, 0);
        for (int sj = 0; sj < sq; ++sj)
          for (int si = 0; si < sq; ++si) {
            Ray r = get_ray(i, j, si, sj);
            pc += ray_color(r, m_max_depth, world, lights);
          }
        Color sc = m_pixel_samples_scale * pc;
        double *o = out + 3 * ((size_t)j * m_image_width + i);
        o[0] = sc.x();
        o[1] = sc.y();
        o[2] = sc.z();
      }
  }
  // StaticCamera::render_cpu's -p loop (StaticCamera.cpp:59-100) on the
  // reference's own ThreadPool (ThreadPool.hpp:6-174), sized by the caller
  // instead of hardware_concurrency(); radiance kept instead of quantised.
  long long trace_pool(HittableList &world, HittableList &lights, int threads, double *out) {
    ThreadPool pool(threads);
    std::vector<Color> row_colors(m_image_width);
    const int sqrt_spp = static_cast<int>(std::sqrt(m_samples_per_pixel));
    for (int j = 0; j < m_image_height; ++j) {
      pool.start();
      for (int i = 0; i < m_image_width; ++i) {
        pool.submit_job([this, &world, &lights, i, j, sqrt_spp, &row_colors]() {
          row_colors[i] = Color(0, 0, 0);
          for (int s_j = 0; s_j < sqrt_spp; ++s_j)
            for (int s_i = 0; s_i < sqrt_spp; ++s_i) {
              Ray ray = get_ray(i, j, s_i, s_j);
              row_colors[i] += ray_color(ray, m_max_depth, world, lights);
            }
        });
      }
      pool.finish();
      for (int i = 0; i < m_image_width; ++i) {
        Color sc = m_pixel_samples_scale * row_colors[i];
        double *o = out + 3 * ((size_t)j * m_image_width + i);
        o[0] = sc.x();
        o[1] = sc.y();
        o[2] = sc.z();
      }
    }
    return (long long)m_image_width * m_image_height * sqrt_spp * sqrt_spp;
  }
  long long trace_parallel(HittableList &world, HittableList &lights, int threads, double *out) {
    int sq = static_cast<int>(std::sqrt(m_samples_per_pixel));
    for (int j = 0; j < m_image_height; ++j) {
      std::atomic<int> next{0};
      std::vector<std::thread> pool;
      for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, j]() {
          for (;;) {
            int i = next.fetch_add(1);
            if (i >= m_image_width) break;
            Color pc(0, 0, 0);
            for (int sj = 0; sj < sq; ++sj)
              for (int si = 0; si < sq; ++si) {
                Ray r = get_ray(i, j, si, sj);
                pc += ray_color(r, m_max_depth, world, lights);
              }
            Color sc = m_pixel_samples_scale * pc;
            double *o = out + 3 * ((size_t)j * m_image_width + i);
            o[0] = sc.x();
            o[1] = sc.y();
            o[2] = sc.z();
          }
        });
      for (auto &th : pool) th.join();
    }
    return (long long)m_image_width * m_image_height * sq * sq;
  }
};

void root_lists(Graph &g, const rt_scene_desc *d, HittableList &world, HittableList &lights) {
  HittablePtr w = g.object(d->world);
  world = *std::static_pointer_cast<HittableList>(w);
  if (d->lights >= 0) lights = *std::static_pointer_cast<HittableList>(g.object(d->lights));
}

} // namespace

extern "C" {

/* INTEGRATION.md's binding against the real classes: rebuild `d` as reference
   objects, convert them back with RtSceneBuilder (ref_binding.hpp).  The tables
   behind *out stay valid until the next call. */
int ref_binding_roundtrip(const rt_scene_desc *d, rt_scene_desc *out) {
  static std::unique_ptr<RtSceneBuilder> builder;
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  builder.reset(new RtSceneBuilder());
  *out = builder->finish(world, lights, d->use_bvh != 0);
  return 0;
}

/* The reference's own scene builders (main.cpp:21-131, compiled from the
   reference's main.cpp text by oracle/Makefile) with the main-thread engine
   seeded by `seed` (the bouncing scene draws its layout from it), converted by
   INTEGRATION.md's binding.  which: 0 = populate_cornell_box_scene, 1 =
   populate_bouncing_spheres_scene.  *cam gets the CameraConfig fields the
   builder sets (CameraConfig.hpp defaults otherwise). */
int ref_populate_scene(int which, uint32_t seed, rt_scene_desc *out, rt_camera_desc *cam) {
  static std::unique_ptr<RtSceneBuilder> builder;
  HittableList world, lights;
  CameraConfig cfg;
  random_engine().seed(seed);
  if (which == 0)
    populate_cornell_box_scene(world, lights, cfg);
  else if (which == 1)
    populate_bouncing_spheres_scene(world, lights, cfg);
  else
    return -1;
  builder.reset(new RtSceneBuilder());
  *out = builder->finish(world, lights, false);
  cam->image_width = cfg.image_width;
  cam->samples_per_pixel = cfg.samples_per_pixel;
  cam->max_depth = cfg.max_depth;
  cam->aspect_ratio = cfg.aspect_ratio;
  cam->vfov = cfg.vfov;
  cam->defocus_angle = cfg.defocus_angle;
  cam->focus_dist = cfg.focus_dist;
  auto cv = [](const Vec3 &v) { return rt_vec3{v.x(), v.y(), v.z()}; };
  cam->lookfrom = cv(cfg.lookfrom);
  cam->lookat = cv(cfg.lookat);
  cam->vup = cv(cfg.vup);
  cam->background = cv(cfg.background);
  return 0;
}

int ref_camera_setup(const rt_camera_desc *cam, rt_frame *f) {
  GoldenCamera c(make_config(cam, false, false));
  c.setup();
  c.frame(f);
  return 0;
}

/* Seeded serial reference render -> scaled float radiance [H][W][3]. */
int ref_render(const rt_scene_desc *d, const rt_camera_desc *cam, uint32_t seed, int use_bvh,
               double *out) {
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  random_engine().seed(seed);
  GoldenCamera c(make_config(cam, use_bvh != 0, false));
  c.setup();
  if (use_bvh) { // StaticCamera.cpp:35-40
    if (!world.get_objects().empty()) world = HittableList(std::make_shared<BVHNode>(world));
    if (!lights.get_objects().empty()) lights = HittableList(std::make_shared<BVHNode>(lights));
  }
  c.trace(world, lights, out);
  return 0;
}

/* The reference's own StaticCamera::render (PPM writer included): writes
   output/<file> relative to the current directory.  parallel=1 is the -p path. */
int ref_render_static(const rt_scene_desc *d, const rt_camera_desc *cam, uint32_t seed,
                      int use_bvh, int parallel, const char *file) {
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  random_engine().seed(seed);
  StaticCamera c(make_config(cam, use_bvh != 0, parallel != 0), std::string(file));
  c.render(world, lights);
  return 0;
}

/* CPU baseline: the reference's own get_ray/ray_color over `threads` host
   threads with the reference's -p decomposition (one task per pixel of a row,
   a barrier per row, StaticCamera.cpp:60-100).  Each thread uses the
   reference's thread_local engine, seeded from random_device as in the
   reference's parallel mode, so the output is not deterministic.  Writes the
   scaled radiance like trace(); returns the number of samples traced. */
long long ref_trace_parallel(const rt_scene_desc *d, const rt_camera_desc *cam, int use_bvh,
                             int threads, double *out) {
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  GoldenCamera c(make_config(cam, use_bvh != 0, true));
  c.setup();
  if (use_bvh) {
    if (!world.get_objects().empty()) world = HittableList(std::make_shared<BVHNode>(world));
    if (!lights.get_objects().empty()) lights = HittableList(std::make_shared<BVHNode>(lights));
  }
  return c.trace_parallel(world, lights, threads, out);
}

/* CPU baseline, quota-sized: render_cpu's -p decomposition on the reference's
   own ThreadPool with `threads` workers (the reference sizes it by
   hardware_concurrency(), StaticCamera.cpp:60). */
long long ref_trace_pool(const rt_scene_desc *d, const rt_camera_desc *cam, int use_bvh,
                         int threads, double *out) {
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  GoldenCamera c(make_config(cam, use_bvh != 0, true));
  c.setup();
  if (use_bvh) {
    if (!world.get_objects().empty()) world = HittableList(std::make_shared<BVHNode>(world));
    if (!lights.get_objects().empty()) lights = HittableList(std::make_shared<BVHNode>(lights));
  }
  return c.trace_pool(world, lights, threads, out);
}

int ref_object_hit(const rt_scene_desc *d, int obj, const double ray[7], double tmin, double tmax,
                   double res[12]) {
  Graph g;
  g.load(d);
  HittablePtr h = g.object(obj);
  Ray r(Point3(ray[0], ray[1], ray[2]), Vec3(ray[3], ray[4], ray[5]), ray[6]);
  HitRecord rec;
  random_engine().seed(1u);
  if (!h->hit(r, Interval(tmin, tmax), rec)) return 0;
  int mi = -1;
  for (int k = 0; k < d->n_materials; ++k)
    if (g.mat[k] && g.mat[k] == rec.material) mi = k;
  // ConstantMedium::hit never writes u, v (ConstantMedium.cpp:25-94): whatever
  // the caller's -- or a HittableList's uninitialised temp -- record held stays.
  // Store 0 for medium hits so the fixtures regenerate byte for byte.  A hit is
  // a medium's when its material is the phase material of a medium reachable
  // from `obj` (through lists and transforms, not into medium boundaries) and
  // no surface reachable that way carries the same material: a surface's own
  // u, v are never overwritten.
  {
    std::vector<int> todo{obj}, seen(d->n_objects, 0);
    bool medium_mat = false, surface_mat = false;
    while (!todo.empty()) {
      const int k = todo.back();
      todo.pop_back();
      if (k < 0 || k >= d->n_objects || seen[k]) continue;
      seen[k] = 1;
      const rt_object_desc &o = d->objects[k];
      if (o.kind == RT_OBJ_MEDIUM) {
        if (o.phase == mi) medium_mat = true;
      } else if (o.kind == RT_OBJ_SPHERE || o.kind == RT_OBJ_QUAD) {
        if (o.material == mi) surface_mat = true;
      } else if (o.kind == RT_OBJ_LIST) {
        for (int c = 0; c < o.count; ++c) todo.push_back(d->children[o.child + c]);
      } else {
        todo.push_back(o.child); // rotate_y / translate
      }
    }
    if (medium_mat && !surface_mat) rec.u = rec.v = 0.0;
  }
  double v[12] = {rec.t,        rec.point.x(),  rec.point.y(),  rec.point.z(),
                  rec.normal.x(), rec.normal.y(), rec.normal.z(), rec.u,
                  rec.v,        rec.frontFace ? 1.0 : 0.0, (double)mi, 0};
  std::memcpy(res, v, sizeof v);
  return 1;
}

/* The two boundary queries of ConstantMedium::hit (ConstantMedium.cpp:28-32)
   for medium object `obj` on n rays (x, y, z, dx, dy, dz, time): the
   boundary's own hit over UNIVERSE_INTERVAL, then over (t1 + 0.0001, INF).
   out per ray: first hit?, t1, second hit?, t2 (0 where not reached). */
int ref_medium_boundary(const rt_scene_desc *d, int obj, const double *rays, int n, double *out) {
  Graph g;
  g.load(d);
  auto cm = std::dynamic_pointer_cast<ConstantMedium>(g.object(obj));
  if (!cm) return -1;
  HittablePtr b = cm->get_boundary();
  for (int k = 0; k < n; ++k) {
    const double *q = rays + 7 * k;
    Ray r(Point3(q[0], q[1], q[2]), Vec3(q[3], q[4], q[5]), q[6]);
    HitRecord rec1, rec2;
    double *o = out + 4 * k;
    o[0] = o[1] = o[2] = o[3] = 0.0;
    if (!b->hit(r, UNIVERSE_INTERVAL, rec1)) continue;
    o[0] = 1.0;
    o[1] = rec1.t;
    if (!b->hit(r, Interval(rec1.t + 0.0001, INF), rec2)) continue;
    o[2] = 1.0;
    o[3] = rec2.t;
  }
  return 0;
}

double ref_object_pdf(const rt_scene_desc *d, int obj, const double org[3], const double dir[3]) {
  Graph g;
  g.load(d);
  return g.object(obj)->pdf_value(Point3(org[0], org[1], org[2]), Vec3(dir[0], dir[1], dir[2]));
}

void ref_object_random(const rt_scene_desc *d, int obj, const double org[3], uint32_t seed,
                       double out[3]) {
  Graph g;
  g.load(d);
  random_engine().seed(seed);
  Vec3 v = g.object(obj)->random(Point3(org[0], org[1], org[2]));
  out[0] = v.x();
  out[1] = v.y();
  out[2] = v.z();
}

void ref_texture_value(const rt_scene_desc *d, int t, double u, double v, const double p[3],
                       double out[3]) {
  Graph g;
  g.load(d);
  Color c = g.texture(t)->value(u, v, Point3(p[0], p[1], p[2]));
  out[0] = c.x();
  out[1] = c.y();
  out[2] = c.z();
}

unsigned char ref_to_byte(double x) { return to_byte(x); }

/* Distribution KATs: n draws of the reference's own samplers from the seeded
   main-thread engine -- kind 0 random_unit_vector (rejection loop,
   Vec3Utility.hpp:53-64), 1 random_in_unit_disk (Vec3Utility.hpp:41-51), 2
   random_cosine_direction (Vec3Utility.hpp:94-103).  out: n x 3. */
int ref_sample_batch(int kind, uint32_t seed, int n, double *out) {
  random_engine().seed(seed);
  for (int k = 0; k < n; ++k) {
    Vec3 v = kind == 0 ? random_unit_vector() : kind == 1 ? random_in_unit_disk()
                                                          : random_cosine_direction();
    out[3 * k] = v.x();
    out[3 * k + 1] = v.y();
    out[3 * k + 2] = v.z();
  }
  return kind >= 0 && kind <= 2 ? 0 : -1;
}

/* n light directions from `org`: the reference's lights.random(org) -- the
   HittableList (HittableList.cpp:58-63) or, with use_bvh, HittableList(BVHNode)
   (BVHNode.cpp:149-166) over Plane::random / Sphere::random (Plane.cpp:128-132,
   Sphere.cpp:160-178) and the RotateY / Translate wrappers.  out: n x 3. */
int ref_light_batch(const rt_scene_desc *d, int use_bvh, const double org[3], uint32_t seed, int n,
                    double *out) {
  if (d->lights < 0) return -1;
  Graph g;
  g.load(d);
  HittableList world, lights;
  root_lists(g, d, world, lights);
  if (use_bvh && !lights.get_objects().empty())
    lights = HittableList(std::make_shared<BVHNode>(lights));
  random_engine().seed(seed);
  Point3 o(org[0], org[1], org[2]);
  for (int k = 0; k < n; ++k) {
    Vec3 v = lights.random(o);
    out[3 * k] = v.x();
    out[3 * k + 1] = v.y();
    out[3 * k + 2] = v.z();
  }
  return 0;
}

} // extern "C"
