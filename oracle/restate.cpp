/* oracle/restate.cpp — CPU RESTATEMENT OF THE REFERENCE HOT PATH.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline.  The product (real-time-ray-tracing-engine_amd/) never links it.
 *
 * What it restates (paths relative to the reference repo, src/):
 *   camera setup            core/camera/Camera.cpp:31-73
 *   get_ray / stratified    core/camera/Camera.cpp:152-230
 *   ray_color (recursive)   core/camera/Camera.cpp:232-309
 *   render loop + scale     core/camera/StaticCamera.cpp:32-134
 *   HittableList            core/HittableList.cpp:26-63
 *   BVHNode build/traverse  optimization/BVHNode.cpp:21-446, BVHNode.hpp:46-170
 *   AABB                    optimization/AABB.cpp:7-175
 *   Sphere                  scene/objects/Sphere.cpp:8-178
 *   Plane (quad)            scene/objects/Plane.cpp:6-132
 *   RotateY / Translate     scene/objects/RotateY.cpp:5-103, Translate.cpp:7-39
 *   ConstantMedium          scene/mediums/ConstantMedium.cpp:25-94
 *   materials               scene/materials/{Lambertian,Metal,Dielectric,DiffuseLight,Isotropic}Material.cpp
 *   textures + Perlin       scene/textures/{SolidColor,Checker,Noise}Texture.cpp, utils/math/PerlinNoise.hpp:43-201
 *   PDFs / ONB / sampling   utils/math/PDF.hpp, ONB.hpp, Vec3Utility.hpp, Vec3.hpp
 *   RNG                     utils/math/Utility.hpp:16-37
 *   quantisation            utils/ColorUtility.hpp:11-36
 *
 * Two RNG modes:
 *   MT      replays the reference's libstdc++ std::mt19937 draws in the order g++
 *           evaluates them (argument lists right to left),
 *           including the rejection loops — bit-parity with the seeded reference.
 *   COUNTER the contract shared with the HIP kernel (DESIGN.md "RNG contract"):
 *           Philox4x32-10 keyed by (seed; pixel, stratum sample, bounce, slot),
 *           analytic unit-vector/disk sampling, one-uniform light-leaf selection.
 * Deliberate, documented deviations from the reference:
 *   - DielectricMaterial's scattered Ray keeps the incoming ray time (the reference
 *     leaves it uninitialised, DielectricMaterial.cpp:82 — UB).
 *   - light pdf_value rays use time 0 (reference: uninitialised, Sphere.cpp:149).
 */
#include "../include/rt_api.h"
#include "philox.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <random>
#include <thread>
#include <vector>

namespace orc {

static const double INF = std::numeric_limits<double>::infinity();
static const double PI = 3.1415926535897932385; // Utility.hpp:9

/* ---------------------------------------------------------------- vectors */
struct V {
  double x, y, z;
  double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  double &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
static inline V mk(double x, double y, double z) { return V{x, y, z}; }
static inline V operator+(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V operator-(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V operator*(V a, V b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V operator*(double t, V v) { return mk(t * v.x, t * v.y, t * v.z); }
static inline V operator*(V v, double t) { return t * v; }
static inline V operator/(V v, double t) { return (1 / t) * v; } // Vec3Utility.hpp:25
static inline V operator-(V v) { return mk(-v.x, -v.y, -v.z); }
static inline double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double len2(V v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
static inline double len(V v) { return std::sqrt(len2(v)); }
static inline V cross(V a, V b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V unit(V v) { // Vec3::normalize, Vec3.hpp:150-158
  double l = len(v);
  if (l > 1e-8) {
    double s = 1.0 / l;
    return mk(v.x * s, v.y * s, v.z * s);
  }
  return mk(1.0, 0.0, 0.0);
}
static inline V from(const rt_vec3 &v) { return mk(v.x, v.y, v.z); }
static inline rt_vec3 to(V v) { return rt_vec3{v.x, v.y, v.z}; }

struct Ival {
  double lo, hi;
  bool contains(double t) const { return lo <= t && t <= hi; }
  bool surrounds(double t) const { return lo < t && t < hi; }
  double size() const { return hi - lo; }
};
static inline Ival ival_expand(Ival a, double delta) {
  double p = delta * 0.5;
  return Ival{a.lo - p, a.hi + p};
}
static inline Ival ival_union(Ival a, Ival b) {
  return Ival{a.lo <= b.lo ? a.lo : b.lo, a.hi >= b.hi ? a.hi : b.hi};
}

struct Ray {
  V o, d;
  double tm;
  V at(double t) const { return mk(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z); }
};

/* ------------------------------------------------------------------ AABB */
struct Box {
  Ival a[3];
};
static inline void box_pad(Box &b) { // AABB::pad_to_minimums, AABB.cpp:167-175
  for (int i = 0; i < 3; ++i)
    if (b.a[i].size() < 0.0001) b.a[i] = ival_expand(b.a[i], 0.0001);
}
static inline Box box_ivals(Ival x, Ival y, Ival z) {
  Box b{{x, y, z}};
  box_pad(b);
  return b;
}
static inline Box box_pts(V p, V q) {
  Box b;
  for (int i = 0; i < 3; ++i) b.a[i] = (p[i] <= q[i]) ? Ival{p[i], q[i]} : Ival{q[i], p[i]};
  box_pad(b);
  return b;
}
static inline Box box_join(const Box &p, const Box &q) {
  return Box{{ival_union(p.a[0], q.a[0]), ival_union(p.a[1], q.a[1]), ival_union(p.a[2], q.a[2])}};
}
static const Box EMPTY_BOX = box_ivals(Ival{INF, -INF}, Ival{INF, -INF}, Ival{INF, -INF});
static inline int box_longest(const Box &b) { // AABB.cpp:43-48
  if (b.a[0].size() > b.a[1].size()) return b.a[0].size() > b.a[2].size() ? 0 : 2;
  return b.a[1].size() > b.a[2].size() ? 1 : 2;
}
static inline V box_center(const Box &b) {
  return mk((b.a[0].lo + b.a[0].hi) * 0.5, (b.a[1].lo + b.a[1].hi) * 0.5,
            (b.a[2].lo + b.a[2].hi) * 0.5);
}
static inline double box_area(const Box &b) {
  double dx = b.a[0].size(), dy = b.a[1].size(), dz = b.a[2].size();
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}
static bool box_hit(const Box &b, const Ray &r, Ival t) { // AABB.cpp:139-165 (scalar path)
  for (int ax = 0; ax < 3; ++ax) {
    const Ival &iv = b.a[ax];
    const double inv = 1.0 / r.d[ax];
    double t0 = (iv.lo - r.o[ax]) * inv;
    double t1 = (iv.hi - r.o[ax]) * inv;
    if (t0 < t1) {
      if (t0 > t.lo) t.lo = t0;
      if (t1 < t.hi) t.hi = t1;
    } else {
      if (t1 > t.lo) t.lo = t1;
      if (t0 < t.hi) t.hi = t0;
    }
    if (t.hi <= t.lo) return false;
  }
  return true;
}

/* -------------------------------------------------------------- sampling */
enum { MODE_MT = 0, MODE_COUNTER = 1 };

// Slots of the counter contract (DESIGN.md "RNG contract").
static const uint32_t CAM_TAG = 0xFFFFFFFFu;
enum { SLOT_SHADE = 0, SLOT_MEDIUM_BASE = 0x100 };

struct Sampler {
  int mode;
  std::mt19937 *eng;
  uint64_t seed;
  uint32_t pixel, sample, bounce;

  // ---- MT mode primitives (Utility.hpp:22-37)
  double rd() { return std::uniform_real_distribution<double>(0.0, 1.0)(*eng); }
  double rd(double a, double b) { return std::uniform_real_distribution<double>(a, b)(*eng); }
  int ri(int a, int b) { return std::uniform_int_distribution<int>(a, b)(*eng); }
  // ---- counter mode primitive
  void ctr(uint32_t bnc, uint32_t slot, double out[4]) const {
    oracle_philox_u01x4(seed, pixel, sample, bnc, slot, out);
  }
};

// Vec3::random(min,max): g++ evaluates the three constructor arguments right to
// left, so z is drawn first (Vec3.hpp:119-126).
static V mt_vec_random(Sampler &s, double a, double b) {
  double z = s.rd(a, b);
  double y = s.rd(a, b);
  double x = s.rd(a, b);
  return mk(x, y, z);
}
// random_unit_vector (Vec3Utility.hpp:53-64), MT: rejection loop.
static V mt_unit_vector(Sampler &s) {
  for (;;) {
    V v = mt_vec_random(s, -1, 1);
    double l2 = len2(v);
    if (1e-160 < l2 && l2 <= 1.0) return v / std::sqrt(l2);
  }
}
// random_in_unit_disk (Vec3Utility.hpp:41-51), MT: y drawn before x.
static V mt_in_unit_disk(Sampler &s) {
  for (;;) {
    double y = s.rd(-1, 1);
    double x = s.rd(-1, 1);
    V p = mk(x, y, 0);
    if (len2(p) < 1) return p;
  }
}
// Counter-mode analytic forms (same distributions; cf. Vec3Utility.cuh:57-72).
static V ctr_unit_vector(double u1, double u2) {
  double z = 1.0 - 2.0 * u1;
  double r = std::sqrt(std::fmax(0.0, 1.0 - z * z));
  double phi = 2.0 * PI * u2;
  return mk(r * std::cos(phi), r * std::sin(phi), z);
}
static V ctr_in_unit_disk(double u1, double u2) {
  double r = std::sqrt(u1);
  double th = 2.0 * PI * u2;
  return mk(r * std::cos(th), r * std::sin(th), 0.0);
}
// random_cosine_direction (Vec3Utility.hpp:94-103)
static V cosine_dir(double r1, double r2) {
  double phi = 2 * PI * r1;
  double x = std::cos(phi) * std::sqrt(r2);
  double y = std::sin(phi) * std::sqrt(r2);
  double z = std::sqrt(1 - r2);
  return mk(x, y, z);
}

/* ------------------------------------------------------------------- ONB */
struct Onb { // ONB.hpp:19-71
  V ax[3];
  explicit Onb(V n) {
    ax[2] = unit(n);
    V a = (std::fabs(ax[2].x) > 0.9) ? mk(0, 1, 0) : mk(1, 0, 0);
    ax[1] = unit(cross(ax[2], a));
    ax[0] = cross(ax[2], ax[1]);
  }
  V xf(V v) const { return (v[0] * ax[0]) + (v[1] * ax[1]) + (v[2] * ax[2]); }
};

/* -------------------------------------------------------------- textures */
struct Scene;
struct Hit {
  V p{0, 0, 0}, n{0, 0, 0};
  double t = 0, u = 0, v = 0;
  int mat = -1;
  bool front = false;
  void set_face(const Ray &r, V outward) { // HitRecord.hpp:42-45
    front = dot(r.d, outward) < 0;
    n = front ? outward : -outward;
  }
};

/* -------------------------------------------------------------- objects */
enum OKind { O_SPHERE, O_QUAD, O_LIST, O_ROT, O_TRANS, O_MEDIUM, O_BVH };

struct FlatNode {
  Box box;
  bool leaf;
  uint32_t a, b; // inner: left,right ; leaf: prim_offset, prim_count
};

struct Obj {
  OKind kind;
  int id = -1; // desc object index (counter-mode medium key); -1 for synthetic nodes
  int mat = -1;
  Box bbox;
  // sphere
  V c0{0, 0, 0}, cdir{0, 0, 0};
  double radius = 0;
  // quad
  V Q{0, 0, 0}, qu{0, 0, 0}, qv{0, 0, 0}, qn{0, 0, 0}, qw{0, 0, 0};
  double D = 0, area = 0;
  // rotate
  double sin_t = 0, cos_t = 1;
  // translate
  V off{0, 0, 0};
  // medium
  double density = 0;
  int phase = -1;
  // composite
  std::vector<Obj *> kids; // list children; rot/trans/medium: kids[0]; bvh: left,right
  // flattened BVH (BVHNode.cpp:322-446)
  bool flat = false;
  std::vector<FlatNode> fnodes;
  std::vector<Obj *> fprims;
};

struct Scene {
  std::vector<std::unique_ptr<Obj>> pool;
  std::vector<rt_texture_desc> tex;
  std::vector<rt_perlin_desc> perlin;
  std::vector<rt_material_desc> mats;
  Obj *world = nullptr;
  Obj *lights = nullptr; // list or nullptr
  // counter mode: flattened light leaves
  struct LightLeaf {
    Obj *prim;
    double weight;
    std::vector<Obj *> chain; // transforms, outermost first
  };
  std::vector<LightLeaf> leaves;
  std::vector<double> leaf_cum;
  Obj *make(OKind k) {
    pool.emplace_back(new Obj());
    pool.back()->kind = k;
    return pool.back().get();
  }
};

/* -------------------------------------------------------- texture eval */
static double perlin_noise(const rt_perlin_desc &P, V p) { // PerlinNoise.hpp:43-60
  double xf = p.x - std::floor(p.x), yf = p.y - std::floor(p.y), zf = p.z - std::floor(p.z);
  int xi = int(std::floor(p.x)), yi = int(std::floor(p.y)), zi = int(std::floor(p.z));
  V c[2][2][2];
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++)
        c[di][dj][dk] = from(P.rand_vec[P.perm_x[(xi + di) & 255] ^ P.perm_y[(yi + dj) & 255] ^
                                        P.perm_z[(zi + dk) & 255]]);
  // perlin_interp, PerlinNoise.hpp:186-201 (scalar branch)
  double uu = xf * xf * (3 - 2 * xf), vv = yf * yf * (3 - 2 * yf), ww = zf * zf * (3 - 2 * zf);
  double acc = 0.0;
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++)
      for (int k = 0; k < 2; k++) {
        V wv = mk(xf - i, yf - j, zf - k);
        acc += (i * uu + (1 - i) * (1 - uu)) * (j * vv + (1 - j) * (1 - vv)) *
               (k * ww + (1 - k) * (1 - ww)) * dot(c[i][j][k], wv);
      }
  return acc;
}
static double perlin_turb(const rt_perlin_desc &P, V p, int depth) { // PerlinNoise.hpp:62-75
  double acc = 0.0, w = 1.0;
  V tp = p;
  for (int i = 0; i < depth; i++) {
    acc += w * perlin_noise(P, tp);
    w *= 0.5;
    tp = mk(tp.x * 2, tp.y * 2, tp.z * 2);
  }
  return std::fabs(acc);
}
static V tex_value(const Scene &S, int t, double u, double v, V p) {
  for (;;) {
    const rt_texture_desc &T = S.tex[t];
    if (T.kind == RT_TEX_SOLID) return from(T.color);
    if (T.kind == RT_TEX_CHECKER) { // CheckerTexture.cpp:41-55
      double inv = 1.0 / T.scale;
      int xi = int(std::floor(inv * p.x)), yi = int(std::floor(inv * p.y)),
          zi = int(std::floor(inv * p.z));
      bool even = (xi + yi + zi) % 2 == 0;
      t = even ? T.even : T.odd;
      continue;
    }
    // NoiseTexture.cpp:31-34
    double f = 1 + std::sin(T.scale * p.z + 10 * perlin_turb(S.perlin[T.perlin], p, 7));
    return mk(0.5, 0.5, 0.5) * f;
  }
}

/* ------------------------------------------------------------- hit code */
struct Ctx {
  const Scene *S;
  Sampler *smp;
};

static bool obj_hit(const Ctx &C, const Obj *o, const Ray &r, Ival t, Hit &rec);

static bool sphere_hit(const Obj *o, const Ray &r, Ival t, Hit &rec) { // Sphere.cpp:101-143
  V cc = mk(o->c0.x + r.tm * o->cdir.x, o->c0.y + r.tm * o->cdir.y, o->c0.z + r.tm * o->cdir.z);
  V oc = cc - r.o;
  double a = len2(r.d);
  double h = dot(r.d, oc);
  double c = len2(oc) - o->radius * o->radius;
  double disc = h * h - a * c;
  if (disc < 0) return false;
  double sq = std::sqrt(disc);
  double root = (h - sq) / a;
  if (!t.surrounds(root)) {
    root = (h + sq) / a;
    if (!t.surrounds(root)) return false;
  }
  rec.t = root;
  rec.p = r.at(rec.t);
  V on = (rec.p - cc) / o->radius;
  rec.set_face(r, on);
  rec.mat = o->mat;
  double theta = std::acos(-on.y);
  double phi = std::atan2(-on.z, on.x) + PI;
  rec.u = phi / (2 * PI);
  rec.v = theta / PI;
  return true;
}

static bool quad_hit(const Obj *o, const Ray &r, Ival t, Hit &rec) { // Plane.cpp:76-113
  double denom = dot(o->qn, r.d);
  if (std::fabs(denom) < 1e-8) return false;
  double tt = (o->D - dot(o->qn, r.o)) / denom;
  if (!t.contains(tt)) return false;
  V ip = r.at(tt);
  V pv = ip - o->Q;
  double alpha = dot(o->qw, cross(pv, o->qv));
  double beta = dot(o->qw, cross(o->qu, pv));
  Ival unit_iv{0, 1};
  if (!unit_iv.contains(alpha) || !unit_iv.contains(beta)) return false;
  rec.u = alpha;
  rec.v = beta;
  rec.t = tt;
  rec.p = ip;
  rec.mat = o->mat;
  rec.set_face(r, o->qn);
  return true;
}

static bool list_hit(const Ctx &C, const std::vector<Obj *> &kids, const Ray &r, Ival t,
                     Hit &rec) { // HittableList.cpp:26-42
  Hit tmp;
  bool any = false;
  double closest = t.hi;
  for (const Obj *k : kids) {
    if (obj_hit(C, k, r, Ival{t.lo, closest}, tmp)) {
      any = true;
      closest = tmp.t;
      rec = tmp;
    }
  }
  return any;
}

static bool bvh_flat_hit(const Ctx &C, const Obj *o, const Ray &r, Ival t, Hit &rec) {
  // BVHNode::hit_flattened, BVHNode.cpp:385-446
  if (o->fnodes.empty()) return false;
  bool any = false;
  struct E {
    uint32_t idx;
    double tmin;
  } st[64];
  int sp = 0;
  st[sp++] = {0, t.lo};
  while (sp > 0) {
    E e = st[--sp];
    if (e.tmin >= t.hi) continue;
    const FlatNode &n = o->fnodes[e.idx];
    Ival nt = t; // AABB::hit takes the interval by value: nt is not narrowed
    if (!box_hit(n.box, r, nt)) continue;
    if (n.leaf) {
      for (uint32_t i = 0; i < n.b; ++i)
        if (obj_hit(C, o->fprims[n.a + i], r, t, rec)) {
          any = true;
          t.hi = rec.t;
        }
    } else {
      uint32_t first = n.a, second = n.b;
      if (r.d[box_longest(n.box)] < 0) std::swap(first, second);
      if (sp < 63) {
        st[sp++] = {second, nt.lo};
        st[sp++] = {first, nt.lo};
      }
    }
  }
  return any;
}

static bool medium_hit(const Ctx &C, const Obj *o, const Ray &r, Ival t, Hit &rec) {
  // ConstantMedium.cpp:25-94
  Hit r1, r2;
  const Obj *bd = o->kids[0];
  if (!obj_hit(C, bd, r, Ival{-INF, INF}, r1)) return false;
  if (!obj_hit(C, bd, r, Ival{r1.t + 0.0001, INF}, r2)) return false;
  if (r1.t < t.lo) r1.t = t.lo;
  if (r2.t > t.hi) r2.t = t.hi;
  if (r1.t >= r2.t) return false;
  if (r1.t < 0) r1.t = 0;
  double rl = len(r.d);
  double dist_inside = (r2.t - r1.t) * rl;
  double nid = -1.0 / o->density;
  double u;
  Sampler &s = *C.smp;
  if (s.mode == MODE_MT) {
    u = s.rd();
  } else {
    double d[4];
    s.ctr(s.bounce, SLOT_MEDIUM_BASE + (uint32_t)o->id, d);
    u = d[0];
  }
  double hd = nid * std::log(u);
  if (hd > dist_inside) return false;
  rec.t = r1.t + hd / rl;
  rec.p = r.at(rec.t);
  rec.n = mk(1, 0, 0);
  rec.front = true;
  rec.mat = o->phase;
  return true;
}

static bool obj_hit(const Ctx &C, const Obj *o, const Ray &r, Ival t, Hit &rec) {
  switch (o->kind) {
  case O_SPHERE:
    return sphere_hit(o, r, t, rec);
  case O_QUAD:
    return quad_hit(o, r, t, rec);
  case O_LIST:
    return list_hit(C, o->kids, r, t, rec);
  case O_ROT: { // RotateY.cpp:41-76
    double s = o->sin_t, c = o->cos_t;
    V org = mk((c * r.o.x) - (s * r.o.z), r.o.y, (s * r.o.x) + (c * r.o.z));
    V dir = mk((c * r.d.x) - (s * r.d.z), r.d.y, (s * r.d.x) + (c * r.d.z));
    Ray rr{org, dir, r.tm};
    if (!obj_hit(C, o->kids[0], rr, t, rec)) return false;
    rec.p = mk((c * rec.p.x) + (s * rec.p.z), rec.p.y, (-s * rec.p.x) + (c * rec.p.z));
    rec.n = mk((c * rec.n.x) + (s * rec.n.z), rec.n.y, (-s * rec.n.x) + (c * rec.n.z));
    return true;
  }
  case O_TRANS: { // Translate.cpp:17-31
    Ray rr{r.o - o->off, r.d, r.tm};
    if (!obj_hit(C, o->kids[0], rr, t, rec)) return false;
    rec.p = rec.p + o->off;
    return true;
  }
  case O_MEDIUM:
    return medium_hit(C, o, r, t, rec);
  case O_BVH: { // BVHNode.cpp:127-147
    if (o->flat) return bvh_flat_hit(C, o, r, t, rec);
    if (!box_hit(o->bbox, r, t)) return false;
    bool lh = obj_hit(C, o->kids[0], r, t, rec);
    bool rh = obj_hit(C, o->kids[1], r, Ival{t.lo, lh ? rec.t : t.hi}, rec);
    return lh || rh;
  }
  }
  return false;
}

/* ------------------------------------------------- pdf_value / random */
static double obj_pdf(const Ctx &C, const Obj *o, V org, V dir) {
  switch (o->kind) {
  case O_SPHERE: { // Sphere.cpp:145-158 (ray time taken as 0)
    Hit rec;
    if (!sphere_hit(o, Ray{org, dir, 0.0}, Ival{0.001, INF}, rec)) return 0;
    V c = mk(o->c0.x + 0 * o->cdir.x, o->c0.y + 0 * o->cdir.y, o->c0.z + 0 * o->cdir.z);
    double dist2 = len2(c - org);
    double ctm = std::sqrt(1 - o->radius * o->radius / dist2);
    double sa = 2 * PI * (1 - ctm);
    return 1 / sa;
  }
  case O_QUAD: { // Plane.cpp:115-126
    Hit rec;
    if (!quad_hit(o, Ray{org, dir, 0.0}, Ival{0.001, INF}, rec)) return 0;
    double d2 = rec.t * rec.t * len2(dir);
    double cosine = std::fabs(dot(dir, rec.n) / len(dir));
    return d2 / (cosine * o->area);
  }
  case O_LIST: { // HittableList.cpp:44-56
    double w = 1.0 / o->kids.size();
    double sum = 0.0;
    for (const Obj *k : o->kids) sum += w * obj_pdf(C, k, org, dir);
    return sum;
  }
  case O_BVH: // BVHNode.cpp:149-157
    return 0.5 * obj_pdf(C, o->kids[0], org, dir) + 0.5 * obj_pdf(C, o->kids[1], org, dir);
  case O_ROT: { // RotateY.cpp:78-89
    double s = o->sin_t, c = o->cos_t;
    V ro = mk(c * org.x - s * org.z, org.y, s * org.x + c * org.z);
    V rd = mk(c * dir.x - s * dir.z, dir.y, s * dir.x + c * dir.z);
    return obj_pdf(C, o->kids[0], ro, rd);
  }
  case O_TRANS:
    return obj_pdf(C, o->kids[0], org - o->off, dir);
  default:
    return 0.0; // Hittable::pdf_value default, Hittable.hpp:37-39
  }
}

// Primitive sampling with explicit uniforms (used by both modes).
static V sphere_random_u(const Obj *o, V org, double r1, double r2) { // Sphere.cpp:160-178
  V c = mk(o->c0.x + 0 * o->cdir.x, o->c0.y + 0 * o->cdir.y, o->c0.z + 0 * o->cdir.z);
  V dir = c - org;
  double d2 = len2(dir);
  Onb uvw(dir);
  double z = 1 + r2 * (std::sqrt(1 - o->radius * o->radius / d2) - 1);
  double phi = 2 * PI * r1;
  double x = std::cos(phi) * std::sqrt(1 - z * z);
  double y = std::sin(phi) * std::sqrt(1 - z * z);
  return uvw.xf(mk(x, y, z));
}
static V quad_random_u(const Obj *o, V org, double su, double sv) { // Plane.cpp:128-132
  V p = o->Q + (su * o->qu) + (sv * o->qv);
  return p - org;
}
static V rot_in(const Obj *o, V p) {
  return mk(o->cos_t * p.x - o->sin_t * p.z, p.y, o->sin_t * p.x + o->cos_t * p.z);
}
static V rot_out(const Obj *o, V d) {
  return mk(o->cos_t * d.x + o->sin_t * d.z, d.y, -o->sin_t * d.x + o->cos_t * d.z);
}

// MT mode: the reference's recursive random() with its own draws.
static V mt_obj_random(const Ctx &C, const Obj *o, V org) {
  Sampler &s = *C.smp;
  switch (o->kind) {
  case O_SPHERE: {
    double r1 = s.rd();
    double r2 = s.rd();
    return sphere_random_u(o, org, r1, r2);
  }
  case O_QUAD: { // v coefficient drawn first (right-to-left operand evaluation)
    double sv = s.rd();
    double su = s.rd();
    return quad_random_u(o, org, su, sv);
  }
  case O_LIST: {
    int n = int(o->kids.size());
    return mt_obj_random(C, o->kids[s.ri(0, n - 1)], org);
  }
  case O_BVH:
    if (s.ri(0, 1) == 0) return mt_obj_random(C, o->kids[0], org);
    return mt_obj_random(C, o->kids[1], org);
  case O_ROT:
    return rot_out(o, mt_obj_random(C, o->kids[0], rot_in(o, org)));
  case O_TRANS:
    return mt_obj_random(C, o->kids[0], org - o->off);
  default:
    return mk(1, 0, 0);
  }
}

// Counter mode: one uniform picks a light leaf by cumulative weight, the DIR slot
// samples it; transforms are applied along the leaf's chain.
static V ctr_light_random(const Ctx &C, V org, double upick, double r1, double r2) {
  const Scene &S = *C.S;
  size_t n = S.leaves.size();
  size_t k = n - 1;
  for (size_t i = 0; i < n; ++i)
    if (upick < S.leaf_cum[i]) {
      k = i;
      break;
    }
  const Scene::LightLeaf &L = S.leaves[k];
  V p = org;
  for (const Obj *t : L.chain) p = (t->kind == O_TRANS) ? p - t->off : rot_in(t, p);
  V d;
  if (L.prim->kind == O_SPHERE)
    d = sphere_random_u(L.prim, p, r1, r2);
  else if (L.prim->kind == O_QUAD)
    d = quad_random_u(L.prim, p, r1, r2);
  else
    d = mk(1, 0, 0);
  for (size_t i = L.chain.size(); i-- > 0;)
    if (L.chain[i]->kind == O_ROT) d = rot_out(L.chain[i], d);
  return d;
}

/* -------------------------------------------------------------- camera */
struct Cam {
  int W, H, spp, depth;
  double scale, defocus_angle;
  V center, p00, du, dv, u, v, w, disk_u, disk_v, bg;
};

static Cam cam_setup(const rt_camera_desc &cd) { // Camera.cpp:31-73
  Cam c;
  c.W = cd.image_width;
  c.spp = cd.samples_per_pixel;
  c.depth = cd.max_depth;
  c.H = int(c.W / cd.aspect_ratio);
  c.H = (c.H < 1) ? 1 : c.H;
  c.scale = 1.0 / c.spp;
  c.center = from(cd.lookfrom);
  double theta = cd.vfov * PI / 180.0;
  double h = std::tan(theta / 2);
  double vh = 2 * h * cd.focus_dist;
  double vw = vh * (double(c.W) / c.H);
  c.w = unit(from(cd.lookfrom) - from(cd.lookat));
  c.u = unit(cross(from(cd.vup), c.w));
  c.v = cross(c.w, c.u);
  V vu = vw * c.u;
  V vv = vh * -c.v;
  c.du = vu / c.W;
  c.dv = vv / c.H;
  V ul = c.center - (cd.focus_dist * c.w) - vu / 2 - vv / 2;
  c.p00 = ul + 0.5 * (c.du + c.dv);
  double rad = cd.focus_dist * std::tan((cd.defocus_angle / 2) * PI / 180.0);
  c.disk_u = c.u * rad;
  c.disk_v = c.v * rad;
  c.defocus_angle = cd.defocus_angle;
  c.bg = from(cd.background);
  return c;
}

static Ray get_ray(const Cam &c, Sampler &s, int i, int j, int si, int sj) { // Camera.cpp:186-216
  int sq = int(std::sqrt(c.spp));
  double rs = 1.0 / sq;
  double a, b, tm = 0;
  V disk{0, 0, 0};
  if (s.mode == MODE_MT) {
    a = s.rd();
    b = s.rd();
  } else { // jitter and time from one block (slot 0)
    double d[4];
    s.ctr(CAM_TAG, 0, d);
    a = d[0];
    b = d[1];
    tm = d[2];
  }
  double px = ((si + a) * rs) - 0.5;
  double py = ((sj + b) * rs) - 0.5;
  V ps = c.p00 + ((i + px) * c.du) + ((j + py) * c.dv);
  V org;
  if (c.defocus_angle <= 0) {
    org = c.center;
  } else {
    if (s.mode == MODE_MT) {
      disk = mt_in_unit_disk(s);
    } else {
      double d[4];
      s.ctr(CAM_TAG, 1, d);
      disk = ctr_in_unit_disk(d[0], d[1]);
    }
    org = c.center + (disk[0] * c.disk_u) + (disk[1] * c.disk_v); // Camera.cpp:226-230
  }
  V dir = ps - org;
  if (s.mode == MODE_MT) tm = s.rd();
  return Ray{org, dir, tm};
}

/* ---------------------------------------------------------- integrator */
struct Counters {
  uint64_t segments = 0;
};

static V ray_color(const Ctx &C, const Cam &cam, const Ray &r, int depth) { // Camera.cpp:232-309
  if (depth <= 0) return mk(0, 0, 0);
  Sampler &s = *C.smp;
  const Scene &S = *C.S;
  s.bounce = (uint32_t)(cam.depth - depth);
  Hit rec;
  if (!obj_hit(C, S.world, r, Ival{0.001, INF}, rec)) return cam.bg;
  const rt_material_desc &M = S.mats[rec.mat];
  V emitted = mk(0, 0, 0);
  if (M.kind == RT_MAT_DIFFUSE_LIGHT) // DiffuseLightMaterial.cpp:12-22
    emitted = rec.front ? tex_value(S, M.texture, rec.u, rec.v, rec.p) : mk(0, 0, 0);

  double ev[2] = {0, 0}, dv[2] = {0, 0};
  if (s.mode == MODE_COUNTER) { // one block per shading event: (e0, e1, d0, d1)
    double d[4];
    s.ctr(s.bounce, SLOT_SHADE, d);
    ev[0] = d[0];
    ev[1] = d[1];
    dv[0] = d[2];
    dv[1] = d[3];
  }
  V att;
  if (M.kind == RT_MAT_DIFFUSE_LIGHT) return emitted; // Material::scatter default false
  if (M.kind == RT_MAT_METAL) {                       // MetalMaterial.cpp:43-62
    V refl = r.d - 2 * dot(r.d, rec.n) * rec.n;
    V uv = (s.mode == MODE_MT) ? mt_unit_vector(s) : ctr_unit_vector(dv[0], dv[1]);
    refl = unit(refl) + (M.fuzz * uv);
    Ray sr{rec.p, refl, r.tm};
    return from(M.albedo) * ray_color(C, cam, sr, depth - 1);
  }
  if (M.kind == RT_MAT_DIELECTRIC) { // DielectricMaterial.cpp:58-85
    double ri = rec.front ? (1.0 / M.refraction_index) : M.refraction_index;
    V ud = unit(r.d);
    double ct = std::fmin(dot(-ud, rec.n), 1.0);
    double st = std::sqrt(1.0 - ct * ct);
    bool cannot = ri * st > 1.0;
    double r0 = (1 - ri) / (1 + ri);
    r0 = r0 * r0;
    double refl = r0 + (1 - r0) * std::pow((1 - ct), 5);
    bool do_reflect = cannot;
    if (!do_reflect) do_reflect = refl > ((s.mode == MODE_MT) ? s.rd() : ev[0]);
    V dir;
    if (do_reflect) {
      dir = ud - 2 * dot(ud, rec.n) * rec.n;
    } else { // refract, Vec3Utility.hpp:80-88
      double c2 = std::fmin(dot(-ud, rec.n), 1.0);
      V perp = ri * (ud + c2 * rec.n);
      V par = -std::sqrt(std::fabs(1.0 - len2(perp))) * rec.n;
      dir = perp + par;
    }
    Ray sr{rec.p, dir, r.tm}; // deviation: reference leaves time uninitialised
    return mk(1.0, 1.0, 1.0) * ray_color(C, cam, sr, depth - 1);
  }
  // Lambertian (cosine PDF) or Isotropic (sphere PDF)
  bool lamb = (M.kind == RT_MAT_LAMBERTIAN);
  att = tex_value(S, M.texture, rec.u, rec.v, rec.p);
  bool have_lights = S.lights && !S.lights->kids.empty();
  Onb uvw(rec.n);
  // MixturePDF::generate (PDF.hpp:145-149): p0 = lights (or material when no lights)
  V gdir;
  if (s.mode == MODE_MT) {
    bool first = s.rd() < 0.5;
    if (first && have_lights) {
      gdir = mt_obj_random(C, S.lights, rec.p);
    } else if (lamb) {
      double r1 = s.rd();
      double r2 = s.rd();
      gdir = uvw.xf(cosine_dir(r1, r2));
    } else {
      gdir = mt_unit_vector(s);
    }
  } else {
    bool first = ev[0] < 0.5;
    if (first && have_lights)
      gdir = ctr_light_random(C, rec.p, ev[1], dv[0], dv[1]);
    else if (lamb)
      gdir = uvw.xf(cosine_dir(dv[0], dv[1]));
    else
      gdir = ctr_unit_vector(dv[0], dv[1]);
  }
  Ray sc{rec.p, gdir, r.tm};
  // MixturePDF::value (PDF.hpp:140-143)
  double mat_pdf;
  if (lamb) {
    double ct = dot(unit(sc.d), uvw.ax[2]);
    mat_pdf = std::fmax(0, ct / PI);
  } else {
    mat_pdf = 1.0 / (4.0 * PI);
  }
  double p0 = have_lights ? obj_pdf(C, S.lights, rec.p, sc.d) : mat_pdf;
  double pdf = 0.5 * p0 + 0.5 * mat_pdf;
  double spdf;
  if (lamb) { // LambertianMaterial.cpp:41-56
    double ct = dot(rec.n, unit(sc.d));
    spdf = ct < 0 ? 0 : ct / PI;
  } else {
    spdf = 1 / (4 * PI);
  }
  if (s.mode == MODE_COUNTER && spdf == 0.0 && pdf > 0.0 && std::isfinite(pdf)) {
    // Counter contract: a zero-weight continuation is not traced (the reference's
    // recursion would multiply a finite sample by exactly 0).
    return emitted;
  }
  V sample = ray_color(C, cam, sc, depth - 1);
  V scat = (att * spdf * sample) / pdf;
  return emitted + scat;
}

/* -------------------------------------------------------- scene build */
struct Builder {
  Scene *S;
  const rt_scene_desc *D;
  std::vector<Obj *> built;
  int use_bvh;
  Obj *build(int idx);
};

static Box obj_bbox(const Obj *o) { return o->bbox; }

// BVHNode construction (BVHNode.cpp:21-123) over a vector of Obj*.
struct BvhBuild {
  Scene *S;
  Obj *node(std::vector<Obj *> &ob, size_t st, size_t en);
  double sah_cost(const Obj *self, std::vector<Obj *> &ob, size_t st, size_t en, int axis,
                  double pos);
};

double BvhBuild::sah_cost(const Obj *self, std::vector<Obj *> &ob, size_t st, size_t en, int axis,
                          double pos) { // BVHNode.cpp:215-254
  Box lb = EMPTY_BOX, rb = EMPTY_BOX;
  size_t lc = 0, rc = 0;
  for (size_t i = st; i < en; ++i) {
    Box b = obj_bbox(ob[i]);
    V c = box_center(b);
    if (c[axis] < pos) {
      lb = box_join(lb, b);
      ++lc;
    } else {
      rb = box_join(rb, b);
      ++rc;
    }
  }
  if (lc == 0 || rc == 0) return INF;
  double tot = box_area(self->bbox);
  if (tot < 1e-9) return INF;
  double pl = box_area(lb) / tot, pr = box_area(rb) / tot;
  return 1.0 + pl * lc * 2.0 + pr * rc * 2.0;
}

static void flatten_into(Obj *root, const Obj *n, uint32_t &off) { // BVHNode.cpp:330-383
  uint32_t mine = off++;
  if (mine >= root->fnodes.size()) root->fnodes.resize(mine + 1);
  root->fnodes[mine].box = n->bbox;
  if (n->kind == O_BVH && n->kids[0] != n->kids[1]) {
    root->fnodes[mine].leaf = false;
    root->fnodes[mine].a = off;
    flatten_into(root, n->kids[0], off);
    root->fnodes[mine].b = off;
    flatten_into(root, n->kids[1], off);
  } else {
    root->fnodes[mine].leaf = true;
    root->fnodes[mine].a = (uint32_t)root->fprims.size();
    if (n->kind == O_BVH) {
      root->fprims.push_back(n->kids[0]);
      root->fnodes[mine].b = 1;
    } else {
      root->fprims.push_back(const_cast<Obj *>(n));
      root->fnodes[mine].b = 1;
    }
  }
}

Obj *BvhBuild::node(std::vector<Obj *> &ob, size_t st, size_t en) {
  Obj *me = S->make(O_BVH);
  me->bbox = EMPTY_BOX;
  for (size_t i = st; i < en; ++i) me->bbox = box_join(me->bbox, obj_bbox(ob[i]));
  size_t span = en - st;
  if (span <= 4) {
    if (span == 1) {
      me->kids = {ob[st], ob[st]};
    } else if (span == 2) {
      me->kids = {ob[st], ob[st + 1]};
    } else {
      size_t mid = st + span / 2;
      Obj *l = node(ob, st, mid);
      Obj *r = node(ob, mid, en);
      me->kids = {l, r};
    }
    return me;
  }
  Box cb = EMPTY_BOX;
  for (size_t i = st; i < en; ++i) {
    V c = box_center(obj_bbox(ob[i]));
    cb = box_join(cb, box_pts(c, c));
  }
  // find_best_sah_split, BVHNode.cpp:168-213
  int best_axis = 0;
  double best_pos = 0, best_cost = INF;
  size_t best_l = 0, best_r = 0;
  for (int axis = 0; axis < 3; ++axis) {
    double amin = cb.a[axis].lo, amax = cb.a[axis].hi;
    if (amax - amin < 1e-9) continue;
    for (int i = 1; i < 16; ++i) {
      double tt = static_cast<double>(i) / 16;
      double pos = amin + tt * (amax - amin);
      double cost = sah_cost(me, ob, st, en, axis, pos);
      if (cost < best_cost) {
        best_axis = axis;
        best_pos = pos;
        best_cost = cost;
        size_t lc = 0, rc = 0;
        for (size_t j = st; j < en; ++j) {
          if (box_center(obj_bbox(ob[j]))[axis] < pos)
            ++lc;
          else
            ++rc;
        }
        best_l = lc;
        best_r = rc;
      }
    }
  }
  size_t mid;
  if (best_cost == INF || best_l == 0 || best_r == 0) {
    int axis = box_longest(me->bbox);
    std::sort(ob.begin() + st, ob.begin() + en, [axis](const Obj *a, const Obj *b) {
      return a->bbox.a[axis].lo < b->bbox.a[axis].lo;
    });
    mid = st + span / 2;
    Obj *l = node(ob, st, mid);
    Obj *r = node(ob, mid, en);
    me->kids = {l, r};
    return me;
  }
  if (span > 1000) {
    // BVHNode::parallel_partition: a stable flag-based partition when each of
    // hardware_concurrency() chunks holds >= 100 objects (BVHNode.cpp:256-320).
    size_t nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (span / nt < 100) {
      auto it = std::partition(ob.begin() + st, ob.begin() + en, [&](const Obj *o) {
        return box_center(obj_bbox(o))[best_axis] < best_pos;
      });
      mid = size_t(it - ob.begin());
    } else {
      auto it = std::stable_partition(ob.begin() + st, ob.begin() + en, [&](const Obj *o) {
        return box_center(obj_bbox(o))[best_axis] < best_pos;
      });
      mid = size_t(it - ob.begin());
    }
  } else {
    auto it = std::partition(ob.begin() + st, ob.begin() + en, [&](const Obj *o) {
      return box_center(obj_bbox(o))[best_axis] < best_pos;
    });
    mid = size_t(it - ob.begin());
  }
  if (mid == st || mid == en) mid = st + span / 2;
  Obj *l = node(ob, st, mid);
  Obj *r = node(ob, mid, en);
  me->kids = {l, r};
  if (span > 100) { // BVHNode.cpp:119-122
    uint32_t off = 0;
    me->fnodes.clear();
    me->fprims.clear();
    flatten_into(me, me, off);
    me->flat = true;
  }
  return me;
}

Obj *Builder::build(int idx) {
  if (idx < 0 || idx >= D->n_objects) return nullptr;
  if (built[idx]) return built[idx];
  const rt_object_desc &d = D->objects[idx];
  Obj *o = nullptr;
  switch (d.kind) {
  case RT_OBJ_SPHERE: {
    o = S->make(O_SPHERE);
    o->mat = d.material;
    V c0 = from(d.a);
    o->radius = std::fmax(0, d.s);
    V rv = mk(d.s, d.s, d.s);
    if (d.moving) { // Sphere.cpp:15-23 (RT_STORED_FORM: b is c1 - c0 itself)
      o->c0 = c0;
      o->cdir = d.moving == RT_STORED_FORM ? from(d.b) : from(d.b) - c0;
      V a0 = mk(o->c0.x + 0 * o->cdir.x, o->c0.y + 0 * o->cdir.y, o->c0.z + 0 * o->cdir.z);
      V a1 = mk(o->c0.x + 1 * o->cdir.x, o->c0.y + 1 * o->cdir.y, o->c0.z + 1 * o->cdir.z);
      o->bbox = box_join(box_pts(a0 - rv, a0 + rv), box_pts(a1 - rv, a1 + rv));
    } else { // Sphere.cpp:8-13
      o->c0 = c0;
      o->cdir = mk(0, 0, 0);
      o->bbox = box_pts(c0 - rv, c0 + rv);
    }
    break;
  }
  case RT_OBJ_QUAD: { // Plane.cpp:6-21
    o = S->make(O_QUAD);
    o->mat = d.material;
    o->Q = from(d.a);
    o->qu = from(d.b);
    o->qv = from(d.c);
    V n = cross(o->qu, o->qv);
    o->qn = unit(n);
    o->D = dot(o->qn, o->Q);
    o->qw = n / dot(n, n);
    o->area = len(n);
    Box b1 = box_pts(o->Q, o->Q + o->qu + o->qv);
    Box b2 = box_pts(o->Q + o->qu, o->Q + o->qv);
    o->bbox = box_join(b1, b2);
    break;
  }
  case RT_OBJ_LIST: {
    o = S->make(O_LIST);
    o->bbox = EMPTY_BOX;
    for (int k = 0; k < d.count; ++k) {
      Obj *c = build(D->children[d.child + k]);
      if (!c) return nullptr;
      o->kids.push_back(c);
      o->bbox = box_join(o->bbox, c->bbox);
    }
    break;
  }
  case RT_OBJ_ROTATE_Y: { // RotateY.cpp:5-35
    o = S->make(O_ROT);
    Obj *c = build(d.child);
    if (!c) return nullptr;
    o->kids = {c};
    if (d.moving == RT_STORED_FORM) { // stored (sin, cos)
      o->sin_t = d.a.x;
      o->cos_t = d.a.y;
    } else {
      double rad = d.s * PI / 180.0;
      o->sin_t = std::sin(rad);
      o->cos_t = std::cos(rad);
    }
    Box bb = c->bbox;
    V mn = mk(INF, INF, INF), mx = mk(-INF, -INF, -INF);
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          double x = i * bb.a[0].hi + (1 - i) * bb.a[0].lo;
          double y = j * bb.a[1].hi + (1 - j) * bb.a[1].lo;
          double z = k * bb.a[2].hi + (1 - k) * bb.a[2].lo;
          double nx = o->cos_t * x + o->sin_t * z;
          double nz = -o->sin_t * x + o->cos_t * z;
          V te = mk(nx, y, nz);
          for (int c3 = 0; c3 < 3; c3++) {
            mn[c3] = std::fmin(mn[c3], te[c3]);
            mx[c3] = std::fmax(mx[c3], te[c3]);
          }
        }
    o->bbox = box_pts(mn, mx);
    break;
  }
  case RT_OBJ_TRANSLATE: { // Translate.cpp:7-10, AABBUtility.hpp:7-11
    o = S->make(O_TRANS);
    Obj *c = build(d.child);
    if (!c) return nullptr;
    o->kids = {c};
    o->off = from(d.a);
    Box bb = c->bbox;
    o->bbox = box_ivals(Ival{bb.a[0].lo + o->off.x, bb.a[0].hi + o->off.x},
                        Ival{bb.a[1].lo + o->off.y, bb.a[1].hi + o->off.y},
                        Ival{bb.a[2].lo + o->off.z, bb.a[2].hi + o->off.z});
    break;
  }
  case RT_OBJ_MEDIUM: {
    o = S->make(O_MEDIUM);
    Obj *c = build(d.child);
    if (!c) return nullptr;
    o->kids = {c};
    o->density = d.s;
    o->phase = d.phase;
    o->bbox = c->bbox;
    break;
  }
  default:
    return nullptr;
  }
  o->id = idx;
  built[idx] = o;
  return o;
}

static void collect_leaves(Scene &S, Obj *o, double w, std::vector<Obj *> &chain) {
  switch (o->kind) {
  case O_LIST: {
    double cw = w * (1.0 / o->kids.size());
    for (Obj *k : o->kids) collect_leaves(S, k, cw, chain);
    return;
  }
  case O_BVH:
    collect_leaves(S, o->kids[0], w * 0.5, chain);
    collect_leaves(S, o->kids[1], w * 0.5, chain);
    return;
  case O_ROT:
  case O_TRANS:
    chain.push_back(o);
    collect_leaves(S, o->kids[0], w, chain);
    chain.pop_back();
    return;
  default:
    S.leaves.push_back(Scene::LightLeaf{o, w, chain});
  }
}

static int build_scene(Scene &S, const rt_scene_desc *D, int use_bvh) {
  S.tex.assign(D->textures, D->textures + D->n_textures);
  S.perlin.assign(D->perlin, D->perlin + D->n_perlin);
  S.mats.assign(D->materials, D->materials + D->n_materials);
  Builder B{&S, D, std::vector<Obj *>(D->n_objects, nullptr), use_bvh};
  Obj *w = B.build(D->world);
  if (!w || w->kind != O_LIST) return -1;
  Obj *l = nullptr;
  if (D->lights >= 0) {
    l = B.build(D->lights);
    if (!l || l->kind != O_LIST) return -1;
  }
  BvhBuild bb{&S};
  if (use_bvh) { // StaticCamera.cpp:35-40
    if (!w->kids.empty()) {
      std::vector<Obj *> ob = w->kids;
      Obj *root = bb.node(ob, 0, ob.size());
      Obj *nw = S.make(O_LIST);
      nw->kids = {root};
      nw->bbox = root->bbox;
      w = nw;
    }
    if (l && !l->kids.empty()) {
      std::vector<Obj *> ob = l->kids;
      Obj *root = bb.node(ob, 0, ob.size());
      Obj *nl = S.make(O_LIST);
      nl->kids = {root};
      nl->bbox = root->bbox;
      l = nl;
    }
  }
  S.world = w;
  S.lights = l;
  if (l && !l->kids.empty()) {
    std::vector<Obj *> chain;
    collect_leaves(S, l, 1.0, chain);
    double c = 0;
    for (auto &lf : S.leaves) {
      c += lf.weight;
      S.leaf_cum.push_back(c);
    }
  }
  return 0;
}

} // namespace orc

/* ======================================================== C entry points */
using namespace orc;

extern "C" {

int oracle_camera_setup(const rt_camera_desc *cd, rt_frame *f) {
  Cam c = cam_setup(*cd);
  f->image_width = c.W;
  f->image_height = c.H;
  f->sqrt_spp = int(std::sqrt(c.spp));
  f->max_depth = c.depth;
  f->center = to(c.center);
  f->pixel00_loc = to(c.p00);
  f->pixel_delta_u = to(c.du);
  f->pixel_delta_v = to(c.dv);
  f->u = to(c.u);
  f->v = to(c.v);
  f->w = to(c.w);
  f->defocus_disk_u = to(c.disk_u);
  f->defocus_disk_v = to(c.disk_v);
  f->defocus_angle = c.defocus_angle;
  f->pixel_samples_scale = c.scale;
  f->background = to(c.bg);
  return 0;
}

/* Render into out[(j-row_begin)*W+i][3].
   mode: 0 = MT (serial, one engine seeded with `seed`, pixels in scanline order,
             exactly StaticCamera::render_cpu's serial loop), 1 = COUNTER.
   output: RT_OUT_SCALED or RT_OUT_SUM.  threads: COUNTER mode only (0 = 1);
   rows are processed one at a time with a barrier per row, pixels of the row
   spread over the threads — the reference's -p decomposition
   (StaticCamera.cpp:60-100). */
int oracle_render(const rt_scene_desc *D, const rt_camera_desc *cd, int mode, uint64_t seed,
                  int use_bvh, int row_begin, int row_end, int sample_begin, int sample_count,
                  int output, int threads, double *out) {
  Scene S;
  if (build_scene(S, D, use_bvh) != 0) return -1;
  Cam cam = cam_setup(*cd);
  if (row_end <= row_begin) {
    row_begin = 0;
    row_end = cam.H;
  }
  int sq = int(std::sqrt(cam.spp));
  int nsamp = sq * sq;
  if (sample_count < 0) sample_count = nsamp - sample_begin;
  if (sample_begin < 0 || sample_begin + sample_count > nsamp) return -1;
  if (mode == MODE_MT && (sample_begin != 0 || sample_count != nsamp)) return -1;
  const double outscale = (output == RT_OUT_SCALED) ? cam.scale : 1.0;

  auto do_pixel = [&](Sampler &s, int i, int j) {
    V acc = mk(0, 0, 0);
    Ctx C{&S, &s};
    for (int k = sample_begin; k < sample_begin + sample_count; ++k) {
      int sj = k / sq, si = k % sq;
      s.pixel = (uint32_t)(j * cam.W + i);
      s.sample = (uint32_t)k;
      Ray r = get_ray(cam, s, i, j, si, sj);
      acc = acc + ray_color(C, cam, r, cam.depth);
    }
    V res = (output == RT_OUT_SCALED) ? (outscale * acc) : acc;
    double *o = out + 3 * ((size_t)(j - row_begin) * cam.W + i);
    o[0] = res.x;
    o[1] = res.y;
    o[2] = res.z;
  };

  if (mode == MODE_MT) {
    std::mt19937 eng((uint32_t)seed);
    Sampler s{MODE_MT, &eng, seed, 0, 0, 0};
    for (int j = row_begin; j < row_end; ++j)
      for (int i = 0; i < cam.W; ++i) do_pixel(s, i, j);
    return 0;
  }
  if (threads <= 1) {
    Sampler s{MODE_COUNTER, nullptr, seed, 0, 0, 0};
    for (int j = row_begin; j < row_end; ++j)
      for (int i = 0; i < cam.W; ++i) do_pixel(s, i, j);
    return 0;
  }
  // threaded: barrier per row
  std::vector<std::thread> pool;
  std::atomic<int> next{0};
  for (int j = row_begin; j < row_end; ++j) {
    next.store(0);
    pool.clear();
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, j]() {
        Sampler s{MODE_COUNTER, nullptr, seed, 0, 0, 0};
        for (;;) {
          int i = next.fetch_add(1);
          if (i >= cam.W) break;
          do_pixel(s, i, j);
        }
      });
    for (auto &th : pool) th.join();
  }
  return 0;
}

/* ---- known-answer helpers used by tests/test_oracle_kat.py ---- */
void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  oracle_philox4x32_10(ctr, key, out);
}
void oracle_u01x4(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce, uint32_t slot,
                  double out[4]) {
  oracle_philox_u01x4(seed, pixel, sample, bounce, slot, out);
}
unsigned char oracle_to_byte(double x) { // ColorUtility.hpp:11-26
  double g = (x > 0) ? std::sqrt(x) : 0;
  if (g < 0.000) g = 0.000;
  if (g > 0.999) g = 0.999;
  return static_cast<unsigned char>(256 * g);
}

/* Evaluate ray hits against one object of a scene (world list child `obj`),
   returning t, p, n, u, v, front, mat.  Used for primitive KATs. */
int oracle_object_hit(const rt_scene_desc *D, int obj, const double ray[7], double tmin,
                      double tmax, double res[12]) {
  Scene S;
  S.tex.assign(D->textures, D->textures + D->n_textures);
  S.perlin.assign(D->perlin, D->perlin + D->n_perlin);
  S.mats.assign(D->materials, D->materials + D->n_materials);
  Builder B{&S, D, std::vector<Obj *>(D->n_objects, nullptr), 0};
  Obj *o = B.build(obj);
  if (!o) return -1;
  std::mt19937 eng(1u);
  Sampler s{MODE_MT, &eng, 1, 0, 0, 0};
  Ctx C{&S, &s};
  Ray r{mk(ray[0], ray[1], ray[2]), mk(ray[3], ray[4], ray[5]), ray[6]};
  Hit h;
  if (!obj_hit(C, o, r, Ival{tmin, tmax}, h)) return 0;
  double v[12] = {h.t, h.p.x, h.p.y, h.p.z, h.n.x, h.n.y, h.n.z, h.u, h.v, h.front ? 1.0 : 0.0,
                  (double)h.mat, 0};
  std::memcpy(res, v, sizeof v);
  return 1;
}

/* Light pdf_value of object `obj` from origin along direction. */
double oracle_object_pdf(const rt_scene_desc *D, int obj, const double org[3], const double dir[3]) {
  Scene S;
  Builder B{&S, D, std::vector<Obj *>(D->n_objects, nullptr), 0};
  Obj *o = B.build(obj);
  if (!o) return -1;
  Sampler s{MODE_COUNTER, nullptr, 0, 0, 0, 0};
  Ctx C{&S, &s};
  return obj_pdf(C, o, mk(org[0], org[1], org[2]), mk(dir[0], dir[1], dir[2]));
}

/* Texture value of texture `t` at (u,v,p). */
void oracle_texture_value(const rt_scene_desc *D, int t, double u, double v, const double p[3],
                          double out[3]) {
  Scene S;
  S.tex.assign(D->textures, D->textures + D->n_textures);
  S.perlin.assign(D->perlin, D->perlin + D->n_perlin);
  V c = tex_value(S, t, u, v, mk(p[0], p[1], p[2]));
  out[0] = c.x;
  out[1] = c.y;
  out[2] = c.z;
}

/* Distribution KATs (tests/test_distributions.py): n draws of the COUNTER-mode
   samplers, draw k from the Philox block (seed; pixel k, sample 0, bounce 0,
   slot) exactly as the integrator consumes it -- kind 0 ctr_unit_vector and 2
   cosine_dir from the shading block's direction uniforms (d2, d3; slot 0,
   ray_color), 1 ctr_in_unit_disk from the camera's defocus block (d0, d1;
   CAM_TAG, slot 1, get_ray).  out: n x 3. */
int oracle_ctr_sample_batch(int kind, uint64_t seed, int n, double *out) {
  for (int k = 0; k < n; ++k) {
    double d[4];
    V v;
    if (kind == 1) {
      oracle_philox_u01x4(seed, (uint32_t)k, 0, CAM_TAG, 1, d);
      v = ctr_in_unit_disk(d[0], d[1]);
    } else {
      oracle_philox_u01x4(seed, (uint32_t)k, 0, 0, SLOT_SHADE, d);
      v = kind == 0 ? ctr_unit_vector(d[2], d[3]) : cosine_dir(d[2], d[3]);
    }
    out[3 * k] = v.x;
    out[3 * k + 1] = v.y;
    out[3 * k + 2] = v.z;
  }
  return kind >= 0 && kind <= 2 ? 0 : -1;
}

/* n COUNTER-mode light directions from `org` (ctr_light_random: leaf pick by
   cumulative weight from d1, direction from d2, d3 of the shading block). */
int oracle_ctr_light_batch(const rt_scene_desc *D, int use_bvh, const double org[3], uint64_t seed,
                           int n, double *out) {
  Scene S;
  if (build_scene(S, D, use_bvh) != 0 || S.leaves.empty()) return -1;
  Sampler s{MODE_COUNTER, nullptr, seed, 0, 0, 0};
  Ctx C{&S, &s};
  V o = mk(org[0], org[1], org[2]);
  for (int k = 0; k < n; ++k) {
    double d[4];
    oracle_philox_u01x4(seed, (uint32_t)k, 0, 0, SLOT_SHADE, d);
    V v = ctr_light_random(C, o, d[1], d[2], d[3]);
    out[3 * k] = v.x;
    out[3 * k + 1] = v.y;
    out[3 * k + 2] = v.z;
  }
  return 0;
}

} // extern "C"
