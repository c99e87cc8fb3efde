// rt_scene.cpp — host scene compiler for the HIP path tracer.
//
// Takes the caller's flat rt_scene_desc (one entry per reference object, see
// include/rt_api.h), validates it, derives the per-object data the reference
// computes in its constructors (Plane.cpp:6-21, Sphere.cpp:8-23, RotateY.cpp:5-35,
// Translate.cpp:7-10, ConstantMedium.cpp:7-21), computes the reference's bounding
// boxes (AABB.cpp:7-27, 167-175), builds a binned-SAH BVH over the world's top-level
// objects and flattens the light list into weighted leaves.
//
// The world BVH is the library's own: closest-hit results do not depend on the
// tree shape.  The LIGHT tree, however, changes the light pdf weights when the
// reference runs with -b (lights = HittableList(BVHNode(lights)),
// StaticCamera.cpp:35-40; BVHNode::pdf_value/random, BVHNode.cpp:149-166), so for
// use_bvh the light list is split exactly as BVHNode's constructor splits it
// (BVHNode.cpp:21-123) and each leaf carries the product of the 1/2 and 1/N
// weights above it.
#include "rt_scene.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>

namespace rtx {
namespace {

int or_default(int32_t v, int dflt) { return v > 0 ? v : dflt; }

const double kInf = std::numeric_limits<double>::infinity();
const double kPi = 3.1415926535897932385;

struct P3 {
  double x, y, z;
};
inline P3 p3(const rt_vec3 &v) { return P3{v.x, v.y, v.z}; }
inline P3 add(P3 a, P3 b) { return P3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline P3 sub(P3 a, P3 b) { return P3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline P3 scl(double t, P3 a) { return P3{t * a.x, t * a.y, t * a.z}; }
inline double dotp(P3 a, P3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline P3 crossp(P3 a, P3 b) {
  return P3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double comp(P3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// Axis-aligned box with the reference's interval semantics.
struct Bx {
  double lo[3], hi[3];
};
Bx bx_empty() {
  Bx b;
  for (int i = 0; i < 3; ++i) {
    b.lo[i] = kInf;
    b.hi[i] = -kInf;
  }
  return b;
}
void bx_pad(Bx &b) { // pad_to_minimums: intervals narrower than 1e-4 grow by 1e-4
  for (int i = 0; i < 3; ++i)
    if (b.hi[i] - b.lo[i] < 0.0001) {
      b.lo[i] -= 0.0001 * 0.5;
      b.hi[i] += 0.0001 * 0.5;
    }
}
Bx bx_points(P3 a, P3 b) {
  Bx r;
  for (int i = 0; i < 3; ++i) {
    double u = comp(a, i), v = comp(b, i);
    r.lo[i] = u <= v ? u : v;
    r.hi[i] = u <= v ? v : u;
  }
  bx_pad(r);
  return r;
}
Bx bx_join(const Bx &a, const Bx &b) {
  Bx r;
  for (int i = 0; i < 3; ++i) {
    r.lo[i] = a.lo[i] <= b.lo[i] ? a.lo[i] : b.lo[i];
    r.hi[i] = a.hi[i] >= b.hi[i] ? a.hi[i] : b.hi[i];
  }
  return r;
}
double bx_area(const Bx &b) {
  double d[3];
  for (int i = 0; i < 3; ++i) d[i] = b.hi[i] - b.lo[i];
  return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
}
P3 bx_center(const Bx &b) {
  return P3{(b.lo[0] + b.hi[0]) * 0.5, (b.lo[1] + b.hi[1]) * 0.5, (b.lo[2] + b.hi[2]) * 0.5};
}
int bx_longest(const Bx &b) {
  double sx = b.hi[0] - b.lo[0], sy = b.hi[1] - b.lo[1], sz = b.hi[2] - b.lo[2];
  if (sx > sy) return sx > sz ? 0 : 2;
  return sy > sz ? 1 : 2;
}

// ---------------------------------------------------------------- world BVH
// Host binned-SAH builder (also the fallback of the device LBVH builder).
struct SahBuilder {
  HostScene &H;
  explicit SahBuilder(HostScene &h) : H(h) {}

  struct BRef {
    Bx b;
    P3 c;
    int32_t obj;
  };
  struct BNode {
    Bx b;
    int left = -1, right = -1; // build-node indices, -1 for leaves
    int first = 0, count = 0;  // leaf ref range
  };
  std::vector<BNode> bn;
  int max_depth_seen = 0;
  // Leaf rules: a range of <= leaf_max items is a leaf; one of <= leaf_split
  // items is a leaf when splitting does not pay (SAH, traversal cost
  // trav_cost, intersection cost 1).  Binary-walk scenes (< kBvh4Min items)
  // use single-item leaves: the wave tests leaves together, so a lane's
  // second leaf item costs the whole wave a trip (C3: 2 / 4 -> 1 / 1 gave
  // +2.1 %, profiles/r02aj_sah_leaf_sweep.log); the 4-wide and device-built
  // trees keep 2 / 4 (the device SAH builder's rules).  Measurement overrides
  // (rt_tuning, via HostScene): sah_leaf_max, sah_leaf_split, sah_trav_x4 (4 x
  // trav_cost), sah_bins.
  int leaf_max = 2, leaf_split = 4;
  double trav_cost = 1.0;
  static constexpr int kMaxBins = 64;
  int sah_bins = 16; // centroid bins per axis (sah_bins override, <= 64)
  void set_leaf_rules(size_t n_items) {
    const bool binary = n_items < (size_t)kBvh4Min;
    leaf_max = or_default(H.sah_leaf_max, binary ? 1 : 2);
    leaf_split = or_default(H.sah_leaf_split, binary ? 1 : 4);
    trav_cost = or_default(H.sah_trav_x4, 4) / 4.0;
    sah_bins = std::min(kMaxBins, std::max(2, or_default(H.sah_bins, 16)));
  }

  int build(std::vector<BRef> &r, int st, int en, int dep) {
    BNode n;
    n.b = bx_empty();
    Bx cb = bx_empty();
    for (int i = st; i < en; ++i) {
      n.b = bx_join(n.b, r[i].b);
      Bx pc{{r[i].c.x, r[i].c.y, r[i].c.z}, {r[i].c.x, r[i].c.y, r[i].c.z}};
      cb = bx_join(cb, pc);
    }
    int cnt = en - st;
    max_depth_seen = std::max(max_depth_seen, dep);
    int id = (int)bn.size();
    bn.push_back(n);
    const int kLeafMax = leaf_max, kLeafSplit = leaf_split;
    const double kTrav = trav_cost;
    // A small world is one flat leaf (the reference's own HittableList walk,
    // in list order): a wavefront's lanes scatter over the whole scene, so a
    // split of a handful of items only adds a node visit and divergent leaf
    // loops (C2: 3.2 wave leaf iterations + 1 node per segment vs 3 flat tests).
    if (cnt <= kLeafMax || (dep == 0 && cnt <= RT_FLAT_MAX)) {
      bn[id].first = st;
      bn[id].count = cnt;
      return id;
    }
    // depth budget: switch to balanced median splits when the SAH tree risks
    // exceeding the per-lane traversal stack (RT_STACK_DEPTH)
    int need = 0;
    while ((1 << need) < cnt) ++need;
    bool force_median = dep + need >= RT_STACK_DEPTH - 2;
    int best_axis = -1, best_bin = -1;
    double best_cost = kInf;
    const int kBins = sah_bins;
    if (!force_median) {
      for (int ax = 0; ax < 3; ++ax) {
        double lo = cb.lo[ax], hi = cb.hi[ax];
        if (!(hi - lo > 1e-12)) continue;
        Bx bb[kMaxBins];
        int bc[kMaxBins];
        for (int k = 0; k < kBins; ++k) {
          bb[k] = bx_empty();
          bc[k] = 0;
        }
        double sc = kBins / (hi - lo);
        for (int i = st; i < en; ++i) {
          int k = std::min(kBins - 1, std::max(0, (int)((comp(r[i].c, ax) - lo) * sc)));
          bb[k] = bx_join(bb[k], r[i].b);
          bc[k]++;
        }
        Bx lb[kMaxBins];
        int lc[kMaxBins];
        Bx acc = bx_empty();
        int a = 0;
        for (int k = 0; k < kBins; ++k) {
          acc = bx_join(acc, bb[k]);
          a += bc[k];
          lb[k] = acc;
          lc[k] = a;
        }
        acc = bx_empty();
        a = 0;
        for (int k = kBins - 1; k > 0; --k) {
          acc = bx_join(acc, bb[k]);
          a += bc[k];
          int nl = lc[k - 1], nr = a;
          if (nl == 0 || nr == 0) continue;
          double cost = bx_area(lb[k - 1]) * nl + bx_area(acc) * nr;
          if (cost < best_cost) {
            best_cost = cost;
            best_axis = ax;
            best_bin = k;
          }
        }
      }
    }
    int mid;
    if (best_axis >= 0) {
      double lo = cb.lo[best_axis], hi = cb.hi[best_axis];
      double sc = kBins / (hi - lo);
      auto it = std::partition(r.begin() + st, r.begin() + en, [&](const BRef &x) {
        int k = std::min(kBins - 1, std::max(0, (int)((comp(x.c, best_axis) - lo) * sc)));
        return k < best_bin;
      });
      mid = int(it - r.begin());
      // leaf if splitting does not pay (SAH with traversal cost 1, isect cost 1)
      double parent_area = bx_area(bn[id].b);
      if (cnt <= kLeafSplit && parent_area > 0 && kTrav + best_cost / parent_area >= (double)cnt) {
        bn[id].first = st;
        bn[id].count = cnt;
        return id;
      }
    } else {
      mid = st + cnt / 2;
    }
    if (mid <= st || mid >= en) {
      int ax = bx_longest(cb);
      std::sort(r.begin() + st, r.begin() + en,
                [ax](const BRef &a, const BRef &b) { return comp(a.c, ax) < comp(b.c, ax); });
      mid = st + cnt / 2;
    }
    int L = build(r, st, mid, dep + 1);
    int R = build(r, mid, en, dep + 1);
    bn[id].left = L;
    bn[id].right = R;
    return id;
  }

  // fp32 box bounds rounded outward, widened by a relative 2^-20 plus 1e-7 so
  // the conservative fp32 slab test (rt_path.h) can never reject a box whose
  // primitives the fp64 test would hit.
  static float f32_lo(double x) {
    double m = x - (std::fabs(x) * 0x1p-20 + 1e-7);
    float f = (float)m;
    if ((double)f > m) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
  }
  static float f32_hi(double x) {
    double m = x + (std::fabs(x) * 0x1p-20 + 1e-7);
    float f = (float)m;
    if ((double)f < m) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
  }

  void emit_world_bvh(const std::vector<Bx> &item_box) {
    std::vector<BRef> r;
    for (size_t i = 0; i < item_box.size(); ++i) {
      BRef x;
      x.b = item_box[i];
      x.c = bx_center(x.b);
      x.obj = (int32_t)i;
      r.push_back(x);
    }
    if (r.empty()) {
      H.root_is_leaf = 1;
      H.n_root_items = 0;
      return;
    }
    bn.clear();
    set_leaf_rules(r.size());
    int root = build(r, 0, (int)r.size(), 0);
    H.bvh_depth = max_depth_seen;
    // store the items in leaf order: a leaf is a contiguous item range
    std::vector<DItem> leaf_order;
    leaf_order.reserve(r.size());
    for (auto &x : r) leaf_order.push_back(H.items[x.obj]);
    H.items.swap(leaf_order);
    if (bn[root].left < 0) {
      H.root_is_leaf = 1;
      H.n_root_items = bn[root].count;
      return;
    }
    // flatten in BFS order (the top levels come first: they are the nodes every
    // ray visits, and the kernel stages a prefix of the array in LDS); each DNode
    // holds both children's boxes
    std::vector<int> map(bn.size(), -1);
    std::vector<int> order;
    order.push_back(root);
    for (size_t q = 0; q < order.size(); ++q) {
      const BNode &p = bn[order[q]];
      map[order[q]] = (int)q;
      if (bn[p.left].left >= 0) order.push_back(p.left);
      if (bn[p.right].left >= 0) order.push_back(p.right);
    }
    H.nodes.resize(order.size());
    for (size_t i = 0; i < order.size(); ++i) {
      const BNode &p = bn[order[i]];
      DNode &d = H.nodes[i];
      std::memset(&d, 0, sizeof d);
      int ch[2] = {p.left, p.right};
      for (int k = 0; k < 2; ++k) {
        const BNode &c = bn[ch[k]];
        for (int a = 0; a < 3; ++a) {
          d.lo[a][k] = f32_lo(c.b.lo[a]);
          d.hi[a][k] = f32_hi(c.b.hi[a]);
        }
        d.entry[k] = c.left < 0 ? ~((c.first << 3) | c.count) : map[ch[k]];
      }
    }
  }

};

struct Compiler {
  const rt_scene_desc *D;
  HostScene &H;
  std::string &err;
  std::vector<Bx> box;
  std::vector<int> state; // 0 unvisited, 1 in progress, 2 done
  std::vector<int> depth; // composite nesting depth of each object

  Compiler(const rt_scene_desc *d, HostScene &h, std::string &e) : D(d), H(h), err(e) {}

  bool fail(const std::string &m) {
    err = m;
    return false;
  }

  bool check_texture(int t, int hops) {
    if (t < 0 || t >= D->n_textures) return fail("texture index out of range");
    if (hops > 64) return fail("checker texture cycle");
    const rt_texture_desc &x = D->textures[t];
    if (x.kind == RT_TEX_CHECKER) {
      if (!(x.scale != 0)) return fail("checker scale must be non-zero");
      return check_texture(x.even, hops + 1) && check_texture(x.odd, hops + 1);
    }
    if (x.kind == RT_TEX_NOISE) {
      if (x.perlin < 0 || x.perlin >= D->n_perlin) return fail("noise texture perlin index out of range");
      return true;
    }
    if (x.kind != RT_TEX_SOLID) return fail("unknown texture kind");
    return true;
  }

  bool check_material(int m, bool allow_none) {
    if (m < 0) return allow_none ? true : fail("world primitive without material");
    if (m >= D->n_materials) return fail("material index out of range");
    const rt_material_desc &x = D->materials[m];
    switch (x.kind) {
    case RT_MAT_LAMBERTIAN:
    case RT_MAT_DIFFUSE_LIGHT:
    case RT_MAT_ISOTROPIC:
      return check_texture(x.texture, 0);
    case RT_MAT_METAL:
    case RT_MAT_DIELECTRIC:
      return true;
    }
    return fail("unknown material kind");
  }

  // Visit object o: compute its box (reference rules) and nesting depth.  The
  // recursion follows the wrapper/list nesting, bounded so that a deep chain in
  // a caller's table cannot overflow the host stack (found by make sanitize).
  static constexpr int kMaxNesting = 1000;
  int nesting = 0;
  struct NestGuard {
    int &n;
    explicit NestGuard(int &c) : n(c) { ++n; }
    ~NestGuard() { --n; }
  };
  bool visit(int o) {
    NestGuard guard(nesting);
    if (nesting > kMaxNesting) return fail("UNSUPPORTED: objects nested deeper than 1000 levels");
    if (o < 0 || o >= D->n_objects) return fail("object index out of range");
    if (state[o] == 2) return true;
    if (state[o] == 1) return fail("object graph has a cycle");
    state[o] = 1;
    const rt_object_desc &x = D->objects[o];
    Bx b = bx_empty();
    int dep = 0;
    switch (x.kind) {
    case RT_OBJ_SPHERE: {
      P3 rv{x.s, x.s, x.s};
      P3 c0 = p3(x.a);
      if (x.moving) { // Sphere.cpp:15-23
        P3 dir = sphere_dir(x);
        P3 a0 = add(c0, scl(0, dir)), a1 = add(c0, scl(1, dir));
        b = bx_join(bx_points(sub(a0, rv), add(a0, rv)), bx_points(sub(a1, rv), add(a1, rv)));
      } else {
        b = bx_points(sub(c0, rv), add(c0, rv));
      }
      if (!(x.s >= 0) && !(x.s < 0)) return fail("sphere radius is NaN");
      break;
    }
    case RT_OBJ_QUAD: { // Plane.cpp:17-20
      P3 Q = p3(x.a), u = p3(x.b), v = p3(x.c);
      b = bx_join(bx_points(Q, add(add(Q, u), v)), bx_points(add(Q, u), add(Q, v)));
      break;
    }
    case RT_OBJ_LIST: {
      if (x.count < 0 || x.child < 0 || x.child + x.count > D->n_children)
        return fail("list child range out of bounds");
      for (int k = 0; k < x.count; ++k) {
        int c = D->children[x.child + k];
        if (!visit(c)) return false;
        b = bx_join(b, box[c]);
        dep = std::max(dep, depth[c] + 1);
      }
      break;
    }
    case RT_OBJ_ROTATE_Y: { // RotateY.cpp:5-35
      if (!visit(x.child)) return false;
      double s, c;
      rot_sincos(x, s, c);
      const Bx &cb = box[x.child];
      double mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
      for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
          for (int k = 0; k < 2; k++) {
            double px = i * cb.hi[0] + (1 - i) * cb.lo[0];
            double py = j * cb.hi[1] + (1 - j) * cb.lo[1];
            double pz = k * cb.hi[2] + (1 - k) * cb.lo[2];
            double t[3] = {c * px + s * pz, py, -s * px + c * pz};
            for (int a = 0; a < 3; a++) {
              mn[a] = std::fmin(mn[a], t[a]);
              mx[a] = std::fmax(mx[a], t[a]);
            }
          }
      b = bx_points(P3{mn[0], mn[1], mn[2]}, P3{mx[0], mx[1], mx[2]});
      dep = depth[x.child] + 1;
      break;
    }
    case RT_OBJ_TRANSLATE: { // Translate.cpp:7-10 + AABBUtility.hpp:7-11
      if (!visit(x.child)) return false;
      const Bx &cb = box[x.child];
      double off[3] = {x.a.x, x.a.y, x.a.z};
      for (int i = 0; i < 3; ++i) {
        b.lo[i] = cb.lo[i] + off[i];
        b.hi[i] = cb.hi[i] + off[i];
      }
      bx_pad(b);
      dep = depth[x.child] + 1;
      break;
    }
    case RT_OBJ_MEDIUM: {
      if (!visit(x.child)) return false;
      if (!(x.s > 0)) return fail("medium density must be > 0");
      if (!check_material(x.phase, false)) return false;
      if (D->materials[x.phase].kind != RT_MAT_ISOTROPIC)
        return fail("medium phase function must be an isotropic material");
      b = box[x.child];
      dep = depth[x.child] + 1;
      break;
    }
    default:
      return fail("unknown object kind");
    }
    box[o] = b;
    depth[o] = dep;
    state[o] = 2;
    return true;
  }

  // World primitives must carry a material (a null MaterialPtr would crash the
  // reference at record.material->emitted, Camera.cpp:248).
  bool check_world_materials(int o) {
    const rt_object_desc &x = D->objects[o];
    switch (x.kind) {
    case RT_OBJ_SPHERE:
    case RT_OBJ_QUAD:
      return check_material(x.material, false);
    case RT_OBJ_LIST:
      for (int k = 0; k < x.count; ++k)
        if (!check_world_materials(D->children[x.child + k])) return false;
      return true;
    case RT_OBJ_ROTATE_Y:
    case RT_OBJ_TRANSLATE:
      return check_world_materials(x.child);
    case RT_OBJ_MEDIUM:
      return true; // boundary materials are never read (ConstantMedium.cpp:88-91)
    }
    return true;
  }

  // ------------------------------------------------------------ flattening
  // The graph below each world object becomes leaf items: primitive or medium +
  // its chain of RotateY/Translate objects (outermost first).  Lists vanish.
  struct FItem {
    int kind; // I_SPHERE / I_QUAD / I_MEDIUM
    int obj;
    std::vector<int> chain;
  };
  std::vector<int> sphere_of, quad_of;

  bool flatten(int o, std::vector<int> &chain, std::vector<FItem> &out, bool in_boundary) {
    const rt_object_desc &x = D->objects[o];
    switch (x.kind) {
    case RT_OBJ_SPHERE:
      out.push_back(FItem{I_SPHERE, o, chain});
      return true;
    case RT_OBJ_QUAD:
      out.push_back(FItem{I_QUAD, o, chain});
      return true;
    case RT_OBJ_LIST:
      for (int k = 0; k < x.count; ++k)
        if (!flatten(D->children[x.child + k], chain, out, in_boundary)) return false;
      return true;
    case RT_OBJ_ROTATE_Y:
    case RT_OBJ_TRANSLATE: {
      if ((int)chain.size() >= RT_MAX_CHAIN)
        return fail("UNSUPPORTED: more than RT_MAX_CHAIN nested rotate_y/translate");
      chain.push_back(o);
      bool ok = flatten(x.child, chain, out, in_boundary);
      chain.pop_back();
      return ok;
    }
    case RT_OBJ_MEDIUM:
      if (in_boundary) return fail("UNSUPPORTED: constant_medium inside a medium boundary");
      out.push_back(FItem{I_MEDIUM, o, chain});
      return true;
    }
    return fail("unknown object kind");
  }

  // Sphere displacement c1 - c0 (Sphere.cpp:15-23: m_center = Ray(c0, c1 - c0));
  // moving == RT_STORED_FORM hands over the stored displacement itself.
  static P3 sphere_dir(const rt_object_desc &x) {
    if (x.moving == RT_STORED_FORM) return p3(x.b);
    return x.moving ? sub(p3(x.b), p3(x.a)) : P3{0, 0, 0};
  }
  // RotateY's (sin, cos) (RotateY.cpp:7-9), or the stored pair.
  static void rot_sincos(const rt_object_desc &x, double &s, double &c) {
    if (x.moving == RT_STORED_FORM) {
      s = x.a.x;
      c = x.a.y;
      return;
    }
    double rad = x.s * kPi / 180.0;
    s = std::sin(rad);
    c = std::cos(rad);
  }

  int sphere_record(int o) {
    if (sphere_of[o] >= 0) return sphere_of[o];
    const rt_object_desc &x = D->objects[o];
    DSphere s;
    P3 c0 = p3(x.a);
    P3 dir = sphere_dir(x);
    s.c0[0] = c0.x, s.c0[1] = c0.y, s.c0[2] = c0.z;
    s.dir[0] = dir.x, s.dir[1] = dir.y, s.dir[2] = dir.z;
    const double r = std::fmax(0, x.s);
    s.inv_r = 1 / r;
    s.rr = r * r;
    sphere_of[o] = (int)H.spheres.size();
    H.spheres.push_back(s);
    return sphere_of[o];
  }

  int quad_record(int o) { // Plane.cpp:6-16
    if (quad_of[o] >= 0) return quad_of[o];
    const rt_object_desc &x = D->objects[o];
    DQuad q;
    std::memset(&q, 0, sizeof q);
    P3 Q = p3(x.a), u = p3(x.b), v = p3(x.c);
    P3 n = crossp(u, v);
    double len = std::sqrt(dotp(n, n));
    P3 nn = (len > 1e-8) ? P3{n.x * (1.0 / len), n.y * (1.0 / len), n.z * (1.0 / len)}
                         : P3{1.0, 0.0, 0.0};
    P3 w = scl(1 / dotp(n, n), n);
    double Qa[3] = {Q.x, Q.y, Q.z}, ua[3] = {u.x, u.y, u.z}, va[3] = {v.x, v.y, v.z};
    double na[3] = {nn.x, nn.y, nn.z}, wa[3] = {w.x, w.y, w.z};
    for (int i = 0; i < 3; ++i) {
      q.Q[i] = Qa[i];
      q.u[i] = ua[i];
      q.v[i] = va[i];
      q.n[i] = na[i];
      q.w[i] = wa[i];
    }
    q.D = dotp(nn, Q);
    q.area = len;
    // axis-aligned: every vector with one nonzero component, on three distinct axes
    auto axis = [](const double a[3]) {
      int k = -1, nz = 0;
      for (int c = 0; c < 3; ++c)
        if (a[c] != 0.0) {
          k = c;
          ++nz;
        }
      return nz == 1 && std::isfinite(a[k]) ? k : -1;
    };
    const int ak = axis(na), ai = axis(ua), aj = axis(va), aw = axis(wa);
    q.aa = -1;
    if (ak >= 0 && ai >= 0 && aj >= 0 && aw == ak && ak != ai && ak != aj && ai != aj &&
        std::isfinite(q.D) && std::isfinite(Qa[0]) && std::isfinite(Qa[1]) && std::isfinite(Qa[2])) {
      const bool even = (ak + 1) % 3 == ai; // (k, i, j) a cyclic shift of (0, 1, 2)
      q.aa = ak | (ai << 2) | (aj << 4) | ((even ? 0 : 1) << 6);
    }
    quad_of[o] = (int)H.quads.size();
    H.quads.push_back(q);
    return quad_of[o];
  }

  std::map<std::vector<int>, int> chain_first; // identical chains share their xforms
  int emit_chain(const std::vector<int> &chain) {
    if (chain.empty()) return 0;
    auto known = chain_first.find(chain);
    if (known != chain_first.end()) return known->second;
    int first = (int)H.xforms.size();
    chain_first[chain] = first;
    for (int o : chain) {
      const rt_object_desc &x = D->objects[o];
      DXform X;
      std::memset(&X, 0, sizeof X);
      if (x.kind == RT_OBJ_TRANSLATE) {
        X.kind = X_TRANSLATE;
        X.a = x.a.x;
        X.b = x.a.y;
        X.c = x.a.z;
      } else { // RotateY.cpp:7-9
        X.kind = X_ROTATE_Y;
        rot_sincos(x, X.a, X.b);
      }
      H.xforms.push_back(X);
    }
    return first;
  }

  // Reference box rules for RotateY (RotateY.cpp:10-34) and Translate
  // (AABBUtility.hpp:7-11), applied innermost transform first.
  Bx rot_box(const Bx &cb, const rt_object_desc &x) {
    double s, c;
    rot_sincos(x, s, c);
    double mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          double px = i * cb.hi[0] + (1 - i) * cb.lo[0];
          double py = j * cb.hi[1] + (1 - j) * cb.lo[1];
          double pz = k * cb.hi[2] + (1 - k) * cb.lo[2];
          double t[3] = {c * px + s * pz, py, -s * px + c * pz};
          for (int a = 0; a < 3; a++) {
            mn[a] = std::fmin(mn[a], t[a]);
            mx[a] = std::fmax(mx[a], t[a]);
          }
        }
    return bx_points(P3{mn[0], mn[1], mn[2]}, P3{mx[0], mx[1], mx[2]});
  }
  Bx trans_box(const Bx &cb, const rt_vec3 &off) {
    Bx b;
    double o[3] = {off.x, off.y, off.z};
    for (int i = 0; i < 3; ++i) {
      b.lo[i] = cb.lo[i] + o[i];
      b.hi[i] = cb.hi[i] + o[i];
    }
    bx_pad(b);
    return b;
  }
  Bx chain_box(Bx b, const std::vector<int> &chain) {
    for (size_t k = chain.size(); k-- > 0;) {
      const rt_object_desc &x = D->objects[chain[k]];
      b = (x.kind == RT_OBJ_ROTATE_Y) ? rot_box(b, x) : trans_box(b, x.a);
    }
    return b;
  }

  // A medium boundary that is a box (make_box, PlaneUtility.hpp:11-39): six
  // axis-aligned quads under one transform chain, two normal to each axis, each
  // face's rectangle spanning the other two axes' face planes.  Sets DMedium::box
  // and the per-axis face constants rt_path.h box_span reads; box_span's range
  // and margin argument needs |D| in {0} U [2^-900, 2^90], |n_a| in [0.5, 2] and
  // equal for both faces of an axis, and rectangle edges within 2^-48 B of the
  // planes (B: the largest |plane coordinate| on that axis).  Anything else
  // keeps the general boundary scan (box = 0).
  void box_of(DMedium &m, const std::vector<DItem> &bs) {
    m.box = 0;
    if (bs.size() != 6) return;
    int nface[3] = {0, 0, 0};
    const DQuad *face[3][2] = {};
    for (const DItem &b : bs) {
      if (b.kind != I_QUAD || b.xf_first != bs[0].xf_first || b.xf_count != bs[0].xf_count) return;
      const DQuad &q = H.quads[b.idx];
      if (q.aa < 0) return;
      const int k = q.aa & 3;
      if (nface[k] == 2) return;
      face[k][nface[k]++] = &q;
    }
    double P[3][2];
    for (int a = 0; a < 3; ++a) {
      if (nface[a] != 2) return;
      for (int f = 0; f < 2; ++f) {
        const DQuad &q = *face[a][f];
        const double n = q.n[a], D = q.D, aD = std::fabs(D);
        if (!(std::fabs(n) >= 0.5 && std::fabs(n) <= 2.0)) return;
        if (!(D == 0.0 || (aD >= 0x1p-900 && aD <= 0x1p90))) return;
        P[a][f] = D / n; // the face's plane coordinate along a
        m.bnk[a][f] = n;
        m.bD[a][f] = D;
      }
      if (std::fabs(m.bnk[a][0]) != std::fabs(m.bnk[a][1]) || !(P[a][0] != P[a][1])) return;
      m.bB[a] = std::fmax(std::fabs(P[a][0]), std::fabs(P[a][1]));
    }
    // every face's rectangle spans the other axes' planes: along its u axis i,
    // {Q_i, Q_i + u_i} = the planes of axis i; along v likewise
    for (int a = 0; a < 3; ++a)
      for (int f = 0; f < 2; ++f) {
        const DQuad &q = *face[a][f];
        const int ax[2] = {(q.aa >> 2) & 3, (q.aa >> 4) & 3};
        const double *side[2] = {q.u, q.v};
        for (int e = 0; e < 2; ++e) {
          const int i = ax[e];
          const double lo = std::fmin(P[i][0], P[i][1]), hi = std::fmax(P[i][0], P[i][1]);
          const double e0 = q.Q[i], e1 = q.Q[i] + side[e][i];
          const double tol = 0x1p-48 * m.bB[i];
          if (!(std::fabs(std::fmin(e0, e1) - lo) <= tol && std::fabs(std::fmax(e0, e1) - hi) <= tol))
            return;
        }
      }
    m.box = 1;
    m.bxf_first = bs[0].xf_first;
    m.bxf_count = bs[0].xf_count;
  }

  bool make_item(const FItem &f, DItem &it, Bx &bb) {
    std::memset(&it, 0, sizeof it);
    const rt_object_desc &x = D->objects[f.obj];
    it.kind = f.kind;
    it.id = f.obj;
    it.mat = -1;
    if (f.kind == I_SPHERE || f.kind == I_QUAD) {
      it.idx = (f.kind == I_SPHERE) ? sphere_record(f.obj) : quad_record(f.obj);
      it.mat = x.material;
      bb = chain_box(box[f.obj], f.chain);
    } else { // medium: boundary items in the medium's local frame
      std::vector<FItem> bs;
      std::vector<int> ch0;
      if (!flatten(x.child, ch0, bs, true)) return false;
      DMedium m;
      std::memset(&m, 0, sizeof m);
      m.neg_inv_density = -1.0 / x.s; // ConstantMedium.cpp:73
      m.phase = x.phase;
      m.id = f.obj;
      Bx ub = bx_empty();
      std::vector<DItem> tmp;
      for (const FItem &b : bs) {
        DItem bi;
        Bx b1;
        if (!make_item(b, bi, b1)) return false;
        tmp.push_back(bi);
        ub = bx_join(ub, b1);
      }
      m.b_first = (int32_t)H.bitems.size();
      m.b_count = (int32_t)tmp.size();
      box_of(m, tmp);
      for (auto &bi : tmp) H.bitems.push_back(bi);
      it.idx = (int32_t)H.media.size();
      H.media.push_back(m);
      bb = chain_box(ub, f.chain);
    }
    it.xf_first = emit_chain(f.chain);
    it.xf_count = (int32_t)f.chain.size();
    return true;
  }

  void emit_materials() {
    for (int i = 0; i < D->n_materials; ++i) {
      const rt_material_desc &m = D->materials[i];
      DMat d;
      std::memset(&d, 0, sizeof d);
      d.kind = m.kind;
      d.tex = m.texture;
      d.ior = m.refraction_index;
      if (m.kind == RT_MAT_DIELECTRIC) { // no albedo/fuzz: the union holds the constants
        d.inv_ior = 1.0 / d.ior;
        for (int f = 0; f < 2; ++f) {
          const double ri = f == 0 ? d.inv_ior : d.ior;
          double r0 = (1 - ri) / (1 + ri);
          d.r0[f] = r0 * r0;
        }
      } else {
        d.albedo[0] = m.albedo.x, d.albedo[1] = m.albedo.y, d.albedo[2] = m.albedo.z;
        d.fuzz = m.fuzz;
      }
      H.mats.push_back(d);
    }
    for (int i = 0; i < D->n_textures; ++i) {
      const rt_texture_desc &t = D->textures[i];
      DTex d;
      std::memset(&d, 0, sizeof d);
      d.kind = t.kind;
      d.even = t.even;
      d.odd = t.odd;
      d.perlin = t.perlin;
      d.scale = t.scale;
      d.inv_scale = 1.0 / t.scale;
      d.color[0] = t.color.x, d.color[1] = t.color.y, d.color[2] = t.color.z;
      H.texs.push_back(d);
    }
    for (int i = 0; i < D->n_perlin; ++i) {
      DPerlin p;
      for (int k = 0; k < 256; ++k) {
        p.rv[k][0] = D->perlin[i].rand_vec[k].x;
        p.rv[k][1] = D->perlin[i].rand_vec[k].y;
        p.rv[k][2] = D->perlin[i].rand_vec[k].z;
        p.px[k] = D->perlin[i].perm_x[k] & 255;
        p.py[k] = D->perlin[i].perm_y[k] & 255;
        p.pz[k] = D->perlin[i].perm_z[k] & 255;
      }
      H.perlin.push_back(p);
    }
  }

  // ------------------------------------------------------------ light leaves
  // BVHNode's split of a light list (BVHNode.cpp:21-123); returns a nested
  // description as a vector of (object, weight) pairs in DFS order.
  void ref_bvh_leaves(std::vector<int32_t> objs, size_t st, size_t en, double w,
                      std::vector<std::pair<int32_t, double>> &out) {
    size_t span = en - st;
    if (span <= 4) {
      if (span == 1) {
        out.push_back({objs[st], w * 0.5});
        out.push_back({objs[st], w * 0.5});
      } else if (span == 2) {
        out.push_back({objs[st], w * 0.5});
        out.push_back({objs[st + 1], w * 0.5});
      } else {
        size_t mid = st + span / 2;
        ref_bvh_leaves(objs, st, mid, w * 0.5, out);
        ref_bvh_leaves(objs, mid, en, w * 0.5, out);
      }
      return;
    }
    // general case: SAH over 15 candidate planes per axis, std::partition
    Bx me = bx_empty(), cb = bx_empty();
    for (size_t i = st; i < en; ++i) {
      me = bx_join(me, box[objs[i]]);
      P3 c = bx_center(box[objs[i]]);
      cb = bx_join(cb, bx_points(c, c));
    }
    auto cost_of = [&](int ax, double pos, size_t &lc, size_t &rc) {
      Bx lb = bx_empty(), rb = bx_empty();
      lc = rc = 0;
      for (size_t i = st; i < en; ++i) {
        const Bx &b = box[objs[i]];
        if (comp(bx_center(b), ax) < pos) {
          lb = bx_join(lb, b);
          ++lc;
        } else {
          rb = bx_join(rb, b);
          ++rc;
        }
      }
      if (lc == 0 || rc == 0) return kInf;
      double tot = bx_area(me);
      if (tot < 1e-9) return kInf;
      return 1.0 + (bx_area(lb) / tot) * lc * 2.0 + (bx_area(rb) / tot) * rc * 2.0;
    };
    int bax = 0;
    double bpos = 0, bcost = kInf;
    size_t bl = 0, br = 0;
    for (int ax = 0; ax < 3; ++ax) {
      double amin = cb.lo[ax], amax = cb.hi[ax];
      if (amax - amin < 1e-9) continue;
      for (int i = 1; i < 16; ++i) {
        double pos = amin + (static_cast<double>(i) / 16) * (amax - amin);
        size_t lc, rc;
        double c = cost_of(ax, pos, lc, rc);
        if (c < bcost) {
          bcost = c;
          bax = ax;
          bpos = pos;
          bl = lc;
          br = rc;
        }
      }
    }
    size_t mid;
    if (bcost == kInf || bl == 0 || br == 0) {
      int ax = bx_longest(me);
      std::sort(objs.begin() + st, objs.begin() + en,
                [&](int32_t a, int32_t b) { return box[a].lo[ax] < box[b].lo[ax]; });
      mid = st + span / 2;
    } else {
      auto it = std::partition(objs.begin() + st, objs.begin() + en, [&](int32_t o) {
        return comp(bx_center(box[o]), bax) < bpos;
      });
      mid = size_t(it - objs.begin());
      if (mid == st || mid == en) mid = st + span / 2;
    }
    ref_bvh_leaves(objs, st, mid, w * 0.5, out);
    ref_bvh_leaves(objs, mid, en, w * 0.5, out);
  }

  bool add_light(int32_t o, double w, std::vector<int32_t> &chain) {
    const rt_object_desc &x = D->objects[o];
    if (x.kind == RT_OBJ_LIST) { // HittableList::pdf_value / random, HittableList.cpp:44-63
      double cw = w * (1.0 / x.count);
      for (int k = 0; k < x.count; ++k)
        if (!add_light(D->children[x.child + k], cw, chain)) return false;
      return true;
    }
    if (x.kind == RT_OBJ_ROTATE_Y || x.kind == RT_OBJ_TRANSLATE) {
      if ((int)chain.size() >= RT_MAX_CHAIN)
        return fail("UNSUPPORTED: light transform chain deeper than RT_MAX_CHAIN");
      chain.push_back(o);
      bool ok = add_light(x.child, w, chain);
      chain.pop_back();
      return ok;
    }
    DLight L;
    std::memset(&L, 0, sizeof L);
    if (x.kind == RT_OBJ_SPHERE) {
      L.kind = I_SPHERE;
      L.idx = sphere_record(o);
    } else if (x.kind == RT_OBJ_QUAD) {
      L.kind = I_QUAD;
      L.idx = quad_record(o);
    } else {
      L.kind = I_NONE; // Hittable defaults: pdf 0, random (1,0,0)
    }
    std::vector<int> ch(chain.begin(), chain.end());
    L.xf_first = emit_chain(ch);
    L.xf_count = (int32_t)chain.size();
    L.weight = w;
    H.lights.push_back(L);
    return true;
  }

  bool emit_lights() {
    if (D->lights < 0) return true;
    const rt_object_desc &lx = D->objects[D->lights];
    if (lx.count == 0) return true;
    std::vector<int32_t> chain;
    if (D->use_bvh) {
      std::vector<int32_t> objs(D->children + lx.child, D->children + lx.child + lx.count);
      std::vector<std::pair<int32_t, double>> leaves;
      ref_bvh_leaves(objs, 0, objs.size(), 1.0, leaves);
      for (auto &p : leaves)
        if (!add_light(p.first, p.second, chain)) return false;
    } else {
      if (!add_light(D->lights, 1.0, chain)) return false;
    }
    double c = 0;
    for (auto &L : H.lights) {
      c += L.weight;
      L.cum = c;
    }
    return true;
  }

  bool run() {
    if (!D) return fail("null scene description");
    if (D->n_objects <= 0 || !D->objects) return fail("scene has no objects");
    if (D->n_textures < 0 || D->n_materials < 0 || D->n_perlin < 0 || D->n_children < 0)
      return fail("negative table size");
    if ((D->n_textures && !D->textures) || (D->n_materials && !D->materials) ||
        (D->n_perlin && !D->perlin) || (D->n_children && !D->children))
      return fail("null table pointer");
    box.assign(D->n_objects, bx_empty());
    state.assign(D->n_objects, 0);
    depth.assign(D->n_objects, 0);
    sphere_of.assign(D->n_objects, -1);
    quad_of.assign(D->n_objects, -1);
    if (D->world < 0 || D->world >= D->n_objects || D->objects[D->world].kind != RT_OBJ_LIST)
      return fail("world must be a list object");
    if (D->lights >= D->n_objects ||
        (D->lights >= 0 && D->objects[D->lights].kind != RT_OBJ_LIST))
      return fail("lights must be a list object or -1");
    for (int o = 0; o < D->n_objects; ++o)
      if (!visit(o)) return false;
    if (!check_world_materials(D->world)) return false;
    std::vector<FItem> fitems;
    std::vector<int> chain;
    if (!flatten(D->world, chain, fitems, false)) return false;
    std::vector<Bx> ibox;
    for (const FItem &f : fitems) {
      DItem it;
      Bx bb;
      if (!make_item(f, it, bb)) return false;
      if (it.kind == I_MEDIUM) {
        H.mitems.push_back(it);
        for (int a = 0; a < 3; ++a) H.mbox.push_back(SahBuilder::f32_lo(bb.lo[a]));
        for (int a = 0; a < 3; ++a) H.mbox.push_back(SahBuilder::f32_hi(bb.hi[a]));
        continue;
      }
      H.items.push_back(it);
      ibox.push_back(bb);
    }
    emit_materials();
    const int builder = D->bvh_builder;
    const bool device = ibox.size() >= 2 &&
                        (builder == RT_BVH_DEVICE || builder == RT_BVH_DEVICE_SAH ||
                         (builder == RT_BVH_AUTO && ibox.size() >= (size_t)kDeviceBuildMin));
    if (device) { // built by the library on the GPU after upload (rt_bvh_sah.hip / rt_bvh_build.hip)
      H.device_bvh = builder == RT_BVH_DEVICE ? RT_BVH_DEVICE : RT_BVH_DEVICE_SAH;
      H.item_boxes.reserve(6 * ibox.size());
      for (int a = 0; a < 3; ++a) {
        H.scene_lo[a] = kInf;
        H.scene_hi[a] = -kInf;
      }
      for (const Bx &bb : ibox) {
        for (int a = 0; a < 3; ++a) H.item_boxes.push_back(bb.lo[a]);
        for (int a = 0; a < 3; ++a) H.item_boxes.push_back(bb.hi[a]);
        for (int a = 0; a < 3; ++a) { // centroid bounds (Morton grid)
          double c = 0.5 * (bb.lo[a] + bb.hi[a]);
          H.scene_lo[a] = std::fmin(H.scene_lo[a], c);
          H.scene_hi[a] = std::fmax(H.scene_hi[a], c);
        }
      }
      H.nodes.assign(ibox.size() - 1, DNode{});
    } else {
      SahBuilder(H).emit_world_bvh(ibox);
    }
    return emit_lights();
  }
};

} // namespace

void build_world_bvh_host(HostScene &H) {
  std::vector<Bx> boxes(H.item_boxes.size() / 6);
  for (size_t i = 0; i < boxes.size(); ++i)
    for (int a = 0; a < 3; ++a) {
      boxes[i].lo[a] = H.item_boxes[6 * i + a];
      boxes[i].hi[a] = H.item_boxes[6 * i + 3 + a];
    }
  H.nodes.clear();
  H.device_bvh = 0;
  SahBuilder(H).emit_world_bvh(boxes);
}

double bvh_sah_cost(const std::vector<DNode> &nodes) {
  if (nodes.empty()) return 0.0;
  auto area = [](const float *lo, const float *hi) {
    const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
    return 2.0 * (x * y + y * z + z * x);
  };
  float rlo[3], rhi[3];
  for (int a = 0; a < 3; ++a) {
    rlo[a] = std::min(nodes[0].lo[a][0], nodes[0].lo[a][1]);
    rhi[a] = std::max(nodes[0].hi[a][0], nodes[0].hi[a][1]);
  }
  const double root = area(rlo, rhi);
  if (!(root > 0.0)) return 0.0;
  double c = 1.0;
  for (const DNode &d : nodes)
    for (int k = 0; k < 2; ++k) {
      const int e = d.entry[k];
      const double w = e >= 0 ? 1.0 : (double)((~e) & 7);
      const float lo[3] = {d.lo[0][k], d.lo[1][k], d.lo[2][k]};
      const float hi[3] = {d.hi[0][k], d.hi[1][k], d.hi[2][k]};
      c += w * area(lo, hi) / root;
    }
  return c;
}

int collapse_bvh4(const std::vector<DNode> &bin, std::vector<DNode4> &out) {
  out.clear();
  if (bin.empty()) return 0;
  struct Child {
    float lo[3], hi[3];
    int32_t e;
  };
  auto child = [&](const DNode &b, int k) {
    Child c;
    for (int a = 0; a < 3; ++a) {
      c.lo[a] = b.lo[a][k];
      c.hi[a] = b.hi[a][k];
    }
    c.e = b.entry[k];
    return c;
  };
  auto area = [](const Child &c) {
    const double x = (double)c.hi[0] - c.lo[0], y = (double)c.hi[1] - c.lo[1],
                 z = (double)c.hi[2] - c.lo[2];
    return x * y + y * z + z * x;
  };
  std::vector<int> src{0}, level{1}; // binary root and level of each 4-wide node
  int depth = 0;
  for (size_t k = 0; k < src.size(); ++k) {
    const DNode &b = bin[src[k]];
    Child c[4];
    int n = 2;
    c[0] = child(b, 0);
    c[1] = child(b, 1);
    while (n < 4) {
      int pick = -1;
      double best = -1.0;
      for (int i = 0; i < n; ++i)
        if (c[i].e >= 0 && area(c[i]) > best) {
          best = area(c[i]);
          pick = i;
        }
      if (pick < 0) break;
      const DNode &m = bin[c[pick].e];
      for (int i = n; i > pick + 1; --i) c[i] = c[i - 1]; // keep the leaf order
      c[pick] = child(m, 0);
      c[pick + 1] = child(m, 1);
      ++n;
    }
    DNode4 q;
    std::memset(&q, 0, sizeof q);
    for (int i = 0; i < 4; ++i) {
      for (int a = 0; a < 3; ++a) {
        q.lo[a][i] = i < n ? c[i].lo[a] : std::numeric_limits<float>::infinity();
        q.hi[a][i] = i < n ? c[i].hi[a] : -std::numeric_limits<float>::infinity();
      }
      if (i >= n) {
        q.entry[i] = -1;
      } else if (c[i].e >= 0) {
        q.entry[i] = (int32_t)src.size();
        src.push_back(c[i].e);
        level.push_back(level[k] + 1);
      } else {
        q.entry[i] = c[i].e;
      }
    }
    depth = std::max(depth, level[k]);
    out.push_back(q);
  }
  return depth;
}

int compile_scene(const rt_scene_desc *desc, HostScene &out, std::string &err) {
  if (desc && desc->bvh_arity != 0 && desc->bvh_arity != 2 && desc->bvh_arity != 4) {
    err = "bvh_arity must be 0 (auto), 2 or 4";
    return RT_ERR_INVALID;
  }
  Compiler c(desc, out, err);
  if (!c.run()) return err.rfind("UNSUPPORTED", 0) == 0 ? RT_ERR_UNSUPPORTED : RT_ERR_INVALID;
  return RT_OK;
}

int camera_setup(const rt_camera_desc *cd, rt_frame *f, std::string &err) {
  if (!cd || !f) {
    err = "null camera";
    return RT_ERR_INVALID;
  }
  if (cd->image_width < 1 || cd->samples_per_pixel < 1 || cd->max_depth < 0 ||
      !(cd->aspect_ratio > 0)) {
    err = "invalid camera (image_width/samples_per_pixel >= 1, aspect_ratio > 0)";
    return RT_ERR_INVALID;
  }
  // Camera::initialize, Camera.cpp:31-73
  int W = cd->image_width;
  int H = int(W / cd->aspect_ratio);
  H = (H < 1) ? 1 : H;
  double theta = cd->vfov * kPi / 180.0;
  double h = std::tan(theta / 2);
  double vh = 2 * h * cd->focus_dist;
  double vw = vh * (double(W) / H);
  auto unit = [](P3 v) {
    double l = std::sqrt(dotp(v, v));
    if (l > 1e-8) {
      double s = 1.0 / l;
      return P3{v.x * s, v.y * s, v.z * s};
    }
    return P3{1.0, 0.0, 0.0};
  };
  P3 from = p3(cd->lookfrom), at = p3(cd->lookat), up = p3(cd->vup);
  P3 w = unit(sub(from, at));
  P3 u = unit(crossp(up, w));
  P3 v = crossp(w, u);
  P3 vu = scl(vw, u);
  P3 vv = scl(vh, P3{-v.x, -v.y, -v.z});
  P3 du = scl(1 / double(W), vu);
  P3 dv = scl(1 / double(H), vv);
  P3 ul = sub(sub(sub(from, scl(cd->focus_dist, w)), scl(1 / 2.0, vu)), scl(1 / 2.0, vv));
  P3 p00 = add(ul, scl(0.5, add(du, dv)));
  double rad = cd->focus_dist * std::tan((cd->defocus_angle / 2) * kPi / 180.0);
  auto rv = [](P3 a) { return rt_vec3{a.x, a.y, a.z}; };
  f->image_width = W;
  f->image_height = H;
  f->sqrt_spp = int(std::sqrt(cd->samples_per_pixel));
  f->max_depth = cd->max_depth;
  f->center = rv(from);
  f->pixel00_loc = rv(p00);
  f->pixel_delta_u = rv(du);
  f->pixel_delta_v = rv(dv);
  f->u = rv(u);
  f->v = rv(v);
  f->w = rv(w);
  f->defocus_disk_u = rv(scl(rad, u));
  f->defocus_disk_v = rv(scl(rad, v));
  f->defocus_angle = cd->defocus_angle;
  f->pixel_samples_scale = 1.0 / cd->samples_per_pixel;
  f->background = cd->background;
  return RT_OK;
}

int device_camera(const rt_frame *f, DCamera &c, std::string &err) {
  if (!f) {
    err = "null frame";
    return RT_ERR_INVALID;
  }
  if (f->image_width < 1 || f->image_height < 1 || f->sqrt_spp < 1 || f->max_depth < 0) {
    err = "invalid frame (width/height/sqrt_spp >= 1, max_depth >= 0)";
    return RT_ERR_INVALID;
  }
  auto cp = [](double *d, const rt_vec3 &v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
  };
  cp(c.center, f->center);
  cp(c.p00, f->pixel00_loc);
  cp(c.du, f->pixel_delta_u);
  cp(c.dv, f->pixel_delta_v);
  cp(c.disk_u, f->defocus_disk_u);
  cp(c.disk_v, f->defocus_disk_v);
  cp(c.bg, f->background);
  c.defocus_angle = f->defocus_angle;
  c.scale = f->pixel_samples_scale;
  c.W = f->image_width;
  c.H = f->image_height;
  c.sqrt_spp = f->sqrt_spp;
  c.rs = 1.0 / c.sqrt_spp;
  c.max_depth = f->max_depth;
  return RT_OK;
}

int launch_geometry(const rt_frame *f, const rt_render_params *p, DLaunch &L, std::string &err) {
  auto bad = [&](int code, const char *m) {
    err = m;
    return code;
  };
  if (!f || !p) return bad(RT_ERR_INVALID, "null frame or params");
  int r0 = p->row_begin, r1 = p->row_end;
  if (r0 == 0 && r1 == 0) r1 = f->image_height;
  if (r0 < 0 || r1 > f->image_height || r1 <= r0) return bad(RT_ERR_INVALID, "row range outside the image");
  int64_t nsamp = (int64_t)f->sqrt_spp * f->sqrt_spp;
  int sb = p->sample_begin;
  int64_t sc = p->sample_count < 0 ? nsamp - sb : p->sample_count;
  if (sb < 0 || sc < 0 || sb + sc > nsamp) return bad(RT_ERR_INVALID, "sample range outside [0, sqrt_spp^2)");
  if (64 * sc > 0x7FFFFFFF) return bad(RT_ERR_UNSUPPORTED, "too many strata in one launch");
  if ((int64_t)f->image_width * f->image_height > 0xFFFFFFFFll)
    return bad(RT_ERR_UNSUPPORTED, "image too large for 32-bit pixel keys");
  if (p->output != RT_OUT_SCALED && p->output != RT_OUT_SUM) return bad(RT_ERR_INVALID, "unknown output mode");
  if (p->strata_chunks < 0)
    return bad(RT_ERR_INVALID, p->strata_chunks == RT_CHUNKS_AUTO
                                   ? "RT_CHUNKS_AUTO is for rt_render_device (RT_LAYOUT_TILES, RT_OUT_SUM) "
                                     "and rt_render_stats (RT_LAYOUT_TILES) only"
                                   : "strata_chunks must be >= 0 (or RT_CHUNKS_AUTO)");
  L.row_begin = r0;
  L.row_end = r1;
  L.sample_begin = sb;
  L.sample_count = (int32_t)sc;
  L.seed_lo = (uint32_t)p->seed;
  L.seed_hi = (uint32_t)(p->seed >> 32);
  L.output = p->output;
  L.accumulate = p->accumulate ? 1 : 0;
  L.tiles_x = (f->image_width + 7) / 8;
  L.tiles_y = (r1 - r0 + 7) / 8;
  int stride = p->tile_stride <= 0 ? 1 : p->tile_stride;
  if (p->tile_first < 0 || p->tile_first >= stride) return bad(RT_ERR_INVALID, "tile_first must be in [0, tile_stride)");
  if (p->layout != RT_LAYOUT_FRAME && p->layout != RT_LAYOUT_TILES) return bad(RT_ERR_INVALID, "unknown output layout");
  const int64_t n_tiles = (int64_t)L.tiles_x * L.tiles_y;
  L.tile_first = p->tile_first;
  L.tile_stride = stride;
  L.n_local_tiles = (int32_t)(n_tiles > p->tile_first ? (n_tiles - p->tile_first + stride - 1) / stride : 0);
  L.compact = p->layout == RT_LAYOUT_TILES;
  int chunks = p->strata_chunks == 0 ? 1 : p->strata_chunks;
  if (chunks > 1 && !L.compact) return bad(RT_ERR_INVALID, "strata_chunks > 1 needs RT_LAYOUT_TILES");
  if (chunks > L.sample_count && L.sample_count > 0)
    return bad(RT_ERR_INVALID, "strata_chunks exceeds the launched strata");
  if ((int64_t)L.n_local_tiles * chunks > 0x7FFFFFFF) return bad(RT_ERR_UNSUPPORTED, "too many work units");
  L.n_chunks = chunks;
  L.chunk_strata = (L.sample_count + chunks - 1) / chunks;
  L.unit_ctr = nullptr;
  L.grid_cap = 0;
  L.tile_order = nullptr;
  L.tile_cost = nullptr;
  // one chunk: every tile is a whole unit; strata_chunks > 1 (tile layout):
  // every tile split, its chunk partials are the caller's output (the launcher
  // points parts at the output buffer)
  L.n_head = chunks > 1 ? 0 : L.n_local_tiles;
  L.head_chunks = 1;
  L.parts = nullptr;
  L.parts_final = chunks > 1 ? 1 : 0;
  return RT_OK;
}

} // namespace rtx
