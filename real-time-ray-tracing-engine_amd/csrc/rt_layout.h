// rt_layout.h — device-side scene layout shared by the host scene compiler
// (rt_scene.cpp) and the HIP kernels (rt_kernel.hip).
//
// Replaces the reference's pointer graph of 256-B sub-allocated CudaHittable /
// CudaSphere / CudaPlane / CudaBVHNode structs (CudaSceneContext.cuh:150-172,
// Hittable.cuh:37-49, BVHNode.cuh:16-22) with flat index-linked arrays.
//
// The object graph is flattened at scene-compile time into leaf ITEMS: a sphere,
// a quad or a constant medium, each with the chain of RotateY/Translate
// transforms above it (outermost first).  Lists disappear: closest hit over
// List(A,B) is closest hit over {A,B}, and Rot(List(A,B)) hits exactly like
// {Rot(A),Rot(B)} because every member sees the identical transformed ray.  A
// medium keeps its boundary as a range of items in the medium's local frame.
// The device code therefore needs no recursion and no function calls.
//
//   - world BVH: binary nodes carrying BOTH children's boxes (one 64-B fetch
//     tests two boxes), children by index, leaves as ranges of items (the item
//     array is permuted into leaf order, so there is no reference indirection);
//     boxes are fp32 rounded outward and tested conservatively (rt_path.h), the
//     primitive tests that decide every hit stay fp64;
//   - lights: flattened to weighted leaves (primitive + transform chain), so light
//     sampling and the light pdf are plain loops.
// Everything but the BVH boxes is fp64, matching the reference arithmetic (Vec3.hpp:184).
#ifndef RT_LAYOUT_H
#define RT_LAYOUT_H
#include <stdint.h>

#define RT_MAX_CHAIN 4    // RotateY/Translate ops above a leaf item
#define RT_N_STATS 24      // counters of the STATS kernel instance (rt_path_stats)
#define RT_STACK_DEPTH 32 // traversal stack entries per lane (BVH depth is capped below it)
#define RT_STACK_DEPTH4 64 // 4-wide walks push up to three entries per level
#define RT_PC_WAVES 16    // waves per block of the persistent instance (one block per CU)
#define RT_PC_BLOCK_WAVES RT_PC_WAVES
#define RT_FLAT_MAX 8 // worlds of at most this many items are one flat leaf (no BVH walk)

enum DItemKind {
  I_SPHERE = 0,
  I_QUAD = 1,
  I_MEDIUM = 2,
  I_NONE = 3 // lights only: Hittable::pdf_value 0, random (1,0,0)
};

struct DItem {       // 32 B
  int32_t kind;
  int32_t idx;       // index into spheres / quads / media
  int32_t xf_first;  // transform chain in xforms[], outermost first
  int32_t xf_count;
  int32_t mat;       // primitive material (-1 for light-only primitives)
  int32_t id;        // caller's object index (medium RNG key)
  int32_t pad[2];
};

enum DXformKind { X_TRANSLATE = 0, X_ROTATE_Y = 1 };
struct DXform {      // 32 B — Translate offset or RotateY (sin, cos)
  int32_t kind, pad;
  double a, b, c;    // translate: offset xyz; rotate: a = sin, b = cos
};

struct DSphere {     // 64 B — Sphere.hpp: m_center Ray (c0, c1-c0), m_radius
  double c0[3];
  double dir[3];     // c1 - c0, 0 for static spheres
  double inv_r;      // 1 / r: the reference's (p - c) / r is (1 / r) * (p - c) (Vec3.hpp:88)
  double rr;         // r*r, as Sphere::hit computes it
};

struct DQuad {       // 144 B — Plane.hpp members
  double Q[3], u[3], v[3];
  double n[3];       // unit normal
  double w[3];       // n / (n.n)
  double D;
  double area;
  int32_t aa;        // axis-aligned quad (u, v, n and w each on one axis; make_box's
                     // faces, the Cornell walls): k | i << 2 | j << 4 | neg << 6 with
                     // k the normal axis, i / j the u / v axes, neg = the permutation
                     // (k, i, j) is odd; -1 otherwise (rt_path.h quad_t)
  int32_t pad_;
};
static_assert(sizeof(DQuad) == 144, "DQuad layout");

struct DMedium {     // ConstantMedium: -1/density, phase material, boundary items
  double neg_inv_density;
  int32_t phase, id;
  int32_t b_first, b_count; // boundary items in bitems[] (medium-local frame)
  // box = 1: the boundary is make_box's six axis-aligned quads (PlaneUtility.hpp:
  // 11-39), all under the one transform chain [bxf_first, +bxf_count), two faces
  // per axis whose rectangles span the other two axes' face planes (checked by
  // the scene compiler, rt_scene.cpp box_of).  rt_path.h box_span then answers
  // both boundary queries from the six face distances alone.  Per axis a and
  // face f (the two faces normal to a): the face's unit-normal component
  // bnk[a][f] = Plane::m_normal[a] (|bnk[a][0]| == |bnk[a][1]|) and its
  // bD[a][f] = Plane::m_D; bB[a] = the largest |plane coordinate| along a.
  int32_t box, bxf_first, bxf_count, pad_;
  double bnk[3][2];
  double bD[3][2];
  double bB[3];
};
static_assert(sizeof(DMedium) == 160, "DMedium layout");

struct DNode {       // 64 B: both children's boxes (fp32, rounded outward) + links
  float lo[3][2];    // lo[axis][child]: the two children's planes of one axis side by
  float hi[3][2];    // side, so one packed fp32 FMA (v_pk_fma_f32) computes both
  int32_t entry[2];  // >= 0: inner node index; < 0: leaf ~((first << 3) | count),
                     // items [first, first + count) (items are stored in leaf order)
  int32_t pad[2];
};
static_assert(sizeof(DNode) == 64, "DNode layout");

// A binary node as the kernels stage it in LDS (80 B): per axis the children's
// lo planes, hi planes and lo planes again, so that a ray's near and far plane
// pairs (sign-picked: near = lo for 1/d_a >= 0, hi otherwise) are adjacent for
// either sign -- one 16-B read per axis at byte 24 a + 8 s_a instead of two
// 8-B reads at unrelated offsets (rt_path.h load_planes_l).  (Staged as
// DNode instead: C3 -1.7 %, profiles/r04l_c3_ab.log.)
struct DNodeL {
  float p[3][3][2]; // p[axis][0] = lo[axis][*], p[axis][1] = hi[axis][*], p[axis][2] = lo[axis][*]
  int32_t entry[2];
};
static_assert(sizeof(DNodeL) == 80, "DNodeL layout");
// (whole: the whole tree is staged -- inner children as DNodeL byte offsets)
inline DNodeL lds_node(const DNode &n, bool whole) {
  DNodeL l;
  for (int a = 0; a < 3; ++a)
    for (int k = 0; k < 2; ++k) {
      l.p[a][0][k] = l.p[a][2][k] = n.lo[a][k];
      l.p[a][1][k] = n.hi[a][k];
    }
  for (int k = 0; k < 2; ++k)
    l.entry[k] = whole && n.entry[k] >= 0 ? n.entry[k] * (int32_t)sizeof(DNodeL) : n.entry[k];
  return l;
}

// 4-wide BVH node (128 B): the boxes of up to four children in SoA order
// (lo x[4], lo y[4], lo z[4], hi x[4], ...), fp32 rounded outward like DNode's,
// and their entries with DNode's encoding (-1 = empty slot).  Collapsed from the
// binary tree for large scenes (rt_scene.cpp collapse_bvh4; RT_FEAT_BVH4).
struct DNode4 {
  float lo[3][4], hi[3][4];
  int32_t entry[4];
  int32_t pad[4];
};
static_assert(sizeof(DNode4) == 128, "DNode4 layout");

struct DMat {        // 48 B
  int32_t kind, tex;
  union {
    struct {         // lambertian / metal / isotropic / diffuse light
      double albedo[3];
      double fuzz;
    };
    struct {         // dielectric: constants formed once on the host with the
                     // kernel's own operations (DielectricMaterial.cpp:62-66, 26-31):
      double inv_ior; // 1/ior (the front-face ratio)
      double r0[2];   // Schlick's ((1 - ri) / (1 + ri))^2 for ri = 1/ior (front), ior (back)
      double pad_;
    };
  };
  double ior;
};
static_assert(sizeof(DMat) == 48, "DMat layout");

struct DTex {        // 48 B
  int32_t kind, even, odd, perlin;
  double scale;
  double color[3];
  double inv_scale; // checker: 1.0 / scale formed on the host (CheckerTexture.cpp:19)
};

struct DPerlin {
  double rv[256][3];
  int32_t px[256], py[256], pz[256];
};

struct DLight {      // flattened light leaf (48 B)
  int32_t kind;      // I_SPHERE / I_QUAD / I_NONE
  int32_t idx;
  int32_t xf_first, xf_count;
  double weight;     // product of 1/N over the list / BVH levels above it
  double cum;        // cumulative weight in DFS order (selection)
  double pad[2];
};

struct DScene {      // kernel argument (by value)
  const DNode *nodes;
  const DItem *items;    // world primitive items, in BVH leaf order
  const DItem *mitems;   // world media (tested after the BVH walk, see rt_path.h)
  const float *mbox;     // per medium: world box lo[3], hi[3] (fp32, rounded outward)
  const DItem *bitems;   // medium boundary items
  const DXform *xforms;
  const DSphere *spheres;
  const DQuad *quads;
  const DMedium *media;
  const DMat *mats;
  const DTex *texs;
  const DPerlin *perlin;
  const DLight *lights;
  int32_t n_lights;
  int32_t n_nodes;
  int32_t root_is_leaf;  // whole world is one leaf: items [0, n_root_items)
  int32_t n_root_items;
  int32_t features;      // RT_FEAT_* bits: selects the specialised kernel instance
  int32_t n_mitems;
  int32_t stack_depth;   // per-lane traversal stack entries (BVH depth + 1)
  int32_t n_lds_nodes;   // nodes [0, n_lds_nodes) are staged in LDS (BFS order: top levels)
  int32_t static_spheres; // 1: every sphere has c1 == c0 (no motion blur): center = c0
  int32_t n_lds_nodes_pc; // nodes staged by the persistent instance's blocks (-1: none)
  int32_t lds_items_pc;   // world items [0, n) and spheres [0, lds_spheres_pc) the persistent
  int32_t lds_spheres_pc; // instance stages after its nodes (0: primitives stay in HBM)
  int32_t pc_waves;       // waves per block of the persistent instance: RT_PC_WAVES (one
                          // block per CU) or 4 (deep trees); 0: no persistent launches
  int32_t lds_perlin;     // 1: the scene's one Perlin table is staged in LDS by the noise
                          // instances' blocks (perlin_lds); 0: read from HBM
};

// Scene features (kernel specialisation keys)
#define RT_FEAT_MEDIA 1  // constant media among the world items
#define RT_FEAT_XFORM 2  // transform chains on world items or lights
#define RT_FEAT_LIGHTS 4 // non-empty light list
#define RT_FEAT_NOISE 8  // Perlin noise textures
#define RT_FEAT_FLAT 16  // flat world (root_is_leaf): no BVH walk
#define RT_FEAT_BVH4 32  // the world BVH is 4-wide (DNode4); never with RT_FEAT_FLAT
// bytes per BVH node staged in LDS (DNode4 / DNodeL / DNode)
#define RT_LDS_NODE_BYTES(features)                                                                \
  (((features) & RT_FEAT_BVH4) ? (int)sizeof(DNode4) : (int)sizeof(DNodeL))

// LDS plan of one render instance (rtk_lds_plan): its occupancy target and
// what the per-block LDS share at that occupancy leaves for staged BVH nodes.
struct RtkLdsPlan {
  int32_t waves_per_simd; // resident waves per SIMD the instance's registers allow
  int32_t block_budget;   // LDS bytes per block at that occupancy (<= 64 KB)
  int32_t fixed_bytes;    // static LDS + traversal stacks per block
  int32_t stack_fits;     // fixed_bytes <= block_budget
  int32_t n_nodes;        // BVH nodes that fit in the rest (BFS prefix)
  int32_t resident_waves_per_cu; // waves resident per CU with no nodes staged (LDS may limit it)
};

struct DCamera {     // the rt_frame values the kernel needs
  double center[3], p00[3], du[3], dv[3], disk_u[3], disk_v[3], bg[3];
  double defocus_angle;
  double scale;
  double rs; // 1.0 / sqrt_spp, formed on the host (Camera::initialize's recip_sqrt_spp)
  int32_t W, H, sqrt_spp, max_depth;
};

struct DLaunch {
  int32_t row_begin, row_end;
  int32_t sample_begin, sample_count;
  uint32_t seed_lo, seed_hi;
  int32_t output, accumulate;
  int32_t tiles_x, tiles_y;
  int32_t tile_first, tile_stride; // tiles rendered: tile_first + k * tile_stride
  int32_t n_local_tiles;           // k in [0, n_local_tiles)
  int32_t compact;                 // RT_LAYOUT_TILES output
  // Work units: the head tiles [0, n_head) in head_chunks stratum chunks each
  // (head_chunks 1: "whole" units whose pixels are final -- frame or compact
  // tile layout, scaled / accumulated as asked); the tail tiles [n_head,
  // n_local_tiles) in n_chunks chunks of chunk_strata strata each.  Chunk units
  // write per-pixel partial sums to parts[u'][64][3], u' = unit when
  // head_chunks > 1, else unit - n_head (raw sums for a frame launch --
  // split_sum_kernel adds them in chunk order; the caller's output when
  // parts_final: RT_LAYOUT_TILES with strata_chunks).
  int32_t n_chunks, chunk_strata;
  int32_t *unit_ctr;               // persistent launch: next work unit (device counter), or null
  int32_t grid_cap;                // persistent launch: resident blocks of the instance (0: none)
  int32_t n_head;
  double *parts;
  int32_t parts_final;
  int32_t head_chunks;
  // Dispatch order (rt_api.cpp "tile order"): the k-th local tile of the plan
  // above is local tile tile_order[k] of the launch (null: k itself); units,
  // chunk partials and the head / tail split follow k, every pixel write goes
  // to the mapped tile.  tile_cost (null: not measured): each unit adds its
  // duration (100 MHz clock ticks) to its mapped tile's counter.
  const int32_t *tile_order;
  uint32_t *tile_cost;
};

#endif
