/*
 * rt_api.h — C ABI of the MI355X-native path-tracing hot path.
 *
 * This is the drop-in boundary that replaces the reference's CUDA entry
 * points for the per-pixel hot path (primary ray -> BVH traversal ->
 * sphere/quad/AABB intersection -> material scatter -> texture eval ->
 * multi-sample accumulation).  Everything here is plain C: fixed-width
 * integers, doubles and pointers, no C++ or torch types.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   rt_camera_setup   <- Camera::initialize             src/core/camera/Camera.cpp:31-73
 *   rt_scene_create   <- initialize_cuda_scene          src/scene/CudaSceneInitialization.cuh:249-300
 *                        (+ HittableConverter::cpu_to_cuda_hittable, HittableConverter.cuh:50-111,
 *                           MaterialConverter.cuh:26-121, TextureConverter.cuh:19-88,
 *                           CudaSceneContext::initialize/finalize_and_upload, CudaSceneContext.cuh:71-123)
 *   rt_scene_create_tuned <- the same with the launch / staging / builder tuning passed
 *                        explicitly (rt_tuning; the reference's CameraConfig,
 *                        src/core/camera/CameraConfig.hpp:9-62, carries its settings the same way)
 *   rt_scene_destroy  <- cleanup_cuda_scene             src/scene/CudaSceneInitialization.cuh:302-308
 *   rt_render         <- cuda_init_rand_states_wrapper  src/core/camera/CameraKernelWrappers.cuh:11-13
 *                        + cuda_static_render_wrapper   src/core/camera/CameraKernelWrappers.cuh:25-34
 *                        + the per-batch memset/sync/D2H copy of StaticCamera::render_gpu
 *                                                       src/core/camera/StaticCamera.cpp:235-300
 *   rt_render_device  <- same, but accumulating raw sample sums into a caller-owned device
 *                        buffer on a caller stream (multi-GPU sample sharding / progressive
 *                        accumulation; the role of dynamic_render_tile_kernel's accumulation
 *                        buffer, CameraKernels.cu:206-236)
 *   rt_multi_create / rt_multi_render / rt_multi_destroy
 *                     <- StaticCamera::render_gpu's single-device batch loop
 *                        (src/core/camera/StaticCamera.cpp:136-313) extended to N devices:
 *                        one scene and one host thread per shard, 8x8 tiles dealt
 *                        round-robin over the shards (SURVEY §8(b) "Threading")
 *   rt_tiles_sum_device / rt_tiles_to_frame_device
 *                     <- the batch assembly of StaticCamera::render_gpu (the D2H copy of each
 *                        64-row batch into its rows of the frame, StaticCamera.cpp:281-299) for
 *                        tile shards: chunk partials summed and tiles reordered into frame rows
 *                        on the device, before the one copy out
 *   rt_last_error     <- replaces CUDA_CHECK's exit() and the converters' exceptions
 *                        (CudaMemoryUtility.cuh:9-15, HittableConverter.cuh:103-108): errors are
 *                        returned as negative codes, never thrown or exit()ed across the ABI.
 *
 * Scene description.  The reference hands the GPU a pointer graph built from
 * shared_ptr<Hittable> objects.  Here the caller serialises that graph into
 * flat tables (textures, Perlin tables, materials, objects, child lists) whose
 * entries mirror the reference classes one to one; rt_scene_create copies them,
 * builds its own acceleration structure and uploads a device layout that the
 * library owns.  The caller owns every pointer it passes in.
 *
 * Threading.  Distinct rt_scene objects are independent and may be used from
 * different host threads (and devices) at once.  One rt_scene is used by one
 * host thread at a time: its kernel-timing events, its scratch / staging
 * buffers, its work-unit counter (persistent launches) and its tile-cost /
 * dispatch-order buffers (rt_tuning.no_tile_order) are per scene.
 * A scene's launches run one after another even on different caller streams:
 * each launch waits for the scene's previous one (an event), since they share
 * the scene's work-unit counter, scratch and tile orders; the caller orders
 * its own buffers' producers and consumers with its streams as for any device
 * work.  Destroying a scene, or a launch that grows its buffers, waits for
 * that scene's own work only -- its stream and its last launch -- never for
 * other scenes' or threads' work on the device: scene memory comes from a
 * library-owned pool per device (hipMallocFromPoolAsync on the scene's
 * stream) because a plain hipFree waits for the whole device, and destroy
 * queues nothing on any stream (a stream may share a hardware queue with a
 * busy one): a destroyed scene's idle buffers are freed by the next
 * allocation on the device, or at process exit.  Tile orders are kept per
 * launch shape (four shapes per scene, least recently used replaced).
 *
 * Numerics.  All arithmetic is fp64, as in the reference (Vec3.hpp:184).  The
 * random stream is a stateless counter-based Philox4x32-10 keyed by
 * (seed, pixel, stratum sample, bounce, slot); see DESIGN.md "RNG contract".
 */
#ifndef RT_API_H
#define RT_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever a struct layout or a signature below changes.  A caller
   checks rt_abi_version() == the RT_ABI_VERSION it was compiled against before
   any other call (rtx/lib.py does): structs are passed by pointer without a
   size field, so a caller built against another version must not proceed.
   2: rt_scene_desc.bvh_arity, rt_path_stats.cyc_*, rt_scene_info's stack and
      LDS fields.
   3: rt_tiles_sum_device, rt_tiles_to_frame_device, rt_multi_gather_ms; the
      rt_multi exchange runs on the devices.
   4: rt_tuning with rt_scene_create_tuned / rt_multi_create_tuned (the
      library reads no environment variables); rt_path_stats.medium_box_*;
      rt_scene_info.lds_node_bytes.
   5: strata_chunks = RT_CHUNKS_AUTO (rt_render_device, RT_LAYOUT_TILES): the
      library's work units for a tile subset, per-tile sums out; rt_tuning
      sub_* and no_tile_order fields (in four of the reserved slots: same size
      and offsets); round 6: rt_tuning.probe_strata (a fifth reserved slot,
      zero = the default, so version 5 callers are unaffected). */
#define RT_ABI_VERSION 5

/* ---- status codes ------------------------------------------------------ */
#define RT_OK 0
#define RT_ERR_INVALID (-1)     /* malformed description / argument */
#define RT_ERR_DEVICE (-2)      /* HIP runtime error (message in rt_last_error) */
#define RT_ERR_OOM (-3)         /* device allocation failed */
#define RT_ERR_UNSUPPORTED (-4) /* valid but not supported (e.g. nesting too deep) */

typedef struct rt_vec3 {
  double x, y, z;
} rt_vec3;

/* ---- textures (Texture.hpp:8-18) ---------------------------------------- */
enum {
  RT_TEX_SOLID = 0,   /* SolidColorTexture   SolidColorTexture.cpp:8-10 */
  RT_TEX_CHECKER = 1, /* CheckerTexture      CheckerTexture.cpp:41-55   */
  RT_TEX_NOISE = 2    /* NoiseTexture        NoiseTexture.cpp:31-34     */
};

typedef struct rt_texture_desc {
  int32_t kind;
  int32_t even;   /* checker: texture index used when the cell parity is even */
  int32_t odd;    /* checker: texture index used when the parity is odd */
  int32_t perlin; /* noise: index into rt_scene_desc.perlin */
  double scale;   /* checker cell size / noise frequency */
  rt_vec3 color;  /* solid colour */
} rt_texture_desc;

/* Perlin gradient + permutation tables (PerlinNoise.hpp:19-33, 150-160). */
#define RT_PERLIN_POINTS 256
typedef struct rt_perlin_desc {
  rt_vec3 rand_vec[RT_PERLIN_POINTS];
  int32_t perm_x[RT_PERLIN_POINTS];
  int32_t perm_y[RT_PERLIN_POINTS];
  int32_t perm_z[RT_PERLIN_POINTS];
} rt_perlin_desc;

/* ---- materials (Material.hpp:11-46) ------------------------------------- */
enum {
  RT_MAT_LAMBERTIAN = 0,    /* LambertianMaterial.cpp:15-59   */
  RT_MAT_METAL = 1,         /* MetalMaterial.cpp:43-62        */
  RT_MAT_DIELECTRIC = 2,    /* DielectricMaterial.cpp:58-85   */
  RT_MAT_DIFFUSE_LIGHT = 3, /* DiffuseLightMaterial.cpp:12-22 */
  RT_MAT_ISOTROPIC = 4      /* IsotropicMaterial.cpp:12-31    */
};

typedef struct rt_material_desc {
  int32_t kind;
  int32_t texture;         /* lambertian / diffuse_light / isotropic */
  rt_vec3 albedo;          /* metal */
  double fuzz;             /* metal */
  double refraction_index; /* dielectric */
} rt_material_desc;

/* ---- hittables (Hittable.hpp:12-50) -------------------------------------- */
enum {
  RT_OBJ_SPHERE = 0,    /* Sphere (static / moving)   Sphere.cpp:8-28, 101-178 */
  RT_OBJ_QUAD = 1,      /* Plane == parallelogram     Plane.cpp:6-132          */
  RT_OBJ_LIST = 2,      /* HittableList               HittableList.cpp:26-63   */
  RT_OBJ_ROTATE_Y = 3,  /* RotateY                    RotateY.cpp:5-103        */
  RT_OBJ_TRANSLATE = 4, /* Translate                  Translate.cpp:7-39       */
  RT_OBJ_MEDIUM = 5     /* ConstantMedium             ConstantMedium.cpp:25-94 */
};

#define RT_STORED_FORM 2

typedef struct rt_object_desc {
  int32_t kind;
  int32_t material; /* sphere / quad: material index, -1 = none (light-list entries) */
  int32_t child;    /* rotate_y / translate / medium: object index of the wrapped object;
                       list: first index into rt_scene_desc.children */
  int32_t count;    /* list: number of children */
  rt_vec3 a;        /* sphere: centre (t=0);  quad: corner Q;  translate: offset */
  rt_vec3 b;        /* sphere: centre at t=1 (moving only);  quad: side u */
  rt_vec3 c;        /* quad: side v */
  double s;         /* sphere: radius;  rotate_y: angle in degrees;  medium: density */
  int32_t moving;   /* sphere: 0 static; 1 = two-centre constructor, b = centre at t=1
                       (Sphere.cpp:15-23); RT_STORED_FORM = b is the stored displacement
                       c1 - c0 (Sphere::get_center().direction()).
                       rotate_y: RT_STORED_FORM = (a.x, a.y) are the stored (sin, cos)
                       (RotateY.hpp m_sin_theta/m_cos_theta) instead of s degrees.
                       The stored forms let a binding hand over the reference objects'
                       own doubles without a lossy round trip. */
  int32_t phase;    /* medium: material index of the phase function (isotropic) */
} rt_object_desc;

typedef struct rt_scene_desc {
  const rt_texture_desc *textures;
  int32_t n_textures;
  int32_t n_perlin;
  const rt_perlin_desc *perlin;
  const rt_material_desc *materials;
  int32_t n_materials;
  int32_t n_objects;
  const rt_object_desc *objects;
  const int32_t *children; /* list child tables */
  int32_t n_children;
  int32_t world;   /* object index of the world list (main.cpp:142 `HittableList world`) */
  int32_t lights;  /* object index of the lights list, -1 = no lights */
  int32_t use_bvh; /* reference -b: lights become HittableList(BVHNode(lights))
                      (StaticCamera.cpp:35-40); the world is always traversed through
                      the library's own BVH (closest hit is structure independent) */
  int32_t bvh_builder; /* RT_BVH_AUTO (0): device binned SAH from 65536 world
                          primitives, host SAH below; RT_BVH_HOST; RT_BVH_DEVICE
                          (linear BVH); RT_BVH_DEVICE_SAH */
  int32_t bvh_arity;   /* world BVH node width: 0 = auto (4 from 4096 world
                          primitives, else 2), 2, or 4 (the binary tree collapsed
                          to 4-wide nodes) */
} rt_scene_desc;

enum {
  RT_BVH_AUTO = 0,
  RT_BVH_HOST = 1,  /* binned SAH on the host (rt_scene.cpp) */
  RT_BVH_DEVICE = 2, /* linear BVH on the GPU (rt_bvh_build.hip) */
  RT_BVH_DEVICE_SAH = 3 /* binned SAH on the GPU, level by level (rt_bvh_sah.hip) */
};

/* ---- camera (CameraConfig.hpp:9-35) ------------------------------------- */
typedef struct rt_camera_desc {
  int32_t image_width;
  int32_t samples_per_pixel;
  int32_t max_depth;
  int32_t _pad0;
  double aspect_ratio;
  double vfov;
  double defocus_angle;
  double focus_dist;
  rt_vec3 lookfrom;
  rt_vec3 lookat;
  rt_vec3 vup;
  rt_vec3 background;
} rt_camera_desc;

/* The camera frame Camera::initialize derives (Camera.hpp:110-141 members);
   exactly the arguments cuda_static_render_wrapper takes. */
typedef struct rt_frame {
  int32_t image_width;
  int32_t image_height;
  int32_t sqrt_spp; /* int(sqrt(samples_per_pixel)) (StaticCamera.cpp:74-76) */
  int32_t max_depth;
  rt_vec3 center;
  rt_vec3 pixel00_loc;
  rt_vec3 pixel_delta_u;
  rt_vec3 pixel_delta_v;
  rt_vec3 u, v, w;
  rt_vec3 defocus_disk_u;
  rt_vec3 defocus_disk_v;
  double defocus_angle;
  double pixel_samples_scale; /* 1/samples_per_pixel (Camera.cpp:35) */
  rt_vec3 background;
} rt_frame;

/* ---- render ---------------------------------------------------------------- */
enum {
  RT_OUT_SCALED = 0, /* out = pixel_samples_scale * sum (StaticCamera.cpp:98) */
  RT_OUT_SUM = 1     /* out = raw sum over the launched samples */
};

enum {
  RT_LAYOUT_FRAME = 0,
  RT_LAYOUT_TILES = 1
};

typedef struct rt_render_params {
  int32_t row_begin;    /* first image row (inclusive) — StaticCamera.cpp:235 batches */
  int32_t row_end;      /* last row (exclusive); 0,0 = whole image */
  int32_t sample_begin; /* first linear stratum index s_j*sqrt_spp+s_i */
  int32_t sample_count; /* number of strata; -1 = all sqrt_spp^2 */
  uint64_t seed;        /* RNG key; replaces curand_init(time(nullptr)+pixel) */
  int32_t output;       /* RT_OUT_SCALED / RT_OUT_SUM */
  int32_t accumulate;   /* rt_render_device only: 1 = add into the buffer, 0 = overwrite */
  /* Tile subset (multi-GPU tile sharding): the 8x8 tiles of the row range, in
     row-major tile order, are rendered for t = tile_first + k*tile_stride only.
     tile_stride 0 or 1 with tile_first 0 = every tile. */
  int32_t tile_first;
  int32_t tile_stride;
  int32_t layout;       /* RT_LAYOUT_FRAME: row-major pixels (index (j-row_begin)*W+i);
                           RT_LAYOUT_TILES: the k-th rendered tile's 64 pixels at
                           [k*64, k*64+64), pixel (x,y) of the tile at k*64 + y*8 + x
                           (slots outside the image hold 0) */
  int32_t strata_chunks; /* RT_LAYOUT_TILES only: split each tile's strata into this
                            many equal consecutive chunks, each traced by its own
                            wavefront (finer work units for small tile subsets);
                            the output becomes [tile k][chunk c][64 px][3], whose
                            chunk sums are the tile's sums.  0 or 1 = one chunk.
                            RT_CHUNKS_AUTO (rt_render_device only, with RT_OUT_SUM
                            and accumulate 0): the library splits the subset into
                            work units sized to the device (a head/tail plan: the
                            last tiles in finer chunks, taken last) and returns
                            the per-tile sums [tile k][64 px][3], the chunk
                            partials added on the device in chunk order on the
                            same stream. */
} rt_render_params;
#define RT_CHUNKS_AUTO (-1)

/* Per-launch traversal/shading counters (for algorithmic-bytes accounting). */
typedef struct rt_path_stats {
  uint64_t samples;        /* camera samples traced */
  uint64_t segments;       /* ray segments (world traversals) */
  uint64_t node_visits;    /* BVH node fetches */
  uint64_t sphere_tests;   /* ray-sphere intersection tests (world traversal) */
  uint64_t quad_tests;     /* ray-quad tests (world traversal) */
  uint64_t other_tests;    /* instance / medium / list object visits */
  uint64_t light_tests;    /* primitive tests done by light pdf_value */
  uint64_t shade_events;   /* material evaluations */
  /* SIMD efficiency: iterations summed over wavefronts (each iteration occupies
     64 lane slots; e.g. node_visits / (64 * wave_node_iters) is the fraction of
     lanes doing useful node work) */
  uint64_t wave_trips;      /* path-loop trips (one segment attempt per lane) */
  uint64_t wave_node_iters; /* traversal node-loop iterations */
  uint64_t wave_leaf_iters; /* leaf-item loop iterations */
  uint64_t wave_shade_iters; /* shading branch executions (lambertian/metal/dielectric/light) */
  /* Where a wavefront's time goes: shader cycles (s_memtime) summed over
     wavefronts, each region counted once per wave visit -- the loop overall,
     camera-ray regeneration, closest-hit queries (traversal + items + media +
     record), the media part of them, material shading, light sampling + light
     pdf, texture evaluation.  Instrumentation adds a few percent; the shares
     are what matters. */
  uint64_t cyc_loop, cyc_regen, cyc_trace, cyc_media, cyc_shade, cyc_lights;
  /* Traversal-SIMD model (summed over wavefronts): model_trace_max = the sum
     over path trips of the largest per-lane node-visit count of the trip (the
     node-loop iterations a wave needs with one walk per lane);
     model_trace_pair_max = the same with each lane's walks of two consecutive
     trips run back to back in one node loop (max over lanes of the pair's
     sum) -- what two walks per lane could at best save. */
  uint64_t model_trace_max, model_trace_pair_max;
  /* Noise-texture albedo evaluations (shading events whose texture is a
     NoiseTexture): lanes, and wavefront executions of that evaluation (their
     ratio / 64 is the evaluation's lane use). */
  uint64_t noise_evals, wave_noise_iters;
  /* Constant media with a box boundary (make_box): lanes whose boundary
     queries took the six-face slab form, and lanes of those it deferred to
     the general boundary scan (edge / corner / parallel rays within its
     margin; ABI 4). */
  uint64_t medium_box_tests, medium_box_deferred;
} rt_path_stats;

typedef struct rt_scene_info {
  int32_t n_nodes;     /* world BVH nodes */
  int32_t n_leaf_refs; /* object references in BVH leaves */
  int32_t n_spheres, n_quads, n_objects, n_light_leaves;
  int32_t bvh_depth;
  int32_t node_bytes;   /* bytes per BVH node in the device layout */
  int32_t sphere_bytes; /* bytes per sphere record */
  int32_t quad_bytes;   /* bytes per quad record */
  int64_t device_bytes; /* total device bytes of the scene */
  int32_t features;     /* kernel instance: bit0 media, bit1 transforms, bit2 lights, bit3 noise,
                           bit4 flat world, bit5 4-wide BVH */
  int32_t lds_nodes;    /* BVH nodes (BFS prefix) the kernel stages in LDS per block */
  int32_t bvh_builder;  /* the builder that made the world BVH: RT_BVH_HOST / RT_BVH_DEVICE /
                           RT_BVH_DEVICE_SAH */
  int32_t bvh_arity;    /* 2 or 4 (n_nodes, lds_nodes and node_bytes count nodes of this width) */
  int32_t stack_depth;  /* traversal stack entries per lane (1 + BVH levels; 3 per 4-wide level) */
  int32_t lds_fixed_bytes;  /* LDS per block the kernel needs before staging nodes: static
                               accumulators + traversal stacks of its 4 wavefronts */
  int32_t lds_block_budget; /* LDS per block at the kernel's occupancy target; the node prefix
                               fills what lds_fixed_bytes leaves (LDS never lowers occupancy) */
  int32_t waves_per_simd;   /* occupancy target of the kernel instance the scene selects */
  int32_t lds_nodes_persistent; /* BVH nodes staged by the persistent frame instance (one
                                   16-wave block per CU owning its 160 KB of LDS); -1: the
                                   scene's frames run one work unit per wavefront */
  int32_t lds_prims_persistent; /* 1: the persistent frame instance also stages every world
                                   item and sphere in LDS (whole tree staged and room left) */
  int32_t persistent_block_waves; /* waves per block of the persistent instance: 16 (one block
                                     per CU) or 4 (traversal stacks too deep for 16); 0: none */
  int32_t lds_perlin; /* 1: the scene's Perlin table (one noise texture source) is staged in
                         LDS by every block of the noise instances; 0: read from HBM */
  int32_t lds_node_bytes; /* bytes per BVH node as staged in LDS (DNodeL 80 / DNode4 128;
                             node_bytes is the HBM layout's, ABI 4) */
} rt_scene_info;

typedef struct rt_scene rt_scene; /* opaque, library-owned */

int rt_abi_version(void);
const char *rt_last_error(void); /* thread-local; valid until the next call */
int rt_device_count(int32_t *count);

int rt_camera_setup(const rt_camera_desc *camera, rt_frame *frame);

/* Tuning of one scene's launches, passed explicitly at creation instead of
   read from the process environment (the reference passes its configuration
   the same way, CameraConfig.hpp:9-62).  A zero-filled struct is the default
   plan of every field -- what rt_scene_create uses.  None of the fields
   changes a rendered value: the frame is the same sum of the same samples,
   only its split into work units, the LDS staging and the BVH builder's
   parameters move (work-unit splits regroup a pixel's fp64 chunk sums, so
   frames of different splits agree to rounding, not bit for bit). */
typedef struct rt_tuning {
  /* frame work units (rt_render*, rt_multi_render) */
  int32_t chunk_target;   /* uniform split: work units per wave slot; 0: 32; < 0: whole tiles only */
  int32_t head_strata;    /* head/tail plan: strata per head unit; 0: 64 up to 64 strata, else 128 */
  int32_t tail_split;     /* tail chunks per head chunk; 0: 8 */
  int32_t no_uniform_tail; /* 1: no finer last chunks in the uniform split */
  int32_t no_persistent;  /* 1: one work unit per wavefront (no persistent unit loop) */
  int32_t grid_cap;       /* persistent launches: at most this many blocks; 0: every resident one */
  double tail_tiles;      /* tail tiles per wave slot; 0: 0.25 (head/tail plan), 0.5 (after the
                             uniform split); < 0: no tail plan */
  /* LDS staging (rt_scene_create) */
  int32_t lds_nodes;      /* one-unit instances: at most this many BVH nodes; 0: the plan; < 0: none */
  int32_t lds_nodes_pc;   /* the persistent instance's node prefix, the same rule */
  int32_t no_lds_prims;   /* 1: the persistent instance stages no items / spheres */
  int32_t no_lds_perlin;  /* 1: the Perlin table stays in HBM */
  int32_t lds_cap;        /* per-block LDS cap in bytes; 0: 64 KB (tests of the stack fallback) */
  int32_t pc_waves;       /* persistent blocks: 0 auto; 4: the 4-wave form on any scene (tests) */
  /* world BVH builders */
  int32_t sah_stack_budget; /* device SAH: depth of the balanced-split switch; 0: RT_STACK_DEPTH-2 */
  int32_t lbvh_max_depth;   /* device trees deeper than this fall back to the host SAH; 0: RT_STACK_DEPTH-1 */
  int32_t sah_leaf_max, sah_leaf_split; /* host SAH leaf rules; 0: the builder's defaults */
  int32_t sah_trav_x4, sah_bins;        /* host SAH traversal cost x4, bins; 0: 4, 16 */
  int32_t extra_features;   /* RT_FEAT_* bits OR'ed into the kernel instance key (debug) */
  /* tile-subset work units (rt_render_device, strata_chunks = RT_CHUNKS_AUTO);
     subsets of more than 4 tiles per wave slot take the frame plan above */
  int32_t sub_head_strata;   /* strata per head unit; 0: 16 x sqrt(strata / 64) */
  int32_t sub_tail_split;    /* tail chunks per head chunk; 0: 2 */
  int32_t sub_tail_permille; /* tail tiles per 1000 wave slots; 0: 125; < 0: none */
  int32_t no_tile_order;     /* 1: launches take their tiles in plan order (default: a probe launch
                                measures the tile costs once per launch shape and the launches of
                                the shape take them most expensive first; the frames are the
                                same bit for bit) */
  int32_t probe_strata;      /* strata per pixel of the probe launch that measures a launch shape's
                                tile costs for its dispatch order, once per shape; 0: 16 */
  int32_t reserved[2];
} rt_tuning;

int rt_scene_create(const rt_scene_desc *desc, int32_t device, rt_scene **scene);
/* rt_scene_create with explicit tuning (NULL: the default, as rt_scene_create) */
int rt_scene_create_tuned(const rt_scene_desc *desc, int32_t device, const rt_tuning *tuning,
                          rt_scene **scene);
int rt_scene_info_get(const rt_scene *scene, rt_scene_info *info);
/* Waits for the scene's own pending work (rt_render_device launches on any
   caller stream included), then releases it; NULL is a no-op. */
int rt_scene_destroy(rt_scene *scene);

/* Render rows [row_begin,row_end) x strata [sample_begin, +sample_count) and
   copy to host_rgb (row-major, 3 doubles per pixel, index (j-row_begin)*W+i).
   Synchronous, like the reference's per-batch loop. */
int rt_render(rt_scene *scene, const rt_frame *frame, const rt_render_params *params,
              double *host_rgb);

/* Same work, asynchronously on `hip_stream` (NULL = the HIP null stream, so work
   is ordered with a framework's default stream, e.g. torch's),
   writing/accumulating into a device buffer of W*(row_end-row_begin)*3 doubles. */
int rt_render_device(rt_scene *scene, const rt_frame *frame,
                     const rt_render_params *params, double *device_rgb,
                     void *hip_stream);

/* SAH cost of the world BVH, relative to the root box: 1 (the root) + the sum
   over every node's two children of area(child) / area(root) x (leaf: its item
   count; inner: 1) -- the tree-quality figure of the reference's builder
   (BVHNode.cpp:215-254, unit traversal and intersection costs).  0 for a flat
   world.  Always the BINARY tree the builder made (for a 4-wide scene, the
   tree before the collapse, costed at creation); otherwise copies the nodes
   back from the device. */
int rt_scene_bvh_cost(const rt_scene *scene, double *cost);

/* Run the counter-instrumented kernel variant (untimed) and return totals. */
int rt_render_stats(rt_scene *scene, const rt_frame *frame,
                    const rt_render_params *params, rt_path_stats *stats);

/* Device time of the last render kernel launched on this scene, measured with
   HIP events recorded on the launch stream around the kernel (ms). */
int rt_last_kernel_ms(rt_scene *scene, double *ms);

/* Quantise a device radiance buffer to 8-bit RGB on the device with the
   reference's write_color rule (ColorUtility.hpp:11-36). */
int rt_to_bytes_device(const double *device_rgb, int64_t n_pixels, double scale,
                       uint8_t *device_bytes, void *hip_stream);

/* ---- tile exchange (multi-GPU tile sharding) ------------------------------ */
/* Tile-layout chunk partials [tile][chunk][64][3] (rt_render_device with
   RT_LAYOUT_TILES and strata_chunks = chunks) -> per-tile sums [tile][64][3],
   each added in chunk order on the device.  parts and device_tiles must not
   overlap (unless chunks == 1). */
int rt_tiles_sum_device(const double *device_parts, int64_t n_tiles, int32_t chunks,
                        double *device_tiles, void *hip_stream);

/* Compact tiles of n_shards tile shards -> frame rows on the device: tile t of
   the row range [params->row_begin, row_end) in row-major tile order (shard
   t % n_shards rendered it as its local tile t / n_shards) is read from
   device_tiles[(t % n_shards) * shard_stride + t / n_shards][64][3] and
   written to device_rgb (index (j-row_begin)*W+i), scaled by
   pixel_samples_scale when params->output is RT_OUT_SCALED, added when
   params->accumulate.  shard_stride (tiles) >= ceil(tiles / n_shards): the
   padded per-shard slot of a gather (RCCL gather into [shard][stride]). */
int rt_tiles_to_frame_device(const double *device_tiles, int32_t n_shards, int64_t shard_stride,
                             const rt_frame *frame, const rt_render_params *params,
                             double *device_rgb, void *hip_stream);

/* ---- multi-device rendering (tile shards) -------------------------------- */
typedef struct rt_multi rt_multi; /* opaque: one rt_scene per shard */

/* One scene per shard, shard k on devices[k % n_devices] (n_shards may exceed
   n_devices: virtual shards share a device; at most RT_MULTI_MAX_SHARDS, since
   each shard holds a device copy of the scene and a host thread).  The scenes
   are compiled and uploaded by one host thread per shard; a failure to start
   one returns RT_ERR_DEVICE (nothing is thrown across the ABI). */
#define RT_MULTI_MAX_SHARDS 256
int rt_multi_create(const rt_scene_desc *desc, const int32_t *devices, int32_t n_devices,
                    int32_t n_shards, rt_multi **multi);
/* ... every shard's scene created with `tuning` (NULL: the default) */
int rt_multi_create_tuned(const rt_scene_desc *desc, const int32_t *devices, int32_t n_devices,
                          int32_t n_shards, const rt_tuning *tuning, rt_multi **multi);

/* rt_render over the shards: shard k renders the 8x8 tiles t = k (mod
   n_shards) of the row range, all launched strata, in (tile, stratum chunk)
   work units, on its own host thread, and adds each of its pixels' chunk
   partials in chunk order on its device; the compact tiles are copied device
   to device (xGMI peer copies) to shard 0's device, reordered into the frame
   there (rt_tiles_to_frame_device's kernel) and copied to host_rgb once.  params->tile_first/tile_stride/
   layout must be 0/0-or-1/RT_LAYOUT_FRAME; params->strata_chunks 0 = the chunk
   split rt_render's frame launch uses on shard 0's device, which makes the
   output bit-identical to rt_render on one device.  Synchronous. */
int rt_multi_render(rt_multi *multi, const rt_frame *frame, const rt_render_params *params,
                    double *host_rgb);

/* Device time (ms) of each shard's last render kernel (HIP events on its
   launch stream); ms must hold n_shards doubles (0 for a shard with no tiles). */
int rt_multi_shard_ms(rt_multi *multi, double *ms);

/* Host time (ms) of the last rt_multi_render's exchange: from the slowest
   shard's render completion to the frame assembled on shard 0's device (the
   peer copies and the reorder; the final D2H copy excluded). */
int rt_multi_gather_ms(rt_multi *multi, double *ms);

int rt_multi_destroy(rt_multi *multi);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
