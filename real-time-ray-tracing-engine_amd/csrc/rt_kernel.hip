// rt_kernel.hip — gfx950 path-tracing megakernel (the hot path).
//
// Replaces static_render_kernel + ray_color_cuda + init_rand_states
// (CameraKernels.cu:15-25, 106-202, 240-278).  Same estimator as the reference CPU
// integrator (Camera.cpp:232-309), restructured for CDNA4:
//
//  * one 64-lane wavefront owns one 8x8-pixel tile; its work queue is the
//    tile's 64 pixels x the launched strata; lanes that finish a path pull the
//    next (pixel, stratum) item with __ballot + mbcnt ("path regeneration"), so
//    the wave stays full until the tile's queue drains instead of idling lanes
//    whose pixels finished early (sky pixels vs multi-bounce pixels);
//  * the recursive integrator becomes an iterative bounce loop carrying a
//    throughput; every lane traces exactly one segment per loop trip;
//  * stateless Philox4x32-10 random numbers keyed by (seed; pixel, stratum,
//    bounce, slot) — no per-pixel curandState traffic (48 B/pixel/sample in the
//    reference) and sample ranges shard across GPUs exactly;
//  * BVH traversal (rt_path.h) with both child boxes per node, near-first
//    while-while order and a per-lane stack in LDS (stack[depth][lane]:
//    consecutive lanes on consecutive banks);
//  * per-pixel fp64 sums in LDS (ds_add_f64), written once per tile with
//    coalesced stores;
//  * scene-feature specialisation: the launcher picks the instance compiled for
//    the features the scene uses (media, transform chains, light sampling,
//    Perlin noise), so e.g. a sphere-only scene runs without the fog and
//    light-sampling code and its register cost.
// All arithmetic is fp64 like the reference (Vec3.hpp:184); built with
// -ffp-contract=off so expression rounding follows the reference's order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <array>
#include <mutex>
#include <set>
#include <utility>

#include "rt_path.h"

namespace {

using namespace rtp;
// Idle lanes that trigger a refill while other lanes still trace (measured:
// 16 for the plain instance, C3 +4 %; the rich instances lose with any delay).
#define RT_REGEN_MIN(F) ((F) == F_FLAT ? 16 : (((F) & ~F_BVH4) == 0 ? 16 : 1))
constexpr int kWaves = 4; // waves (work units) per block
// Flat instances (no BVH, nothing staged in LDS) run one-wave blocks: a
// block's wave slots are released only when all of its waves have ended, so
// with 4-wave blocks a slot idles until the slowest unit of its block is done
// (measured: C2 +2.0 %, C4 +10.4 % over 4-wave blocks; 2-wave blocks +0.5 % /
// +6.3 %; profiles/r03g_ab.log).  BVH instances keep 4-wave blocks: their
// waves share the block's staged BVH prefix.
constexpr int block_waves(unsigned f) { return (f & F_FLAT) ? 1 : kWaves; }
// Waves per block of the persistent instance: one block per CU (16 = 4 SIMDs x
// its 4-waves/SIMD target), so the CU's 160 KB of LDS holds ONE copy of the
// staged BVH beside its 16 waves' stacks instead of four copies for four
// 4-wave blocks (gfx950: a workgroup may own all 160 KB).
constexpr int kPcWaves = RT_PC_WAVES; // rt_layout.h
// the persistent instance also stages the world items and spheres when they fit
constexpr size_t kLdsPerCu = 160 * 1024;

// Occupancy target per instance (waves per SIMD): the compiler may spill a few
// registers to reach it.  Measured: 4 for the plain instance (C3
// +12 % over 3), 3 for the rich ones (C4 +8.6 % over the 2 that 224 VGPRs give).
#define RT_WAVES_PER_EU(F) ((F) == F_FLAT ? 4 : (((F) & ~F_BVH4) == 0 ? 4 : 3))
// Feature sets with a persistent chunked-frame instance (render_tiles<.., PC>,
// whose waves pull work units from a counter): the plain BVH walks (C3 +3.4 %,
// profiles/r02ab-af_*); the flat and the rich instances keep one unit per wave
// -- the unit loop's extra live state cost them 2-20 %.
#define RT_PERSIST_F(F) (((F) & ~F_BVH4) == 0)

// The launch fields read afresh from the kernarg segment at each work unit
// (FRESH, the persistent instances): the asm hides the segment pointer's
// value, so the loads stay inside the unit loop instead of being hoisted out
// of it and held in SGPRs across every path trip.  KArgs mirrors
// render_tiles' explicit arguments (laid out in order, naturally aligned);
// the parameter's own address is never taken (that copies it to scratch).
struct KArgs {
  DScene S;
  DCamera C;
  DLaunch P;
  double *out;
  unsigned long long *stats;
};
// The AMDGPU kernarg segment places explicit arguments in order at their
// natural alignment -- the layout of this struct.  The expected offsets are
// spelled out so a field added to DScene / DCamera / DLaunch breaks the build
// here instead of silently shifting what the persistent instance reads (its
// frames are also checked bit for bit against the one-unit-per-wave instance
// on the GPU: tests/test_persistent.py, and through every BASELINE band).
static_assert(sizeof(DScene) == 160 && alignof(DScene) == 8, "DScene kernarg layout");
static_assert(sizeof(DCamera) == 208 && alignof(DCamera) == 8, "DCamera kernarg layout");
static_assert(sizeof(DLaunch) == 112 && alignof(DLaunch) == 8, "DLaunch kernarg layout");
static_assert(offsetof(KArgs, S) == 0 && offsetof(KArgs, C) == 160 && offsetof(KArgs, P) == 368 &&
                  offsetof(KArgs, out) == 480 && offsetof(KArgs, stats) == 488 &&
                  sizeof(KArgs) == 496,
              "KArgs must mirror render_tiles' kernarg layout");
static_assert(offsetof(DLaunch, n_chunks) == 56 && offsetof(DLaunch, unit_ctr) == 64 &&
                  offsetof(DLaunch, grid_cap) == 72 && offsetof(DLaunch, n_head) == 76 &&
                  offsetof(DLaunch, parts) == 80 && offsetof(DLaunch, parts_final) == 88 &&
                  offsetof(DLaunch, head_chunks) == 92 && offsetof(DLaunch, tile_order) == 96 &&
                  offsetof(DLaunch, tile_cost) == 104,
              "DLaunch field offsets read from the kernarg segment");
template <bool FRESH>
__device__ __forceinline__ DLaunch launch_fields(const DLaunch &P) {
  if constexpr (FRESH) {
    auto ka = (const __attribute__((address_space(4))) KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const __attribute__((address_space(4))) DLaunch &K = ka->P;
    DLaunch L;
    L.row_begin = K.row_begin;
    L.row_end = K.row_end;
    L.sample_begin = K.sample_begin;
    L.sample_count = K.sample_count;
    L.seed_lo = K.seed_lo;
    L.seed_hi = K.seed_hi;
    L.output = K.output;
    L.accumulate = K.accumulate;
    L.tiles_x = K.tiles_x;
    L.tiles_y = K.tiles_y;
    L.tile_first = K.tile_first;
    L.tile_stride = K.tile_stride;
    L.n_local_tiles = K.n_local_tiles;
    L.compact = K.compact;
    L.n_chunks = K.n_chunks;
    L.chunk_strata = K.chunk_strata;
    L.unit_ctr = K.unit_ctr;
    L.grid_cap = K.grid_cap;
    L.n_head = K.n_head;
    L.parts = K.parts;
    L.parts_final = K.parts_final;
    L.head_chunks = K.head_chunks;
    L.tile_order = K.tile_order;
    L.tile_cost = K.tile_cost;
    return L;
  } else {
    return P;
  }
}
// The epilogue's camera fields read afresh from the kernarg segment (FRESH:
// once per work unit, outside the path loop, so the one-unit instances need
// not hold them in SGPRs across every path trip).  Scalar loads through the
// asm-hidden segment pointer: they stay at the use, the scalar cache serves them.
// non-flat instances only: the flat one measured -0.5 % kernel time with it
// (C2; C4 neutral); profiles/r03l_ab.log
#define RT_EPI_FRESH_F(F) (((F) & F_FLAT) == 0)
template <bool FRESH>
__device__ __forceinline__ DCamera camera_fields(const DCamera &C) {
  if constexpr (FRESH) {
    auto ka = (const __attribute__((address_space(4))) KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const __attribute__((address_space(4))) DCamera &K = ka->C;
    DCamera D;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      D.center[k] = K.center[k];
      D.p00[k] = K.p00[k];
      D.du[k] = K.du[k];
      D.dv[k] = K.dv[k];
      D.disk_u[k] = K.disk_u[k];
      D.disk_v[k] = K.disk_v[k];
      D.bg[k] = K.bg[k];
    }
    D.defocus_angle = K.defocus_angle;
    D.scale = K.scale;
    D.rs = K.rs;
    D.W = K.W;
    D.H = K.H;
    D.sqrt_spp = K.sqrt_spp;
    D.max_depth = K.max_depth;
    return D;
  } else {
    return C;
  }
}
// The plan's local tile of work unit `unit` (head units: unit / head_chunks;
// tail units: n_head + (unit - head units) / n_chunks), and the launch's
// local tile it maps to (cost-ordered dispatch: tile_order; null: itself).
__device__ __forceinline__ int plan_tile(const DLaunch &L, int unit) {
  const int head_units = L.n_head * L.head_chunks;
  return unit < head_units ? unit / L.head_chunks : L.n_head + (unit - head_units) / L.n_chunks;
}
__device__ __forceinline__ int order_tile(const DLaunch &L, int k) {
  return L.tile_order != nullptr ? __builtin_amdgcn_readfirstlane(L.tile_order[k]) : k;
}
// Cost-ordered dispatch (rt_api.cpp "tile order"): every instance maps its
// units through the launch's tile order (a scalar load per unit); the STATS
// instance measures tile costs, in the probe launch that orders a launch
// shape once (rt_api.cpp tile_order_probe).  The cost bookkeeping compiled
// into a render instance cost it registers and schedule even when skipped at
// run time: C4 -12.5 % (r05u_ab.log), C2 / C3 / C5 -0.9 % (r06y_ab_C*.log);
// so it lives in one extra instance (COST) of the flat world only, for the
// tile-subset launches of a multi-GPU rank, whose order re-measured after
// every launch beats the probe's (r06ad / r06af: 8-way C2 share).
// rtk_cost_f mirrors it for the host.
#define RT_COST_F(F) ((F) == F_FLAT)
extern "C" int rtk_cost_f(int features) { return RT_COST_F((unsigned)features) ? 1 : 0; }
template <bool FRESH>
__device__ __forceinline__ double *out_arg(double *out) {
  if constexpr (FRESH) {
    auto ka = (const __attribute__((address_space(4))) KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    return ka->out;
  } else {
    return out;
  }
}

#ifndef RT_UNIT_TIMES
#define RT_UNIT_TIMES 0
#endif
#if RT_UNIT_TIMES
// Measurement-only build (make EXTRA=-DRT_UNIT_TIMES=1; tools/unit_timeline.py):
// every work unit's start and end on the device's constant 100 MHz clock
// (s_memrealtime), by unit index, for the launch timeline (how long the
// waves' last units keep the launch open).
constexpr int kUnitTimesMax = 1 << 21;
__device__ unsigned long long g_unit_times[2 * kUnitTimesMax];
extern "C" hipError_t rtk_unit_times(unsigned long long *host, int n_units) {
  const size_t n = 2 * (size_t)(n_units < kUnitTimesMax ? n_units : kUnitTimesMax);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_unit_times), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost);
}
extern "C" hipError_t rtk_unit_times_clear(void) {
  void *p = nullptr;
  hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_unit_times));
  if (e != hipSuccess) return e;
  e = hipMemset(p, 0, sizeof(g_unit_times));
  return e != hipSuccess ? e : hipDeviceSynchronize();
}
#endif

// PC (persistent): the instance for launches of more units than the grid's
// resident waves -- frame launches (head units, then the tail chunks) and
// tile-subset launches (multi-GPU shards) alike -- whose waves persist and
// pull units; it reads the per-unit launch fields afresh from the kernarg
// segment, so they are not live across the path loop.
// PCW: 0 = one work unit per wavefront; else a persistent instance with
// blocks of PCW waves (kPcWaves = one block per CU; kWaves when the traversal
// stacks of 16 waves do not fit the CU's LDS, e.g. deep 4-wide trees)
template <bool STATS, unsigned F, int PCW = 0, bool COST = false>
__global__ __launch_bounds__(64 * (PCW ? PCW : block_waves(F))) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU(F)))) void render_tiles(DScene S_, DCamera C, DLaunch P, double *out,
                                                    unsigned long long *stats) {
  constexpr bool PC = PCW > 0;
  constexpr int BW = PC ? PCW : block_waves(F); // waves per block
  // the persistent instance stages its own (larger) node prefix
  DScene S = S_;
  if constexpr (PC) S.n_lds_nodes = S_.n_lds_nodes_pc;
  // dynamic LDS: traversal stacks [BW][S.stack_depth][64] ints, then the
  // staged BVH prefix nodes [0, S.n_lds_nodes) (sizes: rtk_lds_bytes)
  extern __shared__ int4 dyn_lds[];
  __shared__ double acc_lds[BW][64][3];
  // compacted leaf tests (BVH instances only; 1 KB per wave)
  __shared__ LeafPool leaf_pool[RT_LEAF_SHARE_F(F) ? BW : 1];

  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  int *stack_base = reinterpret_cast<int *>(dyn_lds);
  DNode *lnodes_g = reinterpret_cast<DNode *>(stack_base + BW * S.stack_depth * 64);
  const RT_LDS DNode *lnodes = (const RT_LDS DNode *)lnodes_g; // DNode4 in BVH4 instances
  constexpr int kNodeBytes = RT_LDS_NODE_BYTES(F);
  // persistent instance: world items and spheres after the nodes (LdsPrims)
  LdsPrims lp{nullptr, nullptr};
  int4 *prim_g = reinterpret_cast<int4 *>(lnodes_g) + (size_t)max(0, S.n_lds_nodes) * (kNodeBytes / 16);
  if constexpr (PC) {
    if (S.lds_items_pc > 0) {
      lp.items = (const RT_LDS DItem *)reinterpret_cast<DItem *>(prim_g);
      lp.spheres = (const RT_LDS DSphere *)reinterpret_cast<DSphere *>(prim_g + (size_t)S.lds_items_pc * 2);
    }
  }
  if (S.n_lds_nodes > 0 || (PC && S.lds_items_pc > 0)) { // stage once per block
    if constexpr ((F & F_BVH4) != 0) {
      const int4 *src = reinterpret_cast<const int4 *>(S.nodes);
      int4 *dst = reinterpret_cast<int4 *>(lnodes_g);
      const int n16 = max(0, S.n_lds_nodes) * (kNodeBytes / 16);
      for (int k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
    } else {
      // binary nodes as DNodeL: 8-B unit j of staged node i is, per axis a =
      // j / 3, the lo pair (8a in the DNode), the hi pair (24 + 8a), the lo pair
      // again; unit 9 the child entries (48) -- inner children as DNodeL byte
      // offsets when the whole tree is staged (the LDS-only walk's `cur`)
      const uint2 *src = reinterpret_cast<const uint2 *>(S.nodes);
      uint2 *dst = reinterpret_cast<uint2 *>(lnodes_g);
      const int n8 = max(0, S.n_lds_nodes) * 10;
      const bool whole = S.n_lds_nodes >= S.n_nodes; // trace()'s LDS-only walk
      for (int k = threadIdx.x; k < n8; k += blockDim.x) {
        const int i = k / 10, j = k - 10 * (k / 10);
        const int a = j / 3, m = j - 3 * (j / 3);
        const int u = j == 9 ? 6 : (m == 1 ? 3 + a : a);
        uint2 v = src[8 * i + u];
        if (j == 9 && whole) {
          if ((int)v.x >= 0) v.x *= (unsigned)sizeof(DNodeL);
          if ((int)v.y >= 0) v.y *= (unsigned)sizeof(DNodeL);
        }
        dst[k] = v;
      }
    }
    if constexpr (PC) {
      if (S.lds_items_pc > 0) {
        const int ni = S.lds_items_pc * 2, ns = S.lds_spheres_pc * 4; // int4 per DItem / DSphere
        const int4 *si = reinterpret_cast<const int4 *>(S.items);
        const int4 *ss = reinterpret_cast<const int4 *>(S.spheres);
        for (int k = threadIdx.x; k < ni; k += blockDim.x) prim_g[k] = si[k];
        for (int k = threadIdx.x; k < ns; k += blockDim.x) prim_g[ni + k] = ss[k];
      }
    }
    __syncthreads();
  }
  if constexpr ((F & F_NOISE) != 0) { // the Perlin table (tex_value), once per block
    if (S.lds_perlin) {
      const int4 *src = reinterpret_cast<const int4 *>(S.perlin);
      RT_LDS int4 *dst = (RT_LDS int4 *)perlin_lds();
      for (int k = threadIdx.x; k < (int)(sizeof(DPerlin) / 16); k += blockDim.x) dst[k] = src[k];
      __syncthreads();
    }
  }
  // work unit = (local tile, stratum chunk).  Persistent launches (P.unit_ctr
  // set, grid = the resident waves): a wave's first unit is its static slot,
  // the next ones come from the agent-scope counter (initialised by the host to
  // the grid's wave count), so waves take new units as they finish instead of
  // waiting for their block.
  const int n_units = P.n_head * P.head_chunks + (P.n_local_tiles - P.n_head) * P.n_chunks;
  int unit = blockIdx.x * BW + wv;
  int *stk = stack_base + wv * S.stack_depth * 64 + lane;
  double *acc = &acc_lds[wv][0][0];
  Counters cnt{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t cyc_regen = 0;
  const uint64_t t_start = STATS ? clk() : 0;
  uint32_t n_samples = 0, n_segments = 0, n_trips = 0;
  // traversal-SIMD model (STATS): per trip the largest per-lane visit count,
  // and for trips paired back to back the largest per-lane sum of the pair
  uint64_t m_single = 0, m_pair = 0;
  uint32_t v_prev = 0, m_prev = 0;
  bool have_prev = false;
  auto wave_max = [](uint32_t x) {
    for (int off = 32; off > 0; off >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, off));
    return x;
  };
  while (unit < n_units) { // wave-uniform
#if RT_UNIT_TIMES
  const unsigned long long t_unit0 = __builtin_amdgcn_s_memrealtime();
#endif
  const DLaunch PU = launch_fields<PC>(P);
  // (wave-uniform) head unit: tile unit / head_chunks; tail unit: a chunk of
  // the tail tile n_head + (unit - head units) / n_chunks
  const int head_units = PU.n_head * PU.head_chunks;
  const bool whole = PU.head_chunks == 1 && unit < PU.n_head;
  int local_tile, s_first, s_count;
  {
    const bool head = unit < head_units;
    const int nc = head ? PU.head_chunks : PU.n_chunks;
    const int cs = head ? (PU.sample_count + nc - 1) / nc : PU.chunk_strata;
    const int u = head ? unit : unit - head_units, q = u / nc, chunk = u - q * nc;
    local_tile = head ? q : PU.n_head + q;
    s_first = PU.sample_begin + chunk * cs;
    s_count = min(cs, PU.sample_count - chunk * cs);
  }
  // the plan's k-th tile -> the launch's local tile (cost-ordered dispatch);
  // in the probe (STATS) and the COST instance the unit's cost is its end time
  // minus its start time, both added to the tile's counter (mod 2^32), so no
  // start time is held across the path loop
  local_tile = order_tile(PU, local_tile);
  if constexpr (STATS || COST) {
    if (lane == 0 && PU.tile_cost != nullptr)
      atomicSub(&PU.tile_cost[local_tile], (unsigned)__builtin_amdgcn_s_memrealtime());
  }
  const int tile = PU.tile_first + local_tile * PU.tile_stride;
  const int tx = tile % PU.tiles_x, ty = tile / PU.tiles_x;
  const int x0 = tx * 8, y0 = PU.row_begin + ty * 8;
  acc[lane * 3 + 0] = 0.0;
  acc[lane * 3 + 1] = 0.0;
  acc[lane * 3 + 2] = 0.0;

  const int n_items = 64 * max(0, s_count);
  int next_item = 0; // wave-uniform head of the tile's work queue
  PathState ps;
  ps.active = false;
  Key key{P.seed_lo, P.seed_hi, 0, 0};

  for (;;) {
    // ---- regeneration: idle lanes pull the next (pixel, stratum) items
    const uint64_t t_regen = STATS ? clk() : 0;
    for (;;) {
      unsigned long long idle = __ballot(!ps.active);
      if (idle == 0 || next_item >= n_items) break;
      // refill only once enough lanes are idle: camera-ray generation costs the
      // whole wave, however few lanes take new paths
      if (__popcll(idle) < RT_REGEN_MIN(F) && ~idle != 0ull) break;
      int rank = __popcll(idle & ((1ull << lane) - 1ull));
      int item = next_item + rank;
      next_item += __popcll(idle);
      if (!ps.active && item < n_items) {
        const DCamera &Cr = C;
        int slot = item & 63;
        int i = x0 + (slot & 7), j = y0 + (slot >> 3);
        if (i < Cr.W && j < P.row_end) {
          ps.slot = slot;
          ps.sample = s_first + (item >> 6);
          key.pixel = (uint32_t)(j * Cr.W + i);
          key.sample = (uint32_t)ps.sample;
          ps.ray = camera_ray<RT_KB_F(F), RT_KCONST_MODE(F)>(Cr, key, i, j, ps.sample);
          ps.T = v3(1.0, 1.0, 1.0);
          ps.bounce = 0;
          ps.active = Cr.max_depth > 0;
          if (STATS) n_samples++;
        }
      }
    }
    if (STATS) cyc_regen += clk() - t_regen; // converged here (every lane)
    if (__ballot(ps.active) == 0) break;
    if (STATS) n_trips++; // converged here: every lane counts, lane 0 reports
    uint32_t v_trace = 0;
    if (ps.active) {
      if (STATS) n_segments++;
      const uint32_t nv0 = cnt.nodes;
      bool cont = segment<STATS, F, PC>(
          S, C, ps, key, stk, lnodes, cnt, (RT_LDS LeafPool *)&leaf_pool[RT_LEAF_SHARE_F(F) ? wv : 0], lp);
      if (STATS) v_trace = cnt.nodes - nv0;
      if (!cont) {
        atomicAdd(&acc[ps.slot * 3 + 0], ps.T.x);
        atomicAdd(&acc[ps.slot * 3 + 1], ps.T.y);
        atomicAdd(&acc[ps.slot * 3 + 2], ps.T.z);
        ps.active = false;
      }
    }
    if (STATS) { // converged: every lane
      const uint32_t m1 = wave_max(v_trace);
      m_single += m1;
      if (!have_prev) {
        v_prev = v_trace;
        m_prev = m1;
      } else {
        m_pair += wave_max(v_prev + v_trace);
      }
      have_prev = !have_prev;
    }
  }
  if (STATS && have_prev) {
    m_pair += m_prev;
    have_prev = false;
  }
  __builtin_amdgcn_wave_barrier();

  // ---- tile epilogue: one coalesced store per pixel
  {
    // the epilogue's launch fields, camera width / scale and output pointer
    // read afresh (RT_EPI_FRESH_F): once per unit, outside the path loop, so the
    // one-unit instances need not hold them in SGPRs across every path trip
    constexpr bool kEpiFresh = RT_EPI_FRESH_F(F);
    const DCamera Ce = camera_fields<kEpiFresh>(C);
    const DLaunch PE = launch_fields<PC || kEpiFresh>(P);
    int i = x0 + (lane & 7), j = y0 + (lane >> 3);
    // whole units: the frame (pixels outside the image are not written) or
    // the compact tile layout; split units: their chunk's partial sums
    const bool to_parts = !whole;
    const bool compact = to_parts || PE.compact;
    if (compact || (i < Ce.W && j < PE.row_end)) { // tile slots outside the image hold 0
      double sx = acc[lane * 3 + 0], sy = acc[lane * 3 + 1], sz = acc[lane * 3 + 2];
      const bool final_out = !to_parts || PE.parts_final;
      if (final_out && PE.output == RT_OUT_SCALED) {
        sx = Ce.scale * sx;
        sy = Ce.scale * sy;
        sz = Ce.scale * sz;
      }
      double *const ob = out_arg<PC || kEpiFresh>(out);
      const int part = unit - (PE.head_chunks == 1 ? PE.n_head : 0);
      double *o = to_parts ? PE.parts + 3 * ((size_t)part * 64 + lane)
                  : PE.compact ? ob + 3 * ((size_t)order_tile(PE, unit) * 64 + lane)
                               : ob + 3 * ((size_t)(j - PE.row_begin) * Ce.W + i);
      if (final_out && PE.accumulate) {
        o[0] += sx;
        o[1] += sy;
        o[2] += sz;
      } else {
        o[0] = sx;
        o[1] = sy;
        o[2] = sz;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the unit's duration into its tile's cost (the shape's dispatch order)
  if constexpr (STATS || COST) {
    if (lane == 0) {
      const DLaunch PT = launch_fields<true>(P);
      if (PT.tile_cost != nullptr)
        atomicAdd(&PT.tile_cost[order_tile(PT, plan_tile(PT, unit))], (unsigned)__builtin_amdgcn_s_memrealtime());
    }
  }
#if RT_UNIT_TIMES
  if (lane == 0 && !STATS && unit < kUnitTimesMax) {
    g_unit_times[2 * unit] = t_unit0;
    g_unit_times[2 * unit + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if constexpr (!PC) break;
  int next = n_units;
  if (P.unit_ctr != nullptr && lane == 0)
    next = __hip_atomic_fetch_add(P.unit_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unit = P.unit_ctr != nullptr ? __builtin_amdgcn_readfirstlane(__shfl(next, 0)) : n_units;
  } // unit loop
  if (STATS) {
    const uint64_t cyc_loop = clk() - t_start;
    unsigned long long v[RT_N_STATS] = {n_samples, n_segments, cnt.nodes, cnt.spheres,
                                        cnt.quads, cnt.other,  cnt.light, cnt.shade,
                                        lane == 0 ? n_trips : 0u, cnt.wnode, cnt.wleaf, cnt.wshade,
                                        lane == 0 ? cyc_loop : 0u, lane == 0 ? cyc_regen : 0u,
                                        cnt.ctrace, cnt.cmedia, cnt.cshade, cnt.clights,
                                        lane == 0 ? m_single : 0u, lane == 0 ? m_pair : 0u,
                                        cnt.noise, cnt.wnoise, cnt.mbox, cnt.mbox_fb};
    for (int k = 0; k < RT_N_STATS; ++k) {
      unsigned long long x = v[k];
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
      if (lane == 0) atomicAdd(&stats[k], x);
    }
  }
}

// Frame assembly after a split launch (rtk_launch_render_chunked): each pixel
// of a chunked tile gets its stratum-chunk partial sums added in chunk order
// (scaled / accumulated as the launch asks) -- the head tiles' head_chunks
// partials when head_chunks > 1, the tail tiles' n_chunks partials; whole
// tiles' pixels were written by their own units.  One thread per (chunked
// tile, pixel slot, channel).
__global__ void split_sum_kernel(const double *parts, DCamera C, DLaunch P, double *out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int first = P.head_chunks > 1 ? 0 : P.n_head; // first chunked tile
  if (idx >= (int64_t)(P.n_local_tiles - first) * 64 * 3) return;
  const int ch = (int)(idx % 3);
  const int slot = (int)((idx / 3) & 63);
  const int tile = first + (int)(idx / (64 * 3)); // frame launches: tile_first 0, tile_stride 1
  const int pt = P.tile_order != nullptr ? P.tile_order[tile] : tile; // the plan's tile -> the frame's
  const int i = (pt % P.tiles_x) * 8 + (slot & 7), j = P.row_begin + (pt / P.tiles_x) * 8 + (slot >> 3);
  if (i >= C.W || j >= P.row_end) return;
  const bool head = tile < P.n_head;
  const int nc = head ? P.head_chunks : P.n_chunks;
  const int64_t part0 = head ? (int64_t)tile * nc
                             : (P.head_chunks > 1 ? (int64_t)P.n_head * P.head_chunks : 0) +
                                   (int64_t)(tile - P.n_head) * nc;
  const double *p = parts + (part0 * 64 + slot) * 3 + ch;
  double sum = p[0];
  for (int k = 1; k < nc; ++k) sum += p[(size_t)k * 64 * 3];
  if (P.output == RT_OUT_SCALED) sum = C.scale * sum;
  double *o = out + ((size_t)(j - P.row_begin) * C.W + i) * 3 + ch;
  *o = P.accumulate ? *o + sum : sum;
}

// ---- tile-shard exchange (multi-GPU: rt_multi_render, rtx/dist.py) ----
// Every kernel below adds chunk partials in chunk order (split_sum_kernel's
// order), so a sharded frame is bit-identical to the one-device frame launch.
// A tile's record is 64 pixel slots x 3 channels = 192 doubles; one thread per
// double, consecutive threads on consecutive doubles (coalesced).
constexpr int kTileD = 64 * 3;

// Tile-layout chunk partials [tile][chunk][64][3] -> tile sums [tile][64][3].
__global__ void tiles_sum_kernel(const double *parts, int64_t n_tiles, int chunks, double *out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_tiles * kTileD) return;
  const int64_t tile = idx / kTileD, r = idx - tile * kTileD;
  const double *p = parts + tile * chunks * kTileD + r;
  double sum = p[0];
  for (int c = 1; c < chunks; ++c) sum += p[(int64_t)c * kTileD];
  out[idx] = sum;
}

// One shard's compact tiles finished on its own device: its whole head tiles
// are already in out[lt]; each chunked tile's partials (the launch's parts
// layout, DLaunch) are summed in chunk order into out[lt].
__global__ void shard_finish_kernel(const double *parts, int n_local, int n_head, int head_chunks,
                                    int n_chunks, const int32_t *order, double *out) {
  const int first = head_chunks > 1 ? 0 : n_head; // first chunked local tile
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)(n_local - first) * kTileD) return;
  const int lt = first + (int)(idx / kTileD);
  const int r = (int)(idx % kTileD);
  const bool head = lt < n_head;
  const int nc = head ? head_chunks : n_chunks;
  const int64_t part0 = head ? (int64_t)lt * nc
                             : (head_chunks > 1 ? (int64_t)n_head * head_chunks : 0) + (int64_t)(lt - n_head) * nc;
  const double *p = parts + part0 * kTileD + r;
  double sum = p[0];
  for (int c = 1; c < nc; ++c) sum += p[(int64_t)c * kTileD];
  out[(int64_t)(order != nullptr ? order[lt] : lt) * kTileD + r] = sum; // the plan's tile -> the launch's
}

// Cost-ordered dispatch (rt_api.cpp "tile order"): the local tiles sorted by
// the cost the previous launch of the same shape measured (tile_cost, 100 MHz
// ticks summed over a tile's units), most expensive first -- the next launch
// dispatches them in that order (longest processing time first), so its last
// units are short ones.  Two segments, one block each: the plan's head tiles
// [0, n_head) among themselves and its tail tiles [n_head, n) among
// themselves, so every tile keeps its own unit split (whole / head chunks /
// tail chunks) and so its sums, bit for bit.  Per block: a histogram of 256
// log-spaced buckets (8 per octave), a descending scan, a scatter; ties land in
// any order (scheduling only).
__global__ void tile_order_kernel(const uint32_t *cost, int n, int n_head, int32_t *order) {
  const int lo = blockIdx.x == 0 ? 0 : n_head, hi = blockIdx.x == 0 ? n_head : n;
  if (lo >= hi) return;
  cost += lo;
  order += lo;
  n = hi - lo;
  __shared__ uint32_t hist[256];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  auto bucket = [](uint32_t c) -> int {
    if (c == 0) return 0;
    const int lz = __clz(c);
    return (31 - lz) * 8 + (int)(((c << lz) >> 28) & 7u);
  };
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) { // exclusive scan from the top bucket down
    uint32_t run = 0;
    for (int k = 255; k >= 0; --k) {
      const uint32_t c = hist[k];
      hist[k] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) order[atomicAdd(&hist[bucket(cost[i])], 1u)] = lo + i;
}

extern "C" hipError_t rtk_launch_tile_order(const uint32_t *cost, int n, int n_head, int32_t *order,
                                            hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(tile_order_kernel, dim3(2), dim3(1024), 0, stream, cost, n, n_head, order);
  return hipGetLastError();
}

// Compact tiles of n_shards shards -> frame rows [row_begin, row_end): tile t
// of the row range (row-major tile order) is local tile t / n_shards of shard
// t % n_shards, at tiles[(shard * shard_stride + local) * 192].  One thread per
// frame double: the frame writes are coalesced, the tile reads come in runs
// of 8 pixels (192 B).
__global__ void tiles_to_frame_kernel(const double *tiles, int n_shards, int64_t shard_stride, int W,
                                      int row_begin, int row_end, int tiles_x, double scale, int scaled,
                                      int accumulate, double *out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)(row_end - row_begin) * W * 3) return;
  const int ch = (int)(idx % 3);
  const int64_t pix = idx / 3;
  const int i = (int)(pix % W), jr = (int)(pix / W);
  const int t = (jr >> 3) * tiles_x + (i >> 3), slot = (jr & 7) * 8 + (i & 7);
  const int k = t % n_shards, lt = t / n_shards;
  double v = tiles[((int64_t)k * shard_stride + lt) * kTileD + slot * 3 + ch];
  if (scaled) v = scale * v;
  out[idx] = accumulate ? out[idx] + v : v;
}

__global__ void to_bytes_kernel(const double *rgb, int64_t n, double scale, uint8_t *bytes) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * n) return;
  double x = scale * rgb[i];
  double g = (x > 0) ? sqrt(x) : 0; // ColorUtility.hpp:11-26
  if (g < 0.000) g = 0.000;
  if (g > 0.999) g = 0.999;
  bytes[i] = (uint8_t)(256 * g);
}

using RenderFn = void (*)(DScene, DCamera, DLaunch, double *, unsigned long long *);

// F_BVH4 never comes with F_FLAT (a flat world has no tree): those slots reuse
// the flat instance instead of instantiating a kernel that cannot be launched
constexpr unsigned canonical(unsigned f) { return (f & F_FLAT) ? (f & ~F_BVH4) : f; }
template <bool STATS, unsigned... Fs>
constexpr std::array<RenderFn, sizeof...(Fs)> instance_table(std::integer_sequence<unsigned, Fs...>) {
  return {render_tiles<STATS, canonical(Fs)>...};
}

// the persistent instances (RT_PERSIST_F feature sets), blocks of pcw waves
RenderFn persistent_instance(unsigned f, int pcw) {
  if (pcw == kPcWaves)
    return (f & F_BVH4) ? render_tiles<false, F_BVH4, kPcWaves> : render_tiles<false, 0u, kPcWaves>;
  return (f & F_BVH4) ? render_tiles<false, F_BVH4, kWaves> : render_tiles<false, 0u, kWaves>;
}

// the cost-measuring instance (RT_COST_F: the flat world, never persistent);
// the plain BVH worlds' shares measured as well as by the probe (C3 4- / 8-way
// shares +-0.2 %, profiles/r06ai_sim_C3.log), so they have none
RenderFn cost_instance(unsigned f) { return f == F_FLAT ? render_tiles<false, F_FLAT, 0, true> : nullptr; }

// one instance per feature set (F_MEDIA | F_XFORM | F_LIGHTS | F_NOISE | F_FLAT)
const RenderFn *render_table(bool stats) {
  static constexpr auto plain = instance_table<false>(std::make_integer_sequence<unsigned, F_ALL + 1>{});
  static constexpr auto counted = instance_table<true>(std::make_integer_sequence<unsigned, F_ALL + 1>{});
  return stats ? counted.data() : plain.data();
}

} // namespace

// ---------------------------------------------------------------- launchers
extern "C" size_t rtk_lds_bytes(int features, int stack_depth, int n_lds_nodes) {
  const size_t node = RT_LDS_NODE_BYTES(features);
  return (size_t)block_waves((unsigned)features) * stack_depth * 64 * sizeof(int) +
         (size_t)n_lds_nodes * node;
}
// a persistent instance's dynamic LDS (pcw waves per block)
static size_t lds_bytes_pc(int features, int pcw, int stack_depth, int n_lds_nodes) {
  const size_t node = RT_LDS_NODE_BYTES(features);
  return (size_t)pcw * stack_depth * 64 * sizeof(int) + (size_t)n_lds_nodes * node;
}

// LDS plan per block at the occupancy the instance's register count allows
// (blocks of kWaves waves over the 4 SIMDs): the bytes left for the staged BVH
// prefix after the static LDS and the traversal stacks, and whether those two
// fit at all (the caller then keeps a shallower tree).  lds_cap > 0 lowers the
// per-block cap (rt_tuning.lds_cap: tests of that fallback).
extern "C" hipError_t rtk_lds_plan(int features, int stack_depth, int lds_cap, RtkLdsPlan *plan) {
  hipFuncAttributes a;
  hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(render_table(false)[features & F_ALL]));
  if (e != hipSuccess) return e;
  const int regs = ((a.numRegs + 7) / 8) * 8;
  int waves_per_simd = regs > 0 ? 512 / regs : 8;
  if (waves_per_simd > 8) waves_per_simd = 8;
  if (waves_per_simd < 1) waves_per_simd = 1;
  size_t lds_cu = 160 * 1024, cap = 64 * 1024; // per CU; per block without opt-in
  if (lds_cap > 0 && (size_t)lds_cap < cap) cap = (size_t)lds_cap;
  const int bw = block_waves((unsigned)features);
  const int blocks_per_cu = waves_per_simd * 4 / bw > 0 ? waves_per_simd * 4 / bw : 1;
  size_t per_block = lds_cu / blocks_per_cu;
  if (per_block > cap) per_block = cap;
  const size_t fixed = a.sharedSizeBytes + rtk_lds_bytes(features, stack_depth, 0);
  const size_t node = RT_LDS_NODE_BYTES(features);
  plan->waves_per_simd = waves_per_simd;
  plan->block_budget = (int32_t)per_block;
  plan->fixed_bytes = (int32_t)fixed;
  plan->stack_fits = fixed <= per_block;
  plan->n_nodes = per_block > fixed ? (int)((per_block - fixed) / node) : 0;
  // stacks over the share: fewer blocks per CU (the host then stages no nodes)
  const int lds_blocks = fixed > 0 ? (int)(lds_cu / fixed) : blocks_per_cu;
  plan->resident_waves_per_cu = std::min(blocks_per_cu, std::max(1, lds_blocks)) * bw;
  return hipSuccess;
}

// The persistent instance a scene uses and the LDS it has left for staging
// after its stacks and static LDS: blocks of kPcWaves waves (one per CU, which
// may own the CU's whole LDS) if their stacks fit, else blocks of kWaves waves
// (one per SIMD at the occupancy target: a quarter of the CU's LDS each);
// *pcw = 0 / *free_bytes = -1 when neither fits or the feature set has no
// persistent instance.
extern "C" hipError_t rtk_lds_plan_pc(int features, int stack_depth, int force_waves, int *pcw,
                                      int64_t *free_bytes,
                                      int *blocks_per_cu) {
  *free_bytes = -1;
  *pcw = 0;
  *blocks_per_cu = 0;
  const unsigned f = (unsigned)(features & F_ALL);
  if (!RT_PERSIST_F(f)) return hipSuccess;
  for (int w : {kPcWaves, kWaves}) { // force_waves == kWaves (tests): the 4-wave form on any scene
    if (force_waves == kWaves && w != kWaves) continue;
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(persistent_instance(f, w)));
    if (e != hipSuccess) return e;
    const int regs = ((a.numRegs + 7) / 8) * 8;
    const int waves_per_simd = std::max(1, std::min(8, regs > 0 ? 512 / regs : 8));
    const int bpc = std::max(1, waves_per_simd * 4 / w); // resident blocks per CU
    const size_t per_block = kLdsPerCu / bpc;
    const size_t fixed = a.sharedSizeBytes + lds_bytes_pc(features, w, stack_depth, 0);
    if (fixed <= per_block) {
      *pcw = w;
      *blocks_per_cu = bpc;
      *free_bytes = (int64_t)(per_block - fixed);
      return hipSuccess;
    }
  }
  return hipSuccess;
}
extern "C" int rtk_lds_prims_enabled(void) { return 1; }
extern "C" int rtk_lds_perlin_enabled(void) { return 1; }

// Lets a persistent instance's blocks use more than 64 KB of dynamic LDS: set
// once per device and function, to the most any scene's plan can ask for (the
// CU's LDS less the static part), so scenes of different staged sizes used
// from different host threads never lower it between another launch's check
// and its dispatch.
static hipError_t allow_cu_lds(RenderFn fn) {
  static std::mutex mu;
  static std::set<std::pair<int, const void *>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const void *f = reinterpret_cast<const void *>(fn);
  std::lock_guard<std::mutex> g(mu);
  if (done.count({dev, f})) return hipSuccess;
  hipFuncAttributes a;
  e = hipFuncGetAttributes(&a, f);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsPerCu - a.sharedSizeBytes));
  if (e == hipSuccess) done.insert({dev, f});
  return e;
}

extern "C" hipError_t rtk_launch_render(const DScene *S, const DCamera *C, const DLaunch *P,
                                        double *out, unsigned long long *stats,
                                        hipStream_t stream) {
  const int64_t units = (int64_t)P->n_head * P->head_chunks + (int64_t)(P->n_local_tiles - P->n_head) * P->n_chunks;
  const int bw = block_waves((unsigned)S->features);
  int blocks = (int)((units + bw - 1) / bw);
  if (blocks == 0) return hipSuccess;
  RenderFn fn = render_table(stats != nullptr)[S->features & F_ALL];
  // a launch that measures its tiles' costs (rt_api.cpp: the first tile-subset
  // launch of a shape in the flat world)
  const bool cost = stats == nullptr && P->tile_cost != nullptr;
  if (cost) {
    fn = cost_instance((unsigned)(S->features & F_ALL));
    if (fn == nullptr) return hipErrorInvalidValue;
  }
  size_t lds = rtk_lds_bytes(S->features, S->stack_depth, S->n_lds_nodes);
  int launch_waves = bw;
  DLaunch Q = *P;
  const unsigned f = (unsigned)(S->features & F_ALL);
  if (RT_PERSIST_F(f) && stats == nullptr && Q.unit_ctr != nullptr && Q.grid_cap > 0 &&
      S->pc_waves > 0 && units > (int64_t)Q.grid_cap * S->pc_waves) {
    // persistent: the resident blocks' waves take units [0, grid_cap * pc_waves)
    // statically, the rest from the counter
    fn = persistent_instance(f, S->pc_waves);
    blocks = Q.grid_cap;
    launch_waves = S->pc_waves;
    lds = lds_bytes_pc(S->features, S->pc_waves, S->stack_depth, S->n_lds_nodes_pc) +
          (size_t)S->lds_items_pc * sizeof(DItem) + (size_t)S->lds_spheres_pc * sizeof(DSphere);
    hipError_t e = allow_cu_lds(fn);
    if (e != hipSuccess) return e;
    e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(Q.unit_ctr), blocks * S->pc_waves, 1, stream);
    if (e != hipSuccess) return e;
  } else {
    Q.unit_ctr = nullptr; // every unit has its own wave
  }
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * launch_waves), lds, stream, *S, *C, Q, out, stats);
  return hipGetLastError();
}

// Frame-layout launch over every tile in the host's split plan (rt_api.cpp
// frame_plan): head tiles [0, n_head) in head_chunks units each (1: whole
// units written straight into the frame), then the tail tiles in n_chunks
// finer units -- the units the waves take last, so the launch ends on short
// units; chunk partials go to `scratch` and split_sum_kernel adds them into
// the frame.
extern "C" hipError_t rtk_launch_render_chunked(const DScene *S, const DCamera *C,
                                                const DLaunch *P, int n_head, int head_chunks,
                                                int n_chunks, double *out, double *scratch,
                                                hipStream_t stream) {
  DLaunch Q = *P;
  Q.compact = 0;
  Q.n_head = n_head;
  Q.head_chunks = head_chunks;
  Q.n_chunks = n_chunks;
  Q.chunk_strata = (P->sample_count + n_chunks - 1) / n_chunks;
  Q.parts = scratch;
  Q.parts_final = 0;
  hipError_t e = rtk_launch_render(S, C, &Q, out, nullptr, stream);
  if (e != hipSuccess) return e;
  const int first = head_chunks > 1 ? 0 : n_head;
  const int64_t total = (int64_t)(Q.n_local_tiles - first) * 64 * 3;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(split_sum_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                     scratch, *C, Q, out);
  return hipGetLastError();
}

static unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

extern "C" hipError_t rtk_launch_tiles_sum(const double *parts, int64_t n_tiles, int chunks, double *out,
                                           hipStream_t stream) {
  if (n_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(tiles_sum_kernel, dim3(blocks_for(n_tiles * kTileD)), dim3(256), 0, stream, parts,
                     n_tiles, chunks, out);
  return hipGetLastError();
}

extern "C" hipError_t rtk_launch_shard_finish(const double *parts, int n_local, int n_head, int head_chunks,
                                              int n_chunks, const int32_t *order, double *out,
                                              hipStream_t stream) {
  const int first = head_chunks > 1 ? 0 : n_head;
  const int64_t total = (int64_t)(n_local - first) * kTileD;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(shard_finish_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, parts, n_local,
                     n_head, head_chunks, n_chunks, order, out);
  return hipGetLastError();
}

extern "C" hipError_t rtk_launch_tiles_to_frame(const double *tiles, int n_shards, int64_t shard_stride,
                                                int W, int row_begin, int row_end, double scale, int scaled,
                                                int accumulate, double *out, hipStream_t stream) {
  const int64_t total = (int64_t)(row_end - row_begin) * W * 3;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(tiles_to_frame_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, tiles, n_shards,
                     shard_stride, W, row_begin, row_end, (W + 7) / 8, scale, scaled, accumulate, out);
  return hipGetLastError();
}

extern "C" hipError_t rtk_launch_to_bytes(const double *rgb, int64_t n, double scale,
                                          uint8_t *bytes, hipStream_t stream) {
  int64_t total = 3 * n;
  if (total == 0) return hipSuccess;
  int blocks = (int)((total + 255) / 256);
  hipLaunchKernelGGL(to_bytes_kernel, dim3(blocks), dim3(256), 0, stream, rgb, n, scale, bytes);
  return hipGetLastError();
}

