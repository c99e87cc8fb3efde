// rt_bvh_sah.hip — world BVH built on the GPU with binned SAH (SURVEY §8(f)
// rank 3: "GPU BVH build (binned SAH) for large scenes").
//
// The reference builds a binned-SAH tree on the CPU (BVHNode.cpp:21-123,
// 168-254: 15 candidate planes x 3 axes, leaves <= 4); rt_scene.cpp's host
// builder keeps its rules (16 bins per axis, leaves of <= 2 items, or <= 4 when a
// split does not pay under unit traversal/intersection costs, balanced splits
// near the traversal-stack depth budget).  This builder applies the same rules
// top-down, one tree LEVEL per pair of launches, one wavefront per node:
//
//   sah_decide (wave per node of the level)
//     pass 1: the node's box and centroid bounds (lane-strided loads over the
//             node's reference range, wave min/max reductions);
//     pass 2: 3 axes x 16 bins in the wave's LDS slice -- per item one bin count
//             and six box bounds per axis, as LDS integer atomics on order-
//             preserving float keys (min/max are order independent, so the
//             result is deterministic);
//     SAH:    lane a*16+k evaluates the split of axis a before bin k (45 valid
//             candidates) from prefix/suffix unions; a wave arg-min picks the
//             cheapest (ties: lower axis, then higher k -- the host's scan
//             order); leaf / split / forced balanced split as the host decides.
//   exclusive scan (hipCUB) of the split flags: BFS index of each inner node
//             and the slots of its two children in the next level;
//   sah_apply (wave per node)
//     inner node: a stable partition of its references by the chosen bin
//             (ballot + popcount ranks, chunk by chunk) into the other
//             reference buffer, accumulating both children's boxes on the
//             way; writes its DNode (both child boxes, fp32) and the two child
//             descriptors; a leaf gathers its items into the final leaf-order
//             item array.  Every node writes its own entry into its parent's
//             DNode (inner: its BFS index, leaf: ~(first << 3 | count)).
//
// Item boxes enter as fp32 rounded outward with the host builder's margins
// (f32_lo/f32_hi: a relative 2^-20 + 1e-7 absolute widening, then outward
// rounding).  That rounding is monotone, so the union of the rounded item boxes
// IS the rounded fp64 union the host writes: node boxes are as conservative as
// the host's (rt_path.h's slab test stays exact-safe).  Nodes come out in BFS
// order, as the host emits them (the kernel stages a BFS prefix in LDS).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "rt_layout.h"

namespace {

constexpr int kBins = 16;
constexpr int kWavesPerBlock = 4;
constexpr int kLeafMax = 2;

struct SahNode {   // a node of the level being built (32 B)
  int begin, count;
  int parent, side; // parent's BFS index (-1: the root), which of its entries
  int depth, pad[3];
};

struct SahDecision { // what sah_decide chose for a node (32 B)
  int split;          // 1 inner node, 0 leaf
  int axis, bin, nl;  // axis -1: balanced split of the reference range
  float clo, scale;   // bin = clamp((c[axis] - clo) * scale) on the chosen axis
  int pad[2];
};

// fp32 outward rounding with the host builder's margins (rt_scene.cpp
// SahBuilder::f32_lo / f32_hi; nextafter written on the bits).
__device__ __forceinline__ float next_down(float f) {
  if (f == 0.0f) return __uint_as_float(0x80000001u);
  uint32_t u = __float_as_uint(f);
  return __uint_as_float(f > 0.0f ? u - 1u : u + 1u);
}
__device__ __forceinline__ float next_up(float f) {
  if (f == 0.0f) return __uint_as_float(0x00000001u);
  uint32_t u = __float_as_uint(f);
  return __uint_as_float(f > 0.0f ? u + 1u : u - 1u);
}
__device__ __forceinline__ float f32_lo(double x) {
  double m = x - (fabs(x) * 0x1p-20 + 1e-7);
  float f = (float)m;
  if ((double)f > m) f = next_down(f);
  return f;
}
__device__ __forceinline__ float f32_hi(double x) {
  double m = x + (fabs(x) * 0x1p-20 + 1e-7);
  float f = (float)m;
  if ((double)f < m) f = next_up(f);
  return f;
}

// order-preserving int key of a float (its own inverse)
__device__ __forceinline__ int fkey(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float fval(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

__device__ __forceinline__ float wmin(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ float area(const float lo[3], const float hi[3]) {
  const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  return 2.0f * (x * y + y * z + z * x);
}

__device__ __forceinline__ int bin_of(float c, float clo, float scale) {
  int k = (int)((c - clo) * scale);
  return k < 0 ? 0 : (k > kBins - 1 ? kBins - 1 : k);
}

// fp64 item boxes -> fp32 rounded outward (lo xyz + pad, hi xyz + pad), fp32
// centroids, identity references.
__global__ void sah_prep(const double *box, int n, float4 *blo, float4 *bhi, float4 *cen,
                         int *refs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *b = box + 6 * (size_t)i;
  const float4 lo = make_float4(f32_lo(b[0]), f32_lo(b[1]), f32_lo(b[2]), 0.0f);
  const float4 hi = make_float4(f32_hi(b[3]), f32_hi(b[4]), f32_hi(b[5]), 0.0f);
  blo[i] = lo;
  bhi[i] = hi;
  cen[i] = make_float4(0.5f * (lo.x + hi.x), 0.5f * (lo.y + hi.y), 0.5f * (lo.z + hi.z), 0.0f);
  refs[i] = i;
}

__global__ __launch_bounds__(64 * kWavesPerBlock) void sah_decide(
    const SahNode *level, int n_level, const int *refs, const float4 *blo, const float4 *bhi,
    const float4 *cen, SahDecision *dec, int *is_inner, int stack_budget) {
  __shared__ int bins[kWavesPerBlock][3][kBins][7]; // count, lo xyz keys, hi xyz keys
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int w = blockIdx.x * kWavesPerBlock + wv;
  if (w >= n_level) return; // whole wave
  const SahNode nd = level[w];
  const int begin = nd.begin, end = nd.begin + nd.count, cnt = nd.count;
  // ---- pass 1: node box and centroid bounds
  float nlo[3] = {INFINITY, INFINITY, INFINITY}, nhi[3] = {-INFINITY, -INFINITY, -INFINITY};
  float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = begin + lane; i < end; i += 64) {
    const int r = refs[i];
    const float4 lo = blo[r], hi = bhi[r], c = cen[r];
    const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z}, c3[3] = {c.x, c.y, c.z};
    for (int a = 0; a < 3; ++a) {
      nlo[a] = fminf(nlo[a], l3[a]);
      nhi[a] = fmaxf(nhi[a], h3[a]);
      clo[a] = fminf(clo[a], c3[a]);
      chi[a] = fmaxf(chi[a], c3[a]);
    }
  }
  for (int a = 0; a < 3; ++a) {
    nlo[a] = wmin(nlo[a]);
    nhi[a] = wmax(nhi[a]);
    clo[a] = wmin(clo[a]);
    chi[a] = wmax(chi[a]);
  }
  SahDecision d;
  d.split = 0;
  d.axis = -1;
  d.bin = 0;
  d.nl = 0;
  d.clo = 0.0f;
  d.scale = 0.0f;
  d.pad[0] = d.pad[1] = 0;
  const bool leaf = cnt <= kLeafMax || (nd.depth == 0 && cnt <= RT_FLAT_MAX);
  int need = 0;
  while ((1 << need) < cnt) ++need;
  // depth budget (the host's force_median): near the traversal-stack limit
  // split into count halves -- at the bin boundary of the longest centroid
  // axis closest to the median, or by position when every centroid coincides
  const bool force = nd.depth + need >= stack_budget;
  if (!leaf) {
    // ---- pass 2: bins
    int *B = &bins[wv][0][0][0];
    for (int k = lane; k < 3 * kBins; k += 64) {
      B[7 * k] = 0;
      for (int q = 0; q < 3; ++q) {
        B[7 * k + 1 + q] = fkey(INFINITY);
        B[7 * k + 4 + q] = fkey(-INFINITY);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float scale[3];
    for (int a = 0; a < 3; ++a) {
      const float ext = chi[a] - clo[a];
      scale[a] = ext > 1e-12f ? (float)kBins / ext : 0.0f;
    }
    for (int i = begin + lane; i < end; i += 64) {
      const int r = refs[i];
      const float4 lo = blo[r], hi = bhi[r], c = cen[r];
      const float c3[3] = {c.x, c.y, c.z};
      const int kl[3] = {fkey(lo.x), fkey(lo.y), fkey(lo.z)};
      const int kh[3] = {fkey(hi.x), fkey(hi.y), fkey(hi.z)};
      for (int a = 0; a < 3; ++a) {
        if (scale[a] == 0.0f) continue;
        int *b = B + 7 * (a * kBins + bin_of(c3[a], clo[a], scale[a]));
        atomicAdd(b, 1);
        for (int q = 0; q < 3; ++q) {
          atomicMin(b + 1 + q, kl[q]);
          atomicMax(b + 4 + q, kh[q]);
        }
      }
    }
    // this wave's LDS atomics complete before its lanes read the bins (the
    // waves of a block work on different nodes: no block barrier here)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- SAH: lane a*16 + k, split of axis a before bin k
    float cost = INFINITY;
    int nl = 0;
    const int a = lane / kBins, k = lane % kBins;
    if (lane < 3 * kBins && k > 0 && scale[a] != 0.0f) {
      float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      int nr = 0;
      for (int j = 0; j < kBins; ++j) {
        const int *b = B + 7 * (a * kBins + j);
        if (b[0] == 0) continue;
        float *lo = j < k ? llo : rlo, *hi = j < k ? lhi : rhi;
        for (int q = 0; q < 3; ++q) {
          lo[q] = fminf(lo[q], fval(b[1 + q]));
          hi[q] = fmaxf(hi[q], fval(b[4 + q]));
        }
        if (j < k) nl += b[0];
        else nr += b[0];
      }
      if (nl > 0 && nr > 0) {
        if (!force) {
          cost = area(llo, lhi) * (float)nl + area(rlo, rhi) * (float)nr;
        } else {
          const float e0 = chi[0] - clo[0], e1 = chi[1] - clo[1], e2 = chi[2] - clo[2];
          const int longest = e0 > e1 ? (e0 > e2 ? 0 : 2) : (e1 > e2 ? 1 : 2);
          if (a == longest) cost = (float)abs(2 * nl - cnt);
        }
      }
    }
    // wave arg-min; ties: lower axis, then higher k (the host's scan order)
    float best = cost;
    int who = lane;
    for (int o = 32; o > 0; o >>= 1) {
      const float oc = __shfl_xor(best, o);
      const int ow = __shfl_xor(who, o);
      const int oa = ow / kBins, ok = ow % kBins, ma = who / kBins, mk = who % kBins;
      if (oc < best || (oc == best && (oa < ma || (oa == ma && ok > mk)))) {
        best = oc;
        who = ow;
      }
    }
    const int best_nl = __shfl(nl, who);
    if (best < INFINITY) {
      const float parent_area = area(nlo, nhi);
      if (force || !(cnt <= 4 && parent_area > 0.0f && 1.0f + best / parent_area >= (float)cnt)) {
        d.split = 1;
        d.axis = who / kBins;
        d.bin = who % kBins;
        d.nl = best_nl;
        d.clo = clo[d.axis];
        d.scale = scale[d.axis];
      }
    } else {
      // every centroid in one point: any split is as good; halve the range
      d.split = 1;
      d.nl = cnt / 2;
    }
  }
  if (lane == 0) {
    dec[w] = d;
    is_inner[w] = d.split;
  }
}

__global__ __launch_bounds__(64 * kWavesPerBlock) void sah_apply(
    const SahNode *level, int n_level, const SahDecision *dec, const int *rank, int level_base,
    const int *refs_in, int *refs_out, const float4 *blo, const float4 *bhi, const float4 *cen,
    const DItem *items_in, DItem *items_out, DNode *nodes, SahNode *next, int *root_leaf) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int w = blockIdx.x * kWavesPerBlock + wv;
  if (w >= n_level) return;
  const SahNode nd = level[w];
  const SahDecision d = dec[w];
  const int begin = nd.begin, cnt = nd.count, end = begin + cnt;
  const int me = level_base + rank[w];
  if (lane == 0) {
    const int entry = d.split ? me : ~((begin << 3) | cnt);
    if (nd.parent >= 0) nodes[nd.parent].entry[nd.side] = entry;
    else if (!d.split) *root_leaf = cnt;
  }
  if (!d.split) { // leaf: its items, in place, in the final leaf-order array
    for (int i = begin + lane; i < end; i += 64) items_out[i] = items_in[refs_in[i]];
    return;
  }
  // stable partition by the chosen bin (axis -1: the first nl references)
  float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
  float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
  int left = 0, right = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int base = begin; base < end; base += 64) {
    const int i = base + lane;
    const bool valid = i < end;
    int r = 0;
    bool go_left = false;
    float4 lo = make_float4(0, 0, 0, 0), hi = lo;
    if (valid) {
      r = refs_in[i];
      lo = blo[r];
      hi = bhi[r];
      if (d.axis >= 0) {
        const float4 c = cen[r];
        const float ca = d.axis == 0 ? c.x : (d.axis == 1 ? c.y : c.z);
        go_left = bin_of(ca, d.clo, d.scale) < d.bin;
      } else {
        go_left = i - begin < d.nl;
      }
    }
    const unsigned long long L = __ballot(valid && go_left), R = __ballot(valid && !go_left);
    if (valid) {
      const int dst = go_left ? begin + left + __popcll(L & below)
                              : begin + d.nl + right + __popcll(R & below);
      refs_out[dst] = r;
      float *bl = go_left ? llo : rlo, *bh = go_left ? lhi : rhi;
      const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
      for (int q = 0; q < 3; ++q) {
        bl[q] = fminf(bl[q], l3[q]);
        bh[q] = fmaxf(bh[q], h3[q]);
      }
    }
    left += __popcll(L);
    right += __popcll(R);
  }
  for (int q = 0; q < 3; ++q) {
    llo[q] = wmin(llo[q]);
    lhi[q] = wmax(lhi[q]);
    rlo[q] = wmin(rlo[q]);
    rhi[q] = wmax(rhi[q]);
  }
  if (lane == 0) {
    DNode n;
    for (int q = 0; q < 3; ++q) {
      n.lo[q][0] = llo[q];
      n.hi[q][0] = lhi[q];
      n.lo[q][1] = rlo[q];
      n.hi[q][1] = rhi[q];
    }
    n.entry[0] = n.entry[1] = -1; // written by the children at the next level
    n.pad[0] = n.pad[1] = 0;
    nodes[me] = n;
    SahNode c;
    c.parent = me;
    c.depth = nd.depth + 1;
    c.pad[0] = c.pad[1] = c.pad[2] = 0;
    c.begin = begin;
    c.count = left;
    c.side = 0;
    next[2 * rank[w]] = c;
    c.begin = begin + left;
    c.count = cnt - left;
    c.side = 1;
    next[2 * rank[w] + 1] = c;
  }
}

__global__ void sah_root(SahNode *level, int n) {
  SahNode r;
  r.begin = 0;
  r.count = n;
  r.parent = -1;
  r.side = 0;
  r.depth = 0;
  r.pad[0] = r.pad[1] = r.pad[2] = 0;
  *level = r;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Temp {
  size_t blo, bhi, cen, refs0, refs1, lvl0, lvl1, dec, inner, rank, misc, cub, total;
};

size_t scan_bytes(int n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (int *)nullptr, (int *)nullptr, n);
  return b;
}

Temp layout(int n) {
  Temp t;
  size_t o = 0;
  auto take = [&](size_t b) {
    size_t at = o;
    o += align256(b ? b : 1);
    return at;
  };
  t.blo = take(sizeof(float4) * n);
  t.bhi = take(sizeof(float4) * n);
  t.cen = take(sizeof(float4) * n);
  t.refs0 = take(sizeof(int) * n);
  t.refs1 = take(sizeof(int) * n);
  t.lvl0 = take(sizeof(SahNode) * n);
  t.lvl1 = take(sizeof(SahNode) * n);
  t.dec = take(sizeof(SahDecision) * n);
  t.inner = take(sizeof(int) * n);
  t.rank = take(sizeof(int) * n);
  t.misc = take(sizeof(int) * 4);
  t.cub = take(scan_bytes(n));
  t.total = o;
  return t;
}

} // namespace

extern "C" size_t rtk_sah_temp_bytes(int n) { return layout(n).total; }

// boxes: n x (lo xyz, hi xyz) fp64 in item order; items_in: n items.  Writes the
// inner nodes in BFS order (root = node 0) into `nodes` (room for n - 1), the
// items in leaf order into items_out, and on the host: the inner-node count,
// the depth of the deepest node, and root_leaf (n when the whole world is one
// leaf, else 0).  Synchronises `st` once per tree level.
extern "C" hipError_t rtk_build_sah(const double *boxes, const DItem *items_in, int n,
                                    DNode *nodes, DItem *items_out, void *temp,
                                    size_t temp_bytes, int stack_budget, int *n_nodes,
                                    int *depth, int *root_leaf, hipStream_t st) {
  if (n < 1) return hipErrorInvalidValue;
  const Temp t = layout(n);
  if (temp_bytes < t.total) return hipErrorInvalidValue;
  char *base = (char *)temp;
  auto P = [&](size_t off) { return (void *)(base + off); };
  float4 *blo = (float4 *)P(t.blo), *bhi = (float4 *)P(t.bhi), *cen = (float4 *)P(t.cen);
  int *refs[2] = {(int *)P(t.refs0), (int *)P(t.refs1)};
  SahNode *lvl[2] = {(SahNode *)P(t.lvl0), (SahNode *)P(t.lvl1)};
  SahDecision *dec = (SahDecision *)P(t.dec);
  int *inner = (int *)P(t.inner), *rank = (int *)P(t.rank), *misc = (int *)P(t.misc);
  hipError_t e;
  hipLaunchKernelGGL(sah_prep, dim3((n + 255) / 256), dim3(256), 0, st, boxes, n, blo, bhi, cen,
                     refs[0]);
  hipLaunchKernelGGL(sah_root, dim3(1), dim3(1), 0, st, lvl[0], n);
  if ((e = hipMemsetAsync(misc, 0, sizeof(int) * 4, st)) != hipSuccess) return e;
  int level_size = 1, level_base = 0, cur = 0, lev = 0;
  while (level_size > 0) {
    const int blocks = (level_size + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(sah_decide, dim3(blocks), dim3(64 * kWavesPerBlock), 0, st, lvl[cur],
                       level_size, refs[cur], blo, bhi, cen, dec, inner, stack_budget);
    size_t cb = scan_bytes(level_size);
    if ((e = hipcub::DeviceScan::ExclusiveSum(P(t.cub), cb, inner, rank, level_size, st)) !=
        hipSuccess)
      return e;
    int tail[2];
    if ((e = hipMemcpyAsync(&tail[0], rank + level_size - 1, sizeof(int), hipMemcpyDeviceToHost,
                            st)) != hipSuccess ||
        (e = hipMemcpyAsync(&tail[1], inner + level_size - 1, sizeof(int), hipMemcpyDeviceToHost,
                            st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
      return e;
    const int n_inner = tail[0] + tail[1];
    hipLaunchKernelGGL(sah_apply, dim3(blocks), dim3(64 * kWavesPerBlock), 0, st, lvl[cur],
                       level_size, dec, rank, level_base, refs[cur], refs[cur ^ 1], blo, bhi, cen,
                       items_in, items_out, nodes, lvl[cur ^ 1], misc);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    level_base += n_inner;
    level_size = 2 * n_inner;
    cur ^= 1;
    if (level_size > 0) ++lev;
  }
  *n_nodes = level_base;
  *depth = lev;
  if ((e = hipMemcpyAsync(root_leaf, misc, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess)
    return e;
  return hipStreamSynchronize(st);
}
