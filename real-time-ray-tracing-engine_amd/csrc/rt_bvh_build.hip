// rt_bvh_build.hip — world BVH built on the GPU (linear BVH, Karras 2012).
//
// the reference builds its BVH on the CPU, single-threaded
// below 1k objects (BVHNode.cpp:81-112); the host SAH builder here (rt_scene.cpp)
// is O(n log n) but still serial.  For large scenes the library builds instead
// on the device:
//   1. morton_keys:   30-bit Morton code of each item's box centre in the scene
//                     bounds, item index in the low 32 bits (unique keys);
//   2. radix sort of the keys (hipCUB);
//   3. karras_nodes:  the n-1 internal nodes of the binary radix tree, each
//                     from its own key range (longest-common-prefix search);
//   4. refit_boxes:   bottom-up fp64 boxes — each leaf walks to the root and the
//                     second arrival at a node unions its children (agent-scope
//                     acq_rel counter, since the 8 XCDs' L2s are not coherent);
//   5. emit_nodes:    DNode records (both children's boxes in fp32 rounded
//                     outward exactly as the host builder does) and the items
//                     permuted into leaf (= sorted) order;
//   6. tree_depth:    the deepest leaf, for the per-lane traversal stack size.
// Leaves hold one item.  The closest hit does not depend on the tree (every hit
// is decided by the fp64 primitive tests), so images match the host-built tree
// up to exact-t ties.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "rt_layout.h"

namespace {

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) { // 10 bits -> every 3rd bit
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void morton_keys(const double *box, int n, double lx, double ly, double lz, double sx,
                            double sy, double sz, unsigned long long *keys) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *b = box + 6 * (size_t)i;
  double c[3] = {0.5 * (b[0] + b[3]), 0.5 * (b[1] + b[4]), 0.5 * (b[2] + b[5])};
  double lo[3] = {lx, ly, lz}, sc[3] = {sx, sy, sz};
  uint32_t q[3];
  for (int a = 0; a < 3; ++a) {
    double u = (c[a] - lo[a]) * sc[a];
    u = u > 0 ? (u < 1 ? u : 1) : 0; // NaN -> 0
    double x = u * 1024.0;
    q[a] = (uint32_t)(x < 1023.0 ? x : 1023.0);
  }
  uint32_t m = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
  keys[i] = ((unsigned long long)m << 32) | (uint32_t)i;
}

__device__ __forceinline__ int lcp(const unsigned long long *k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  return __clzll(k[i] ^ k[j]); // keys are unique: < 64
}

// Internal node i: children (>= 0 internal, < 0 leaf ~k), parents of both.
__global__ void karras_nodes(const unsigned long long *keys, int n, int *left, int *right,
                             int *parent_int, int *parent_leaf) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (lcp(keys, n, i, i + 1) - lcp(keys, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = lcp(keys, n, i, i - d);
  int lmax = 2;
  while (lcp(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (lcp(keys, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = lcp(keys, n, i, j);
  int s = 0;
  for (int t = (l + 1) / 2;; t = (t + 1) / 2) { // ceil halving down to 1
    if (lcp(keys, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int gamma = i + s * d + (d < 0 ? -1 : 0);
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  if (lo == gamma) {
    left[i] = ~gamma;
    parent_leaf[gamma] = i;
  } else {
    left[i] = gamma;
    parent_int[gamma] = i;
  }
  if (hi == gamma + 1) {
    right[i] = ~(gamma + 1);
    parent_leaf[gamma + 1] = i;
  } else {
    right[i] = gamma + 1;
    parent_int[gamma + 1] = i;
  }
}

__device__ __forceinline__ const double *child_box(int c, const double *leaf_box,
                                                   const double *node_box) {
  return c < 0 ? leaf_box + 6 * (size_t)(~c) : node_box + 6 * (size_t)c;
}

// leaf_box: boxes in sorted order.  Second arrival at a node writes its union.
__global__ void refit_boxes(const double *leaf_box, int n, const int *left, const int *right,
                            const int *parent_int, const int *parent_leaf, unsigned *visits,
                            double *node_box) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int p = parent_leaf[k];
  while (p >= 0) {
    // acq_rel at agent scope: releases this thread's earlier box writes and,
    // for the second arrival, acquires the sibling subtree's (other XCD's L2)
    unsigned prev = __hip_atomic_fetch_add(&visits[p], 1u, __ATOMIC_ACQ_REL,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (prev == 0) return;
    const double *a = child_box(left[p], leaf_box, node_box);
    const double *b = child_box(right[p], leaf_box, node_box);
    double *o = node_box + 6 * (size_t)p;
    for (int q = 0; q < 3; ++q) {
      o[q] = fmin(a[q], b[q]);
      o[q + 3] = fmax(a[q + 3], b[q + 3]);
    }
    p = p == 0 ? -1 : parent_int[p];
  }
}

__global__ void gather_sorted(const unsigned long long *keys, int n, const double *box,
                              const DItem *items, double *box_sorted, DItem *items_sorted) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t src = (uint32_t)keys[k];
  for (int q = 0; q < 6; ++q) box_sorted[6 * (size_t)k + q] = box[6 * (size_t)src + q];
  items_sorted[k] = items[src];
}

// Outward fp32 rounding with the host builder's margins (rt_scene.cpp f32_lo/f32_hi;
// std::nextafter toward -inf / +inf, written on the bits).
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

__global__ void emit_nodes(int n, const int *left, const int *right, const double *leaf_box,
                           const double *node_box, DNode *nodes) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  DNode d;
  const int ch[2] = {left[i], right[i]};
  for (int k = 0; k < 2; ++k) {
    const double *b = child_box(ch[k], leaf_box, node_box);
    for (int q = 0; q < 3; ++q) {
      d.lo[q][k] = f32_lo(b[q]);
      d.hi[q][k] = f32_hi(b[q + 3]);
    }
    d.entry[k] = ch[k] >= 0 ? ch[k] : ~(((~ch[k]) << 3) | 1);
  }
  d.pad[0] = d.pad[1] = 0;
  nodes[i] = d;
}

__global__ void tree_depth(int n, const int *parent_int, const int *parent_leaf, int *depth) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int dep = 0;
  for (int p = parent_leaf[k]; p >= 0; p = p == 0 ? -1 : parent_int[p]) {
    if (++dep > 4096) break; // malformed tree guard: the host rejects the result
  }
  atomicMax(depth, dep);
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Temp {
  size_t keys_in, keys_out, left, right, pint, pleaf, visits, leaf_box, node_box, depth, cub, total;
};

Temp layout(int n, size_t cub_bytes) {
  Temp t;
  size_t o = 0;
  auto take = [&](size_t b) {
    size_t at = o;
    o += align256(b ? b : 1);
    return at;
  };
  t.keys_in = take(sizeof(unsigned long long) * n);
  t.keys_out = take(sizeof(unsigned long long) * n);
  t.left = take(sizeof(int) * n);
  t.right = take(sizeof(int) * n);
  t.pint = take(sizeof(int) * n);
  t.pleaf = take(sizeof(int) * n);
  t.visits = take(sizeof(unsigned) * n);
  t.leaf_box = take(sizeof(double) * 6 * n);
  t.node_box = take(sizeof(double) * 6 * n);
  t.depth = take(sizeof(int));
  t.cub = take(cub_bytes);
  t.total = o;
  return t;
}

size_t cub_temp_bytes(int n) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (unsigned long long *)nullptr,
                                    (unsigned long long *)nullptr, n);
  return b;
}

} // namespace

extern "C" size_t rtk_lbvh_temp_bytes(int n) { return layout(n, cub_temp_bytes(n)).total; }

// boxes: n x (lo xyz, hi xyz) fp64 in item order; items_in: n items.  Writes the
// n-1 internal nodes (root = node 0), the items in leaf order, and the depth
// (internal nodes on the longest root-to-leaf path) to *depth_dev.
extern "C" hipError_t rtk_build_lbvh(const double *boxes, const DItem *items_in, int n,
                                     const double *scene_lo, const double *scene_hi,
                                     DNode *nodes, DItem *items_out, int *depth_dev, void *temp,
                                     size_t temp_bytes, hipStream_t st) {
  if (n < 2) return hipErrorInvalidValue;
  const size_t cub_bytes = cub_temp_bytes(n);
  Temp t = layout(n, cub_bytes);
  if (temp_bytes < t.total) return hipErrorInvalidValue;
  char *base = (char *)temp;
  auto P = [&](size_t off) { return (void *)(base + off); };
  unsigned long long *kin = (unsigned long long *)P(t.keys_in), *kout = (unsigned long long *)P(t.keys_out);
  int *left = (int *)P(t.left), *right = (int *)P(t.right);
  int *pint = (int *)P(t.pint), *pleaf = (int *)P(t.pleaf);
  unsigned *visits = (unsigned *)P(t.visits);
  double *leaf_box = (double *)P(t.leaf_box), *node_box = (double *)P(t.node_box);
  const int B = 256, G = (n + B - 1) / B;
  double sc[3];
  for (int a = 0; a < 3; ++a) {
    double ext = scene_hi[a] - scene_lo[a];
    sc[a] = ext > 0 ? 1.0 / ext : 0.0;
  }
  hipLaunchKernelGGL(morton_keys, dim3(G), dim3(B), 0, st, boxes, n, scene_lo[0], scene_lo[1],
                     scene_lo[2], sc[0], sc[1], sc[2], kin);
  size_t cb = cub_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(P(t.cub), cb, kin, kout, n, 0, 64, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gather_sorted, dim3(G), dim3(B), 0, st, kout, n, boxes, items_in, leaf_box,
                     items_out);
  if ((e = hipMemsetAsync(pint, 0xFF, sizeof(int) * n, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(visits, 0, sizeof(unsigned) * n, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(P(t.depth), 0, sizeof(int), st)) != hipSuccess) return e;
  hipLaunchKernelGGL(karras_nodes, dim3(G), dim3(B), 0, st, kout, n, left, right, pint, pleaf);
  hipLaunchKernelGGL(refit_boxes, dim3(G), dim3(B), 0, st, leaf_box, n, left, right, pint, pleaf,
                     visits, node_box);
  hipLaunchKernelGGL(emit_nodes, dim3(G), dim3(B), 0, st, n, left, right, leaf_box, node_box,
                     nodes);
  hipLaunchKernelGGL(tree_depth, dim3(G), dim3(B), 0, st, n, pint, pleaf, (int *)P(t.depth));
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return hipMemcpyAsync(depth_dev, P(t.depth), sizeof(int), hipMemcpyDeviceToDevice, st);
}
