// rt_path.h — the per-path hot-path functions of the HIP megakernel, as
// host+device code.
//
// rt_kernel.hip includes this to build the gfx950 kernels.  The same source also
// compiles on the host (g++) into a TEST-ONLY emulator (tests/native/), which runs
// the kernel's exact per-path code sequentially so a logic error can be told apart
// from a code-generation problem.  Nothing on the product path uses the host
// build: the library launches only the gfx950 kernels.
#ifndef RT_PATH_H
#define RT_PATH_H
#include <math.h>
#include <stdint.h>

#include "../../include/rt_api.h"
#include "rt_layout.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__
#define RT_FI __forceinline__
#else
#define RT_HD
#define RT_FI inline
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_LDS __attribute__((address_space(3))) // LDS pointer: ds_read, not flat loads
#else
#define RT_LDS
#endif

namespace rtp {

constexpr double kInf = __builtin_huge_val();
constexpr double kPi = 3.1415926535897932385;
constexpr uint32_t kCamTag = 0xFFFFFFFFu;
constexpr uint32_t kSlotShade = 0, kSlotMediumBase = 0x100;

struct V3 {
  double x, y, z;
};
RT_HD RT_FI V3 v3(double x, double y, double z) { return V3{x, y, z}; }
RT_HD RT_FI V3 ld3(const double *p) { return V3{p[0], p[1], p[2]}; }
RT_HD RT_FI V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD RT_FI V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD RT_FI V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD RT_FI V3 operator*(double t, V3 a) { return v3(t * a.x, t * a.y, t * a.z); }
RT_HD RT_FI V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
RT_HD RT_FI double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD RT_FI double len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
RT_HD RT_FI V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Correctly rounded fp64 sqrt for x == 0 or x >= 2^-767 (and +inf, NaN, x < 0):
// the compiler's own lowering (v_rsq_f64, Goldschmidt step, two Newton
// corrections, zero/+inf class fixup) without its input scaling by 2^256 and
// output scaling by 2^-128, which only matter below 2^-767 — 5 of 18
// instructions.  Used where the input is a unit-range quantity known to be 0 or
// far above 2^-767 (u = k 2^-32, 1 - u, 1 - x^2 of a double |x| <= 1, a squared
// length compared against 1e-16); the root of a discriminant keeps sqrt().
RT_HD RT_FI double sqrt_n(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  return __builtin_isfpclass(x, 0x260) ? x : g; // +-0, +inf: x itself
#else
  return sqrt(x);
#endif
}
// Correctly rounded 1/x for x in [2^-600, 2^600] or +inf: the compiler's fp64
// division lowering with numerator 1 (v_rcp_f64, two Newton steps, one
// Markstein correction) without v_div_scale (a no-op in that range) and with a
// +inf class select in place of v_div_fixup — 7 of 11 instructions.
RT_HD RT_FI double rcp_n(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y0 = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y0, 1.0);
  const double y1 = fma(y0, e, y0);
  e = fma(-x, y1, 1.0);
  const double y2 = fma(y1, e, y1);
  const double r = fma(-x, y2, 1.0);
  const double q = fma(r, y2, y2);
  return __builtin_isfpclass(x, 0x200) ? 0.0 : q; // 1/+inf = +0
#else
  return 1.0 / x;
#endif
}
RT_HD RT_FI V3 unitv(V3 a) { // Vec3::normalize (Vec3.hpp:150-158)
  double l = sqrt_n(len2(a)); // l <= 1e-8 (incl. every input below 2^-767) -> (1, 0, 0)
  if (l > 1e-8) {
    double s = rcp_n(l); // l in (1e-8, 2^512] or +inf
    return v3(a.x * s, a.y * s, a.z * s);
  }
  return v3(1.0, 0.0, 0.0);
}

struct Ray {
  V3 o, d;
  double tm;
};
RT_HD RT_FI V3 at(const Ray &r, double t) {
  return v3(r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z);
}

struct Hit {
  double t;
  V3 p, n;
  int mat;
  bool front;
};

// ------------------------------------------------------- uniform loads
// A scene-table record whose index is the same in every lane of the wavefront
// (the flat list walk, the media and light-pdf loops): read through the
// constant address space, so the compiler issues one scalar load (s_load)
// into SGPRs instead of a vector load per lane into VGPRs -- no VMEM
// instruction, no per-lane address arithmetic, no VGPRs for the record.  The
// scene tables are never written while a kernel runs.  U = false: a plain load.
template <bool U>
struct UTag {
  static constexpr bool value = U;
};
template <bool U, class T>
RT_HD RT_FI T ldu(const T *p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (U) {
    T t;
    __builtin_memcpy(&t, (const __attribute__((address_space(4))) T *)(p + i), sizeof(T));
    return t;
  }
#endif
  return p[i];
}

// ---------------------------------------------------------------- RNG
struct Key {
  uint32_t k0, k1, pixel, sample;
};
// KB ("key barrier"): hide the wave-uniform key from the optimiser at entry,
// so the round keys are re-derived with scalar adds in every call.  Without it
// the 20 round keys are hoisted out of the path loop, spill to VGPR lanes and
// cost a v_readlane (plus hazard nops) per use.  Measured per instance: the
// plain flat instance gains (C2 +3 %); the rich instances lose badly (C4 -25 %,
// more SGPR pressure there), so only the former sets it.
// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96) instead of two v_xor_b32
RT_HD RT_FI uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
// the key barrier per instance: the plain flat one only (every instance with
// it: C4 -8.6 %, C3 -0.5 %, C2 +-0.5 %, profiles/r05e_kb_ab.log)
#define RT_KB_F(F) ((F) == F_FLAT)
template <bool KB = false>
RT_HD RT_FI void philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                         uint32_t k0, uint32_t k1, uint32_t out[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KB) asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int r = 0; r < 10; ++r) { // Philox4x32-10 (Random123 default)
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // one 32x32->64 product per multiplier (v_mad_u64_u32), not a separate
    // mul_hi + mul_lo pair: half the quarter-rate integer multiplies
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0), n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}
// Four uniforms in [0,1) (x * 2^-32, exact in fp64) from one Philox block for
// (bounce, slot) — DESIGN.md "RNG contract".
template <bool KB = false>
RT_HD RT_FI void u01x4(const Key &k, uint32_t bounce, uint32_t slot, double u[4]) {
  uint32_t x[4];
  philox10<KB>(k.pixel, k.sample, bounce, slot, k.k0, k.k1, x);
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = (double)x[q] * 0x1.0p-32;
}

// sin and cos of 2*pi*u for a uniform u = k * 2^-32 in [0, 1) (every angle the
// path draws: disk, cosine, unit-vector and light-cone directions).  Quadrant
// reduction in u is exact (4u and 4u - q are exact doubles), so no Cody-Waite or
// Payne-Hanek reduction is needed; the kernels on [-pi/4, pi/4] are the
// fdlibm/FreeBSD k_sin/k_cos minimax polynomials.  Max |error| 1.4e-16 against
// the exact sin(2 pi u) (the reference's sin(fl(2 pi u)) is itself up to 4.4e-16
// from it); tested in tests/test_emulator.py.
// Polynomial constants at their use (device, RT_KCONST_MODE 1): fma(a, b, K) as ONE
// v_fma_f64 whose addend K is put into an SGPR pair by two s_mov_b32 right
// there (volatile, so not hoisted).  Written as plain fma, the compiler hoists
// each fp64 coefficient out of the path loop into a VGPR pair (sincos: 10
// pairs, 20 VGPRs live across the whole loop in every instance) and, because
// it selects the tied v_fmac_f64 form, copies the constant into the
// accumulator before every step (v_mov_b64 + v_fmac_f64).  Same correctly
// rounded fma, same bits.
#if defined(__HIP_DEVICE_COMPILE__)
template <uint64_t K>
__device__ __forceinline__ double kconst_s() { // K's double in an SGPR pair, materialised here
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3" : "=s"(lo), "=s"(hi) : "i"((uint32_t)K), "i"((uint32_t)(K >> 32)));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <uint64_t K>
__device__ __forceinline__ double fma_k(double a, double b) { // fma(a, b, K)
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(kconst_s<K>()));
  return r;
}
template <uint64_t B, uint64_t K>
__device__ __forceinline__ double fma_kk(double a) { // fma(a, B, K): B from SGPRs, K copied to a VGPR
  double r;
  const double k = kconst_s<K>();
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(kconst_s<B>()), "v"(k));
  return r;
}
#define RT_KB(x) __builtin_bit_cast(uint64_t, (double)(x))
#define FMA_K(a, b, K) fma_k<RT_KB(K)>((a), (b))
#define FMA_KK(a, B, K) fma_kk<RT_KB(B), RT_KB(K)>((a))
#endif
// Measured (profiles/r03v_ab.log): the plain BVH instances C3 +2.3 % (their
// VGPR spills 20 -> 4), the flat instance C2 -1 %, the rich C4 -8 % (its SGPRs
// are already spilled into VGPR lanes; constants put into VGPRs by v_mov at
// their use instead: C4 -7.6 %, r03x_ab.log): used by the plain BVH instances only.
#define RT_KCONST_F(F) (((F) & ~F_BVH4) == 0)
// KC: 1 = the polynomial constants at their use in SGPRs (above), 0 = plain fma
#define RT_KCONST_MODE(F) (RT_KCONST_F(F) ? 1 : 0)
template <int KC = 0>
RT_HD RT_FI void sincos_2pi(double u, double &s, double &c) {
  const double t = 4.0 * u;
  const double q = floor(t + 0.5);
  const double x = (t - q) * 1.5707963267948966;
  const double z = x * x;
  double ps, sn, pc;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (KC == 1) {
    ps = FMA_K(z, FMA_K(z, FMA_K(z, FMA_KK(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                 2.75573137070700676789e-06), -1.98412698298579493134e-04),
               8.33333333332248946124e-03);
    sn = fma(z * x, FMA_K(z, ps, -1.66666666666666324348e-01), x);
    pc = z * FMA_K(z, FMA_K(z, FMA_K(z, FMA_K(z, FMA_KK(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                              -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                          -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  } else
#endif
  {
    ps = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                           2.75573137070700676789e-06), -1.98412698298579493134e-04),
             8.33333333332248946124e-03);
    sn = fma(z * x, fma(z, ps, -1.66666666666666324348e-01), x);
    pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                         -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                        -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  }
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cn = w + (((1.0 - w) - hz) + z * pc);
  const int qi = (int)q & 3;
  s = (qi & 1) ? cn : sn;
  c = (qi & 1) ? sn : cn;
  if (qi >= 2) s = -s;
  if (qi == 1 || qi == 2) c = -c;
}

// ---------------------------------------------------------------- features
enum : unsigned {
  F_MEDIA = 1u,  // constant media in the world
  F_XFORM = 2u,  // RotateY/Translate chains on world items or lights
  F_LIGHTS = 4u, // a non-empty light list (mixture with light sampling)
  F_NOISE = 8u,  // Perlin noise textures
  F_FLAT = 16u,  // flat world (root_is_leaf): every item tested in list order, no BVH walk
  F_BVH4 = 32u,  // 4-wide world BVH (DNode4); never with F_FLAT
  F_ALL = 63u
};

// ---------------------------------------------------------------- textures
// sin(x) for NoiseTexture::value (NoiseTexture.cpp:33), within 1 ulp (checked
// against long double in tests/test_emulator.py).  The library's double sin
// carries a Payne-Hanek reduction for huge arguments whose temporaries are live
// beside the whole path state at this point -- 16 of the rich instance's 28
// spilled VGPRs.  Here: Cody-Waite reduction by pi/2 = P1 + P2 + P3 (P1 the
// double nearest pi/2, so x - n P1 is exact for |x| < 2^20: both are multiples
// of 2^-53 and the difference is below 1), the rest as a double-double
// (TwoSum, exact product tail by FMA), then the fdlibm kernels (k_sin.c /
// k_cos.c, Sun Microsystems 1993, freely redistributable) on |r| <= pi/4.
// Larger or non-finite arguments go to the library sin out of line.
RT_HD __attribute__((noinline)) double sin_wide(double x) { return sin(x); }
RT_HD RT_FI double sin_n(double x) {
  if (!(fabs(x) < 0x1p20)) return sin_wide(x);
  const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54,
               P3 = -0x1.f1976b7ed8fbcp-110;
  const double n = rint(x * 0x1.45f306dc9c883p-1);
  const double r1 = fma(-n, P1, x); // exact
  const double p = n * P2, pe = fma(n, P2, -p);
  const double hi = r1 - p, bb = hi - r1;
  const double lo = ((r1 - (hi - bb)) + (-p - bb)) - pe - n * P3;
  const double y0 = hi + lo, y1 = lo - (y0 - hi); // r = y0 + y1
  const double z = y0 * y0;
  double v;
  const int q = (int)n & 3;
  if ((q & 1) == 0) { // k_sin(y0, y1)
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double w = z * y0;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    v = y0 - ((z * (0.5 * y1 - w * r) - y1) - w * S1);
  } else { // k_cos(y0, y1)
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double zz = z * z;
    const double r = z * (C1 + z * (C2 + z * C3)) + zz * zz * (C4 + z * (C5 + z * C6));
    const double hz = 0.5 * z, w = 1.0 - hz;
    v = w + (((1.0 - w) - hz) + (z * r - y0 * y1));
  }
  v = (q & 2) ? -v : v;
  return fabs(x) < 0x1p-26 ? x : v; // sin x = x to 1/2 ulp there; keeps -0
}

// PerlinNoise::noise + perlin_interp (PerlinNoise.hpp:43-60, 186-201).  The
// reference's corner weight i*uu + (1-i)*(1-uu) is uu or 1-uu and (u - i) is u or
// u-1: the same doubles for every input (0*x + y == y, x - 0 == x here; NaN stays
// NaN), without the dead multiplies.  Corner order and the ((fi*fj)*fk)*dot
// grouping are the reference's.
// The device build: the same trilinear Hermite blend as
// repeated linear interpolation -- 8 corner dot products as FMAs, then 4 + 2 +
// 1 lerps a + t (b - a) -- instead of 8 products of three weights: about 40
// instead of 70 fp64 operations per octave.  The grouping and the FMAs change
// the rounding of the noise value (relative differences ~1e-16; nothing
// branches on it, it only scales the albedo), so the host build (emulator)
// keeps the reference's order and images agree with the oracle to ~1e-15.
#if defined(__HIP_DEVICE_COMPILE__)
// The device form's blend of one octave from its cell offsets (u, v, w), their
// Hermite weights and the six permutation entries of the cell's corners.
template <class PP>
__device__ __forceinline__ double perlin_blend(PP P, double u, double v, double w, double uu, double vv,
                                               double ww, int px0, int px1, int py0, int py1, int pz0,
                                               int pz1) {
  const double u1 = u - 1, v1 = v - 1, w1 = w - 1;
  auto dotc = [&](int h, double di, double dj, double dk) {
    const auto *g = P->rv[h];
    return fma(g[0], di, fma(g[1], dj, g[2] * dk));
  };
  auto lerp = [](double a, double b, double t) { return fma(t, b - a, a); };
  const double c000 = dotc(px0 ^ py0 ^ pz0, u, v, w), c100 = dotc(px1 ^ py0 ^ pz0, u1, v, w);
  const double c010 = dotc(px0 ^ py1 ^ pz0, u, v1, w), c110 = dotc(px1 ^ py1 ^ pz0, u1, v1, w);
  const double c001 = dotc(px0 ^ py0 ^ pz1, u, v, w1), c101 = dotc(px1 ^ py0 ^ pz1, u1, v, w1);
  const double c011 = dotc(px0 ^ py1 ^ pz1, u, v1, w1), c111 = dotc(px1 ^ py1 ^ pz1, u1, v1, w1);
  const double x00 = lerp(c000, c100, uu), x10 = lerp(c010, c110, uu);
  const double x01 = lerp(c001, c101, uu), x11 = lerp(c011, c111, uu);
  return lerp(lerp(x00, x10, vv), lerp(x01, x11, vv), ww);
}
#endif
template <class PP> // const DPerlin *, or the LDS copy's pointer (RT_LDS)
RT_HD double perlin_noise(PP P, V3 p) {
  double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
  double u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int xi = (int)fx, yi = (int)fy, zi = (int)fz;
  double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
#if defined(__HIP_DEVICE_COMPILE__)
  const int px0 = P->px[xi & 255], px1 = P->px[(xi + 1) & 255];
  const int py0 = P->py[yi & 255], py1 = P->py[(yi + 1) & 255];
  const int pz0 = P->pz[zi & 255], pz1 = P->pz[(zi + 1) & 255];
  return perlin_blend(P, u, v, w, uu, vv, ww, px0, px1, py0, py1, pz0, pz1);
#endif
  double acc = 0.0;
  for (int i = 0; i < 2; i++) {
    int pxi = P->px[(xi + i) & 255];
    double fi = i ? uu : 1 - uu, di = i ? u - 1 : u;
    for (int j = 0; j < 2; j++) {
      int pyj = P->py[(yi + j) & 255];
      double fj = j ? vv : 1 - vv, dj = j ? v - 1 : v;
      for (int k = 0; k < 2; k++) {
        const auto *g = P->rv[pxi ^ pyj ^ P->pz[(zi + k) & 255]];
        double fk = k ? ww : 1 - ww, dk = k ? w - 1 : w;
        acc += fi * fj * fk * (g[0] * di + g[1] * dj + g[2] * dk);
      }
    }
  }
  return acc;
}

using PerlinLds = DPerlin;
#if defined(__HIP__)
// The block's LDS copy of the scene's Perlin table (9 KB; allocated in the noise instances only -- the ones that call this).
__device__ __forceinline__ const RT_LDS PerlinLds *perlin_lds() {
  __shared__ PerlinLds table;
  return (const RT_LDS PerlinLds *)&table;
}
#endif

// The octave loop stays rolled: unrolled, the scheduler overlaps the octaves'
// independent LDS reads and the noise instances spill ~100 VGPRs; software-
// pipelined (the next octave's cell and permutation reads issued while this
// octave blends) it measured C4 -1.5 % with 7 more spilled VGPRs
// (profiles/r03s_ab.log).  fp32 octaves on an fp32 gradient copy: C4 +0.25 %,
// within noise (r03r_ab.log), so the reference's fp64 arithmetic is kept.

template <unsigned F>
RT_HD V3 tex_value(const DScene &S, int t, V3 p) {
  for (int guard = 0; guard < 64; ++guard) {
    const DTex &T = S.texs[t];
    if (T.kind == RT_TEX_SOLID) return ld3(T.color);
    if (T.kind == RT_TEX_CHECKER) { // CheckerTexture.cpp:41-55
      const double inv = T.inv_scale; // 1.0 / scale, host-formed
      int xi = (int)floor(inv * p.x), yi = (int)floor(inv * p.y), zi = (int)floor(inv * p.z);
      t = ((xi + yi + zi) % 2 == 0) ? T.even : T.odd;
      continue;
    }
    if constexpr ((F & F_NOISE) != 0) {
      // NoiseTexture.cpp:31-34: 0.5 * (1 + sin(scale*z + 10*turb(p, 7)))
      auto turb = [&](auto P) { // PerlinNoise::turb(p, 7)
        double acc = 0.0, wgt = 1.0;
        V3 q = p;
#pragma unroll 1
        for (int i = 0; i < 7; i++) {
          acc += wgt * perlin_noise(P, q);
          wgt *= 0.5;
          q = v3(q.x * 2, q.y * 2, q.z * 2);
        }
        return acc;
      };
#if defined(__HIP_DEVICE_COMPILE__)
      // the scene's one Perlin table staged in LDS by the block (S.lds_perlin):
      // 7 octaves x (6 permutation + 8 gradient reads), two dependent rounds
      // each, at LDS rather than L1/L2 latency
      const double acc = S.lds_perlin ? turb(perlin_lds()) : turb(&S.perlin[T.perlin]);
#else
      const double acc = turb(&S.perlin[T.perlin]);
#endif
      double f = 1 + sin_n(T.scale * p.z + 10 * fabs(acc));
      return f * v3(0.5, 0.5, 0.5);
    }
    break;
  }
  return v3(0, 0, 0);
}

// ------------------------------------------------------------ primitives
// Sphere::hit root search (Sphere.cpp:101-127).
// The center at the ray's time, center.at(time) = c0 + tm * (c1 - c0): exactly
// c0 for a static sphere (dir = 0), so scenes without motion skip the six ops
// (DScene::static_spheres, wave-uniform).
RT_HD RT_FI V3 sphere_center(const DSphere &s, double tm, bool moving) {
  if (!moving) return ld3(s.c0);
  return v3(s.c0[0] + tm * s.dir[0], s.c0[1] + tm * s.dir[1], s.c0[2] + tm * s.dir[2]);
}
// x / b from y = RN(1/b): q = x*y is within one ulp of x/b, the remainder
// x - b*q is exact in one FMA, and one correction q + r*y rounds to the correctly
// rounded quotient (Markstein, IBM J. R&D 34(1), 1990; Muller et al., Handbook of
// Floating-Point Arithmetic, "Markstein's theorem") — the division's own double,
// in 3 fp64 ops instead of a full division's ~11 (scale, rcp, Newton steps,
// fixup), wherever one divisor serves several quotients.  The theorem needs q and
// the remainder to stay normal: |x| >= 2^-960 and |x/b| < 2^1000.  Outside that
// (x = 0, NaN, inf, subnormal-range operands) the quotient may differ from the
// division's; for the sphere roots such cases are rejected by the
// tmin < t < tmax test either way (|t| far below tmin while |d|^2 >= 2^-900,
// or NaN where the division gives +-inf), and for ct/pi (|ct| <= 1) only
// |ct| < 2^-960 could differ.  A
// per-call operand check with a division fallback was measured and costs more
// than the saving (C2 -3 %).  Checked on the host over 4e8 random operand pairs
// (incl. all-ones significands): 0 differences.
RT_HD RT_FI double div_mk(double x, double b, double y) {
  const double q = x * y;
  const double r = fma(-q, b, x);
  return fma(r, y, q);
}
constexpr double kInvPi = 1.0 / kPi; // correctly rounded at compile time

RT_HD RT_FI bool sphere_root(const DSphere &s, const Ray &r, double a, double tmin,
                                            double tmax, double &root, bool moving = true,
                                            bool mk = false, double ya = 0.0) {
  V3 cc = sphere_center(s, r.tm, moving);
  V3 oc = cc - r.o;
  double h = dot(r.d, oc);
  double c = len2(oc) - s.rr;
  double disc = h * h - a * c;
  if (disc < 0) return false;
  double sq = sqrt(disc);
  // mk: ya = RN(1/a) shared by every root of one ray (div_mk), else the division
  double t = mk ? div_mk(h - sq, a, ya) : (h - sq) / a;
  if (!(tmin < t && t < tmax)) {
    t = mk ? div_mk(h + sq, a, ya) : (h + sq) / a;
    if (!(tmin < t && t < tmax)) return false;
  }
  root = t;
  return true;
}
RT_HD RT_FI void sphere_record(const DSphere &s, const Ray &r, double t, int mat,
                                              Hit &h, bool moving = true) {
  V3 cc = sphere_center(s, r.tm, moving);
  h.t = t;
  h.p = at(r, t);
  V3 on = s.inv_r * (h.p - cc); // inv_r = 1 / r, the same double the reference forms
  h.front = dot(r.d, on) < 0;
  h.n = h.front ? on : -on;
  h.mat = mat;
  // u,v (Sphere.cpp:136-140) are not computed: no texture kind reads them.
}

// Axis-aligned quads (DQuad::aa >= 0; make_box faces, the Cornell walls): with
// n, w on axis k and u, v on axes i, j, every other term of Plane::hit's dot and
// cross products is a product with an exact zero, so
//   denom = n_k d_k,  t = (D - n_k o_k) / denom,
//   alpha = w_k (+-(pv_i v_j)),  beta = w_k (+-(u_i pv_j))   (sign: parity of (k, i, j))
// at a third of the operations, with the same outcome for EVERY ray:
//  * finite ray: the dropped terms are +-0 and vanish from the sums exactly
//    (a + +-0 == a for a != 0; a zero result may flip sign, which no test
//    reads: 0 <= -0, and a zero t fails t >= tmin / enters the medium span as
//    the same value);
//  * non-finite ray: both forms reject.  The full form turns 0 * inf into a
//    NaN dot product; this form rejects an infinite denominator explicitly
//    (t would be 0) and otherwise accepts only with d_k, o_k (finite t) and
//    o_i, d_i, o_j, d_j (finite alpha, beta) finite -- every component.
// The quad's own values are finite (checked when aa is set).
// ... in the plain flat instance (C2 +2.7 %); the rich flat instances have no
// SGPRs to spare for the records (C4 -1.6 %; profiles/r03d_ab.log)
#define RT_UNIFORM_LOADS_F(F) ((F) == F_FLAT)
RT_HD RT_FI double comp(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); } // no private array
// SEL: the quad's axis components picked by value selects, not by an indexed
// load -- for a record held in registers (a uniform scalar load, ldu), where
// an indexed access would put it in scratch memory
template <bool SEL = false>
RT_HD RT_FI bool quad_t_aa(const DQuad &q, const Ray &r, double tmin, double tmax, double &t) {
  const int k = q.aa & 3, i = (q.aa >> 2) & 3, j = (q.aa >> 4) & 3;
  const double nk = SEL ? comp(ld3(q.n), k) : q.n[k], wk = SEL ? comp(ld3(q.w), k) : q.w[k];
  const double Qi = SEL ? comp(ld3(q.Q), i) : q.Q[i], Qj = SEL ? comp(ld3(q.Q), j) : q.Q[j];
  const double vj = SEL ? comp(ld3(q.v), j) : q.v[j], ui = SEL ? comp(ld3(q.u), i) : q.u[i];
  const double denom = nk * comp(r.d, k);
  // |denom| = inf: the full form's denom is NaN (0 * inf in the dot product)
  if (fabs(denom) < 1e-8 || fabs(denom) == kInf) return false;
  const double tt = (q.D - nk * comp(r.o, k)) / denom;
  if (!(tmin <= tt && tt <= tmax)) return false;
  const double pvi = (comp(r.o, i) + tt * comp(r.d, i)) - Qi;
  const double pvj = (comp(r.o, j) + tt * comp(r.d, j)) - Qj;
  const double ca = pvi * vj, cb = ui * pvj;
  const bool neg = (q.aa >> 6) & 1;
  const double alpha = wk * (neg ? -ca : ca);
  const double beta = wk * (neg ? -cb : cb);
  if (!(0 <= alpha && alpha <= 1) || !(0 <= beta && beta <= 1)) return false;
  t = tt;
  return true;
}
// quad_t_aa with the axes (k, i, j) as constants: the ray's components and the
// record's fields are picked at compile time, not by per-lane selects (four
// v_cndmask per double component read by an axis held in a register, 24 per
// test), and the sign `neg` is the permutation's parity.  The same operations
// on the same values as quad_t_aa, so the same t and the same verdict.
RT_HD RT_FI constexpr double comp_c(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
template <int K, int I, int J>
RT_HD RT_FI bool quad_t_aa_c(const DQuad &q, const Ray &r, double tmin, double tmax, double &t) {
  constexpr bool neg = !((K + 1) % 3 == I); // (k, i, j) not a cyclic shift of (0, 1, 2)
  const double nk = q.n[K], wk = q.w[K], Qi = q.Q[I], Qj = q.Q[J], vj = q.v[J], ui = q.u[I];
  const double denom = nk * comp_c(r.d, K);
  if (fabs(denom) < 1e-8 || fabs(denom) == kInf) return false;
  const double tt = (q.D - nk * comp_c(r.o, K)) / denom;
  if (!(tmin <= tt && tt <= tmax)) return false;
  const double pvi = (comp_c(r.o, I) + tt * comp_c(r.d, I)) - Qi;
  const double pvj = (comp_c(r.o, J) + tt * comp_c(r.d, J)) - Qj;
  const double ca = pvi * vj, cb = ui * pvj;
  const double alpha = wk * (neg ? -ca : ca);
  const double beta = wk * (neg ? -cb : cb);
  if (!(0 <= alpha && alpha <= 1) || !(0 <= beta && beta <= 1)) return false;
  t = tt;
  return true;
}
// Dispatch on a WAVE-UNIFORM aa (the flat list walk, the light loops: one
// record for every lane): scalar branches to the constant-axis form.  A
// per-lane aa (BVH leaves) keeps quad_t_aa: a switch would serialise there.
RT_HD RT_FI bool quad_t_aa_u(const DQuad &q, const Ray &r, double tmin, double tmax, double &t) {
  switch (q.aa & 63) {
  case 0 | 1 << 2 | 2 << 4: return quad_t_aa_c<0, 1, 2>(q, r, tmin, tmax, t);
  case 0 | 2 << 2 | 1 << 4: return quad_t_aa_c<0, 2, 1>(q, r, tmin, tmax, t);
  case 1 | 2 << 2 | 0 << 4: return quad_t_aa_c<1, 2, 0>(q, r, tmin, tmax, t);
  case 1 | 0 << 2 | 2 << 4: return quad_t_aa_c<1, 0, 2>(q, r, tmin, tmax, t);
  case 2 | 0 << 2 | 1 << 4: return quad_t_aa_c<2, 0, 1>(q, r, tmin, tmax, t);
  default: return quad_t_aa_c<2, 1, 0>(q, r, tmin, tmax, t);
  }
}
template <bool SEL = false, bool UAX = false> // UAX: q is the same record in every lane
RT_HD RT_FI bool quad_t(const DQuad &q, const Ray &r, double tmin, double tmax,
                                       double &t) { // Plane.cpp:76-100
  if constexpr (UAX) {
    if (q.aa >= 0) return quad_t_aa_u(q, r, tmin, tmax, t);
  }
  if (q.aa >= 0) return quad_t_aa<SEL>(q, r, tmin, tmax, t);
  V3 n = ld3(q.n);
  double denom = dot(n, r.d);
  if (fabs(denom) < 1e-8) return false;
  double tt = (q.D - dot(n, r.o)) / denom;
  if (!(tmin <= tt && tt <= tmax)) return false;
  V3 pv = at(r, tt) - ld3(q.Q);
  V3 w = ld3(q.w);
  double alpha = dot(w, cross(pv, ld3(q.v)));
  double beta = dot(w, cross(ld3(q.u), pv));
  if (!(0 <= alpha && alpha <= 1) || !(0 <= beta && beta <= 1)) return false;
  t = tt;
  return true;
}
RT_HD RT_FI void quad_record(const DQuad &q, const Ray &r, double t, int mat,
                                            Hit &h) {
  h.t = t;
  h.p = at(r, t);
  V3 n = ld3(q.n);
  h.front = dot(r.d, n) < 0;
  h.n = h.front ? n : -n;
  h.mat = mat;
}

// ------------------------------------------------------ transform chains
// RotateY (RotateY.cpp:41-76) / Translate (Translate.cpp:17-31) as flattened
// chains: world -> local applies ops outermost first, the record goes back
// innermost first.
RT_HD RT_FI V3 rot_in(double s, double c, V3 p) {
  return v3((c * p.x) - (s * p.z), p.y, (s * p.x) + (c * p.z));
}
RT_HD RT_FI V3 rot_out(double s, double c, V3 p) {
  return v3((c * p.x) + (s * p.z), p.y, (-s * p.x) + (c * p.z));
}
template <bool U = false>
RT_HD RT_FI Ray to_local(const DScene &S, int f, int n, Ray r) {
  for (int k = 0; k < n; ++k) {
    const DXform X = ldu<U>(S.xforms, f + k);
    if (X.kind == X_TRANSLATE) {
      r.o = r.o - v3(X.a, X.b, X.c);
    } else {
      r.o = rot_in(X.a, X.b, r.o);
      r.d = rot_in(X.a, X.b, r.d);
    }
  }
  return r;
}
RT_HD RT_FI void to_world(const DScene &S, int f, int n, Hit &h) {
  for (int k = n - 1; k >= 0; --k) {
    const DXform X = S.xforms[f + k];
    if (X.kind == X_TRANSLATE) {
      h.p = h.p + v3(X.a, X.b, X.c);
    } else {
      h.p = rot_out(X.a, X.b, h.p);
      h.n = rot_out(X.a, X.b, h.n);
    }
  }
}

// Closest t over a set of items (sphere/quad + chain), no record: one boundary
// query of ConstantMedium::hit (ConstantMedium.cpp:28-32).  Used only as the
// fallback of boundary_span.
RT_HD bool items_closest_t(const DScene &S, const DItem *its, int first, int n, const Ray &r,
                           double tmin, double tmax, double &tbest) {
  bool any = false;
  for (int k = 0; k < n; ++k) {
    const DItem it = its[first + k];
    Ray lr = it.xf_count ? to_local(S, it.xf_first, it.xf_count, r) : r;
    double t;
    bool hit;
    if (it.kind == I_SPHERE)
      hit = sphere_root(S.spheres[it.idx], lr, len2(lr.d), tmin, tmax, t);
    else
      hit = quad_t(S.quads[it.idx], lr, tmin, tmax, t);
    if (hit) {
      any = true;
      tmax = t;
      tbest = t;
    }
  }
  return any;
}

// Both boundary queries of ConstantMedium::hit in ONE pass over the boundary
// items: t1 = closest boundary hit on (-inf, inf), t2 = closest beyond t1+1e-4
// (ConstantMedium.cpp:28-32).  A scan's result is the minimum over the items'
// distances that pass its interval test (a sphere offers both roots, open
// interval; a quad its plane distance, closed interval), so the three smallest
// candidates decide both; only when more than three candidates exist and none
// of the kept ones passes the second test does the exact second scan run.
RT_HD RT_FI bool boundary_span(const DScene &S, const DMedium &M, const Ray &r, double &t1,
                               double &t2) {
  // the three smallest candidates, ascending; bit k of kf: candidate k is a quad
  // distance (closed interval).  Flags as bits of one integer: three bools
  // shifted by the insertion were kept in scratch memory by the compiler.
  double c0 = 0, c1 = 0, c2 = 0;
  uint32_t kf = 0;
  int n_cand = 0;
  auto keep = [&](double t, uint32_t cl) {
    ++n_cand;
    if (n_cand == 1 || t < c0) {
      c2 = c1, c1 = c0, c0 = t;
      kf = ((kf << 1) | cl) & 7u;
    } else if (n_cand == 2 || t < c1) {
      c2 = c1, c1 = t;
      kf = (kf & 1u) | (cl << 1) | ((kf & 2u) << 1);
    } else if (n_cand == 3 || t < c2) {
      c2 = t;
      kf = (kf & 3u) | (cl << 2);
    }
  };
  Ray lr = r;
  int lr_first = -1, lr_count = 0; // chain lr is in (boundary items often share one)
  for (int k = 0; k < M.b_count; ++k) {
    const DItem it = S.bitems[M.b_first + k];
    if (it.xf_first != lr_first || it.xf_count != lr_count) {
      lr = it.xf_count ? to_local(S, it.xf_first, it.xf_count, r) : r;
      lr_first = it.xf_first;
      lr_count = it.xf_count;
    }
    if (it.kind == I_SPHERE) { // sphere_root's two roots
      const DSphere &sp = S.spheres[it.idx];
      V3 cc = v3(sp.c0[0] + lr.tm * sp.dir[0], sp.c0[1] + lr.tm * sp.dir[1],
                 sp.c0[2] + lr.tm * sp.dir[2]);
      V3 oc = cc - lr.o;
      double a = len2(lr.d);
      double h = dot(lr.d, oc);
      double cc2 = len2(oc) - sp.rr;
      double disc = h * h - a * cc2;
      if (disc < 0) continue;
      double sq = sqrt(disc);
      double r1 = (h - sq) / a, r2 = (h + sq) / a;
      if (-kInf < r1 && r1 < kInf) keep(r1, 0u);
      if (-kInf < r2 && r2 < kInf) keep(r2, 0u);
    } else { // quad_t without its interval test
      const DQuad &q = S.quads[it.idx];
      double tt;
      if (q.aa >= 0) {
        if (!quad_t_aa(q, lr, -kInf, kInf, tt)) continue;
      } else {
        V3 n = ld3(q.n);
        double denom = dot(n, lr.d);
        if (fabs(denom) < 1e-8) continue;
        tt = (q.D - dot(n, lr.o)) / denom;
        if (!(-kInf <= tt && tt <= kInf)) continue;
        V3 pv = at(lr, tt) - ld3(q.Q);
        V3 w = ld3(q.w);
        double alpha = dot(w, cross(pv, ld3(q.v)));
        double beta = dot(w, cross(ld3(q.u), pv));
        if (!(0 <= alpha && alpha <= 1) || !(0 <= beta && beta <= 1)) continue;
      }
      keep(tt, 1u);
    }
  }
  if (n_cand == 0) return false;
  t1 = c0;
  const double thr = t1 + 0.0001;
  auto pass = [&](double t, uint32_t cl) {
    return cl ? (thr <= t && t <= kInf) : (thr < t && t < kInf);
  };
  if (pass(c0, kf & 1u)) {
    t2 = c0;
    return true;
  }
  if (n_cand >= 2 && pass(c1, kf & 2u)) {
    t2 = c1;
    return true;
  }
  if (n_cand >= 3 && pass(c2, kf & 4u)) {
    t2 = c2;
    return true;
  }
  if (n_cand <= 3) return false;
  return items_closest_t(S, S.bitems, M.b_first, M.b_count, r, thr, kInf, t2);
}

// Both boundary queries of ConstantMedium::hit for a make_box boundary
// (DMedium::box), from the six face distances alone -- the same doubles as
// boundary_span's, at a third of its work.  Returns 1 (span: t1, t2 set), 0 (no
// span: boundary_span would return false) or -1 (undecided here: the caller runs
// boundary_span).  `r` is the medium-frame ray; the boundary's own chain is
// applied here.
//
// 1. Exact face distances.  Plane::hit's t for a face normal to axis a is
//    RN(RN(D - RN(n_a o_a)) / RN(n_a d_a)) (its dot products with the unit
//    normal's exact zeros drop out, as in quad_t_aa).  Both faces of an axis
//    have |n_a| equal, so their denominators are b and +-b exactly, and one
//    correctly rounded reciprocal y = RN(1/b) (rcp_n) gives each quotient by
//    Markstein's correction (div_mk) -- the division's own double as long as
//    |x| >= 2^-960 or x = 0, and |x/b| < 2^1000.  The lane check `ok`
//    guarantees that: 1e-8 <= |b| <= 2^90 (1e-8 is Plane::hit's own parallel
//    test, so no face is skipped here that the reference would test), |o_a| <=
//    2^90 and o_a = 0 or |o_a| >= 2^-898, and the scene compiler admits only
//    |D| in {0} U [2^-900, 2^90] and |n_a| in [0.5, 2]: then D and RN(n_a o_a)
//    are both 0 or multiples of 2^-952, so x is 0 or |x| >= 2^-952.  Any other
//    lane (non-finite rays included: every check fails on NaN) returns -1.
// 2. Which faces pass Plane::hit's interior test.  The six distances form a
//    slab test: per axis tn = min, tf = max of its two faces; entry = max tn,
//    exit = min tf.  A face's hit point lies inside the box's extent along
//    another axis c exactly when its t lies in [tn_c, tf_c] -- in real
//    arithmetic.  Plane::hit decides it on rounded values: the t's above carry
//    relative errors of ~2^-52 in (B_a + |o_a|) / |d_a| (B_a: the box's largest
//    |plane coordinate| along a), the interior test's point, alpha / beta
//    (RN(w (pv x v))) and the rectangle edges (Q + u vs. the other axis's plane:
//    the compiler admits at most 2^-48 B apart) another ~2^-50 (B_c + |o_c| +
//    |t d_c|) / |d_c| in t.  With s_a = (B_a + |o_a|) |y_a| (|y_a| >= 1 / (2
//    |d_a|)) every such error is below 2^-45 (s_0 + s_1 + s_2), 32x below the
//    margin del = 2^-40 (s_0 + s_1 + s_2).  So, with del:
//    * every near face but the entry axis's, t < entry - del: its point lies
//      before the entry axis's slab -- fails; likewise every far face but the
//      exit axis's, t > exit + del -- fails (cn, cf: exactly one face each
//      within del of entry / exit, else -1);
//    * entry < exit - del: the entry and exit faces pass (their points lie
//      inside the other two slabs by more than del), and only they: the
//      candidates are {entry, exit};
//    * entry > exit + del: no face passes (the entry face lies beyond the exit
//      axis's slab and vice versa);
//    * otherwise -1.
// 3. boundary_span's candidate rules on {entry, exit} (two quads: closed
//    intervals): t1 = entry, t2 = the first candidate >= RN(t1 + 0.0001).
// Proven on the host against the reference's own ConstantMedium boundary
// queries (tests/test_medium_box.py: edge, corner, grazing and axis-parallel
// rays, oracle/_ref) and on the device against boundary_span bit for bit.
RT_HD RT_FI int box_span(const DScene &S, const DMedium &M, const Ray &mr, double &t1,
                         double &t2) {
  const Ray r = M.bxf_count ? to_local(S, M.bxf_first, M.bxf_count, mr) : mr;
  double tn[3], tf[3], s = 0.0;
  bool ok = true;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double o = comp(r.o, a), d = comp(r.d, a);
    const double n0 = M.bnk[a][0], n1 = M.bnk[a][1];
    const double b = n0 * d; // RN(n_a d_a): face 0's denominator; face 1's is +-b
    const double ab = fabs(b), ao = fabs(o);
    ok = ok && ab >= 1e-8 && ab <= 0x1p90 && ao <= 0x1p90 && (o == 0.0 || ao >= 0x1p-898);
    const double y = rcp_n(b); // |b| in [1e-8, 2^90]: correctly rounded
    const double x0 = M.bD[a][0] - n0 * o, x1 = M.bD[a][1] - n1 * o;
    const double u0 = div_mk(x0, b, y);
    const double u1 = (n1 == n0) ? div_mk(x1, b, y) : div_mk(x1, -b, -y);
    tn[a] = fmin(u0, u1);
    tf[a] = fmax(u0, u1);
    s += (M.bB[a] + ao) * fabs(y);
  }
  if (!ok) return -1;
  const double entry = fmax(fmax(tn[0], tn[1]), tn[2]);
  const double exit_ = fmin(fmin(tf[0], tf[1]), tf[2]);
  const double del = 0x1p-40 * s;
  const double elo = entry - del, xhi = exit_ + del;
  const int cn = (tn[0] >= elo) + (tn[1] >= elo) + (tn[2] >= elo);
  const int cf = (tf[0] <= xhi) + (tf[1] <= xhi) + (tf[2] <= xhi);
  if (cn != 1 || cf != 1) return -1;
  if (entry > xhi) return 0;
  if (!(entry < exit_ - del)) return -1;
  t1 = entry;
  const double thr = entry + 0.0001;
  if (thr <= entry) { // |entry| >= 2^39: the closed interval keeps t1 itself
    t2 = entry;
    return 1;
  }
  if (thr <= exit_) {
    t2 = exit_;
    return 1;
  }
  return 0;
}

// ConstantMedium::hit (ConstantMedium.cpp:25-94) in the medium's local frame:
// the scattering distance only (hit_t); medium_record builds the record of
// the winning medium once, after every medium has been tested.
// (box_path, STATS: 1 box_span decided, 0 box_span deferred to boundary_span,
// -1 not a box)
template <bool KB = false>
RT_HD bool medium_t(const DScene &S, const DItem &it, const Ray &wr, double tmin,
                    double tmax, const Key &key, uint32_t bounce, double &hit_t,
                    int &box_path) {
  const DMedium M = S.media[it.idx];
  Ray r = it.xf_count ? to_local(S, it.xf_first, it.xf_count, wr) : wr;
  double t1, t2;
  const int rc = M.box ? box_span(S, M, r, t1, t2) : -2;
  box_path = rc == -2 ? -1 : rc >= 0;
  if (rc == 0) return false;
  if (rc < 0 && !boundary_span(S, M, r, t1, t2)) return false;
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (t1 >= t2) return false;
  if (t1 < 0) t1 = 0;
  double rl = sqrt(len2(r.d));
  double inside = (t2 - t1) * rl;
  double uu[4];
  u01x4<KB>(key, bounce, kSlotMediumBase + (uint32_t)M.id, uu);
  double hd = M.neg_inv_density * log(uu[0]);
  if (hd > inside) return false;
  hit_t = t1 + hd / rl;
  return true;
}

// The record ConstantMedium::hit fills (ConstantMedium.cpp:80-92) at the
// distance medium_t returned: the same local ray, so the same point.
RT_HD RT_FI void medium_record(const DScene &S, const DItem &it, const Ray &wr, double t,
                               Hit &h) {
  Ray r = it.xf_count ? to_local(S, it.xf_first, it.xf_count, wr) : wr;
  h.t = t;
  h.p = at(r, t);
  h.n = v3(1, 0, 0);
  h.front = true;
  h.mat = S.media[it.idx].phase;
  if (it.xf_count) to_world(S, it.xf_first, it.xf_count, h);
}

// ------------------------------------------------------------ traversal
// Conservative fp32 slab test.  Node boxes are fp32 rounded outward with a
// relative 2^-20 + 1e-7 margin (rt_scene.cpp); per ray the origin is rounded up
// for the lo planes and down for the hi planes, so (lo - o) and (hi - o) are
// bracketed before the fp32 subtraction/multiply, whose relative error (< 4
// ulp) the 1 + 2^-20 growth of the far distance absorbs (Ize, "Robust BVH Ray
// Traversal", JCGT 2013).  A box can thus only be visited MORE often than under
// exact arithmetic, never less; every hit is still decided by the fp64
// primitive tests, so the closest hit is unchanged.
RT_HD RT_FI uint32_t f32_bits(float f) {
  union {
    float f;
    uint32_t u;
  } x{f};
  return x.u;
}
RT_HD RT_FI float f32_from(uint32_t u) {
  union {
    uint32_t u;
    float f;
  } x{u};
  return x.f;
}
RT_HD RT_FI float f32_up(double x) { // smallest float >= x (x not NaN)
  float f = (float)x;
  if ((double)f < x) f = (f == 0.0f) ? f32_from(1u) : f32_from(f > 0.0f ? f32_bits(f) + 1u : f32_bits(f) - 1u);
  return f;
}
RT_HD RT_FI float f32_dn(double x) { // largest float <= x (x not NaN)
  float f = (float)x;
  if ((double)f > x) f = (f == 0.0f) ? f32_from(0x80000001u) : f32_from(f > 0.0f ? f32_bits(f) - 1u : f32_bits(f) + 1u);
  return f;
}
// 1/d for the slab test in fp32: v_rcp_f32 (1 ulp) of the rounded direction,
// instead of an fp64 division rounded to fp32 (relative error <= 2^-22.4 vs
// 2^-24; the far-distance growth below still covers the slab error with room).
RT_HD RT_FI float rcp32(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
constexpr float kSlabGrow = 1.0f + 0x1p-19f;
constexpr float kInvClamp = 1e30f; // finite 1/d: a 0 * inf NaN would drop a box

// Slab form (FMA): t = fma(plane, 1/d, -P) with P = RN32(o/d) per ray
// and axis — one fp32 FMA per plane instead of a subtract and a multiply.  P's
// rounding is an ABSOLUTE error eps <= |P| 2^-23 in every plane distance (the
// subtract form's errors are all relative), so the test adds an absolute slack
// E = 2^-21 max|P| (>= 4 eps; floor 1e-30 for P = 0) to the far side:
// tl <= fma(th, 1 + 2^-19, E).  With tl <= th exact, the computed
// tl <= T(1 + 2^-24) + eps and th >= T(1 - 2^-24) - eps, so the relative terms
// (rcp32 2^-22.4 per axis, the fma and final roundings 2^-24 each) stay inside
// the 2^-19 growth and 2 eps inside E: a box is still only ever visited MORE
// often than under exact arithmetic.  P is clamped to +-1e37 before the
// conversion (finite, so lo * inv - P is never inf - inf); a clamped P only
// widens E, i.e. visits more boxes.
// FMA: the BVH instances (one ray feeds many box tests); the flat instances
// single medium-box cull keeps the subtract form, whose per-ray setup is
// cheaper (measured: C3 +2.8 %, C4 -6.5 % with FMA everywhere).
template <bool FMA> struct RayF;
template <> struct RayF<false> { // per-ray fp32 slab-test constants, subtract form
  float oa[3], ob[3], inv[3];
};
template <> struct RayF<true> { // FMA form
  float p[3], inv[3], slack;
};
template <bool FMA>
RT_HD RT_FI RayF<FMA> ray_f32(const Ray &r) {
  RayF<FMA> q;
  const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
  float pm = 0.0f;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float iv = rcp32((float)d[a]);
    q.inv[a] = fminf(fmaxf(iv, -kInvClamp), kInvClamp);
    if constexpr (FMA) {
      const double pd = fmin(fmax((double)q.inv[a] * o[a], -1e37), 1e37); // NaN o: NaN
      q.p[a] = (float)pd;
      pm = fmaxf(pm, fabsf(q.p[a]));
    } else {
      q.oa[a] = f32_up(o[a]);
      q.ob[a] = f32_dn(o[a]);
    }
  }
  if constexpr (FMA) q.slack = fmaxf(pm * 0x1p-21f, 1e-30f);
  return q;
}
// Entry distance if the ray may hit [lo,hi] within [tmin32, cl32], else +inf.
template <bool FMA>
RT_HD RT_FI float slab(const RayF<FMA> &q, const float *lo, const float *hi, float tmin32,
                                      float cl32) {
  float a0, b0, a1, b1, a2, b2;
  if constexpr (FMA) {
    a0 = fmaf(lo[0], q.inv[0], -q.p[0]), b0 = fmaf(hi[0], q.inv[0], -q.p[0]);
    a1 = fmaf(lo[1], q.inv[1], -q.p[1]), b1 = fmaf(hi[1], q.inv[1], -q.p[1]);
    a2 = fmaf(lo[2], q.inv[2], -q.p[2]), b2 = fmaf(hi[2], q.inv[2], -q.p[2]);
  } else {
    a0 = (lo[0] - q.oa[0]) * q.inv[0], b0 = (hi[0] - q.ob[0]) * q.inv[0];
    a1 = (lo[1] - q.oa[1]) * q.inv[1], b1 = (hi[1] - q.ob[1]) * q.inv[1];
    a2 = (lo[2] - q.oa[2]) * q.inv[2], b2 = (hi[2] - q.ob[2]) * q.inv[2];
  }
  float tl = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), tmin32));
  float th = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), cl32));
  if constexpr (FMA)
    return tl <= fmaf(th, kSlabGrow, q.slack) ? tl : __builtin_huge_valf();
  else
    return tl <= th * kSlabGrow ? tl : __builtin_huge_valf();
}
// The same test as slab<FMA=true> with the verdict and the entry distance
// returned apart: the binary node visit branches on the verdict and orders the
// two children by the entry distances, so selecting +inf for a miss and
// comparing against it again (two VALU per box) is not needed.
RT_HD RT_FI bool slab_hit(const RayF<true> &q, const float *lo, const float *hi, float tmin32,
                          float cl32, float &tl) {
  const float a0 = fmaf(lo[0], q.inv[0], -q.p[0]), b0 = fmaf(hi[0], q.inv[0], -q.p[0]);
  const float a1 = fmaf(lo[1], q.inv[1], -q.p[1]), b1 = fmaf(hi[1], q.inv[1], -q.p[1]);
  const float a2 = fmaf(lo[2], q.inv[2], -q.p[2]), b2 = fmaf(hi[2], q.inv[2], -q.p[2]);
  tl = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), tmin32));
#if defined(__HIP_DEVICE_COMPILE__)
  // min(x, cl32) as v_min3_f32 in asm: cl32 is a loop-carried value the
  // compiler cannot prove canonical, so fminf re-canonicalised it (one v_max)
  // at every node visit; both operands are the results of float operations
  float th;
  const float m01 = fminf(fmaxf(a0, b0), fmaxf(a1, b1));
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(th) : "v"(fmaxf(a2, b2)), "v"(cl32), "v"(m01));
#else
  const float th = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), cl32));
#endif
  return tl <= fmaf(th, kSlabGrow, q.slack);
}
// Both children of a binary node (slab_hit each).  As six packed fp32 FMAs
// (v_pk_fma_f32 on the child-interleaved planes) the visit is 5 VALU shorter
// but the persistent instance spills 3 more VGPRs: C3 -2.1 % (r03k_ab.log).
RT_HD RT_FI void slab_hit2(const RayF<true> &q, const DNode &N, float tmin32, float cl32, float &t0,
                           float &t1, bool &h0, bool &h1) {
  const float lo0[3] = {N.lo[0][0], N.lo[1][0], N.lo[2][0]}, hi0[3] = {N.hi[0][0], N.hi[1][0], N.hi[2][0]};
  const float lo1[3] = {N.lo[0][1], N.lo[1][1], N.lo[2][1]}, hi1[3] = {N.hi[0][1], N.hi[1][1], N.hi[2][1]};
  h0 = slab_hit(q, lo0, hi0, tmin32, cl32, t0);
  h1 = slab_hit(q, lo1, hi1, tmin32, cl32, t1);
}
// Node planes picked by the ray's direction signs -- the
// binary walk over a fully staged tree (C3: +8 %, C5: +8 %, profiles/
// r04b_slab_sign_ab.log) and every 4-wide visit (100k / 1M spheres +10 %,
// r04c_arity_sign_ab.log): for an axis with 1/d >= 0 the lo plane
// gives the entry distance and the hi plane the exit, the other way round for
// 1/d < 0 -- fma(plane, 1/d, -P) is monotone in the plane for a fixed 1/d, and
// every operand is finite (1/d and P are clamped, ray_f32), so min / max of
// the two plane distances ARE these picks, value for value.  Each lane reads
// its near and far plane pairs (both children, 8 B) at per-ray byte offsets
// `po` into the node (lo[a][*] at 8a, hi[a][*] at 24 + 8a): six 8-B LDS reads
// instead of the twelve planes, and no min / max per plane pair -- the visit
// drops from 36 to 24 slab VALU plus the six read addresses.
struct PlaneOff { // per-ray byte offsets of the near planes of each axis in a DNode / DNode4
  int n[3];
};
// W: children per node (2: DNode, lo[a][*] at 8a, hi at 24 + 8a; 4: DNode4,
// lo[a][*] at 16a, hi at 48 + 16a); the far planes are at 2 W 4 a + 3 W 4 - n
template <int W>
RT_HD RT_FI PlaneOff plane_offsets(const RayF<true> &q) {
  PlaneOff o;
#pragma unroll
  for (int a = 0; a < 3; ++a) o.n[a] = 4 * W * a + (q.inv[a] < 0.0f ? 12 * W : 0);
  return o;
}
// in a DNodeL (binary nodes staged in LDS, rt_layout.h): the near pair at
// 24 a + 8 s_a, the far pair 8 B after it
RT_HD RT_FI PlaneOff plane_offsets_l(const RayF<true> &q) {
  PlaneOff o;
#pragma unroll
  for (int a = 0; a < 3; ++a) o.n[a] = 24 * a + (q.inv[a] < 0.0f ? 8 : 0);
  return o;
}
template <int W>
RT_HD RT_FI int far_offset(const PlaneOff &po, int a) { return 8 * W * a + 12 * W - po.n[a]; }
RT_HD RT_FI float max3f(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return fmaxf(fmaxf(a, b), c);
#endif
}
RT_HD RT_FI float min3f(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return fminf(fminf(a, b), c);
#endif
}
// One node's sign-picked planes and child entries, read through a byte
// pointer into the LDS copy (PS = const RT_LDS char *) or into the node table
// in memory (const char *): a lane's node may be staged or not; the loads
// differ by address space, the slab math after them is shared, so lanes that
// diverge on staging repeat only the loads (W = 2: DNode, W = 4: DNode4).
template <int W>
struct NodePlanes {
  float nr[3][W], fr[3][W]; // near / far plane of each axis, per child
  int en[W];
};
template <class T, class PS>
RT_HD RT_FI T load_at(PS b, int off) { // a T at byte offset off, in b's address space
  T v;
  __builtin_memcpy(&v, b + off, sizeof(T));
  return v;
}
// (base: the wave-uniform start of the LDS copy or of the table, node: the
// lane's node byte offset -- a 32-bit per-lane offset from a scalar base)
template <int W, class PS>
RT_HD RT_FI void load_planes(NodePlanes<W> &pl, PS base, int node, const PlaneOff &po) {
  struct E {
    int e[W];
  };
  struct P {
    float f[W];
  };
  // the child entries first (at 48 in a DNode, 96 in a DNode4): their latency
  // overlaps the plane reads and the slab math
  const E e = load_at<E>(base, node + 24 * W);
#pragma unroll
  for (int c = 0; c < W; ++c) pl.en[c] = e.e[c];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const P n = load_at<P>(base, node + po.n[a]), f = load_at<P>(base, node + far_offset<W>(po, a));
#pragma unroll
    for (int c = 0; c < W; ++c) {
      pl.nr[a][c] = n.f[c];
      pl.fr[a][c] = f.f[c];
    }
  }
}
// The same from a DNodeL in LDS: per axis the near and far pairs as one 16-B
// read (ds_read2_b64), the entries at 72
template <class PS>
RT_HD RT_FI void load_planes_l(NodePlanes<2> &pl, PS base, int node, const PlaneOff &po) {
  struct E {
    int e[2];
  };
  struct P {
    float n[2], f[2];
  };
#if defined(__HIP_DEVICE_COMPILE__)
  // DNodeL offsets are multiples of 80 (the copy is 16-B aligned), the pair
  // offsets of 8: each axis read is an 8-B aligned ds_read2_b64 (not an
  // unaligned ds_read_b128)
  __builtin_assume((node & 15) == 0);
#endif
  const E e = load_at<E>(base, node + 72);
  pl.en[0] = e.e[0];
  pl.en[1] = e.e[1];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_assume((po.n[a] & 7) == 0);
#endif
    const P v = load_at<P>(base, node + po.n[a]);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      pl.nr[a][c] = v.n[c];
      pl.fr[a][c] = v.f[c];
    }
  }
}
// Both children of a binary node from their picked planes, verdicts returned
// as two bools (an array of them made the compiler build the visit's branch
// masks with VALU selects: C3 -1.6 %, profiles/r04g_c3_build_ab.log)
#ifndef RT_PK_SLAB
#define RT_PK_SLAB 0
#endif
RT_HD RT_FI void slab2_planes(const RayF<true> &q, const NodePlanes<2> &pl, float tmin32, float cl32,
                              float &t0, float &t1, bool &h0, bool &h1) {
  float th[2];
  float tl[2];
#if defined(__HIP_DEVICE_COMPILE__) && RT_PK_SLAB
  // both children's plane of an axis in one v_pk_fma_f32 (the pair the
  // DNodeL read puts in adjacent registers): the same fma per plane, half
  // the instructions
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 n[3], f[3];
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {
    const f2 inv = {q.inv[ax], q.inv[ax]}, mp = {-q.p[ax], -q.p[ax]};
    n[ax] = __builtin_elementwise_fma(f2{pl.nr[ax][0], pl.nr[ax][1]}, inv, mp);
    f[ax] = __builtin_elementwise_fma(f2{pl.fr[ax][0], pl.fr[ax][1]}, inv, mp);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    tl[c] = max3f(n[0][c], n[1][c], fmaxf(n[2][c], tmin32));
    th[c] = min3f(f[0][c], f[1][c], min3f(f[2][c], cl32, cl32));
  }
#else
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float ax = fmaf(pl.nr[0][c], q.inv[0], -q.p[0]), bx = fmaf(pl.fr[0][c], q.inv[0], -q.p[0]);
    const float ay = fmaf(pl.nr[1][c], q.inv[1], -q.p[1]), by = fmaf(pl.fr[1][c], q.inv[1], -q.p[1]);
    const float az = fmaf(pl.nr[2][c], q.inv[2], -q.p[2]), bz = fmaf(pl.fr[2][c], q.inv[2], -q.p[2]);
    tl[c] = max3f(ax, ay, fmaxf(az, tmin32));
    th[c] = min3f(bx, by, min3f(bz, cl32, cl32));
  }
#endif
  t0 = tl[0];
  t1 = tl[1];
  h0 = tl[0] <= fmaf(th[0], kSlabGrow, q.slack);
  h1 = tl[1] <= fmaf(th[1], kSlabGrow, q.slack);
}
// The slab verdicts and entry distances of the W children from their planes.
template <int W>
RT_HD RT_FI void slab_planes(const RayF<true> &q, const NodePlanes<W> &pl, float tmin32, float cl32,
                             float tl[W], bool hit[W]) {
#pragma unroll
  for (int c = 0; c < W; ++c) {
    const float ax = fmaf(pl.nr[0][c], q.inv[0], -q.p[0]), bx = fmaf(pl.fr[0][c], q.inv[0], -q.p[0]);
    const float ay = fmaf(pl.nr[1][c], q.inv[1], -q.p[1]), by = fmaf(pl.fr[1][c], q.inv[1], -q.p[1]);
    const float az = fmaf(pl.nr[2][c], q.inv[2], -q.p[2]), bz = fmaf(pl.fr[2][c], q.inv[2], -q.p[2]);
    tl[c] = max3f(ax, ay, fmaxf(az, tmin32));
    const float th = min3f(bx, by, min3f(bz, cl32, cl32));
    hit[c] = tl[c] <= fmaf(th, kSlabGrow, q.slack);
  }
}
// f32_up(x) as a canonical float (the min/max operations take it as is
// instead of re-canonicalising it at every box test)
RT_HD RT_FI float f32_up_c(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_canonicalizef(f32_up(x));
#else
  return f32_up(x);
#endif
}

// Per-wave LDS scratch of the compacted leaf tests (trace, leaf_share): the
// round's (item << 6 | owner lane) table and each owner's running closest t
// (as order-preserving bits: every t is positive), its tie key and its item.
struct LeafPool {
  unsigned long long bt[64];
  int bk[64]; // tie key of the owner's current hit (leaf_share)
  int bi[64];
  int tab[64];
};
// Which instances compact their leaf tests across the wave (BVH walks only; a
// flat world's items are wave-uniform already).  Off in the product build:
// measured C3 -11 % (-19 % when every leaf phase compacts), since moving a ray
// between lanes (9 doubles through ds_bpermute) plus the LDS merge costs about
// as much as the sphere test it saves, and leaf-phase lane use rose only
// 0.39 -> 0.52 (profiles/r02y_*, r02z_*).  Built as the variant
// build/variants/librtx_hip_leafshare.so, parity-tested on the GPU
// (tests/test_leaf_share.py).
#ifndef RT_LEAF_SHARE
#define RT_LEAF_SHARE 0
#endif
#ifndef RT_LEAF_SHARE_F
#define RT_LEAF_SHARE_F(F) (RT_LEAF_SHARE != 0 && ((F) & F_FLAT) == 0)
#endif

struct Counters {
  uint32_t nodes, spheres, quads, other, light, shade;
  uint32_t wnode, wleaf, wshade; // wave-level iterations (counted by one lane per wave)
  uint64_t ctrace, cmedia, cshade, clights; // wave-level cycles (first active lane adds)
  uint32_t noise, wnoise; // noise-texture albedo evaluations: lanes, wave executions
  uint32_t mbox, mbox_fb; // box-boundary medium tests: lanes, lanes box_span deferred
};
// shader clock for the STATS instance's phase cycles (s_memtime)
RT_HD RT_FI uint64_t clk() {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_readcyclecounter();
#else
  return 0;
#endif
}
// true when no active lane of the wavefront has `pred` (a single-lane host build: !pred)
RT_HD RT_FI bool wave_none(bool pred) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(pred) == 0;
#else
  return !pred;
#endif
}
// STATS only: 1 on the first active lane of the wavefront, else 0 (wave-level counts)
RT_HD RT_FI uint32_t wave_once() {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)(__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id()));
#else
  return 1u;
#endif
}

// World items and spheres staged in LDS by the persistent instance (one
// 16-wave block per CU owns the CU's LDS: C3's whole scene -- 485 nodes, 486
// items, 486 spheres -- fits beside the traversal stacks).  items == nullptr:
// nothing staged, every load goes to the scene tables in HBM / L2.
struct LdsPrims {
  const RT_LDS DItem *items;
  const RT_LDS DSphere *spheres;
};
template <bool LP>
RT_HD RT_FI DItem load_item(const DScene &S, const LdsPrims &lp, int i) {
  if constexpr (LP) {
    if (lp.items != nullptr) {
      const RT_LDS DItem &L = lp.items[i];
      DItem d;
      d.kind = L.kind;
      d.idx = L.idx;
      d.xf_first = L.xf_first;
      d.xf_count = L.xf_count;
      d.mat = L.mat;
      d.id = L.id;
      d.pad[0] = d.pad[1] = 0;
      return d;
    }
  }
  return S.items[i];
}
template <bool LP>
RT_HD RT_FI DSphere load_sphere(const DScene &S, const LdsPrims &lp, int i) {
  if constexpr (LP) {
    if (lp.items != nullptr) {
      const RT_LDS DSphere &L = lp.spheres[i];
      DSphere d;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        d.c0[k] = L.c0[k];
        d.dir[k] = L.dir[k];
      }
      d.inv_r = L.inv_r;
      d.rr = L.rr;
      return d;
    }
  }
  return S.spheres[i];
}

// The end of a closest-hit query: constant media tested against the final
// primitive distance `closest` (the closest hit is the minimum over items in any
// order, and a medium's free-flight draw is keyed by its id, not by visiting
// order -- keeps the medium code out of the traversal loop's register budget),
// then the hit record of the winning item, built once.
template <bool STATS, unsigned F, bool LP = false>
RT_HD RT_FI bool trace_tail(const DScene &S, const Ray &r, Hit &h, const Key &key,
                                           uint32_t bounce, double closest, int best,
                                           Counters &cnt, const LdsPrims &lp = LdsPrims{}) {
  const double tmin = 0.001;
  constexpr bool kFlat = (F & F_FLAT) != 0;
  const bool moving = kFlat ? !S.static_spheres : true;
  bool best_full = false;
  if constexpr ((F & F_MEDIA) != 0) {
    const uint64_t t0 = STATS ? clk() : 0;
    constexpr bool kFma = !kFlat;
    const RayF<kFma> q = ray_f32<kFma>(r);
    const float tmin32 = f32_dn(tmin);
    float cl32 = f32_up(closest);
    int best_m = -1;
    for (int m = 0; m < S.n_mitems; ++m) {
      if (slab(q, S.mbox + 6 * m, S.mbox + 6 * m + 3, tmin32, cl32) == __builtin_huge_valf())
        continue;
      if (STATS) cnt.other++;
      double tm_hit;
      int box_path;
      const bool mh = medium_t<RT_KB_F(F)>(S, S.mitems[m], r, tmin, closest, key, bounce, tm_hit, box_path);
      if (STATS) {
        cnt.mbox += box_path >= 0;
        cnt.mbox_fb += box_path == 0;
      }
      if (mh) {
        closest = tm_hit;
        cl32 = f32_up(closest);
        best_m = m;
      }
    }
    if (best_m >= 0) {
      medium_record(S, S.mitems[best_m], r, closest, h);
      best = best_m;
      best_full = true;
    }
    if (STATS && wave_once()) cnt.cmedia += clk() - t0;
  }
  if (best < 0) return false;
  if (!best_full) {
    const DItem it = load_item<LP>(S, lp, best);
    Ray lr = r;
    if constexpr ((F & F_XFORM) != 0) {
      if (it.xf_count) lr = to_local(S, it.xf_first, it.xf_count, r);
    }
    if (it.kind == I_SPHERE)
      sphere_record(load_sphere<LP>(S, lp, it.idx), lr, closest, it.mat, h, moving);
    else
      quad_record(S.quads[it.idx], lr, closest, it.mat, h);
    if constexpr ((F & F_XFORM) != 0) {
      if (it.xf_count) to_world(S, it.xf_first, it.xf_count, h);
    }
  }
  return true;
}

// Stack entry: >= 0 inner node; < 0 a leaf ~(first << 3 | count) (DNode::entry).

// Closest hit over the world BVH.  Primitive items record only (t, item) during
// traversal and build the hit record once at the end; media build theirs when hit.
// `lnodes` is the LDS copy of nodes [0, S.n_lds_nodes): DNode4 for 4-wide trees,
// DNodeL for binary ones (the host emulator passes the same forms
// of the whole tree).
template <bool STATS, unsigned F, bool LP = false>
RT_HD RT_FI bool trace(const DScene &S, const Ray &r, Hit &h, const Key &key,
                                      uint32_t bounce, int *stk, const RT_LDS DNode *lnodes,
                                      Counters &cnt, RT_LDS LeafPool *pool = nullptr,
                                      const LdsPrims &lp = LdsPrims{}) {
  const double tmin = 0.001; // Camera.cpp:242
  double closest = kInf;
  int best = -1;
  const double a = len2(r.d);
  const double ya = 1.0 / a; // one reciprocal per ray for every sphere root
  // F_FLAT instances (small worlds, SAH root is one leaf) have no BVH walk; they
  // need the fp32 slab constants only for the medium box cull, and they skip
  // the center.at(time) arithmetic when no sphere moves (a wave-uniform flag).
  constexpr bool kFlat = (F & F_FLAT) != 0;
  constexpr bool kBoxes = !kFlat || (F & F_MEDIA) != 0;
  const bool moving = kFlat ? !S.static_spheres : true;
  constexpr bool kFma = !kFlat;
  RayF<kFma> q{};
  float tmin32 = 0.0f;
  float cl32 = __builtin_huge_valf(); // f32_up(closest)
  if constexpr (kBoxes) {
    q = ray_f32<kFma>(r);
    tmin32 = f32_dn(tmin);
  }

  // hit test of world item ii against ray rr (|d|^2 = ra, its reciprocal ry)
  // in (tmin, tmax): the root in t
  // (uniform: UTag<true> where ii is the same in every lane -- the flat walk)
  auto item_root_t = [&](auto uniform, int ii, const Ray &rr, double ra, double ry, double tmax,
                         double &t) -> bool {
    constexpr bool U = decltype(uniform)::value && RT_UNIFORM_LOADS_F(F);
    const DItem it = U ? ldu<U>(S.items, ii) : load_item<LP>(S, lp, ii);
    Ray lr = rr;
    double al = ra;
    bool local = false;
    if constexpr ((F & F_XFORM) != 0) {
      if (it.xf_count) {
        lr = to_local<U>(S, it.xf_first, it.xf_count, rr);
        al = len2(lr.d);
        local = true;
      }
    }
    if (it.kind == I_SPHERE) {
      if (STATS) cnt.spheres++;
      // a local ray has its own |d|^2 and so its own reciprocal (a value, not
      // a pointer to one of two locals: that pointer kept ya in scratch memory)
      const double yl = local ? 1.0 / al : ry;
      return sphere_root(U ? ldu<U>(S.spheres, it.idx) : load_sphere<LP>(S, lp, it.idx), lr, al,
                         tmin, tmax, t, moving, true, yl);
    }
    if (STATS) cnt.quads++;
    constexpr bool UA = decltype(uniform)::value; // the flat walk: the same quad in every lane
    if constexpr (U) return quad_t<true, UA>(ldu<true>(S.quads, it.idx), lr, tmin, tmax, t);
    return quad_t<false, UA>(S.quads[it.idx], lr, tmin, tmax, t);
  };
  [[maybe_unused]] auto item_root = [&](int ii, const Ray &rr, double ra, double ry, double tmax,
                                        double &t) -> bool {
    return item_root_t(UTag<false>{}, ii, rr, ra, ry, tmax, t);
  };
  // closest-hit test of one world item (records only t and the item index)
  auto test_item = [&](auto uniform, int ii) {
    if (STATS) cnt.wleaf += wave_once();
    double t;
    const bool hit = item_root_t(uniform, ii, r, a, ya, closest, t);
    if (hit) {
      closest = t;
      if constexpr (kBoxes) cl32 = f32_up_c(closest);
      best = ii;
    }
  };

  [[maybe_unused]] constexpr bool kShare = RT_LEAF_SHARE_F(F);
#if defined(__HIP_DEVICE_COMPILE__)
  // Leaf tests compacted with ballot + ds_bpermute: the lanes' parked leaves
  // (ln items from lf) are numbered by a ballot prefix sum; each round, every
  // lane of the query takes the next item number, reads (item, owner) from the
  // wave's LDS table, borrows the owner's ray with ds_bpermute and tests it
  // against the owner's current bound; hits are merged per owner in LDS.  The
  // merge reproduces the per-lane loop over the leaf exactly: the smallest t
  // wins, and among equal t the loop's replacement rules decide -- a sphere
  // replaces the closest hit only on t < closest (Sphere.cpp), a quad also on
  // t == closest (Plane.cpp's closed interval) -- so the winner is the last
  // quad in item order at that t, else the first sphere, and a quad at the
  // previous closest t replaces the previous hit while a sphere does not.
  // Tie keys: quad 2^26-1-item < previous hit 2^26 < sphere 2^26+1+item.
  auto leaf_share = [&](int &ln_, int &lf_) {
    constexpr int kPrev = 1 << 26;
    const int lane = (int)__lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t ex = __ballot(1);
    int pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) { // counts are <= 7 (3-bit leaf field)
      const uint64_t m = __ballot((ln_ >> b) & 1);
      pre += __popcll(m & below) << b;
      tot += __popcll(m) << b;
    }
    const int nx = __popcll(ex), rk = __popcll(ex & below);
    unsigned long long cbits = (unsigned long long)__double_as_longlong(closest);
    int ckey = kPrev;
    pool->bt[lane] = cbits;
    pool->bk[lane] = kPrev;
    for (int base = 0; base < tot; base += nx) {
      if (STATS) cnt.wleaf += wave_once();
      for (int k = base > pre ? base - pre : 0; k < ln_ && pre + k < base + nx; ++k)
        pool->tab[pre + k - base] = ((lf_ + k) << 6) | lane;
      __builtin_amdgcn_wave_barrier();
      const int w = base + rk;
      int o = lane, ii = 0;
      if (w < tot) {
        const int e = pool->tab[rk];
        o = e & 63;
        ii = e >> 6;
      }
      Ray ro;
      ro.o = v3(__shfl(r.o.x, o), __shfl(r.o.y, o), __shfl(r.o.z, o));
      ro.d = v3(__shfl(r.d.x, o), __shfl(r.d.y, o), __shfl(r.d.z, o));
      ro.tm = __shfl(r.tm, o);
      const double ra = __shfl(a, o), ry = __shfl(ya, o);
      bool hit = false;
      double t = 0.0;
      unsigned long long tb = 0;
      int key = 0;
      if (w < tot) {
        const double tmax = __longlong_as_double((long long)pool->bt[o]);
        hit = item_root(ii, ro, ra, ry, tmax, t);
        tb = (unsigned long long)__double_as_longlong(t);
        key = S.items[ii].kind == I_SPHERE ? kPrev + 1 + ii : kPrev - 1 - ii;
        if (hit)
          __hip_atomic_fetch_min(&pool->bt[o], tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
      __builtin_amdgcn_wave_barrier();
      // a new closest t: the previous hit's key no longer competes
      if (pool->bt[lane] != cbits) pool->bk[lane] = 0x7fffffff;
      __builtin_amdgcn_wave_barrier();
      const bool at_min = hit && pool->bt[o] == tb;
      if (at_min)
        __hip_atomic_fetch_min(&pool->bk[o], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      __builtin_amdgcn_wave_barrier();
      if (at_min && pool->bk[o] == key) pool->bi[o] = ii; // keys are unique per item
      __builtin_amdgcn_wave_barrier();
      const unsigned long long nb = pool->bt[lane];
      const int nk = pool->bk[lane];
      if (nb != cbits || nk != ckey) {
        cbits = nb;
        ckey = nk;
        closest = __longlong_as_double((long long)nb);
        best = pool->bi[lane];
        if constexpr (kBoxes) cl32 = f32_up_c(closest);
      }
      __builtin_amdgcn_wave_barrier();
    }
    lf_ += ln_;
    ln_ = 0;
  };
#endif

  if constexpr (kFlat) {
    // the reference's HittableList walk (HittableList.cpp), wave-uniform items
    for (int ii = 0; ii < S.n_root_items; ++ii) test_item(UTag<true>{}, ii);
  } else {
    // Speculative while-while traversal (Aila & Laine 2009, "postponed leaves"):
    // a lane that reaches its first leaf parks it in (lf, ln) and keeps walking
    // its stack; the wave leaves the node loop only once every lane still walking
    // holds a leaf (or has finished), so node-loop slots that lanes with a leaf
    // would otherwise idle through do useful visits.  Stack pops happen eagerly
    // inside the visiting iteration (no separate pop iterations).  Entries: >= 0
    // inner node, -1 none (stack empty: done after the parked leaf), <= -2 a leaf
    // ~(first << 3 | count) (count >= 1).  Visiting order only changes how much
    // the closest-hit bound culls, never the closest hit.
    // The stack as a pointer to the next free entry (stk[64 k]: this lane's
    // k-th entry): a push is a store and one add, a pop one add and a load --
    // no sp * 256 address arithmetic per access.  No overflow guard: the host
    // sizes S.stack_depth to what the walk can push -- one entry per level of
    // the binary tree (a pushed entry is the sibling of a node on the current
    // root path), three per 4-wide level -- plus one, from the depth of the
    // tree it built (a per-push check measured C3 -2.3 %, profiles/r03h_ab.log).
    int *top = stk;
    auto push = [&](int e) {
      *top = e;
      top += 64;
    };
    auto pop = [&]() -> int {
      if (top == stk) return -1;
      top -= 64;
      return *top;
    };
    [[maybe_unused]] PlaneOff po{};
    if constexpr (kFma)
      po = (F & F_BVH4) == 0 ? plane_offsets_l(q) : plane_offsets<(F & F_BVH4) ? 4 : 2>(q);
    int cur;
    int lf = 0, ln = 0;
    if (S.root_is_leaf) {
      cur = -1;
      ln = S.n_root_items;
    } else {
      cur = 0;
    }
    for (;;) {
      if constexpr ((F & F_BVH4) != 0) {
        // 4-wide node: four slab tests, the hits sorted near to far by a
        // 5-comparator network, the far ones pushed (farthest first), the
        // nearest walked next -- the binary walk's near-first order per level
        const RT_LDS DNode4 *lnodes4 = (const RT_LDS DNode4 *)lnodes;
        const DNode4 *nodes4 = (const DNode4 *)S.nodes;
        while (cur >= 0) {
          if (STATS) cnt.wnode += wave_once();
          if (wave_none(ln == 0)) break;
          if (STATS) cnt.nodes++;
          float tn[4];
          int en[4];
          if constexpr (kFma) {
            NodePlanes<4> pl;
            if (cur < S.n_lds_nodes)
              load_planes<4>(pl, (const RT_LDS char *)lnodes4, cur * (int)sizeof(DNode4), po);
            else
              load_planes<4>(pl, (const char *)nodes4, cur * (int)sizeof(DNode4), po);
            bool hh[4];
            slab_planes<4>(q, pl, tmin32, cl32, tn, hh);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              en[c] = pl.en[c];
              if (en[c] == -1 || !hh[c]) tn[c] = __builtin_huge_valf();
            }
          } else {
            DNode4 N;
            if (cur < S.n_lds_nodes) {
              const RT_LDS DNode4 &L = lnodes4[cur];
#pragma unroll
              for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                  N.lo[a][c] = L.lo[a][c];
                  N.hi[a][c] = L.hi[a][c];
                }
#pragma unroll
              for (int c = 0; c < 4; ++c) N.entry[c] = L.entry[c];
            } else {
              N = nodes4[cur];
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float lo[3] = {N.lo[0][c], N.lo[1][c], N.lo[2][c]};
              const float hi[3] = {N.hi[0][c], N.hi[1][c], N.hi[2][c]};
              en[c] = N.entry[c];
              tn[c] = en[c] == -1 ? __builtin_huge_valf() : slab(q, lo, hi, tmin32, cl32);
            }
          }
          auto cswap = [&](int x, int y) {
            const bool sw = tn[y] < tn[x];
            const float tx = tn[x], ty = tn[y];
            const int ex = en[x], ey = en[y];
            tn[x] = sw ? ty : tx;
            tn[y] = sw ? tx : ty;
            en[x] = sw ? ey : ex;
            en[y] = sw ? ex : ey;
          };
          cswap(0, 1);
          cswap(2, 3);
          cswap(0, 2);
          cswap(1, 3);
          cswap(1, 2);
#pragma unroll
          for (int c = 3; c >= 1; --c)
            if (tn[c] != __builtin_huge_valf()) push(en[c]);
          cur = tn[0] != __builtin_huge_valf() ? en[0] : pop();
          if (cur < -1 && ln == 0) { // first leaf: park it, keep walking
            lf = (~cur) >> 3;
            ln = (~cur) & 7;
            cur = pop();
          }
        }
      } else {
        // the binary walk; LDS_ONLY: every node is staged (a wave-uniform
        // property of the scene and launch, so the loop is entered in one of
        // two forms and the per-visit LDS / HBM branch is gone when the whole
        // tree is in LDS -- C3's persistent instance)
        auto walk = [&](auto lds_only) {
          constexpr bool LDS_ONLY = decltype(lds_only)::value;
          while (cur >= 0) {
            if (STATS) cnt.wnode += wave_once();
            if (wave_none(ln == 0)) break; // every walking lane holds a leaf: test them
            if (STATS) cnt.nodes++;
            float tn0, tn1;
            bool h0, h1;
            int e0, e1;
            if constexpr (kFma && LDS_ONLY) {
              // the whole tree staged: sign-picked planes from LDS.  (From the
              // node table in memory the six 8-B loads instead of four 16-B
              // ones lost 14-17 % on 100k-1M spheres, and a per-lane choice
              // between the two forms runs both slab passes in a mixed wave:
              // -6.5 %, profiles/r04b_arity_sign_ab.log, r04c_arity_sign_ab.log.)
              NodePlanes<2> pl;
              load_planes_l(pl, (const RT_LDS char *)lnodes, cur, po); // cur: the node's byte offset (entries staged so)
              slab2_planes(q, pl, tmin32, cl32, tn0, tn1, h0, h1);
              e0 = pl.en[0];
              e1 = pl.en[1];
            } else {
              DNode N;
              if (cur < S.n_lds_nodes) {
                const RT_LDS DNodeL &L = ((const RT_LDS DNodeL *)lnodes)[cur];
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                  for (int k = 0; k < 2; ++k) {
                    N.lo[a][k] = L.p[a][0][k];
                    N.hi[a][k] = L.p[a][1][k];
                  }
                N.entry[0] = L.entry[0];
                N.entry[1] = L.entry[1];
              } else {
                N = S.nodes[cur];
              }
              slab_hit2(q, N, tmin32, cl32, tn0, tn1, h0, h1);
              e0 = N.entry[0];
              e1 = N.entry[1];
            }
            if (h0 && h1) {
              const bool first0 = tn0 <= tn1;
              push(first0 ? e1 : e0);
              cur = first0 ? e0 : e1;
            } else if (h0 || h1) {
              cur = h0 ? e0 : e1;
            } else {
              cur = pop();
            }
            if (cur < -1 && ln == 0) { // first leaf: park it, keep walking
              lf = (~cur) >> 3;
              ln = (~cur) & 7;
              cur = pop();
            }
          }
        };
        if (kFma && S.n_lds_nodes >= S.n_nodes)
          walk(UTag<true>{});
        else
          walk(UTag<false>{});
      }
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (kShare) {
        // ---- the single leaf-test site, compacted across the wave: every
        // lane of the query (finished walks included) tests one of the wave's
        // parked leaf items per round instead of its own leaf's items in turn
        if (__ballot(ln > 0) == 0) break; // no lane holds a leaf: all walks done
        // compact only when it takes fewer rounds than the per-lane loop's
        // max(ln) trips (each round also moves rays between lanes)
        int mx = 1;
#pragma unroll
        for (int k = 2; k <= 7; ++k)
          if (__ballot(ln >= k) != 0) mx = k;
        int tot = 0;
#pragma unroll
        for (int b = 0; b < 3; ++b) tot += __popcll(__ballot((ln >> b) & 1)) << b;
        const int nx = __popcll(__ballot(1));
        if ((tot + nx - 1) / nx < mx) {
          leaf_share(ln, lf);
        } else {
          while (ln > 0) {
            const int ii = lf;
            ++lf;
            --ln;
            test_item(UTag<false>{}, ii);
          }
        }
      } else
#endif
      {
        if (ln == 0) break; // nothing parked and nothing left to walk: done
        while (ln > 0) { // ---- the single leaf-test site
          const int ii = lf;
          ++lf;
          --ln;
          test_item(UTag<false>{}, ii);
        }
      }
      if (cur < -1) { // a second leaf met while one was parked: it is next
        lf = (~cur) >> 3;
        ln = (~cur) & 7;
        cur = pop();
      }
    }
  }
  return trace_tail<STATS, F, LP>(S, r, h, key, bounce, closest, best, cnt, lp);
}

// ------------------------------------------------------------ lights
// Sum over light leaves of weight * pdf_value (Plane.cpp:115-126, Sphere.cpp:145-158).
template <bool STATS>
RT_HD double lights_pdf(const DScene &S, V3 org, V3 dir, Counters &cnt) {
  double sum = 0.0;
  for (int i = 0; i < S.n_lights; ++i) {
    const DLight L = S.lights[i];
    Ray lr = to_local(S, L.xf_first, L.xf_count, Ray{org, dir, 0.0});
    double p = 0.0;
    if (L.kind == I_SPHERE) {
      if (STATS) cnt.light++;
      const DSphere &s = S.spheres[L.idx];
      double t;
      if (sphere_root(s, lr, len2(lr.d), 0.001, kInf, t)) {
        V3 c0 = v3(s.c0[0] + 0 * s.dir[0], s.c0[1] + 0 * s.dir[1], s.c0[2] + 0 * s.dir[2]);
        double dist2 = len2(c0 - lr.o);
        double ctm = sqrt(1 - s.rr / dist2);
        double sa = 2 * kPi * (1 - ctm);
        p = 1 / sa;
      }
    } else if (L.kind == I_QUAD) {
      if (STATS) cnt.light++;
      const DQuad &q = S.quads[L.idx];
      double t;
      if (quad_t<false, true>(q, lr, 0.001, kInf, t)) { // the same light in every lane
        V3 n = ld3(q.n);
        V3 fn = dot(lr.d, n) < 0 ? n : -n;
        double d2 = t * t * len2(lr.d);
        double cosine = fabs(dot(lr.d, fn) / sqrt(len2(lr.d)));
        p = d2 / (cosine * q.area);
      }
    }
    sum += L.weight * p;
  }
  return sum;
}

// SC: sincos(2 pi r1) arrives precomputed in (sp1, cp1) -- the caller's one
// sincos shared with the other shading branches (shade, kSc)
template <int KC = 0, bool SC = false>
RT_HD V3 lights_random(const DScene &S, V3 org, double upick, double r1, double r2,
                       double sp1 = 0.0, double cp1 = 0.0) {
  int k = S.n_lights - 1;
  for (int i = 0; i < S.n_lights; ++i)
    if (upick < S.lights[i].cum) {
      k = i;
      break;
    }
  const DLight L = S.lights[k];
  V3 p = to_local(S, L.xf_first, L.xf_count, Ray{org, v3(0, 0, 0), 0.0}).o;
  V3 d;
  if (L.kind == I_SPHERE) { // Sphere::random, Sphere.cpp:160-178
    const DSphere &s = S.spheres[L.idx];
    V3 c0 = v3(s.c0[0] + 0 * s.dir[0], s.c0[1] + 0 * s.dir[1], s.c0[2] + 0 * s.dir[2]);
    V3 dir = c0 - p;
    double d2 = len2(dir);
    V3 w = unitv(dir);
    V3 a = (fabs(w.x) > 0.9) ? v3(0, 1, 0) : v3(1, 0, 0);
    V3 vv = unitv(cross(w, a));
    V3 uu = cross(w, vv);
    double z = 1 + r2 * (sqrt(1 - s.rr / d2) - 1);
    double sphi = sp1, cphi = cp1;
    if constexpr (!SC) sincos_2pi<KC>(r1, sphi, cphi);
    double x = cphi * sqrt(1 - z * z);
    double y = sphi * sqrt(1 - z * z);
    d = ((x * uu) + (y * vv)) + (z * w);
  } else if (L.kind == I_QUAD) { // Plane::random, Plane.cpp:128-132
    const DQuad &q = S.quads[L.idx];
    V3 pt = (ld3(q.Q) + (r1 * ld3(q.u))) + (r2 * ld3(q.v));
    d = pt - p;
  } else {
    d = v3(1, 0, 0);
  }
  for (int c = L.xf_count - 1; c >= 0; --c) {
    const DXform X = S.xforms[L.xf_first + c];
    if (X.kind == X_ROTATE_Y) d = rot_out(X.a, X.b, d);
  }
  return d;
}

// ------------------------------------------------------------ integrator
struct PathState {
  Ray ray;
  V3 T; // throughput; when the path ends: its radiance (T x terminal value)
  uint32_t bounce;
  int slot;   // tile pixel slot 0..63
  int sample; // linear stratum index
  bool active;
};

// Continue to the next segment unless the depth budget is spent (ray_color at
// depth 0 returns 0, Camera.cpp:236-237; T * 0 keeps a NaN/inf weight alive).
RT_HD RT_FI bool advance(PathState &ps, const DCamera &C) {
  ps.bounce++;
  if ((int)ps.bounce >= C.max_depth) {
    ps.T = ps.T * v3(0.0, 0.0, 0.0);
    return false;
  }
  return true;
}

// One segment of Camera::ray_color in forward (throughput) form.  Returns false
// when the path ends; its radiance is then in ps.T.  The recursion's
// L = e + a*L' sums emission only where a path ends (lights never scatter), so the
// forward form needs no radiance register: the terminal T x value is the sample.
// The material half of a segment, after the closest hit `h` of ps.ray.
// Measured (profiles/r02w_shade_merge_ab.log): C3 (plain BVH instance, mixed
// Lambertian / metal / glass) +2 %; C2 (flat, Lambertian only: the selects are
// pure overhead) -2 %, C4 -1 % (more spills): merged in the plain BVH instances only.
// Re-measured on the round-6 build (profiles/r06am_*): C2 -2.9 %, C4 -2.4 %.
#define RT_SHADE_MERGE_F(F) (((F) & ~F_BVH4) == 0)
template <bool STATS, unsigned F>
RT_HD RT_FI bool shade(const DScene &S, const DCamera &C, PathState &ps, const Key &key,
                       const Hit &h, Counters &cnt) {
  const uint32_t b = ps.bounce;
  const DMat M = S.mats[h.mat];
  if (STATS) cnt.shade++;
  if (M.kind == RT_MAT_DIFFUSE_LIGHT) { // emits on the front face, never scatters
    if (STATS) cnt.wshade += wave_once();
    // Always add T * emitted (0 on the back face): a NaN/inf throughput must
    // poison the sample as the reference recursion does (NaN * 0 = NaN).
    V3 e = h.front ? tex_value<F>(S, M.tex, h.p) : v3(0.0, 0.0, 0.0);
    ps.T = ps.T * e;
    return false;
  }
  double rn[4]; // one block per shading event: (e0, e1, d0, d1)
  u01x4<RT_KB_F(F)>(key, b, kSlotShade, rn);
  const double e0 = rn[0], e1 = rn[1], d0 = rn[2], d1 = rn[3];
  const Ray &r = ps.ray;
  constexpr bool kMerge = RT_SHADE_MERGE_F(F);
  // Merged shading (kMerge): a wave whose lanes shade different materials
  // runs each material's branch; the expensive steps they have in common run
  // ONCE for all lanes here, each lane feeding its own operand -- the same
  // operations on the same values as in the per-material code below:
  //   unit vector: metal's reflection, the dielectric's ray, the ONB normal;
  //   sincos(2 pi a): metal / isotropic a = d1, Lambertian a = d0;
  //   first root: metal / isotropic 1 - z^2 (>= 0), Lambertian d1, dielectric
  //   1 - ct^2.
  V3 u1{};
  double sp1 = 0.0, cp1 = 0.0, s1 = 0.0, z1 = 0.0, ct1 = 0.0;
  if constexpr (kMerge) {
    const bool metal = M.kind == RT_MAT_METAL, diel = M.kind == RT_MAT_DIELECTRIC;
    const bool lamb = M.kind == RT_MAT_LAMBERTIAN;
    V3 x1 = diel ? r.d : h.n;
    if (metal) x1 = r.d - (2 * dot(r.d, h.n)) * h.n;
    u1 = unitv(x1);
    if (!diel) sincos_2pi<RT_KCONST_MODE(F)>(lamb ? d0 : d1, sp1, cp1);
    z1 = 1.0 - 2.0 * d0;
    if (diel) ct1 = fmin(dot(-u1, h.n), 1.0);
    s1 = sqrt_n(lamb ? d1 : (diel ? 1.0 - ct1 * ct1 : fmax(0.0, 1.0 - z1 * z1)));
  }
  if (kMerge && M.kind == RT_MAT_METAL) {
    if (STATS) cnt.wshade += wave_once();
    V3 uv = v3(s1 * cp1, s1 * sp1, z1);
    V3 refl = u1 + (M.fuzz * uv);
    ps.T = ps.T * ld3(M.albedo);
    ps.ray = Ray{h.p, refl, r.tm};
    return advance(ps, C);
  }
  if (kMerge && M.kind == RT_MAT_DIELECTRIC) {
    if (STATS) cnt.wshade += wave_once();
    double ri = h.front ? M.inv_ior : M.ior;
    const V3 ud = u1;
    const double ct = ct1, st = s1;
    bool reflect_it = ri * st > 1.0;
    if (!reflect_it) {
      const double r0 = h.front ? M.r0[0] : M.r0[1];
      double x = 1 - ct;
      double x2 = x * x;
      double refl = r0 + (1 - r0) * (x2 * x2 * x);
      reflect_it = refl > e0;
    }
    V3 dir;
    if (reflect_it) {
      dir = ud - (2 * dot(ud, h.n)) * h.n;
    } else {
      V3 perp = ri * (ud + ct * h.n);
      V3 par = (-sqrt_n(fabs(1.0 - len2(perp)))) * h.n;
      dir = perp + par;
    }
    ps.ray = Ray{h.p, dir, r.tm};
    return advance(ps, C);
  }
  if (!kMerge && M.kind == RT_MAT_METAL) { // MetalMaterial.cpp:43-62
    if (STATS) cnt.wshade += wave_once();
    V3 refl = r.d - (2 * dot(r.d, h.n)) * h.n;
    double z = 1.0 - 2.0 * d0;
    double rr = sqrt_n(fmax(0.0, 1.0 - z * z));
    double sp, cp;
    sincos_2pi<RT_KCONST_MODE(F)>(d1, sp, cp);
    V3 uv = v3(rr * cp, rr * sp, z);
    refl = unitv(refl) + (M.fuzz * uv);
    ps.T = ps.T * ld3(M.albedo);
    ps.ray = Ray{h.p, refl, r.tm};
    return advance(ps, C);
  }
  if (!kMerge && M.kind == RT_MAT_DIELECTRIC) { // DielectricMaterial.cpp:58-85
    if (STATS) cnt.wshade += wave_once();
    double ri = h.front ? M.inv_ior : M.ior; // 1/ior formed on the host
    V3 ud = unitv(r.d);
    double ct = fmin(dot(-ud, h.n), 1.0);
    double st = sqrt_n(1.0 - ct * ct);
    bool reflect_it = ri * st > 1.0;
    if (!reflect_it) {
      const double r0 = h.front ? M.r0[0] : M.r0[1]; // ((1 - ri) / (1 + ri))^2, host-formed
      double x = 1 - ct;
      double x2 = x * x;
      double refl = r0 + (1 - r0) * (x2 * x2 * x);
      reflect_it = refl > e0;
    }
    V3 dir;
    if (reflect_it) {
      dir = ud - (2 * dot(ud, h.n)) * h.n;
    } else {
      V3 perp = ri * (ud + ct * h.n);
      V3 par = (-sqrt_n(fabs(1.0 - len2(perp)))) * h.n;
      dir = perp + par;
    }
    ps.ray = Ray{h.p, dir, r.tm};
    return advance(ps, C);
  }
  // Lambertian (CosinePDF) or Isotropic (SpherePDF), mixed 50/50 with the lights
  const bool lamb = (M.kind == RT_MAT_LAMBERTIAN);
  if (STATS) cnt.wshade += wave_once();
  // albedo: fetched early when a noise texture may run (its long evaluation
  // overlaps less live state there), late otherwise (shorter live range)
  V3 att;
  if constexpr ((F & F_NOISE) != 0) {
    if (STATS && S.texs[M.tex].kind == RT_TEX_NOISE) {
      cnt.noise++;
      cnt.wnoise += wave_once();
    }
    att = tex_value<F>(S, M.tex, h.p);
  }
  V3 w = kMerge ? u1 : unitv(h.n); // ONB(n), ONB.hpp:25-37
  V3 a = (fabs(w.x) > 0.9) ? v3(0, 1, 0) : v3(1, 0, 0);
  V3 ov = unitv(cross(w, a));
  V3 ou = cross(w, ov);
  bool have_lights = false;
  if constexpr ((F & F_LIGHTS) != 0) have_lights = S.n_lights > 0;
  V3 gd;
  bool from_light = false;
  // one sincos(2 pi a) for whichever of the light sample (a sphere light's
  // azimuth, a = d0), the cosine direction (a = d0) and the isotropic
  // direction (a = d1) a lane takes: the wave runs it once instead of once
  // per branch that any lane takes -- the same operation on the same operand
  // for every lane (the merged-shading instances have theirs).
  // C4 +2.4 %, frames bit-identical (profiles/r05h_*).
  constexpr bool kSc = !kMerge && (F & F_LIGHTS) != 0;
  [[maybe_unused]] double sps = 0.0, cps = 0.0;
  if constexpr (kSc) {
    const bool to_light = e0 < 0.5 && have_lights;
    sincos_2pi<RT_KCONST_MODE(F)>((to_light || lamb) ? d0 : d1, sps, cps);
  }
  if constexpr ((F & F_LIGHTS) != 0) {
    if (e0 < 0.5 && have_lights) {
      const uint64_t t0 = STATS ? clk() : 0;
      gd = lights_random<RT_KCONST_MODE(F), kSc>(S, h.p, e1, d0, d1, sps, cps);
      from_light = true;
      if (STATS && wave_once()) cnt.clights += clk() - t0;
    }
  }
  if (!from_light) {
    if (kSc) {
      if (lamb) { // random_cosine_direction, Vec3Utility.hpp:94-103
        double sr = sqrt_n(d1);
        V3 lc = v3(cps * sr, sps * sr, sqrt_n(1 - d1));
        gd = ((lc.x * ou) + (lc.y * ov)) + (lc.z * w);
      } else {
        double z = 1.0 - 2.0 * d0;
        double rr = sqrt_n(fmax(0.0, 1.0 - z * z));
        gd = v3(rr * cps, rr * sps, z);
      }
    } else if (kMerge) { // the shared sincos and first root (above)
      if (lamb) {
        V3 lc = v3(cp1 * s1, sp1 * s1, sqrt_n(1 - d1));
        gd = ((lc.x * ou) + (lc.y * ov)) + (lc.z * w);
      } else {
        gd = v3(s1 * cp1, s1 * sp1, z1);
      }
    } else if (lamb) { // random_cosine_direction, Vec3Utility.hpp:94-103
      double sp, cp;
      sincos_2pi<RT_KCONST_MODE(F)>(d0, sp, cp);
      double sr = sqrt_n(d1);
      V3 lc = v3(cp * sr, sp * sr, sqrt_n(1 - d1));
      gd = ((lc.x * ou) + (lc.y * ov)) + (lc.z * w);
    } else {
      double z = 1.0 - 2.0 * d0;
      double rr = sqrt_n(fmax(0.0, 1.0 - z * z));
      double sp, cp;
      sincos_2pi<RT_KCONST_MODE(F)>(d1, sp, cp);
      gd = v3(rr * cp, rr * sp, z);
    }
  }
  double mat_pdf;
  if (lamb) {
    double ct = dot(unitv(gd), w);
    mat_pdf = fmax(0.0, div_mk(ct, kPi, kInvPi));
  } else {
    mat_pdf = 1.0 / (4.0 * kPi);
  }
  double p0 = mat_pdf;
  if constexpr ((F & F_LIGHTS) != 0) {
    if (have_lights) {
      const uint64_t t0 = STATS ? clk() : 0;
      p0 = lights_pdf<STATS>(S, h.p, gd, cnt);
      if (STATS && wave_once()) cnt.clights += clk() - t0;
    }
  }
  double pdf = 0.5 * p0 + 0.5 * mat_pdf;
  double spdf;
  if (lamb) {
    double ct = dot(h.n, unitv(gd));
    spdf = ct < 0 ? 0 : div_mk(ct, kPi, kInvPi);
  } else {
    spdf = 1 / (4 * kPi);
  }
  if (spdf == 0.0 && pdf > 0.0 && pdf < kInf) { // zero-weight continuation
    ps.T = ps.T * v3(0.0, 0.0, 0.0);             // (keeps an earlier NaN/inf alive)
    return false;
  }
  if constexpr ((F & F_NOISE) == 0) att = tex_value<F>(S, M.tex, h.p);
  V3 wgt = (1 / pdf) * (spdf * att);
  ps.T = ps.T * wgt;
  ps.ray = Ray{h.p, gd, r.tm};
  return advance(ps, C);
}

template <bool STATS, unsigned F, bool LP = false>
RT_HD RT_FI bool segment(const DScene &S, const DCamera &C, PathState &ps,
                                        const Key &key, int *stk, const RT_LDS DNode *lnodes,
                                        Counters &cnt, RT_LDS LeafPool *pool = nullptr,
                                        const LdsPrims &lp = LdsPrims{}) {
  Hit h;
  const uint64_t t0 = STATS ? clk() : 0;
  const bool hit = trace<STATS, F, LP>(S, ps.ray, h, key, ps.bounce, stk, lnodes, cnt, pool, lp);
  const uint64_t t1 = STATS ? clk() : 0;
  if (STATS && wave_once()) cnt.ctrace += t1 - t0;
  if (!hit) {
    ps.T = ps.T * ld3(C.bg); // miss -> background (Camera.cpp:242-243)
    return false;
  }
  const bool cont = shade<STATS, F>(S, C, ps, key, h, cnt);
  if (STATS && wave_once()) cnt.cshade += clk() - t1;
  return cont;
}

// The camera ray of stratum k of pixel (i, j) from its slot-0 block jt
// (jitter x, jitter y, time); the defocus block (slot 1) is drawn here.
template <bool KB = false, int KC = 0> // KB: philox10; KC: sincos_2pi
RT_HD RT_FI Ray camera_ray_jt(const DCamera &C, const Key &key, int i, int j, int k, const double jt[4]) {
  int si = k % C.sqrt_spp, sj = k / C.sqrt_spp;
  const double rs = C.rs; // 1.0 / sqrt_spp (host-formed)
  const double ja = jt[0], jb = jt[1];
  double px = ((si + ja) * rs) - 0.5;
  double py = ((sj + jb) * rs) - 0.5;
  V3 ps = (ld3(C.p00) + ((i + px) * ld3(C.du))) + ((j + py) * ld3(C.dv)); // Camera.cpp:186-205
  V3 org = ld3(C.center);
  if (!(C.defocus_angle <= 0)) {
    double dk[4]; // slot 1: defocus disk (r^2, angle)
    u01x4<KB>(key, kCamTag, 1, dk);
    const double a = dk[0], b = dk[1];
    double rr = sqrt_n(a);
    double s, c;
    sincos_2pi<KC>(b, s, c);
    double dx = rr * c, dy = rr * s;
    org = (org + (dx * ld3(C.disk_u))) + (dy * ld3(C.disk_v)); // Camera.cpp:226-230
  }
  return Ray{org, ps - org, jt[2]};
}
template <bool KB = false, int KC = 0>
RT_HD RT_FI Ray camera_ray(const DCamera &C, const Key &key, int i, int j, int k) {
  double jt[4]; // slot 0: jitter x, jitter y, time
  u01x4<KB>(key, kCamTag, 0, jt);
  return camera_ray_jt<KB, KC>(C, key, i, j, k, jt);
}


} // namespace rtp
#endif
