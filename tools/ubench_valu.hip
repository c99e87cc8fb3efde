// ubench_valu.hip — issue cost of the VALU instructions the megakernel leans on
// (fp64 FMA/MUL/ADD, fp64 rsq/rcp, the 32x32->64 integer product Philox uses,
// fp32 FMA and min3), measured on the MI355X itself: the guide's cost table
// lists fp32 and transcendental fp32 costs only.
//
// Each wave runs 8 independent dependency chains of one instruction for `iters`
// iterations; 4 waves per SIMD (blocks of 256 threads, 4 blocks per CU) keep the
// issue port busy.  Reported: SIMD cycles per wave-instruction =
// shader cycles of the timed loop (s_memtime) x waves per SIMD / instructions
// per wave.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(256) void kern(unsigned long long *cycles, double *sink, int iters) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  double d[CHAINS];
  float f[CHAINS];
  unsigned long long u[CHAINS];
  for (int c = 0; c < CHAINS; ++c) {
    d[c] = 1.0 + 1e-9 * (t + c);
    f[c] = 1.0f + 1e-6f * (t + c);
    u[c] = 0x9E3779B97F4A7C15ull * (t + c + 1);
  }
  const double db = 0.999999999, dc = 1e-12;
  const float fb = 0.9999f, fc = 1e-6f;
  const unsigned mb = 0xD2511F53u;
  __syncthreads();
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc));
      if constexpr (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[c]) : "v"(db));
      if constexpr (OP == 2) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dc));
      if constexpr (OP == 3) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[c]));
      if constexpr (OP == 4) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[c]));
      if constexpr (OP == 5) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "+v"(u[c]) : "v"(mb), "v"((unsigned)u[c]) : "vcc");
      if constexpr (OP == 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc));
      if constexpr (OP == 7) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc));
      if constexpr (OP == 8) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(*(unsigned *)&u[c]) : "v"(mb));
      if constexpr (OP == 9) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(*(unsigned *)&u[c]) : "v"(mb));
      if constexpr (OP == 10) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[c]) : "v"((unsigned)u[c]));
      if constexpr (OP == 11) asm volatile("v_cmp_lt_f64 vcc, %0, %1\n v_cndmask_b32 %2, %2, %3, vcc" : : "v"(d[c]), "v"(db), "v"(f[c]), "v"(fb) : "vcc");
      if constexpr (OP == 12) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(*(unsigned *)&u[c]) : "v"(mb));
      if constexpr (OP == 13) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[c]));
      if constexpr (OP == 14) asm volatile("v_floor_f64 %0, %0" : "+v"(d[c]));
      if constexpr (OP == 15) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(d[c]));
      if constexpr (OP == 16) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc));
      if constexpr (OP == 17) asm volatile("v_mov_b64 %0, %1" : "=v"(d[c]) : "v"(d[(c + 1) % CHAINS]));
      if constexpr (OP == 18) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(*(unsigned *)&u[c]) : "v"(mb), "v"(mb));
      if constexpr (OP == 19) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(*(unsigned *)&u[c]) : "v"(mb));
      if constexpr (OP == 20) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fb));
      if constexpr (OP == 21) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(f[c]) : "v"(fb));
      if constexpr (OP == 22) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(u[c]) : "v"(u[(c + 1) % CHAINS]));
      if constexpr (OP == 23) asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(d[c]) : "v"(db) : "vcc");
      if constexpr (OP == 24) asm volatile("v_div_fmas_f64 %0, %0, %1, %0" : "+v"(d[c]) : "v"(db));
      if constexpr (OP == 25) asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(d[c]));
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  double s = 0;
  for (int c = 0; c < CHAINS; ++c) s += d[c] + f[c] + (double)u[c];
  sink[t] = s;
  if ((threadIdx.x & 63) == 0) cycles[t / 64] = t1 - t0;
}

template <int OP> void run(const char *name, int cus) {
  const int blocks = cus * 4, threads = 256, iters = 4096;
  const int waves = blocks * threads / 64;
  unsigned long long *cyc;
  double *sink;
  (void)hipMalloc(&cyc, waves * sizeof(unsigned long long));
  (void)hipMalloc(&sink, blocks * threads * sizeof(double));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, cyc, sink, iters); // warm
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, cyc, sink, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(waves);
  (void)hipMemcpy(h.data(), cyc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto x : h) avg += (double)x;
  avg /= waves;
  const double per_wave_instr = (double)iters * CHAINS;
  // 4 waves per SIMD share the issue port: SIMD cycles per wave-instruction
  std::printf("%-16s %6.2f SIMD cyc/wave-instr (s_memtime)   %6.2f (events, 2.4 GHz)   %.3f ms\n", name,
              avg * 4.0 / per_wave_instr, ms * 1e-3 * 2.4e9 / (per_wave_instr * 4 /*waves/SIMD*/) * 4.0 / 4.0,
              ms);
  (void)hipFree(cyc);
  (void)hipFree(sink);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::printf("CUs %d; 8 independent chains per wave, 4 waves per SIMD\n", cus);
  run<0>("v_fma_f64", cus);
  run<1>("v_mul_f64", cus);
  run<2>("v_add_f64", cus);
  run<3>("v_rsq_f64", cus);
  run<4>("v_rcp_f64", cus);
  run<13>("v_sqrt_f64", cus);
  run<14>("v_floor_f64", cus);
  run<10>("v_cvt_f64_u32", cus);
  run<15>("v_cvt_f32_f64", cus);
  run<11>("v_cmp_f64+cndmask", cus);
  run<5>("v_mad_u64_u32", cus);
  run<8>("v_mul_lo_u32", cus);
  run<9>("v_mul_hi_u32", cus);
  run<12>("v_xor_b32", cus);
  run<6>("v_fma_f32", cus);
  run<7>("v_min3_f32", cus);
  run<16>("v_pk_fma_f32", cus);
  run<17>("v_mov_b64", cus);
  run<18>("v_bitop3_b32", cus);
  run<19>("v_mul_u32_u24", cus);
  run<20>("v_mul_f32", cus);
  run<21>("v_cndmask_b32", cus);
  run<22>("v_lshl_add_u64", cus);
  run<23>("v_div_scale_f64", cus);
  run<24>("v_div_fmas_f64", cus);
  run<25>("v_ldexp_f64", cus);
  return 0;
}
