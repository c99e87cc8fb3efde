// ubench_issue.hip -- VALU issue-rate calibration of the SQ counters on gfx950.
//
// Each kernel streams ONE instruction kind with 16 independent dependency
// chains per wave at 8 waves per SIMD (256-thread blocks, 8 blocks per CU), so
// the SIMD's VALU issue port, not latency, limits it.  Run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE ... -- ./ubench_issue
// the per-kernel counters give, for a saturated stream of each kind, the
// value of 4 * SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs) that
// bench.py reports for the render kernel (its "issue ratio"), and
// SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU (what the counter adds per
// instruction).  Printed: the event time and wave-instructions per SIMD per
// microsecond; with the kernel-trace clock (GRBM_GUI_ACTIVE / 8 / duration)
// that is the SIMD cycles each wave-instruction of the kind occupies.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHAINS 16

template <int OP>
__global__ __launch_bounds__(256) void issue(double *sink, int iters) {
  const int t = threadIdx.x + blockIdx.x * blockDim.x;
  double d[CHAINS];
  float f[CHAINS];
  unsigned u[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    d[c] = 1.0 + 1e-9 * (t + c);
    f[c] = 1.0f + 1e-6f * (t + c);
    u[c] = 0x9E3779B9u * (t + c + 1);
  }
  const double db = 0.999999999, dc = 1e-12;
  const float fb = 0.9999f, fc = 1e-6f;
  const unsigned mb = 0xD2511F53u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc));
      if constexpr (OP == 1) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc));
      if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(mb));
      if constexpr (OP == 3) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc));
      if constexpr (OP == 4) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc));
      if constexpr (OP == 5) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dc));
      if constexpr (OP == 6) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(mb));
      if constexpr (OP == 7) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[c]));
      // half the lanes active (odd lanes): do the FLOPS / THREAD counters count lanes?
      if constexpr (OP == 8) if (threadIdx.x & 1) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc));
      if constexpr (OP == 9) if (threadIdx.x & 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc));
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += d[c] + f[c] + (double)u[c];
  sink[t] = s;
}

template <int OP>
void run(const char *name, int cus) {
  const int blocks = cus * 8, threads = 256, iters = 2048;
  double *sink;
  (void)hipMalloc(&sink, (size_t)blocks * threads * sizeof(double));
  hipLaunchKernelGGL(issue<OP>, dim3(blocks), dim3(threads), 0, 0, sink, iters); // warm
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(issue<OP>, dim3(blocks), dim3(threads), 0, 0, sink, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double wave_instr = (double)blocks * threads / 64 * iters * CHAINS;
  const double per_simd = wave_instr / (cus * 4);
  std::printf("%-14s %8.3f ms  %.4g wave-instr per SIMD per us\n", name, ms, per_simd / (ms * 1e3));
  (void)hipFree(sink);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::printf("CUs %d; %d independent chains per wave, 8 waves per SIMD\n", cus, CHAINS);
  run<0>("v_fma_f32", cus);
  run<1>("v_fma_f64", cus);
  run<2>("v_xor_b32", cus);
  run<3>("v_min3_f32", cus);
  run<4>("v_pk_fma_f32", cus);
  run<5>("v_add_f64", cus);
  run<6>("v_add_u32", cus);
  run<7>("v_rcp_f64", cus);
  run<8>("v_fma_f64 1/2", cus);
  run<9>("v_fma_f32 1/2", cus);
  return 0;
}
