// free_probe.hip — does freeing one buffer wait for unrelated work on the device?
// (rt_scene_destroy should wait only for its own scene's work.)
//
// A spin kernel runs ~300 ms on stream B.  Meanwhile, from the host, on other
// buffers: hipFree (hipMalloc'd), hipFreeAsync on stream A (hipMalloc'd and
// hipMallocAsync'd), each timed.  A free that returns in << 300 ms does not
// wait for B's kernel.
//   hipcc --offload-arch=gfx950 -O2 -o build/free_probe tools/free_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                                   \
      return 1;                                                                             \
    }                                                                                       \
  } while (0)

__global__ void spin(long long cycles, int *out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  int *flag;
  CK(hipMalloc(&flag, 1024 * sizeof(int)));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const long long cycles = (long long)rate_khz * 300; // 300 ms
  std::printf("wall clock %d kHz\n", rate_khz);
  const char *names[] = {"hipFree(hipMalloc)", "hipFreeAsync(hipMalloc, A)", "hipFreeAsync(hipMallocAsync, A)",
                         "hipEventSynchronize(A's event)"};
  for (int mode = 0; mode < 4; ++mode) {
    void *p = nullptr;
    if (mode == 2) {
      CK(hipMallocAsync(&p, 64 << 20, A));
      CK(hipStreamSynchronize(A));
    } else {
      CK(hipMalloc(&p, 64 << 20));
    }
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipMemsetAsync(p, 0, 64 << 20, A));
    CK(hipEventRecord(ev, A));
    CK(hipStreamSynchronize(A));
    hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, B, cycles, flag);
    CK(hipGetLastError());
    const double t0 = now_ms();
    if (mode == 0) CK(hipFree(p));
    if (mode == 1 || mode == 2) CK(hipFreeAsync(p, A));
    if (mode == 3) CK(hipEventSynchronize(ev));
    const double t1 = now_ms();
    CK(hipStreamSynchronize(B));
    const double t2 = now_ms();
    if (mode == 3) CK(hipFree(p));
    CK(hipEventDestroy(ev));
    std::printf("%-36s returned after %8.2f ms (spin kernel ended at %8.2f ms)\n", names[mode], t1 - t0, t2 - t0);
  }
  // the whole release sequence of a scene while B's kernel runs: frees on A,
  // then synchronise A, then destroy A's objects -- with the device's default
  // pool (release threshold 0: a sync may hand freed memory back to the
  // system) and with a pool that keeps its memory (threshold UINT64_MAX)
  hipMemPool_t own;
  hipMemPoolProps props = {};
  props.allocType = hipMemAllocationTypePinned;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = 0;
  CK(hipMemPoolCreate(&own, &props));
  uint64_t keep = ~0ull;
  CK(hipMemPoolSetAttribute(own, hipMemPoolAttrReleaseThreshold, &keep));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipStream_t S;
      CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
      void *p[4];
      for (int i = 0; i < 4; ++i) {
        if (mode == 0) CK(hipMallocAsync(&p[i], (size_t)(64 + 32 * i) << 20, S));
        else CK(hipMallocFromPoolAsync(&p[i], (size_t)(64 + 32 * i) << 20, own, S));
      }
      CK(hipMemsetAsync(p[0], 0, 1 << 20, S));
      CK(hipStreamSynchronize(S));
      hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, B, cycles, flag);
      CK(hipGetLastError());
      const double t0 = now_ms();
      for (int i = 0; i < 4; ++i) CK(hipFreeAsync(p[i], S));
      CK(hipStreamSynchronize(S));
      const double t1 = now_ms();
      CK(hipStreamDestroy(S));
      const double t2 = now_ms();
      CK(hipStreamSynchronize(B));
      const double t3 = now_ms();
      std::printf("%-36s rep %d: frees + sync %8.2f ms, stream destroy %8.2f ms (spin ended at %8.2f ms)\n",
                  mode == 0 ? "default pool (threshold 0)" : "own pool (threshold max)", rep, t1 - t0,
                  t2 - t1, t3 - t0);
    }
  }
  CK(hipMemPoolDestroy(own));
  CK(hipFree(flag));
  CK(hipStreamDestroy(A));
  CK(hipStreamDestroy(B));
  return 0;
}
