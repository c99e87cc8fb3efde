// TEST-ONLY gfx950 build of rt_path.h's arithmetic helpers, to check on the
// GPU that the kernel's shortened sequences equal the full IEEE operations bit
// for bit (tests/test_gpu_arith.py):
//   sqrt_n(x)           vs sqrt(x)      (the compiler's correctly rounded lowering)
//   div_mk(x, b, 1/b)   vs x / b
//   rcp_n(x)            vs 1.0 / x      (returned in the div_mk slot when b == 0)
//   sincos_2pi<1>, <2>  vs sincos_2pi<0> (the polynomial constants materialised at
//                       their use in SGPRs / VGPRs vs held, rt_path.h RT_KCONST)
// Nothing on the product path links this.
#include <hip/hip_runtime.h>

#include "../../real-time-ray-tracing-engine_amd/csrc/rt_path.h"

namespace {
__global__ void arith_kernel(const double *x, const double *b, int n, double *sq_n, double *sq,
                             double *dq, double *dv) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double xv = x[k], bv = b[k];
  sq_n[k] = rtp::sqrt_n(xv);
  sq[k] = sqrt(xv);
  if (bv == 0.0) { // reciprocal mode
    dq[k] = rtp::rcp_n(xv);
    dv[k] = 1.0 / xv;
  } else {
    dq[k] = rtp::div_mk(xv, bv, 1.0 / bv);
    dv[k] = xv / bv;
  }
}
__global__ void sincos_kernel(const double *u, int n, double *out) { // out: [6][n]
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double s0, c0, s1, c1, s2, c2;
  rtp::sincos_2pi<0>(u[k], s0, c0);
  rtp::sincos_2pi<1>(u[k], s1, c1);
  rtp::sincos_2pi<2>(u[k], s2, c2);
  out[k] = s0;
  out[n + k] = c0;
  out[2 * n + k] = s1;
  out[3 * n + k] = c1;
  out[4 * n + k] = s2;
  out[5 * n + k] = c2;
}
} // namespace

// sincos_2pi's three constant forms on the device: out [6][n] = s0, c0, s1, c1, s2, c2
extern "C" int devcheck_sincos(const double *u, int n, double *out) {
  if (n <= 0) return 0;
  double *d = nullptr;
  const size_t bytes = sizeof(double) * (size_t)n;
  if (hipMalloc(&d, 7 * bytes) != hipSuccess) return -1;
  int rc = 0;
  if (hipMemcpy(d, u, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(sincos_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d, n, d + n);
    if (hipDeviceSynchronize() != hipSuccess) rc = -3;
  }
  if (!rc && hipMemcpy(out, d + n, 6 * bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -4;
  hipFree(d);
  return rc;
}

// Host buffers in, host buffers out; returns 0 or a negative hipError_t.
extern "C" int devcheck_arith(const double *x, const double *b, int n, double *sq_n, double *sq,
                              double *dq, double *dv) {
  if (n <= 0) return 0;
  double *d = nullptr;
  const size_t bytes = sizeof(double) * (size_t)n;
  if (hipMalloc(&d, 6 * bytes) != hipSuccess) return -1;
  double *dx = d, *db = d + n, *o0 = d + 2 * (size_t)n, *o1 = d + 3 * (size_t)n,
         *o2 = d + 4 * (size_t)n, *o3 = d + 5 * (size_t)n;
  int rc = 0;
  if (hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(db, b, bytes, hipMemcpyHostToDevice) != hipSuccess)
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(arith_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dx, db, n, o0, o1, o2, o3);
    if (hipDeviceSynchronize() != hipSuccess) rc = -3;
  }
  if (!rc && (hipMemcpy(sq_n, o0, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
              hipMemcpy(sq, o1, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
              hipMemcpy(dq, o2, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
              hipMemcpy(dv, o3, bytes, hipMemcpyDeviceToHost) != hipSuccess))
    rc = -4;
  hipFree(d);
  return rc;
}
