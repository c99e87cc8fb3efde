// TEST-ONLY gfx950 build of rt_path.h's arithmetic helpers, to check on the
// GPU that the kernel's shortened sequences equal the full IEEE operations bit
// for bit (tests/test_gpu_arith.py):
//   sqrt_n(x)           vs sqrt(x)      (the compiler's correctly rounded lowering)
//   div_mk(x, b, 1/b)   vs x / b
//   rcp_n(x)            vs 1.0 / x      (returned in the div_mk slot when b == 0)
//   sincos_2pi<1>, <2>  vs sincos_2pi<0> (the polynomial constants materialised at
//                       their use in SGPRs / VGPRs vs held, rt_path.h RT_KCONST)
//   box_span            vs boundary_span (a make_box medium's boundary queries,
//                       tests/test_medium_box.py; the scene compiled on the host
//                       by csrc/rt_scene.cpp, linked in)
// Nothing on the product path links this.
#include <hip/hip_runtime.h>

#include "../../real-time-ray-tracing-engine_amd/csrc/rt_path.h"
#include "../../real-time-ray-tracing-engine_amd/csrc/rt_scene.h"

#include <string>
#include <vector>

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
// one ray per thread: out[6] as emu_medium_spans (tests/native/rt_emulate.cpp)
__global__ void medium_kernel(DScene S, int m, const double *rays, int n, double *out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const DMedium M = S.media[m];
  const double *q = rays + 7 * k;
  rtp::Ray r{rtp::v3(q[0], q[1], q[2]), rtp::v3(q[3], q[4], q[5]), q[6]};
  double a1 = 0, a2 = 0, g1 = 0, g2 = 0;
  const int rc = M.box ? rtp::box_span(S, M, r, a1, a2) : -2;
  const bool g = rtp::boundary_span(S, M, r, g1, g2);
  double *o = out + 6 * k;
  o[0] = rc;
  o[1] = rc == 1 ? a1 : 0.0;
  o[2] = rc == 1 ? a2 : 0.0;
  o[3] = g ? 1.0 : 0.0;
  o[4] = g ? g1 : 0.0;
  o[5] = g ? g2 : 0.0;
}
} // namespace

template <class T>
static int upload(const std::vector<T> &v, void **d) {
  *d = nullptr;
  if (v.empty()) return 0;
  if (hipMalloc(d, v.size() * sizeof(T)) != hipSuccess) return -1;
  return hipMemcpy(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess ? 0 : -2;
}

// Both boundary queries of medium m on n medium-frame rays, on the device:
// out per ray as emu_medium_spans.  Returns 0, or a negative code.
extern "C" int devcheck_medium_spans(const rt_scene_desc *desc, int m, const double *rays, int n,
                                     double *out) {
  rtx::HostScene H;
  std::string err;
  if (rtx::compile_scene(desc, H, err) != RT_OK) return -10;
  if (m < 0 || m >= (int)H.media.size() || n <= 0) return -11;
  void *b[7] = {};
  int rc = upload(H.bitems, &b[0]);
  if (!rc) rc = upload(H.xforms, &b[1]);
  if (!rc) rc = upload(H.spheres, &b[2]);
  if (!rc) rc = upload(H.quads, &b[3]);
  if (!rc) rc = upload(H.media, &b[4]);
  if (!rc) rc = upload(std::vector<double>(rays, rays + 7 * (size_t)n), &b[5]);
  if (!rc && hipMalloc(&b[6], 6 * sizeof(double) * (size_t)n) != hipSuccess) rc = -3;
  if (!rc) {
    DScene S{};
    S.bitems = (const DItem *)b[0];
    S.xforms = (const DXform *)b[1];
    S.spheres = (const DSphere *)b[2];
    S.quads = (const DQuad *)b[3];
    S.media = (const DMedium *)b[4];
    hipLaunchKernelGGL(medium_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, S, m,
                       (const double *)b[5], n, (double *)b[6]);
    if (hipDeviceSynchronize() != hipSuccess) rc = -4;
  }
  if (!rc && hipMemcpy(out, b[6], 6 * sizeof(double) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
    rc = -5;
  for (void *p : b)
    if (p) (void)hipFree(p);
  return rc;
}

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
