// Shared device/host helpers for the MI355X (gfx950) droid_backends library.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <string>

namespace droid {

// ---------------------------------------------------------------------------
// Error plumbing for the C ABI: every entry point returns a status code and
// leaves a message retrievable through droid_last_error().
// ---------------------------------------------------------------------------
enum Status : int {
  kOk = 0,
  kInvalidArgument = 1,
  kUnsupported = 2,
  kHipError = 3,
  kNotContiguous = 4,
};

void set_last_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define DROID_HIP_CHECK(expr)                                                   \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess)                                                       \
      return ::droid::fail(::droid::kHipError,                                  \
                           std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

#define DROID_LAUNCH_CHECK()                                                    \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess)                                                       \
      return ::droid::fail(::droid::kHipError,                                  \
                           std::string("kernel launch failed: ") + hipGetErrorString(_e)); \
  } while (0)

// ---------------------------------------------------------------------------
// A/B builds.  The product library (make) takes every kernel choice from its
// arguments and compiled defaults - nothing from the environment - and ships
// only the kernels the defaults run.  `make ab` (lib/ab/libdroid_hip.so,
// -DDROID_AB=1) adds the measured-and-dropped variants and the experiment
// knobs (env DROID_*) that select them, for A/B runs and bitwise cross-checks.
// ---------------------------------------------------------------------------
#ifndef DROID_AB
#define DROID_AB 0
#endif
#ifndef DROID_CONV_PROFILE
#define DROID_CONV_PROFILE 0
#endif
// The testing builds (make ab, make prof) also export the hooks declared in
// include/droid_backends_testing.h (A/B variant and tile setters, fault
// injection, profile buffers); the product library exports none of them.
#define DROID_TESTING (DROID_AB || DROID_CONV_PROFILE)
inline int ab_knob(const char* name, int dflt) {
#if DROID_AB
  const char* e = getenv(name);
  return (e && e[0]) ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

constexpr int kWave = 64;
constexpr float kMinDepth = 0.25f;  // droid_kernels.cu:26

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// fp32 value -> nearest fp16 -> fp32, with the fp32 operand materialised first.
// Without the empty asm, hipcc folds round(a*b) / round(a+b) into one
// v_fma_mixlo_f16 that rounds the EXACT result once - not the reference's
// fp32-then-half double rounding (at::Half arithmetic), so 1-ulp differences
// appear on rare ties.  Used by the bit-exact correlation lookups.
__device__ __forceinline__ float rnd16(float x) {
  asm volatile("" : "+v"(x));
  return __half2float(__float2half(x));
}

// compute units of the current device (grid size of persistent kernels)
inline int device_cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// ---------------------------------------------------------------------------
// SE3 device helpers.  Pose layout [tx,ty,tz,qx,qy,qz,qw], twist [tau,phi].
// Formulas restate droid_kernels.cu:58-175 (actSO3, actSE3, adjSE3, relSE3,
// expSO3, expSE3) and :877-895 (retrSE3); the arithmetic order follows the
// reference so fp32 results agree to rounding.
// ---------------------------------------------------------------------------
struct SE3f {
  float t[3];
  float q[4];
};

__device__ __forceinline__ void act_so3(const float* q, const float* X, float* Y) {
  float uv0 = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  float uv1 = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  float uv2 = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  Y[0] = X[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  Y[1] = X[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  Y[2] = X[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

// Homogeneous point [X, W] -> [R X + t W, W]
__device__ __forceinline__ void act_se3(const SE3f& T, const float* X, float* Y) {
  act_so3(T.q, X, Y);
  Y[3] = X[3];
  Y[0] += X[3] * T.t[0];
  Y[1] += X[3] * T.t[1];
  Y[2] += X[3] * T.t[2];
}

// Tij = Tj * Ti^-1
__device__ __forceinline__ SE3f rel_se3(const float* pi, const float* pj) {
  SE3f r;
  const float* qi = pi + 3;
  const float* qj = pj + 3;
  r.q[0] = -qj[3] * qi[0] + qj[0] * qi[3] - qj[1] * qi[2] + qj[2] * qi[1];
  r.q[1] = -qj[3] * qi[1] + qj[1] * qi[3] - qj[2] * qi[0] + qj[0] * qi[2];
  r.q[2] = -qj[3] * qi[2] + qj[2] * qi[3] - qj[0] * qi[1] + qj[1] * qi[0];
  r.q[3] = qj[3] * qi[3] + qj[0] * qi[0] + qj[1] * qi[1] + qj[2] * qi[2];
  float ti[3] = {pi[0], pi[1], pi[2]};
  float y[3];
  act_so3(r.q, ti, y);
  r.t[0] = pj[0] - y[0];
  r.t[1] = pj[1] - y[1];
  r.t[2] = pj[2] - y[2];
  return r;
}

__device__ __forceinline__ SE3f stereo_se3() {
  SE3f r;
  r.t[0] = -0.1f; r.t[1] = 0.f; r.t[2] = 0.f;
  r.q[0] = 0.f; r.q[1] = 0.f; r.q[2] = 0.f; r.q[3] = 1.f;
  return r;
}

// Y = Adj-transposed action used to map Jj rows to Ji rows (adjSE3).
__device__ __forceinline__ void adj_se3(const SE3f& T, const float* X, float* Y) {
  const float qinv[4] = {-T.q[0], -T.q[1], -T.q[2], T.q[3]};
  act_so3(qinv, X, Y);
  act_so3(qinv, X + 3, Y + 3);
  float u[3], v[3];
  u[0] = T.t[2] * X[1] - T.t[1] * X[2];
  u[1] = T.t[0] * X[2] - T.t[2] * X[0];
  u[2] = T.t[1] * X[0] - T.t[0] * X[1];
  act_so3(qinv, u, v);
  Y[3] += v[0];
  Y[4] += v[1];
  Y[5] += v[2];
}

__device__ __forceinline__ void exp_so3(const float* phi, float* q) {
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta_p4 = theta_sq * theta_sq;
  float theta = sqrtf(theta_sq);
  float imag, real;
  if (theta_sq < 1e-8f) {
    imag = 0.5f - (1.0f / 48.0f) * theta_sq + (1.0f / 3840.0f) * theta_p4;
    real = 1.0f - (1.0f / 8.0f) * theta_sq + (1.0f / 384.0f) * theta_p4;
  } else {
    imag = sinf(0.5f * theta) / theta;
    real = cosf(0.5f * theta);
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}

__device__ __forceinline__ void cross_inplace(const float* a, float* b) {
  float x0 = a[1] * b[2] - a[2] * b[1];
  float x1 = a[2] * b[0] - a[0] * b[2];
  float x2 = a[0] * b[1] - a[1] * b[0];
  b[0] = x0; b[1] = x1; b[2] = x2;
}

__device__ __forceinline__ void exp_se3(const float* xi, float* t, float* q) {
  exp_so3(xi + 3, q);
  float tau[3] = {xi[0], xi[1], xi[2]};
  const float phi[3] = {xi[3], xi[4], xi[5]};
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  t[0] = tau[0]; t[1] = tau[1]; t[2] = tau[2];
  if (theta > 1e-4f) {
    float a = (1.0f - cosf(theta)) / theta_sq;
    cross_inplace(phi, tau);
    t[0] += a * tau[0]; t[1] += a * tau[1]; t[2] += a * tau[2];
    float b = (theta - sinf(theta)) / (theta * theta_sq);
    cross_inplace(phi, tau);
    t[0] += b * tau[0]; t[1] += b * tau[1]; t[2] += b * tau[2];
  }
}

// T <- Exp(xi) * T   (retrSE3)
__device__ __forceinline__ void retr_se3(const float* xi, float* pose) {
  float dt[3] = {0.f, 0.f, 0.f};
  float dq[4] = {0.f, 0.f, 0.f, 1.f};
  exp_se3(xi, dt, dq);
  const float t[3] = {pose[0], pose[1], pose[2]};
  const float q[4] = {pose[3], pose[4], pose[5], pose[6]};
  float q1[4], t1[3];
  q1[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
  q1[1] = dq[3] * q[1] + dq[1] * q[3] + dq[2] * q[0] - dq[0] * q[2];
  q1[2] = dq[3] * q[2] + dq[2] * q[3] + dq[0] * q[1] - dq[1] * q[0];
  q1[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
  act_so3(dq, t, t1);
  pose[0] = t1[0] + dt[0];
  pose[1] = t1[1] + dt[1];
  pose[2] = t1[2] + dt[2];
  pose[3] = q1[0]; pose[4] = q1[1]; pose[5] = q1[2]; pose[6] = q1[3];
}

__device__ __forceinline__ SE3f load_pose(const float* poses, int k) {
  SE3f T;
  const float* p = poses + 7 * k;
  T.t[0] = p[0]; T.t[1] = p[1]; T.t[2] = p[2];
  T.q[0] = p[3]; T.q[1] = p[4]; T.q[2] = p[5]; T.q[3] = p[6];
  return T;
}

// Round an fp32 value to the nearest fp16 and return it widened again.
__device__ __forceinline__ float round_half(float x) {
  return __half2float(__float2half(x));
}

}  // namespace droid
