// Instance normalisation of NHWC fp16 feature maps fused with the ReLU and
// residual adds around it in the MotionFilter's feature encoder
// (modules/extractor.py: BasicEncoder(norm_fn='instance') = fnet, its
// ResidualBlocks; nn.InstanceNorm2d(affine=False, eps=1e-5): per image and
// channel, (x - mean) / sqrt(var + eps) with the biased variance over H x W).
//
// Two launches, both HBM-bound streaming passes over the map:
//   * instnorm_stats_kernel: grid (S pixel ranges, N images); each thread sums
//     8 channels (one 16-B piece) over a strided set of pixels in fp32, the
//     workgroup reduces through LDS and writes (sum, sum of squares) per channel
//     and range;
//   * instnorm_apply_kernel: grid (pixel blocks, N); the workgroup first turns
//     the S partials of its image into mean / rstd per channel (in LDS, ranges
//     added in order: deterministic), then streams the map once more:
//       mode 0  out = relu(n(x))                (norm1/norm2 + ReLU)
//       mode 1  out = relu(res + relu(n(x)))    (stride-1 block: conv2 branch + identity)
//       mode 2  out = relu(n(x) + res)          (stride-2 block: norm3 of the downsample + branch)
//       mode 3  out = n(x)
#include "common.hpp"

#include <algorithm>

namespace droid {

constexpr int kNormThreads = 256;

__global__ void __launch_bounds__(kNormThreads) instnorm_stats_kernel(const __half* __restrict__ x, int HW, int C,
                                                                      float2* __restrict__ part) {
  __shared__ float2 red[kNormThreads * 8];
  const int n = blockIdx.y, s = blockIdx.x, S = gridDim.x;
  const int G = C / 8;                      // 16-B pieces per pixel
  const int t = threadIdx.x;
  const int P = kNormThreads / G;           // pixels in flight per step
  const int g = t % G, pl = t / G;
  const long p0 = (long)HW * s / S, p1 = (long)HW * (s + 1) / S;
  float sm[8] = {}, sq[8] = {};
  if (pl < P) {
    const __half* xb = x + (long)n * HW * C + g * 8;
    for (long p = p0 + pl; p < p1; p += P) {
      const uint4 v = *reinterpret_cast<const uint4*>(xb + p * C);
      const __half* h = reinterpret_cast<const __half*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = __half2float(h[k]);
        sm[k] += f;
        sq[k] += f * f;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[t * 8 + k] = make_float2(sm[k], sq[k]);
  __syncthreads();
  for (int c = t; c < C; c += kNormThreads) {  // channel c = 8 g + k: add the P pixel lanes in order
    const int gg = c / 8, k = c % 8;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < P; ++q) {
      const float2 v = red[(q * G + gg) * 8 + k];
      a += v.x;
      b += v.y;
    }
    part[((long)n * S + s) * C + c] = make_float2(a, b);
  }
}

__global__ void __launch_bounds__(kNormThreads) instnorm_apply_kernel(const __half* __restrict__ x,
                                                                      const __half* __restrict__ res,
                                                                      __half* __restrict__ out,
                                                                      const float2* __restrict__ part, int S, int HW,
                                                                      int C, int mode, float eps) {
  __shared__ float2 mr[512];   // mean, rstd per channel
  const int n = blockIdx.y, t = threadIdx.x;
  for (int c = t; c < C; c += kNormThreads) {
    float a = 0.f, b = 0.f;
    for (int s = 0; s < S; ++s) {
      const float2 v = part[((long)n * S + s) * C + c];
      a += v.x;
      b += v.y;
    }
    const float mean = a / (float)HW;
    const float var = fmaxf(b / (float)HW - mean * mean, 0.f);
    mr[c] = make_float2(mean, rsqrtf(var + eps));
  }
  __syncthreads();
  const int G = C / 8;
  const long npieces = (long)HW * G;
  const long base = (long)n * HW * C;
  for (long q = (long)blockIdx.x * kNormThreads + t; q < npieces; q += (long)gridDim.x * kNormThreads) {
    const int g = (int)(q % G);
    const long off = base + q * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(x + off);
    const __half* h = reinterpret_cast<const __half*>(&v);
    uint4 rv = make_uint4(0, 0, 0, 0);
    if (mode == 1 || mode == 2) rv = *reinterpret_cast<const uint4*>(res + off);
    const __half* r = reinterpret_cast<const __half*>(&rv);
    uint4 o;
    __half* oh = reinterpret_cast<__half*>(&o);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float2 m = mr[g * 8 + k];
      // the normalised value rounds to fp16 first, as the module's output does
      const float y = __half2float(__float2half((__half2float(h[k]) - m.x) * m.y));
      float z;
      if (mode == 0) z = fmaxf(y, 0.f);
      else if (mode == 1) z = fmaxf(__half2float(r[k]) + fmaxf(y, 0.f), 0.f);
      else if (mode == 2) z = fmaxf(y + __half2float(r[k]), 0.f);
      else z = y;
      oh[k] = __float2half(z);
    }
    *reinterpret_cast<uint4*>(out + off) = o;
  }
}

}  // namespace droid

using namespace droid;

extern "C" {

// Bytes of workspace droid_instance_norm_act_f16 needs.
size_t droid_instance_norm_workspace(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0) return 0;
  const int S = std::max(1, std::min(64, HW / 1024));
  return (size_t)N * S * C * sizeof(float2);
}

// x, res, out: (N, HW, C) fp16 NHWC (channels_last), C % 8 == 0, C <= 512,
// 16-B aligned; res needed for modes 1 and 2 (may alias nothing); out may be x.
int droid_instance_norm_act_f16(const void* x, const void* res, void* out, int N, int HW, int C, int mode, float eps,
                                void* ws, size_t ws_bytes, hipStream_t stream) {
  if (N < 0 || HW <= 0 || C <= 0 || C % 8 || C > 512 || mode < 0 || mode > 3 || !x || !out ||
      ((mode == 1 || mode == 2) && !res) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 15) || (res && (reinterpret_cast<uintptr_t>(res) & 15)))
    return fail(kInvalidArgument, "instance_norm_act_f16: bad arguments (C % 8, C <= 512, 16-B aligned NHWC)");
  if (N == 0) return kOk;
  if ((long)N * HW * C > 0x7fffffffL) return fail(kUnsupported, "instance_norm_act_f16: map too large");
  const int S = std::max(1, std::min(64, HW / 1024));
  if (!ws || ws_bytes < (size_t)N * S * C * sizeof(float2))
    return fail(kInvalidArgument, "instance_norm_act_f16: workspace too small");
  float2* part = static_cast<float2*>(ws);
  instnorm_stats_kernel<<<dim3(S, N), kNormThreads, 0, stream>>>((const __half*)x, HW, C, part);
  DROID_LAUNCH_CHECK();
  const long pieces = (long)HW * (C / 8);
  const int nb = (int)std::min<long>(std::max<long>(1, pieces / (4 * kNormThreads)), 1024);
  instnorm_apply_kernel<<<dim3(nb, N), kNormThreads, 0, stream>>>((const __half*)x, (const __half*)res,
                                                                   (__half*)out, part, S, HW, C, mode, eps);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
