// Batched fp16 transposes for the reference-layout drop-in
// (droid_mi355x.fused.ReferenceLayoutUpdateModule): the reference's
// factor_graph.py hands the update operator NCHW state (net, inp, the 196-channel
// lookup, droid_net.py:111-143) while the MI355X operator runs channels-last.
// torch's permute + contiguous runs these as strided element copies at ~2 TB/s;
// here a 64 x 64 tile goes through LDS, read and written as 16-B row pieces.
//
//   dst[b][c][r] = src[b][r][c]   (r < R),   dst[b][c][r] = 0   (R <= r < ldd)
//   src (B, R, C) fp16 contiguous, dst (B, C, ldd) fp16 contiguous.
// NCHW -> NHWC: R = channels, C = H*W (ldd >= channels pads them with zeros);
// NHWC -> NCHW: R = H*W, C = channels.
#include "lds_dma.hpp"

namespace droid {

constexpr int kTrT = 64;            // tile edge
constexpr int kTrS = kTrT + 2;      // LDS row stride (halves): column reads spread over banks

__global__ void __launch_bounds__(256) transpose_f16_kernel(const _Float16* __restrict__ src, _Float16* __restrict__ dst,
                                                            int R, int C, int ldd) {
  __shared__ _Float16 tile[kTrT * kTrS];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * kTrT, c0 = blockIdx.x * kTrT;
  const int tid = threadIdx.x;
  const _Float16* s = src + (long)b * R * C;
  _Float16* d = dst + (long)b * C * ldd;
  // load: 64 rows x 8 pieces of 8 halves; thread -> (row, piece), two rounds
  const bool cvec = (C & 7) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k, rr = idx >> 3, pc = idx & 7;
    const int r = r0 + rr, c = c0 + pc * 8;
    half8 v = {};
    if (r < R) {
      if (cvec && c + 8 <= C) {
        v = *reinterpret_cast<const half8*>(s + (long)r * C + c);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (c + q < C) ? s[(long)r * C + c + q] : (_Float16)0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) tile[rr * kTrS + pc * 8 + q] = v[q];
  }
  __syncthreads();
  // store: 64 dst rows (c) x 8 pieces of 8 halves (r), rows r >= R (up to ldd) zero
  const bool rvec = (ldd & 7) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k, cc = idx >> 3, pr = idx & 7;
    const int c = c0 + cc, r = r0 + pr * 8;
    if (c >= C || r >= ldd) continue;
    half8 v;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = (r + q < R) ? tile[(pr * 8 + q) * kTrS + cc] : (_Float16)0.f;
    if (rvec && r + 8 <= ldd) {
      *reinterpret_cast<half8*>(d + (long)c * ldd + r) = v;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (r + q < ldd) d[(long)c * ldd + r + q] = v[q];
    }
  }
}

}  // namespace droid

using namespace droid;

extern "C" int droid_transpose_f16(const void* src, void* dst, int B, int R, int C, int ldd, hipStream_t stream) {
  if (B < 0 || R < 0 || C < 0 || ldd < R || !src || !dst)
    return fail(kInvalidArgument, "transpose_f16: bad arguments");
  if (B == 0 || C == 0 || ldd == 0) return kOk;
  if (B > 65535 || (long)B * R * C > 0x7fffffffffL) return fail(kUnsupported, "transpose_f16: too many batches");
  const int rt = ceil_div(ldd, kTrT);   // row tiles cover the zero padding up to ldd
  if (rt > 65535) return fail(kUnsupported, "transpose_f16: too many rows");
  transpose_f16_kernel<<<dim3(ceil_div(C, kTrT), rt, B), 256, 0, stream>>>(static_cast<const _Float16*>(src),
                                                                           static_cast<_Float16*>(dst), R, C, ldd);
  DROID_LAUNCH_CHECK();
  return kOk;
}
