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

// ---------------------------------------------------------------------------
// Round 4: the update operator's corr_encoder[0] (1x1 conv 196 -> 128 + bias +
// ReLU, droid_net.py:84-86) straight from the reference's NCHW lookup tensor
// (1, E, 196, H, W) - the reference-layout drop-in otherwise transposes the
// 2.5 GB lookup to channels-last (droid_transpose_f16) and reads it again.
// Persistent, one 4-wave workgroup per CU: the 128 x K weights stay in LDS; a
// tile = 128 pixels of one edge: its C channel rows (256 B each, coalesced)
// land in LDS as [K][128 px] (rows >= C zero), and the MFMA A fragments (8
// consecutive channels of one pixel) are gathered from that channel-major tile
// with 2-byte LDS reads - the transpose happens on the LDS read side.  The next
// tile's rows are loaded into registers during this tile's MFMAs.
// src (E, C, HW) fp16, w [128][K] fp16 (K % 32 == 0, columns >= C zero), bias
// [128] f32 -> out (E, HW, 128) fp16; HW % 128 == 0.
// ---------------------------------------------------------------------------
constexpr int kC1TP = 128;                 // pixels per tile
constexpr int kC1XS = kC1TP + 8;           // LDS row stride of the [K][px] tile (halves)
constexpr int kC1Rows = 16;                // global-load rounds per thread (C <= 256 rows of 16 uint4)
typedef float c1f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) conv1x1_nchw_kernel(const _Float16* __restrict__ src, int C,
                                                           const _Float16* __restrict__ w, int K,
                                                           const float* __restrict__ bias, _Float16* __restrict__ out,
                                                           int HW, long ntiles, int relu) {
  extern __shared__ __attribute__((aligned(16))) _Float16 c1_smem[];
  const int WS = K + 8;
  _Float16* Ws = c1_smem;                 // [128][WS]
  _Float16* Xs = c1_smem + 128 * WS;      // [K][kC1XS]; the output staging [128][kC1XS] reuses it
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fq = lane >> 4;
  const int tpe = HW / kC1TP;
  for (int idx = tid; idx < 128 * (K / 8); idx += 256) {
    const int r = idx / (K / 8), q = idx - r * (K / 8);
    *reinterpret_cast<half8*>(&Ws[r * WS + q * 8]) = *reinterpret_cast<const half8*>(w + (long)r * K + q * 8);
  }
  for (int idx = tid; idx < (K - C) * (kC1TP / 8); idx += 256) {   // channel rows past C: zero
    const int r = C + idx / (kC1TP / 8), q = idx % (kC1TP / 8);
    *reinterpret_cast<half8*>(&Xs[r * kC1XS + q * 8]) = half8{};
  }
  float bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = bias[wn * 64 + j * 16 + fr];
  // round q of thread tid: channel row (tid + 256 q) >> 4, 16-B piece tid & 15
  // branch-free loads against a per-tile descriptor (rows >= C and tiles past
  // the end read zeros), so the registers are never conditionally assigned
  uint4 pre[kC1Rows];
#define C1_LOAD(T_)                                                                                           \
  do {                                                                                                        \
    const long tt_ = (T_) < ntiles ? (T_) : 0;                                                                \
    const _Float16* sb_ = src + (tt_ / tpe) * (long)C * HW + (tt_ % tpe) * kC1TP;                             \
    const __amdgpu_buffer_rsrc_t rs_ = __builtin_amdgcn_make_buffer_rsrc(                                    \
        const_cast<_Float16*>(sb_), (short)0, (T_) < ntiles ? (int)(((long)(C - 1) * HW + kC1TP) * 2) : 0, \
        kBufFlags);                                                                                           \
    _Pragma("unroll") for (int q = 0; q < kC1Rows; ++q) {                                                     \
      const int idx = tid + 256 * q, r = idx >> 4, pc = idx & 15;                                             \
      const unsigned off = r < C ? (unsigned)(((long)r * HW + pc * 8) * 2) : kOob;                           \
      pre[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_, (int)off, 0, 0));        \
    }                                                                                                         \
  } while (0)
  long t = blockIdx.x;
  C1_LOAD(t);
  for (; t < ntiles; t += gridDim.x) {
#pragma unroll
    for (int q = 0; q < kC1Rows; ++q) {
      const int idx = tid + 256 * q, r = idx >> 4, pc = idx & 15;
      if (r < C) *reinterpret_cast<uint4*>(&Xs[r * kC1XS + pc * 8]) = pre[q];
    }
    __syncthreads();
    C1_LOAD(t + gridDim.x);   // the next tile's rows, in flight during the MFMAs
    c1f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = c1f4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < K / 32; ++ks) {
      half8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const _Float16* col = Xs + (ks * 32 + fq * 8) * kC1XS + wm * 64 + i * 16 + fr;
#pragma unroll
        for (int q = 0; q < 8; ++q) af[i][q] = col[q * kC1XS];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const half8*>(&Ws[(wn * 64 + j * 16 + fr) * WS + ks * 32 + fq * 8]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();   // every wave is done reading Xs: it becomes the output staging tile
    // lane (fr, fq) of fragment (i, j): pixels wm*64 + 16 i + 4 fq + q, channel wn*64 + 16 j + fr
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[i][j][q] + bv[j];
          if (relu) v = fmaxf(v, 0.f);
          Xs[(wm * 64 + i * 16 + fq * 4 + q) * kC1XS + wn * 64 + j * 16 + fr] = (_Float16)v;
        }
    __syncthreads();
    const long pix0 = (t / tpe) * (long)HW + (t % tpe) * kC1TP;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + 256 * q, r = idx >> 4, pc = idx & 15;
      *reinterpret_cast<uint4*>(out + (pix0 + r) * 128 + pc * 8) = *reinterpret_cast<const uint4*>(&Xs[r * kC1XS + pc * 8]);
    }
    __syncthreads();   // staging reads done before the next tile's rows land
    if (C < kC1TP) {   // the staging overwrote zero rows past C (only rows < 128 are staging)
      for (int idx = tid; idx < (K - C) * (kC1TP / 8); idx += 256) {
        const int r = C + idx / (kC1TP / 8), q = idx % (kC1TP / 8);
        *reinterpret_cast<half8*>(&Xs[r * kC1XS + q * 8]) = half8{};
      }
    }
  }
#undef C1_LOAD
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

// corr_encoder[0] on an NCHW lookup tensor (conv1x1_nchw_kernel): src (E, C, HW)
// fp16, w [128][K] fp16 (K % 32 == 0, K >= C, columns >= C zero), bias [128]
// f32 -> out (E, HW, 128) fp16 = act(w . src + bias), act = ReLU when relu.
extern "C" int droid_conv1x1_nchw_f16(const void* src, int C, const void* w, int K, const float* bias, void* out,
                                      int E, int HW, int relu, hipStream_t stream) {
  if (!src || !w || !bias || !out || E < 0 || HW <= 0 || C <= 0 || K < C || K % 32 || C > 16 * kC1Rows)
    return fail(kInvalidArgument, "conv1x1_nchw_f16: bad arguments (C <= 256, K % 32 == 0, K >= C)");
  if (HW % kC1TP) return fail(kUnsupported, "conv1x1_nchw_f16: needs H*W % 128 == 0");
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(out)) & 15)
    return fail(kInvalidArgument, "conv1x1_nchw_f16: operands must be 16-B aligned");
  if (E == 0) return kOk;
  const int lds = (128 * (K + 8) + K * kC1XS) * 2;
  if (lds > 160 * 1024 || 128 * kC1XS > K * kC1XS) return fail(kUnsupported, "conv1x1_nchw_f16: K too large / small");
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_nchw_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const long ntiles = (long)E * (HW / kC1TP);
  const long grid = std::min<long>(ntiles, device_cu_count());
  conv1x1_nchw_kernel<<<dim3((unsigned)grid), 256, lds, stream>>>(static_cast<const _Float16*>(src), C,
                                                                  static_cast<const _Float16*>(w), K, bias,
                                                                  static_cast<_Float16*>(out), HW, ntiles, relu);
  DROID_LAUNCH_CHECK();
  return kOk;
}
