// Correlation lookup kernels for gfx950.
//
//  corr_index_forward / backward  — drop-in for correlation_kernels.cu:19-185
//  corr_pyramid_lookup            — CorrBlock.__call__ (modules/corr.py:40-50) for all
//                                   levels in ONE launch, writing the concatenated
//                                   (E, L*(2r+1)^2, H, W) tensor directly
//  altcorr_forward / backward     — drop-in for altcorr_kernel.cu:27-356
//
// Lookup arithmetic (all dtypes) follows the reference loop order: taps are
// visited i = x-offset outer, j = y-offset inner, and every output (a,b)
// receives its four bilinear terms in the order
//     (a,b)*(1-dx)(1-dy), (a,b+1)*(1-dx)dy, (a+1,b)*dx(1-dy), (a+1,b+1)*dx*dy.
// fp16 reproduces at::Half semantics bit-exactly (weight rounded to half,
// product rounded to half, every += rounded to half); fp32/fp64 use the fused
// multiply-add nvcc emits for `corr += s * w`.
#include "common.hpp"
#include "lds_dma.hpp"

// Bit-exact at::Half semantics need every product and sum rounded separately:
// forbid fusing them into v_fma_mix / v_fma_f16 (hipcc contracts by default).
#pragma clang fp contract(off)

// cache policy of the volume window loads (buffer-op aux bits) in the fused and
// the reference-layout cooperative lookups (A/B builds: 2 = nt; each
// wave-instruction there reads whole 128-B tiles, so no line is re-read later)
#ifndef DROID_VOL_LOAD_AUX
#define DROID_VOL_LOAD_AUX 2
#endif
// DROID_CE0_OUT_NT (A/B builds): the fused lookup's 128-channel output rows as
// non-temporal stores (0.8 GB at C3, past the caches)
#ifndef DROID_CE0_OUT_NT
#define DROID_CE0_OUT_NT 0
#endif

namespace droid {
typedef unsigned u32x4nt __attribute__((ext_vector_type(4)));  // non-temporal 16-B stores

template <typename T> struct Acc;
template <> struct Acc<__half> {
  // weight -> half, product -> half, sum -> half (at::Half operator semantics)
  __device__ static float weight(float w) { return rnd16(w); }
  __device__ static float madd(float acc, float s, float w) {
    return rnd16(acc + rnd16(s * w));
  }
  __device__ static float load(const __half* p) { return __half2float(*p); }
  __device__ static __half store(float v) { return __float2half(v); }
};
template <> struct Acc<float> {
  __device__ static float weight(float w) { return w; }
  __device__ static float madd(float acc, float s, float w) { return fmaf(s, w, acc); }
  __device__ static float load(const float* p) { return *p; }
  __device__ static float store(float v) { return v; }
};
template <> struct Acc<double> {
  __device__ static double weight(float w) { return (double)w; }
  __device__ static double madd(double acc, double s, double w) { return fma(s, w, acc); }
  __device__ static double load(const double* p) { return *p; }
  __device__ static double store(double v) { return v; }
};

template <typename T> struct Compute { using type = float; };
template <> struct Compute<double> { using type = double; };

// ---------------------------------------------------------------------------
// Generic per-level lookup: one thread per (n, y, x).  `out_bstride` lets the
// pyramid path write level i straight into its channel slice of the
// concatenated output.  Taps outside the volume are skipped (adding an exact
// zero is identical: the running sum can never be -0).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
corr_index_fwd_kernel(const T* __restrict__ volume, const float* __restrict__ coords,
                      int coords_layout_hw2, float scale, T* __restrict__ corr,
                      long out_bstride, int B, int H, int W, int H2, int W2, int r) {
  using C = typename Compute<T>::type;
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  if (p >= HW) return;
  float x0, y0;
  if (coords_layout_hw2) {  // (B, H, W, 2)
    x0 = coords[((long)n * HW + p) * 2 + 0] * scale;
    y0 = coords[((long)n * HW + p) * 2 + 1] * scale;
  } else {  // (B, 2, H, W)
    x0 = coords[((long)n * 2 + 0) * HW + p] * scale;
    y0 = coords[((long)n * 2 + 1) * HW + p] * scale;
  }
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xi0 = (int)fx0, yi0 = (int)fy0;
  const int rd = 2 * r + 1;
  const C w11 = Acc<T>::weight(dx * dy);
  const C w10 = Acc<T>::weight(dx * (1.0f - dy));
  const C w01 = Acc<T>::weight((1.0f - dx) * dy);
  const C w00 = Acc<T>::weight((1.0f - dx) * (1.0f - dy));
  const T* vol = volume + ((long)n * HW + p) * (long)H2 * W2;
  T* out = corr + (long)n * out_bstride + p;
  // Gather the (rd+1)^2 taps one x-column at a time, producing column a = i-1
  // once column i is known.  Columns of the window live in registers only
  // for the fixed radius-3 instantiation; generic radii use a small local
  // array (r <= 7 supported).
  C prev[16], cur[16];
  for (int i = 0; i <= rd; ++i) {
    const int x1 = xi0 - r + i;
    for (int j = 0; j <= rd; ++j) {
      const int y1 = yi0 - r + j;
      C s = 0;
      if (x1 >= 0 && x1 < W2 && y1 >= 0 && y1 < H2) s = (C)Acc<T>::load(vol + (long)y1 * W2 + x1);
      cur[j] = s;
    }
    if (i > 0) {
      const int a = i - 1;
      for (int b = 0; b < rd; ++b) {
        C acc = 0;
        acc = Acc<T>::madd(acc, prev[b], w00);
        acc = Acc<T>::madd(acc, prev[b + 1], w01);
        acc = Acc<T>::madd(acc, cur[b], w10);
        acc = Acc<T>::madd(acc, cur[b + 1], w11);
        out[(long)(a * rd + b) * HW] = Acc<T>::store(acc);
      }
    }
    for (int j = 0; j <= rd; ++j) prev[j] = cur[j];
  }
}

// ---------------------------------------------------------------------------
// Fast fp16 radius-3 pyramid lookup: one thread per (edge, pixel), all levels.
// Each window row (8 taps = 16 B at an arbitrary 2-B offset) is fetched as the
// two aligned 16-B chunks that cover it (requires W2 % 8 == 0) and funnel-
// shifted into place; arithmetic identical to corr_index_fwd_kernel<__half>.
// ---------------------------------------------------------------------------
struct PyramidArgs {
  const __half* vol[4];
  int H2[4];
  int W2[4];
  int levels;
  int fast;  // bit l: level l rows are 16-B aligned (W2 % 8 == 0)
};

__device__ __forceinline__ void load_row8_f16_scalar(const __half* row, int xs, int W2, float* t) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int x = xs + i;
    t[i] = (x >= 0 && x < W2) ? __half2float(row[x]) : 0.f;
  }
}

__device__ __forceinline__ void load_row8_f16(const __half* row, int xs, int W2, float* t) {
  // taps x = xs .. xs+7 of one volume row; zero outside [0, W2)
  const int c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);  // floor(xs/8)
  const int off = xs - 8 * c0;                                // 0..7
  const int nch = W2 >> 3;
  uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
  if (c0 >= 0 && c0 < nch) a = *reinterpret_cast<const uint4*>(row + 8 * c0);
  if (c0 + 1 >= 0 && c0 + 1 < nch) b = *reinterpret_cast<const uint4*>(row + 8 * (c0 + 1));
  unsigned u[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const int k = off >> 1;
  unsigned v[6], w[5];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[i] = (k & 2) ? u[i + 2] : u[i];
#pragma unroll
  for (int i = 0; i < 5; ++i) w[i] = (k & 1) ? v[i + 1] : v[i];
  const unsigned sh = (off & 1) ? 16u : 0u;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const unsigned o = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
    t[2 * m + 0] = __half2float(__ushort_as_half((unsigned short)(o & 0xffffu)));
    t[2 * m + 1] = __half2float(__ushort_as_half((unsigned short)(o >> 16)));
  }
}

template <bool NHWC>
__global__ void __launch_bounds__(256)
corr_pyramid_f16_r3_kernel(PyramidArgs args, const float* __restrict__ coords,
                           __half* __restrict__ out, int H, int W, int ocs) {
  constexpr int R = 3, RD = 7, L = 4;
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = blockIdx.y;
  if (p >= HW) return;
  const float cx = coords[((long)e * HW + p) * 2 + 0];
  const float cy = coords[((long)e * HW + p) * 2 + 1];
  const int nch = args.levels * RD * RD;
  __half* o = out + (long)e * nch * HW + p;
  // NHWC: the pixel's channels are packed in registers and written as 16-B rows
  unsigned pk[NHWC ? (L * RD * RD + 7) / 2 + 4 : 1];
  if (NHWC) {
#pragma unroll
    for (int q = 0; q < (int)(sizeof(pk) / sizeof(unsigned)); ++q) pk[q] = 0u;
  }
#pragma unroll
  for (int lvl = 0; lvl < L; ++lvl) {
    if (lvl >= args.levels) break;
    const float s = 1.0f / (float)(1 << lvl);
    const float x0 = cx * s, y0 = cy * s;
    const float fx0 = floorf(x0), fy0 = floorf(y0);
    const float dx = x0 - fx0, dy = y0 - fy0;
    const int xi0 = (int)fx0, yi0 = (int)fy0;
    const float w11 = rnd16(dx * dy);
    const float w10 = rnd16(dx * (1.0f - dy));
    const float w01 = rnd16((1.0f - dx) * dy);
    const float w00 = rnd16((1.0f - dx) * (1.0f - dy));
    const int H2 = args.H2[lvl], W2 = args.W2[lvl];
    const __half* vol = args.vol[lvl] + ((long)e * HW + p) * (long)H2 * W2;
    float prev[8], cur[8];
    __half* ol = o + (long)lvl * RD * RD * HW;
#pragma unroll
    for (int j = 0; j <= RD; ++j) {
      const int y1 = yi0 - R + j;
      if (y1 >= 0 && y1 < H2) {
        if ((args.fast >> lvl) & 1) load_row8_f16(vol + (long)y1 * W2, xi0 - R, W2, cur);
        else load_row8_f16_scalar(vol + (long)y1 * W2, xi0 - R, W2, cur);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = 0.f;
      }
      if (j > 0) {
        const int b = j - 1;
#pragma unroll
        for (int a = 0; a < RD; ++a) {
          float acc = 0.f + rnd16(prev[a] * w00);
          acc = rnd16(acc + rnd16(cur[a] * w01));
          acc = rnd16(acc + rnd16(prev[a + 1] * w10));
          acc = rnd16(acc + rnd16(cur[a + 1] * w11));
          if (NHWC) {
            const int ch = lvl * RD * RD + a * RD + b;
            const unsigned hv = (unsigned)__half_as_ushort(__float2half(acc));
            pk[ch >> 1] |= (ch & 1) ? (hv << 16) : hv;
          } else {
            ol[(long)(a * RD + b) * HW] = __float2half(acc);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) prev[i] = cur[i];
    }
  }
  if (NHWC) {
    uint4* dst = reinterpret_cast<uint4*>(out + ((long)e * HW + p) * ocs);
    const int n16 = ocs / 8;
#pragma unroll
    for (int q = 0; q < (L * RD * RD + 7) / 8; ++q)
      if (q < n16) dst[q] = make_uint4(pk[4 * q], pk[4 * q + 1], pk[4 * q + 2], pk[4 * q + 3]);
  }
}

// ---------------------------------------------------------------------------
// Round 4: fp16 radius-3 lookup of ONE level per thread (grid z = level) in the
// reference layout - the reference-layout drop-in's lookup (CorrBlock.__call__,
// modules/corr.py:40-50, and the per-level corr_index_forward it calls).  The
// 4-level kernel above walks a pixel's levels one after another with 16 loads
// in flight per thread and guarded loads (divergent branches + waits); here each
// (pixel, level) is its own thread, its 8 window rows (2 aligned 16-B pieces
// each) are 16 branch-free buffer loads against a per-block descriptor (pieces
// outside the slice use an out-of-range offset and load zeros), all in flight
// at once - 4x the memory-level parallelism.  Arithmetic identical to
// corr_pyramid_f16_r3_kernel (bit-exact at::Half semantics).  Needs W2 % 8 == 0
// and 16-B aligned levels; PLANAR: coords (B,2,H,W) (corr_index_forward),
// else (E,H,W,2) at level-0 scale.
// ---------------------------------------------------------------------------
// window row taps x = xs .. xs + 7: dwords off/2 .. of the row's two 16-B pieces, funnel-shifted
__device__ __forceinline__ void coop_taps(uint4 p0v, uint4 p1v, int off, float* t) {
  // plain values and selects (an array indexed under a select becomes a
  // scratch-memory array)
  const bool k2 = off & 4, k1 = off & 2;
  const unsigned v0 = k2 ? p0v.z : p0v.x, v1 = k2 ? p0v.w : p0v.y, v2 = k2 ? p1v.x : p0v.z;
  const unsigned v3 = k2 ? p1v.y : p0v.w, v4 = k2 ? p1v.z : p1v.x, v5 = k2 ? p1v.w : p1v.y;
  const unsigned w0 = k1 ? v1 : v0, w1 = k1 ? v2 : v1, w2 = k1 ? v3 : v2, w3 = k1 ? v4 : v3, w4 = k1 ? v5 : v4;
  const unsigned sh = (off & 1) ? 16u : 0u;
  const unsigned q0 = __builtin_amdgcn_alignbit(w1, w0, sh), q1 = __builtin_amdgcn_alignbit(w2, w1, sh);
  const unsigned q2 = __builtin_amdgcn_alignbit(w3, w2, sh), q3 = __builtin_amdgcn_alignbit(w4, w3, sh);
  const unsigned q[4] = {q0, q1, q2, q3};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    t[2 * m + 0] = __half2float(__ushort_as_half((unsigned short)(q[m] & 0xffffu)));
    t[2 * m + 1] = __half2float(__ushort_as_half((unsigned short)(q[m] >> 16)));
  }
}
__device__ __forceinline__ uint4 dpp_next_lane(uint4 v) {   // lane + 1's value (DPP row_shl:1)
  uint4 r;
  r.x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x101, 0xF, 0xF, false);
  r.y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x101, 0xF, 0xF, false);
  r.z = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x101, 0xF, 0xF, false);
  r.w = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x101, 0xF, 0xF, false);
  return r;
}

struct LookupLvlArgs {
  const __half* vol[4];
  int H2[4], W2[4];
  const int* slot;    // TILED: volume row of each edge (a slot pool) or null = e
  const float* coords;
  __half* out;
  long out_estride;   // output halves per edge
  int H, W;
  float coord_scale;  // PLANAR: coordinates already at the level's scale (1); else 1 / 2^l per level
};

// TILED (round 4): the same lookup reading the 8x8-tiled slot pool of the fused
// path, (R,H,W,ceil(H2/8),W2/8,8,8): a window row is still two 16-B pieces (one
// tile row of tile columns c0, c0 + 1), but a window's 8 rows lie in at most
// 2 x 2 tiles = four 128-B lines instead of 8-16 lines of the row-major slice -
// the reference API's lookup (CorrBlock.__call__, NCHW output) at the fused
// path's line efficiency.
template <bool PLANAR, bool TILED = false>
__global__ void __launch_bounds__(256) corr_lookup_lvl_kernel(LookupLvlArgs a) {
  constexpr int R = 3, RD = 7;
  const int HW = a.H * a.W;
  const int p0 = blockIdx.x * 256;
  const int p = p0 + threadIdx.x;
  const int e = blockIdx.y;
  const int lvl = blockIdx.z;
  const int H2 = a.H2[lvl], W2 = a.W2[lvl], nch = W2 >> 3;
  const long slice = TILED ? (long)((H2 + 7) >> 3) * 8 * W2 : (long)H2 * W2;
  const long vrow = (TILED && a.slot) ? (long)a.slot[e] : (long)e;
  const bool live = p < HW;
  const int pc = live ? p : HW - 1;
  float cx, cy;
  if (PLANAR) {
    cx = a.coords[((long)e * 2 + 0) * HW + pc];
    cy = a.coords[((long)e * 2 + 1) * HW + pc];
  } else {
    cx = a.coords[((long)e * HW + pc) * 2 + 0];
    cy = a.coords[((long)e * HW + pc) * 2 + 1];
  }
  const float s = PLANAR ? a.coord_scale : 1.0f / (float)(1 << lvl);
  const float x0 = cx * s, y0 = cy * s;
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xi0 = (int)fx0, yi0 = (int)fy0;
  const float w11 = rnd16(dx * dy);
  const float w10 = rnd16(dx * (1.0f - dy));
  const float w01 = rnd16((1.0f - dx) * dy);
  const float w00 = rnd16((1.0f - dx) * (1.0f - dy));
  // the block's 256 pixel slices as one descriptor (wave-uniform base)
  const long nblk = min(256, HW - p0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__half*>(a.vol[lvl] + (vrow * HW + p0) * slice), (short)0, (int)(nblk * slice * 2), kBufFlags);
  const unsigned pbase = (unsigned)((p - p0) * slice) * 2u;
  const int xs = xi0 - R;
  const int c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);
  const int off = xs - 8 * c0;
  const bool ok0 = live && c0 >= 0 && c0 < nch, ok1 = live && c0 + 1 >= 0 && c0 + 1 < nch;
  uint4 raw[8][2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int y1 = yi0 - R + j;
    const bool yok = y1 >= 0 && y1 < H2;
    // piece (row y1, tile column c): row-major y1 * W2 + 8 c; tiled (tile (y1/8, c), row y1 % 8)
    const int rb = TILED ? (y1 >> 3) * 8 * W2 + (y1 & 7) * 8 : y1 * W2;
    const int cm = TILED ? 64 : 8;
    const unsigned o0 = (yok && ok0) ? pbase + (unsigned)(rb + cm * c0) * 2u : kOob;
    const unsigned o1 = (yok && ok1) ? pbase + (unsigned)(rb + cm * (c0 + 1)) * 2u : kOob;
    raw[j][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o0, 0, 0));
    raw[j][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o1, 0, 0));
  }
  __half* o = a.out + (long)e * a.out_estride + (long)lvl * RD * RD * HW + pc;
  auto taps = [&](int j, float* t) { coop_taps(raw[j][0], raw[j][1], off, t); };
  float prev[8], cur[8];
  taps(0, prev);
#pragma unroll
  for (int j = 1; j <= RD; ++j) {
    taps(j, cur);
    const int b = j - 1;
#pragma unroll
    for (int x = 0; x < RD; ++x) {
      float acc = 0.f + rnd16(prev[x] * w00);
      acc = rnd16(acc + rnd16(cur[x] * w01));
      acc = rnd16(acc + rnd16(prev[x + 1] * w10));
      acc = rnd16(acc + rnd16(cur[x + 1] * w11));
      if (live) o[(long)(x * RD + b) * HW] = __float2half(acc);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) prev[i] = cur[i];
  }
}

// ---------------------------------------------------------------------------
// Cooperative NCHW lookup (round 4, the reference-layout CorrBlock.__call__):
// the same (pixel, level) arithmetic as corr_lookup_lvl_kernel, bit for bit,
// with the fused path's cooperative gather and staged stores.  A wave owns 64
// consecutive pixels of one edge and level; in round r lane (pp = lane >> 3,
// j = lane & 7) loads window row j (two 16-B pieces) of pixel 8 r + pp, so a
// load instruction touches 8 pixels x <= 2 lines each instead of 64 pixels x
// 4 lines (the per-thread kernel's TA / line pressure).  Window row j + 1 comes
// from the next lane (DPP row_shl:1, the 8-lane groups never straddle a DPP
// row), lane j < 7 forms the 7 outputs of window row j, and they go through
// an LDS tile [49 channels][64 px] so every global store is a 16-B piece of a
// 128-B channel row.  Needs H*W % 64 == 0 and a 16-B aligned output.
// ---------------------------------------------------------------------------
constexpr int kCoopPitch = 72;   // staging row pitch in halves (144 B: 16-B aligned rows)
template <bool TILED>
__global__ void __launch_bounds__(256) corr_lookup_coop_kernel(LookupLvlArgs a) {
  constexpr int R = 3, RD = 7, SP = kCoopPitch;
  __shared__ __attribute__((aligned(16))) __half stage[4][RD * RD * SP];
  const int HW = a.H * a.W;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pw0 = blockIdx.x * 256 + wave * 64;
  if (pw0 >= HW) return;   // wave-uniform (HW % 64 == 0); no workgroup barrier below
  const int e = blockIdx.y, lvl = blockIdx.z;
  const int H2 = a.H2[lvl], W2 = a.W2[lvl], nch = W2 >> 3;
  const long slice = TILED ? (long)((H2 + 7) >> 3) * 8 * W2 : (long)H2 * W2;
  const long vrow = (TILED && a.slot) ? (long)a.slot[e] : (long)e;
  const int pp = lane >> 3, j = lane & 7;
  const float s = 1.0f / (float)(1 << lvl);
  float2 cc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r)
    cc[r] = *reinterpret_cast<const float2*>(a.coords + ((long)e * HW + pw0 + 8 * r + pp) * 2);
  // the wave's 64 pixel slices as one descriptor
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__half*>(a.vol[lvl] + (vrow * HW + pw0) * slice), (short)0, (int)(64 * slice * 2), kBufFlags);
  auto geom = [&](int r, int& xs, int& c0, float& dx, float& dy, int& yi0) {
    const float x0 = cc[r].x * s, y0 = cc[r].y * s;
    const float fx0 = floorf(x0), fy0 = floorf(y0);
    dx = x0 - fx0;
    dy = y0 - fy0;
    yi0 = (int)fy0;
    xs = (int)fx0 - R;
    c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);
  };
  uint4 raw[8][2];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int xs, c0, yi0;
    float dx, dy;
    geom(r, xs, c0, dx, dy, yi0);
    const bool ok0 = c0 >= 0 && c0 < nch, ok1 = c0 + 1 >= 0 && c0 + 1 < nch;
    const int y1 = yi0 - R + j;
    const bool yok = y1 >= 0 && y1 < H2;
    const unsigned pbase = (unsigned)((8 * r + pp) * slice) * 2u;
    const int rb = TILED ? (y1 >> 3) * 8 * W2 + (y1 & 7) * 8 : y1 * W2;
    const int cm = TILED ? 64 : 8;
    const unsigned o0 = (yok && ok0) ? pbase + (unsigned)(rb + cm * c0) * 2u : kOob;
    const unsigned o1 = (yok && ok1) ? pbase + (unsigned)(rb + cm * (c0 + 1)) * 2u : kOob;
    raw[r][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o0, 0, DROID_VOL_LOAD_AUX));
    raw[r][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o1, 0, DROID_VOL_LOAD_AUX));
  }
  __half* const st = stage[wave];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int xs, c0, yi0;
    float dx, dy;
    geom(r, xs, c0, dx, dy, yi0);
    const int off = xs - 8 * c0;
    const float w11 = rnd16(dx * dy);
    const float w10 = rnd16(dx * (1.0f - dy));
    const float w01 = rnd16((1.0f - dx) * dy);
    const float w00 = rnd16((1.0f - dx) * (1.0f - dy));
    // window row j + 1 of the same pixel is lane + 1's row
    const uint4 n0 = dpp_next_lane(raw[r][0]), n1 = dpp_next_lane(raw[r][1]);
    float prev[8], cur[8];
    coop_taps(raw[r][0], raw[r][1], off, prev);
    coop_taps(n0, n1, off, cur);
    if (j < RD) {
#pragma unroll
      for (int x = 0; x < RD; ++x) {
        float acc = 0.f + rnd16(prev[x] * w00);
        acc = rnd16(acc + rnd16(cur[x] * w01));
        acc = rnd16(acc + rnd16(prev[x + 1] * w10));
        acc = rnd16(acc + rnd16(cur[x + 1] * w11));
        st[(x * RD + j) * SP + 8 * r + pp] = __float2half(acc);   // channel x*7 + b, b = j
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  __half* const o = a.out + (long)e * a.out_estride + (long)lvl * RD * RD * HW + pw0;
#pragma unroll
  for (int k0 = 0; k0 < RD * RD * 8; k0 += 64) {
    const int k = k0 + lane;
    if (k < RD * RD * 8) {
      const int ch = k >> 3, seg = k & 7;
      *reinterpret_cast<uint4*>(o + (long)ch * HW + seg * 8) = *reinterpret_cast<const uint4*>(&st[ch * SP + seg * 8]);
    }
  }
}

// ---------------------------------------------------------------------------
// corr_index_backward: scatter bilinear-weighted gradients into the volume
// (correlation_kernels.cu:73-124).  Each (n,y,x) owns its volume slice, so no
// atomics are needed.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
corr_index_bwd_kernel(const float* __restrict__ coords, const T* __restrict__ grad,
                      T* __restrict__ vgrad, int B, int H, int W, int H2, int W2, int r) {
  using C = typename Compute<T>::type;
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  if (p >= HW) return;
  const float x0 = coords[((long)n * 2 + 0) * HW + p];
  const float y0 = coords[((long)n * 2 + 1) * HW + p];
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xi0 = (int)fx0, yi0 = (int)fy0;
  const int rd = 2 * r + 1;
  const T* g = grad + (long)n * rd * rd * HW + p;
  T* vg = vgrad + ((long)n * HW + p) * (long)H2 * W2;
  for (int i = 0; i <= rd; ++i) {
    for (int j = 0; j <= rd; ++j) {
      const int x1 = xi0 - r + i, y1 = yi0 - r + j;
      if (!(x1 >= 0 && x1 < W2 && y1 >= 0 && y1 < H2)) continue;
      C acc = 0;
      if (i > 0 && j > 0) acc += (C)Acc<T>::load(g + (long)((i - 1) * rd + (j - 1)) * HW) * (C)(dx * dy);
      if (i > 0 && j < rd) acc += (C)Acc<T>::load(g + (long)((i - 1) * rd + j) * HW) * (C)(dx * (1.0f - dy));
      if (i < rd && j > 0) acc += (C)Acc<T>::load(g + (long)(i * rd + (j - 1)) * HW) * (C)((1.0f - dx) * dy);
      if (i < rd && j < rd) acc += (C)Acc<T>::load(g + (long)(i * rd + j) * HW) * (C)((1.0f - dx) * (1.0f - dy));
      T* dst = vg + (long)y1 * W2 + x1;
      *dst = Acc<T>::store((C)Acc<T>::load(dst) + acc);
    }
  }
}

// ---------------------------------------------------------------------------
// altcorr_forward: corr[b,s,7*ix+iy,h,w] = bilinear sample of <f1(h,w), f2(.)>
// over the radius window, computed on the fly from channels-last fmaps
// (altcorr_kernel.cu:27-149, race-free).  One thread per (b, s, pixel); the
// 64 per-tap dot products are accumulated over 32-channel chunks in fp32.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(64)
altcorr_fwd_kernel(const T* __restrict__ fmap1, const T* __restrict__ fmap2,
                   const float* __restrict__ coords, T* __restrict__ corr,
                   int B, int S, int H, int W, int H2, int W2, int C) {
  constexpr int R = 3, RD = 7, NT = 8;
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const int b = blockIdx.z;
  if (p >= HW) return;
  const float x = coords[(((long)b * S + s) * HW + p) * 2 + 0];
  const float y = coords[(((long)b * S + s) * HW + p) * 2 + 1];
  const float fx0 = floorf(x), fy0 = floorf(y);
  const float dx = x - fx0, dy = y - fy0;
  const int xi0 = (int)fx0, yi0 = (int)fy0;
  float dots[NT * NT];
#pragma unroll
  for (int k = 0; k < NT * NT; ++k) dots[k] = 0.f;
  const T* f1 = fmap1 + ((long)b * HW + p) * C;
  const T* f2b = fmap2 + (long)b * H2 * W2 * C;
  for (int c0 = 0; c0 < C; c0 += 8) {
    float a[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) a[c] = (c0 + c < C) ? (float)f1[c0 + c] : 0.f;
#pragma unroll
    for (int iy = 0; iy < NT; ++iy) {
      const int h2 = yi0 - R + iy;
#pragma unroll
      for (int ix = 0; ix < NT; ++ix) {
        const int w2 = xi0 - R + ix;
        if (h2 < 0 || h2 >= H2 || w2 < 0 || w2 >= W2) continue;
        const T* f2 = f2b + ((long)h2 * W2 + w2) * C + c0;
        float acc = dots[iy * NT + ix];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c0 + c < C) acc = fmaf(a[c], (float)f2[c], acc);
        dots[iy * NT + ix] = acc;
      }
    }
  }
  T* out = corr + (((long)b * S + s) * RD * RD) * HW + p;
#pragma unroll
  for (int ix = 0; ix < RD; ++ix) {
#pragma unroll
    for (int iy = 0; iy < RD; ++iy) {
      // output (iy, ix) collects taps (iy,ix) se, (iy+1,ix) ne, (iy,ix+1) sw, (iy+1,ix+1) nw
      float v = dots[iy * NT + ix] * ((1.f - dy) * (1.f - dx));
      v += dots[(iy + 1) * NT + ix] * (dy * (1.f - dx));
      v += dots[iy * NT + ix + 1] * ((1.f - dy) * dx);
      v += dots[(iy + 1) * NT + ix + 1] * (dy * dx);
      out[(long)(iy + RD * ix) * HW] = (T)v;
    }
  }
}

// altcorr_backward (fp32): g1 owned per pixel, g2 scattered with atomics.
__global__ void __launch_bounds__(64)
altcorr_bwd_kernel(const float* __restrict__ fmap1, const float* __restrict__ fmap2,
                   const float* __restrict__ coords, const float* __restrict__ grad,
                   float* __restrict__ g1, float* __restrict__ g2,
                   int B, int S, int H, int W, int H2, int W2, int C) {
  constexpr int R = 3, RD = 7, NT = 8;
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.z;
  if (p >= HW) return;
  for (int s = 0; s < S; ++s) {
    const float x = coords[(((long)b * S + s) * HW + p) * 2 + 0];
    const float y = coords[(((long)b * S + s) * HW + p) * 2 + 1];
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float dx = x - fx0, dy = y - fy0;
    const int xi0 = (int)fx0, yi0 = (int)fy0;
    const float* G = grad + (((long)b * S + s) * RD * RD) * HW + p;
    for (int iy = 0; iy < NT; ++iy) {
      for (int ix = 0; ix < NT; ++ix) {
        const int h2 = yi0 - R + iy, w2 = xi0 - R + ix;
        if (h2 < 0 || h2 >= H2 || w2 < 0 || w2 >= W2) continue;
        float g = 0.f;
        if (iy > 0 && ix > 0) g += G[(long)((iy - 1) + RD * (ix - 1)) * HW] * dy * dx;
        if (iy > 0 && ix < RD) g += G[(long)((iy - 1) + RD * ix) * HW] * dy * (1 - dx);
        if (iy < RD && ix > 0) g += G[(long)(iy + RD * (ix - 1)) * HW] * (1 - dy) * dx;
        if (iy < RD && ix < RD) g += G[(long)(iy + RD * ix) * HW] * (1 - dy) * (1 - dx);
        if (g == 0.f) continue;
        const float* f2 = fmap2 + (((long)b * H2 + h2) * W2 + w2) * C;
        const float* f1 = fmap1 + ((long)b * HW + p) * C;
        float* d1 = g1 + ((long)b * HW + p) * C;
        float* d2 = g2 + (((long)b * H2 + h2) * W2 + w2) * C;
        for (int c = 0; c < C; ++c) {
          d1[c] += g * f2[c];
          atomicAdd(d2 + c, g * f1[c]);
        }
      }
    }
  }
}

}  // namespace droid

// ===========================================================================
// C ABI
// ===========================================================================
using namespace droid;

// A/B build, DROID_LOOKUP_V1=1: the round-3 one-launch kernel
// (corr_pyramid_f16_r3_kernel, NCHW out) for the reference-layout lookups; the
// product library takes corr_lookup_lvl / corr_lookup_coop there (the r3 kernel
// stays the channels-last fallback, droid_corr_pyramid_lookup_nhwc)
static bool lookup_lvl_on() {
  static const bool on = ab_knob("DROID_LOOKUP_V1", 0) != 1;
  return on;
}

// the cooperative NCHW lookup (corr_lookup_coop_kernel) for the 4-level
// reference lookups; droid_lookup_set_coop(0) (or DROID_LOOKUP_COOP=0 in the
// A/B build) for the per-thread kernel (A/B and the bitwise test)
static int& lookup_coop() {
  static int v = ab_knob("DROID_LOOKUP_COOP", 1) == 0 ? 0 : 1;
  return v;
}
static bool coop_ok(int HW, const void* out, long maxslice) {
  return lookup_coop() && HW % 64 == 0 && !(reinterpret_cast<uintptr_t>(out) & 15u) && 64 * maxslice * 2 < 0x7fffffffL;
}

extern "C" {

#if DROID_TESTING
int droid_lookup_set_coop(int on) {
  lookup_coop() = on ? 1 : 0;
  return kOk;
}
#endif  // DROID_TESTING

// dtype codes: 0 = fp16, 1 = fp32, 2 = fp64
int droid_corr_index_forward(int dtype, const void* volume, const float* coords, void* corr,
                             int B, int H, int W, int H2, int W2, int radius, hipStream_t stream) {
  if (B < 0 || H <= 0 || W <= 0 || H2 <= 0 || W2 <= 0 || radius < 0 || radius > 7)
    return fail(kInvalidArgument, "corr_index_forward: bad shape or radius (0..7)");
  if (B == 0) return kOk;
  const int rd = 2 * radius + 1;
  const long bstride = (long)rd * rd * H * W;
  if (dtype == 0 && radius == 3 && W2 % 8 == 0 && !(reinterpret_cast<uintptr_t>(volume) & 15) && lookup_lvl_on() &&
      (long)256 * H2 * W2 * 2 < 0x7fffffffL) {
    LookupLvlArgs a{};
    a.vol[0] = (const __half*)volume;
    a.H2[0] = H2;
    a.W2[0] = W2;
    a.coords = coords;
    a.out = (__half*)corr;
    a.out_estride = bstride;
    a.H = H;
    a.W = W;
    a.coord_scale = 1.0f;
    corr_lookup_lvl_kernel<true><<<dim3(ceil_div(H * W, 256), B, 1), 256, 0, stream>>>(a);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  dim3 grid(ceil_div(H * W, 256), B);
  switch (dtype) {
    case 0: corr_index_fwd_kernel<__half><<<grid, 256, 0, stream>>>((const __half*)volume, coords, 0, 1.0f, (__half*)corr, bstride, B, H, W, H2, W2, radius); break;
    case 1: corr_index_fwd_kernel<float><<<grid, 256, 0, stream>>>((const float*)volume, coords, 0, 1.0f, (float*)corr, bstride, B, H, W, H2, W2, radius); break;
    case 2: corr_index_fwd_kernel<double><<<grid, 256, 0, stream>>>((const double*)volume, coords, 0, 1.0f, (double*)corr, bstride, B, H, W, H2, W2, radius); break;
    default: return fail(kUnsupported, "corr_index_forward: dtype must be fp16/fp32/fp64");
  }
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_corr_index_backward(int dtype, const float* coords, const void* corr_grad, void* volume_grad,
                              int B, int H, int W, int H2, int W2, int radius, hipStream_t stream) {
  if (B < 0 || H <= 0 || W <= 0 || H2 <= 0 || W2 <= 0 || radius < 0)
    return fail(kInvalidArgument, "corr_index_backward: bad shape");
  if (B == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), B);
  switch (dtype) {
    case 0: corr_index_bwd_kernel<__half><<<grid, 256, 0, stream>>>(coords, (const __half*)corr_grad, (__half*)volume_grad, B, H, W, H2, W2, radius); break;
    case 1: corr_index_bwd_kernel<float><<<grid, 256, 0, stream>>>(coords, (const float*)corr_grad, (float*)volume_grad, B, H, W, H2, W2, radius); break;
    case 2: corr_index_bwd_kernel<double><<<grid, 256, 0, stream>>>(coords, (const double*)corr_grad, (double*)volume_grad, B, H, W, H2, W2, radius); break;
    default: return fail(kUnsupported, "corr_index_backward: dtype must be fp16/fp32/fp64");
  }
  DROID_LAUNCH_CHECK();
  return kOk;
}

// CorrBlock.__call__ over the fused path's 8x8-tiled slot pool (see
// corr_lookup_lvl_kernel<.., TILED>): fp16, radius 3, levels[l] (R,H,W,
// ceil(H2/8),W2/8,8,8), edge e's volume at row slot[e] (slot null: row e);
// out (E, L*49, H, W) fp16, bit-exact with droid_corr_pyramid_lookup on the
// row-major volume.
int droid_corr_pyramid_lookup_tiled(const void* const* levels, const int* H2s, const int* W2s, const int* slot,
                                    int num_levels, const float* coords, void* out, int E, int H, int W,
                                    hipStream_t stream) {
  if (num_levels < 1 || num_levels > 4 || E < 0 || H <= 0 || W <= 0)
    return fail(kInvalidArgument, "corr_pyramid_lookup_tiled: bad arguments");
  if (E == 0) return kOk;
  long maxslice = 0;
  LookupLvlArgs a{};
  for (int l = 0; l < num_levels; ++l) {
    if (H2s[l] <= 0 || W2s[l] <= 0 || W2s[l] % 8 != 0 || (reinterpret_cast<uintptr_t>(levels[l]) & 15u))
      return fail(kInvalidArgument, "corr_pyramid_lookup_tiled: levels need W2 % 8 == 0 and 16-B alignment");
    maxslice = std::max(maxslice, (long)((H2s[l] + 7) / 8) * 8 * W2s[l]);
    a.vol[l] = (const __half*)levels[l];
    a.H2[l] = H2s[l];
    a.W2[l] = W2s[l];
  }
  if (256 * maxslice * 2 >= 0x7fffffffL) return fail(kInvalidArgument, "corr_pyramid_lookup_tiled: slice too large");
  a.slot = slot;
  a.coords = coords;
  a.out = (__half*)out;
  a.out_estride = (long)num_levels * 49 * H * W;
  a.H = H;
  a.W = W;
  a.coord_scale = 1.0f;
  if (coop_ok(H * W, out, maxslice))
    corr_lookup_coop_kernel<true><<<dim3(ceil_div(H * W, 256), E, num_levels), 256, 0, stream>>>(a);
  else
    corr_lookup_lvl_kernel<false, true><<<dim3(ceil_div(H * W, 256), E, num_levels), 256, 0, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_corr_pyramid_lookup(int dtype, const void* const* levels, const int* H2s, const int* W2s,
                              int num_levels, const float* coords, void* out,
                              int E, int H, int W, int radius, hipStream_t stream) {
  if (num_levels < 1 || num_levels > 4 || E < 0 || H <= 0 || W <= 0 || radius < 0 || radius > 7)
    return fail(kInvalidArgument, "corr_pyramid_lookup: bad arguments");
  if (E == 0) return kOk;
  const int rd = 2 * radius + 1;
  bool fast = (dtype == 0 && radius == 3);
  for (int l = 0; l < num_levels; ++l) {
    if (H2s[l] <= 0 || W2s[l] <= 0) return fail(kInvalidArgument, "corr_pyramid_lookup: empty level");
    if (W2s[l] % 8 != 0 || (reinterpret_cast<uintptr_t>(levels[l]) & 15u)) fast = false;
  }
  dim3 grid(ceil_div(H * W, 256), E);
  long maxslice = 0;
  for (int l = 0; l < num_levels; ++l) maxslice = std::max(maxslice, (long)H2s[l] * W2s[l]);
  if (fast && lookup_lvl_on() && 256 * maxslice * 2 < 0x7fffffffL) {
    LookupLvlArgs a{};
    for (int l = 0; l < num_levels; ++l) {
      a.vol[l] = (const __half*)levels[l];
      a.H2[l] = H2s[l];
      a.W2[l] = W2s[l];
    }
    a.coords = coords;
    a.out = (__half*)out;
    a.out_estride = (long)num_levels * rd * rd * H * W;
    a.H = H;
    a.W = W;
    a.coord_scale = 1.0f;
    if (coop_ok(H * W, out, maxslice))
      corr_lookup_coop_kernel<false><<<dim3(ceil_div(H * W, 256), E, num_levels), 256, 0, stream>>>(a);
    else
      corr_lookup_lvl_kernel<false><<<dim3(ceil_div(H * W, 256), E, num_levels), 256, 0, stream>>>(a);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  if (fast) {
    PyramidArgs a;
    for (int l = 0; l < 4; ++l) {
      a.vol[l] = (const __half*)levels[l < num_levels ? l : 0];
      a.H2[l] = H2s[l < num_levels ? l : 0];
      a.W2[l] = W2s[l < num_levels ? l : 0];
    }
    a.levels = num_levels;
    a.fast = 0xf;
    corr_pyramid_f16_r3_kernel<false><<<grid, 256, 0, stream>>>(a, coords, (__half*)out, H, W, 0);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  const long bstride = (long)num_levels * rd * rd * H * W;
  for (int l = 0; l < num_levels; ++l) {
    const float scale = 1.0f / (float)(1 << l);
    const long off = (long)l * rd * rd * H * W;
    switch (dtype) {
      case 0: corr_index_fwd_kernel<__half><<<grid, 256, 0, stream>>>((const __half*)levels[l], coords, 1, scale, (__half*)out + off, bstride, E, H, W, H2s[l], W2s[l], radius); break;
      case 1: corr_index_fwd_kernel<float><<<grid, 256, 0, stream>>>((const float*)levels[l], coords, 1, scale, (float*)out + off, bstride, E, H, W, H2s[l], W2s[l], radius); break;
      case 2: corr_index_fwd_kernel<double><<<grid, 256, 0, stream>>>((const double*)levels[l], coords, 1, scale, (double*)out + off, bstride, E, H, W, H2s[l], W2s[l], radius); break;
      default: return fail(kUnsupported, "corr_pyramid_lookup: dtype must be fp16/fp32/fp64");
    }
    DROID_LAUNCH_CHECK();
  }
  return kOk;
}

// CorrBlock lookup writing channels-last (E, H, W, out_cstride) fp16 rows with
// zero padding past L*(2r+1)^2 channels: the A operand layout of the fused
// update operator.  fp16 volumes, radius 3, 4 levels, W2 % 8 == 0.
int droid_corr_pyramid_lookup_nhwc(const void* const* levels, const int* H2s, const int* W2s,
                                   int num_levels, const float* coords, void* out, int out_cstride,
                                   int E, int H, int W, hipStream_t stream) {
  if (num_levels != 4 || out_cstride % 8 || out_cstride < 196 || out_cstride > 200)
    return fail(kUnsupported, "corr_pyramid_lookup_nhwc: needs 4 levels and channel stride 200");
  PyramidArgs a;
  a.fast = 0;
  for (int l = 0; l < 4; ++l) {
    if (H2s[l] <= 0 || W2s[l] <= 0) return fail(kInvalidArgument, "corr_pyramid_lookup_nhwc: empty level");
    a.vol[l] = (const __half*)levels[l];
    a.H2[l] = H2s[l];
    a.W2[l] = W2s[l];
    if (W2s[l] % 8 == 0 && (reinterpret_cast<uintptr_t>(levels[l]) & 15) == 0) a.fast |= 1 << l;
  }
  a.levels = 4;
  if (E == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), E);
  corr_pyramid_f16_r3_kernel<true><<<grid, 256, 0, stream>>>(a, coords, (__half*)out, H, W, out_cstride);
  DROID_LAUNCH_CHECK();
  return kOk;
}

extern "C++" {  // (inside the extern "C" block: the kernel below is a template)
namespace droid {

// ---------------------------------------------------------------------------
// Fused CorrBlock lookup + corr_encoder[0] (modules/corr.py:40-50 feeding
// droid_net.py:84-86: conv1x1 196 -> 128, bias, ReLU): the 196-channel
// lookup of a 128-pixel tile is built in LDS (bit-identical to
// corr_pyramid_f16_r3_kernel) and multiplied on MFMA by the resident 1x1
// weights, so the 2.5 GB lookup tensor of a 2048-edge graph is never written
// or re-read.  Persistent: one 8-wave workgroup per CU keeps the 128x224
// weight tile in LDS and walks the pixel tiles; while tile t is multiplied and
// stored, the window rows of tile t+1 (issued right after t's gather) and the
// coordinates of tile t+2 are in flight.
// Gather: wave w handles level w & 3 for pixels 64 (w >> 2) + lane; each
// lane loads its 8 window rows as 2 aligned 16-B chunks (W2 % 8 == 0).
// ---------------------------------------------------------------------------
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

struct CorrCe0Args {
  const __half* vol[4];
  int H2[4], W2[4];
  const float* coords;  // (E, H, W, 2)
  int fast;             // bit l: level l rows are 16-B aligned (W2 % 8 == 0)
  int tiled;            // bit l: level l slices stored in 8x8 tiles (droid_corr_lookup_ce0_tiled)
  const __half* w;      // [128][224], columns >= 196 zero
  const float* bias;    // [128]
  __half* out;          // (E, H, W, 128)
  const int* slot;      // (E) volume row of edge e (a slot pool, droid_corr_lookup_ce0_tiled_slots), or null = e
  int HW;
  long ntiles;
};

constexpr int kCeTP = 128, kCeKS = 232, kCeOS = 136;
constexpr unsigned kCeOob = 0x80000000u;  // buffer offset past any descriptor: the load returns 0
// + coordinate staging Cs [2 slots][8 waves][64 px] float2 (LDS-DMA), private
// per wave: the four waves of a pixel half would otherwise share a slot, and a
// wave ahead could overwrite it (tile t + 4g) before a wave behind has read it
// (tile t + 2g) - nothing orders different waves' reads and DMAs in between
constexpr int kCeLds = (2 * 128 * kCeKS + kCeTP * kCeOS) * 2 + 2 * 8 * 64 * 8;
static_assert(kCeLds <= 160 * 1024, "corr_ce0 LDS budget");

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// LDS-DMA of 4 B per lane (buffer_load_dword ... lds): lane l's dword lands at
// LDS byte `lds` + 4 l.  Preceded by lgkmcnt(0) so that the issuing wave's
// earlier ds_reads of the destination have returned (write-after-read).
__device__ __forceinline__ void ce_dma4(rsrc_t rs, unsigned lds, unsigned voff) {
  const rsrc_t r = {__builtin_amdgcn_readfirstlane(rs.x), __builtin_amdgcn_readfirstlane(rs.y),
                    __builtin_amdgcn_readfirstlane(rs.z), __builtin_amdgcn_readfirstlane(rs.w)};
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// FAST: every level's rows are 16-B aligned (W2 % 8 == 0) - the gather is
// branch-free buffer loads only, which keeps the compiler's vmcnt accounting
// exact across the loop (a CFG join with the generic path makes it wait for 0)
#ifndef DROID_CE0_ABLATE_TA
#define DROID_CE0_ABLATE_TA 0
#endif
// Cooperative gather (FAST path): lane (pixel pp = lane >> 3, window row j =
// lane & 7) loads one window row of eight pixels per instruction instead of
// one pixel's row per lane: an instruction then touches ~16 128-B lines
// instead of 64 - the texture-address path was full for ~53 % of the kernel's
// cycles (SQ_VMEM_TA_ADDR_FIFO_FULL, profiles/r03/pmc_sq_r03bj.txt); the row
// below comes from the next lane by one DPP shift.  DROID_CE0_COOP=0: one
// pixel per lane (A/B builds).  Outputs are bitwise the same.
#ifndef DROID_CE0_COOP
#define DROID_CE0_COOP 1
#endif
template <bool FAST>
__global__ void __launch_bounds__(512) corr_ce0_kernel(CorrCe0Args a) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem_ce[];
  _Float16* Ws = smem_ce;                 // [128 co][kCeKS]
  _Float16* As = Ws + 128 * kCeKS;        // [128 px][kCeKS] lookup tile (cols 196.. zero)
  _Float16* Os = As + kCeTP * kCeKS;      // [128 px][kCeOS] output staging
  float2* Cs = reinterpret_cast<float2*>(Os + kCeTP * kCeOS);  // [2 slots][8 waves][64 px]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // level is wave-uniform: keep it (and everything derived from it) in SGPRs
  const int lvl = __builtin_amdgcn_readfirstlane(wave & 3), px = (wave >> 2) * 64 + lane;
  const int HW = a.HW, tpe = HW / kCeTP;  // tiles per edge

  for (int idx = tid; idx < 128 * 29; idx += 512) {
    const int r = idx / 29, q = idx - r * 29;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < 28) v = *reinterpret_cast<const uint4*>(a.w + r * 224 + q * 8);
    *reinterpret_cast<uint4*>(&Ws[r * kCeKS + q * 8]) = v;
  }
  // the K padding 196..223 the MFMA reads; columns 224..231 (never read by it)
  // are the cooperative gather's coordinate parking slots, written below
  // without a barrier in between - zeroing them here would race with those writes
  for (int idx = tid; idx < kCeTP * 28; idx += 512) {
    const int r = idx / 28, c = idx - r * 28;
    As[r * kCeKS + 196 + c] = (_Float16)0.f;
  }

  const int H2 = a.H2[lvl], W2 = a.W2[lvl], nch = W2 >> 3;
  const bool fast = FAST || ((a.fast >> lvl) & 1);  // rows 16-B aligned
  const __half* vol = a.vol[lvl];
  // 8x8-tiled slices (tiled bit): element (y, x) at ((y>>3) * W2/8 + (x>>3)) * 64
  // + (y&7) * 8 + (x&7), H2 padded to a multiple of 8 - a window's 8 rows then
  // touch ~3.5 128-B lines instead of 8 (one per row of the row-major slice)
  const bool tiled = (a.tiled >> lvl) & 1;
  const long slice = tiled ? (long)((H2 + 7) & ~7) * W2 : (long)H2 * W2;
  const float scl = 1.0f / (float)(1 << lvl);

  // per-lane gather state of the two tiles in flight (slot = iteration parity)
  uint4 raw[2][8][2];
  float wdx[2] = {0.f, 0.f}, wdy[2] = {0.f, 0.f};  // bilinear fractions
  int woff[2] = {0, 0};                             // window x offset within the first chunk
  auto tile_pixel = [&](long t) { return (t / tpe) * (long)HW + (t % tpe) * kCeTP + px; };
  // the volume row of tile t's edge (wave-uniform scalar load when the volume is a slot pool)
  auto vol_row = [&](long t) -> long {
    const long e = t / tpe;
    return a.slot ? (long)__builtin_amdgcn_readfirstlane(a.slot[e]) : e;
  };
  auto load_coords = [&](long t, float& x, float& y) {
    if (t < a.ntiles) {
      const float2 c = *reinterpret_cast<const float2*>(a.coords + tile_pixel(t) * 2);
      x = c.x; y = c.y;
    }
  };
  // Coordinates of the tile a slot issues next are staged in this wave's own LDS
  // region by its own LDS-DMA (its 64 pixels, 2 x 4 B per lane), issued right BEFORE the slot's
  // window rows: when the wave has waited for those rows (the bilinear step),
  // the coordinates have landed too (vmcnt retires in order) and no VGPR holds a
  // load across the loop - a loop-carried loaded value costs a vmcnt wait on its
  // copy at the back edge, which would drain the other slot's rows.
  const int half = wave >> 2;
  const unsigned cs_lds = lds_addr(Cs) + (unsigned)(wave * 512);
  auto stage_coords = [&](const int sl, long t) __attribute__((always_inline)) {
    if (t >= a.ntiles) return;
    const long p0 = (t / tpe) * (long)HW + (t % tpe) * kCeTP + half * 64;
    const rsrc_t rs = make_rsrc(a.coords + p0 * 2, 512);
    const unsigned dst = cs_lds + (unsigned)(sl * 4096);
    ce_dma4(rs, dst, (unsigned)lane * 4u);
    ce_dma4(rs, dst + 256, 256u + (unsigned)lane * 4u);
  };
  auto issue = [&](const int sl, long t, float cx, float cy) __attribute__((always_inline)) {
    const bool valid = t < a.ntiles;  // uniform; FAST: past the last tile every offset is out of range
    if (!FAST && !valid) return;
    const float x0 = cx * scl, y0 = cy * scl;
    const float fx0 = floorf(x0), fy0 = floorf(y0);
    wdx[sl] = x0 - fx0; wdy[sl] = y0 - fy0;
    const int xi0 = (int)fx0, yi0 = (int)fy0;
    const int xs = xi0 - 3;
    const int c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);
    woff[sl] = xs - 8 * c0;
    if (fast) {
      // buffer loads relative to the tile's first slice (wave-uniform descriptor;
      // a tile never crosses an edge since HW % 128 == 0): window pieces outside
      // the slice get an out-of-range offset and return zeros - no branches, so
      // all 16 loads of the lane stay in flight together
      const long tp0 = valid ? vol_row(t) * (long)HW + (t % tpe) * kCeTP : 0;
      const unsigned long long pa = (unsigned long long)(vol + tp0 * slice);
      const unsigned long long pu = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(pa >> 32)) << 32) |
                                    (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)pa);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(pu), (short)0, __builtin_amdgcn_readfirstlane((int)(kCeTP * slice * 2)), 0x00020000);
#if DROID_CE0_ABLATE_TA   // timing ablation only (results invalid): 8 lanes share one pixel's slice
      const unsigned pbase = (unsigned)((px & ~7) * slice) * 2u;
#else
      const unsigned pbase = (unsigned)(px * slice) * 2u;
#endif
      const bool ok0 = valid && c0 >= 0 && c0 < nch, ok1 = valid && c0 + 1 >= 0 && c0 + 1 < nch;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int y1 = yi0 - 3 + j;
        const bool yok = y1 >= 0 && y1 < H2;
        // 16-B piece c of row y1: row-major y1*W2 + 8c, tiled ((y1>>3)*nch + c)*64 + (y1&7)*8
        const int re = tiled ? (y1 >> 3) * nch * 64 + (y1 & 7) * 8 : y1 * W2;
        const int cs = tiled ? 64 : 8;
        const unsigned o0 = (yok && ok0) ? pbase + (unsigned)(re + cs * c0) * 2u : kCeOob;
        const unsigned o1 = (yok && ok1) ? pbase + (unsigned)(re + cs * (c0 + 1)) * 2u : kCeOob;
        raw[sl][j][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o0, 0, DROID_VOL_LOAD_AUX));
        raw[sl][j][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o1, 0, DROID_VOL_LOAD_AUX));
      }
    } else if constexpr (!FAST) {
      const __half* base = vol + (vol_row(t) * (long)HW + (t % tpe) * kCeTP + px) * slice;
      // rows not 16-B aligned (W2 % 8 != 0): the 8 taps one by one, packed as an
      // aligned chunk (window offset 0)
      woff[sl] = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int y1 = yi0 - 3 + j;
        const bool yok = y1 >= 0 && y1 < H2;
        const unsigned short* row = reinterpret_cast<const unsigned short*>(base + (long)y1 * W2);
        unsigned u[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int xa = xs + 2 * m, xb = xa + 1;
          const unsigned lo = (yok && xa >= 0 && xa < W2) ? row[xa] : 0u;
          const unsigned hi = (yok && xb >= 0 && xb < W2) ? row[xb] : 0u;
          u[m] = lo | (hi << 16);
        }
        raw[sl][j][0] = make_uint4(u[0], u[1], u[2], u[3]);
        raw[sl][j][1] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  // row j of slot sl's window as 8 floats (the taps x = xs .. xs+7)
  // Row j of slot sl's window as fp16 pairs: T[m] = (tap 2m, tap 2m+1) and
  // S[m] = (tap 2m+1, tap 2m+2) of the taps x = xs .. xs+7 (S[3].x = tap 7).
  auto row_pairs = [&](const int sl, int j, h2_t* T, h2_t* S) __attribute__((always_inline)) {
    // dword m + k of the two pieces, k = woff / 2 in 0..3, as explicit selects on
    // scalars (a select over an array index becomes a dynamic index into scratch,
    // whose vmcnt waits would drain the window loads still in flight)
    const uint4 p0 = raw[sl][j][0], p1 = raw[sl][j][1];
    const int k = woff[sl] >> 1;
    const bool k2 = k & 2, k1 = k & 1;
    const unsigned v0 = k2 ? p0.z : p0.x, v1 = k2 ? p0.w : p0.y, v2 = k2 ? p1.x : p0.z;
    const unsigned v3 = k2 ? p1.y : p0.w, v4 = k2 ? p1.z : p1.x, v5 = k2 ? p1.w : p1.y;
    const unsigned w[5] = {k1 ? v1 : v0, k1 ? v2 : v1, k1 ? v3 : v2, k1 ? v4 : v3, k1 ? v5 : v4};
    const unsigned sh = (woff[sl] & 1) ? 16u : 0u;
    unsigned o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) o[m] = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      T[m] = __builtin_bit_cast(h2_t, o[m]);
      S[m] = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(m < 3 ? o[m + 1] : 0u, o[m], 16));
    }
  };

  // ---- cooperative gather (FAST, DROID_CE0_COOP): lane = (pixel pp, row jr);
  // pixel group g of the wave's 64 = pixel 64 half + 8 g + pp.  The per-pixel
  // window state of an in-flight tile is not held in registers (8 pixels per
  // lane): the pixel's coordinates are parked in columns 224..231 of its As row
  // (never read by the K <= 224 MFMA; float2 per slot) and the state is
  // recomputed at the bilinear step.
  constexpr bool kCoop = FAST && DROID_CE0_COOP;
  const int pp = lane >> 3, jr = lane & 7;
  // cg: this wave's staged coordinates of tile t (64 px, LDS), read one pixel
  // group at a time
  auto issue_co = [&](const int sl, long t, const float2* cg) __attribute__((always_inline)) {
    const bool valid = t < a.ntiles;
    const long tp0 = valid ? vol_row(t) * (long)HW + (t % tpe) * kCeTP : 0;
    const unsigned long long pa = (unsigned long long)(vol + tp0 * slice);
    const unsigned long long pu = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(pa >> 32)) << 32) |
                                  (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)pa);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pu), (short)0, __builtin_amdgcn_readfirstlane((int)(kCeTP * slice * 2)), 0x00020000);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float2 cc = cg[8 * g + pp];
      const float x0 = cc.x * scl, y0 = cc.y * scl;
      const int xi0 = (int)floorf(x0), yi0 = (int)floorf(y0);
      const int xs = xi0 - 3;
      const int c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);
      const unsigned pbase = (unsigned)((half * 64 + 8 * g + pp) * slice) * 2u;
      const bool ok0 = valid && c0 >= 0 && c0 < nch, ok1 = valid && c0 + 1 >= 0 && c0 + 1 < nch;
      const int y1 = yi0 - 3 + jr;
      const bool yok = y1 >= 0 && y1 < H2;
      const int re = tiled ? (y1 >> 3) * nch * 64 + (y1 & 7) * 8 : y1 * W2;
      const int cs = tiled ? 64 : 8;
      const unsigned o0 = (yok && ok0) ? pbase + (unsigned)(re + cs * c0) * 2u : kCeOob;
      const unsigned o1 = (yok && ok1) ? pbase + (unsigned)(re + cs * (c0 + 1)) * 2u : kCeOob;
      raw[sl][g][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o0, 0, DROID_VOL_LOAD_AUX));
      raw[sl][g][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o1, 0, DROID_VOL_LOAD_AUX));
    }
  };
  // bilinear windows of slot sl's tile -> As: lane (pp, jr) forms output row jr
  // (jr < 7) of pixel group g from its row (jr) and the next lane's (jr + 1),
  // the same products and sums, in the same order, as the per-pixel path
  auto bilinear_co = [&](const int sl) __attribute__((always_inline)) {
#pragma clang fp contract(off)
    const h2_t Z = {(_Float16)0.f, (_Float16)0.f};
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int pxg = half * 64 + 8 * g + pp;
      const float2 c = *reinterpret_cast<const float2*>(&As[pxg * kCeKS + 224 + 4 * sl]);
      const float x0 = c.x * scl, y0 = c.y * scl;
      const float fx0 = floorf(x0), fy0 = floorf(y0);
      const float dx = x0 - fx0, dy = y0 - fy0;
      const int xs = (int)fx0 - 3;
      const int c0 = (xs >= 0) ? (xs >> 3) : -((-xs + 7) >> 3);
      const int wo = xs - 8 * c0;
      const _Float16 h11 = (_Float16)rnd16(dx * dy);
      const _Float16 h10 = (_Float16)rnd16(dx * (1.0f - dy));
      const _Float16 h01 = (_Float16)rnd16((1.0f - dx) * dy);
      const _Float16 h00 = (_Float16)rnd16((1.0f - dx) * (1.0f - dy));
      const h2_t W00 = {h00, h00}, W01 = {h01, h01}, W10 = {h10, h10}, W11 = {h11, h11};
      // this row's tap pairs (dword m + wo/2 of the two pieces, funnel-shifted)
      const uint4 p0 = raw[sl][g][0], p1 = raw[sl][g][1];
      const int k = wo >> 1;
      const bool k2 = k & 2, k1 = k & 1;
      const unsigned v0 = k2 ? p0.z : p0.x, v1 = k2 ? p0.w : p0.y, v2 = k2 ? p1.x : p0.z;
      const unsigned v3 = k2 ? p1.y : p0.w, v4 = k2 ? p1.z : p1.x, v5 = k2 ? p1.w : p1.y;
      const unsigned w[5] = {k1 ? v1 : v0, k1 ? v2 : v1, k1 ? v3 : v2, k1 ? v4 : v3, k1 ? v5 : v4};
      const unsigned sh = (wo & 1) ? 16u : 0u;
      unsigned o[4], q[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) o[m] = __builtin_amdgcn_alignbit(w[m + 1], w[m], sh);
#pragma unroll
      for (int m = 0; m < 4; ++m) q[m] = __builtin_amdgcn_alignbit(m < 3 ? o[m + 1] : 0u, o[m], 16);
      _Float16* arow = As + pxg * kCeKS + lvl * 49;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        // the row below: the next lane's pairs (row_shl:1; lane jr = 7 outputs nothing)
        const unsigned oc = (unsigned)__builtin_amdgcn_update_dpp(0, (int)o[m], 0x101, 0xF, 0xF, false);
        const unsigned qc = (unsigned)__builtin_amdgcn_update_dpp(0, (int)q[m], 0x101, 0xF, 0xF, false);
        h2_t acc = Z + __builtin_bit_cast(h2_t, o[m]) * W00;
        acc = acc + __builtin_bit_cast(h2_t, oc) * W01;
        acc = acc + __builtin_bit_cast(h2_t, q[m]) * W10;
        acc = acc + __builtin_bit_cast(h2_t, qc) * W11;
        if (jr < 7) {
          arow[(2 * m) * 7 + jr] = acc.x;
          if (m < 3) arow[(2 * m + 1) * 7 + jr] = acc.y;
        }
      }
    }
  };

  // GEMM geometry: waves 4 (32 px) x 2 (64 co)
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fq = lane >> 4;
  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = a.bias[wn * 64 + j * 16 + fr];

  // one tile: windows of slot sl -> As, then (with the tile two steps ahead
  // issued into the same slot) the 1x1 conv on MFMA and the coalesced store
  auto process = [&](const int sl, long t) __attribute__((always_inline)) {
   if constexpr (kCoop) {
    bilinear_co(sl);
   } else {
    // (1) bilinear windows of tile t -> As (corr_pyramid_f16_r3_kernel arithmetic)
    //     on packed fp16 pairs of x offsets (q, q+1).  The reference rounds every
    //     product and sum of two halves to half through float (at::Half ops);
    //     a native half op rounds the exact result once, and float carries 24 >=
    //     2*11 + 2 bits, so the double rounding is innocuous: bit-identical.
    //     No contraction (an fma would round once where the reference rounds twice).
    {
#pragma clang fp contract(off)
      const _Float16 h11 = (_Float16)rnd16(wdx[sl] * wdy[sl]);
      const _Float16 h10 = (_Float16)rnd16(wdx[sl] * (1.0f - wdy[sl]));
      const _Float16 h01 = (_Float16)rnd16((1.0f - wdx[sl]) * wdy[sl]);
      const _Float16 h00 = (_Float16)rnd16((1.0f - wdx[sl]) * (1.0f - wdy[sl]));
      const h2_t W00 = {h00, h00}, W01 = {h01, h01}, W10 = {h10, h10}, W11 = {h11, h11};
      const h2_t Z = {(_Float16)0.f, (_Float16)0.f};
      _Float16* arow = As + px * kCeKS + lvl * 49;
      h2_t Tp[4], Sp[4], Tc[4], Sc[4];
      row_pairs(sl, 0, Tp, Sp);
#pragma unroll
      for (int j = 1; j <= 7; ++j) {
        row_pairs(sl, j, Tc, Sc);
        const int b = j - 1;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          h2_t acc = Z + Tp[m] * W00;   // (0 + p w00: +0 for a -0 product, as in float)
          acc = acc + Tc[m] * W01;
          acc = acc + Sp[m] * W10;
          acc = acc + Sc[m] * W11;
          arow[(2 * m) * 7 + b] = acc.x;
          if (m < 3) arow[(2 * m + 1) * 7 + b] = acc.y;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          Tp[m] = Tc[m];
          Sp[m] = Sc[m];
        }
      }
    }
   }
    // (2) the tile two steps ahead goes into this slot while this one is multiplied
    // and stored; its coordinates were staged before the rows just consumed.
    const float2 c2 = Cs[sl * 512 + wave * 64 + lane];  // staged with the rows just consumed
    if constexpr (kCoop) {
      // the rows first, then the coordinates' DMA over the staging slot they
      // were read from (ce_dma4 waits for this wave's LDS reads; the rows'
      // vmcnt wait at the bilinear step covers the later DMA: in-order retirement)
      issue_co(sl, t + 2L * gridDim.x, Cs + sl * 512 + wave * 64);
      stage_coords(sl, t + 4L * gridDim.x);
    } else {
      stage_coords(sl, t + 4L * gridDim.x);
      issue(sl, t + 2L * gridDim.x, c2.x, c2.y);
    }
    __syncthreads();
    // coop: park the coordinates of the tile just issued (read by its bilinear
    // step two steps on; every wave of this one's bilinear step is past the barrier)
    if (kCoop && lvl == 0) *reinterpret_cast<float2*>(&As[(half * 64 + lane) * kCeKS + 224 + 4 * sl]) = c2;
    // (3) 128 px x 128 co x 224 on MFMA
    floatx4_t acc[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[f][j] = floatx4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) {
      half8_t af[2], bf[4];
#pragma unroll
      for (int f = 0; f < 2; ++f)
        af[f] = *reinterpret_cast<const half8_t*>(&As[(wm * 32 + f * 16 + fr) * kCeKS + ks * 32 + fq * 8]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const half8_t*>(&Ws[(wn * 64 + j * 16 + fr) * kCeKS + ks * 32 + fq * 8]);
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[f], bf[j], acc[f][j], 0, 0, 0);
    }
    // (4) bias + ReLU -> Os -> coalesced 16-B stores
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          Os[(wm * 32 + f * 16 + fq * 4 + k) * kCeOS + wn * 64 + j * 16 + fr] =
              (_Float16)fmaxf(acc[f][j][k] + bias[j], 0.f);
    __syncthreads();
    if (t >= a.ntiles) return;  // uniform: the odd step past the last tile computes but stores nothing
    const long pix0 = (t / tpe) * (long)HW + (t % tpe) * kCeTP;
    for (int idx = tid; idx < kCeTP * 16; idx += 512) {
      const int r = idx >> 4, q = idx & 15;
      const uint4 ov = *reinterpret_cast<const uint4*>(&Os[r * kCeOS + q * 8]);
      if constexpr (DROID_CE0_OUT_NT) __builtin_nontemporal_store(__builtin_bit_cast(u32x4nt, ov), reinterpret_cast<u32x4nt*>(a.out + (pix0 + r) * 128 + q * 8));
      else *reinterpret_cast<uint4*>(a.out + (pix0 + r) * 128 + q * 8) = ov;
    }
  };

  const long g = gridDim.x;
  long t = blockIdx.x;
  if constexpr (kCoop) {
    // the first two tiles' coordinates straight from memory: eight pixels per
    // lane for the gather, the lane's own pixel for the As parking slot
    // (the gather reads 64 coordinates per wave straight from memory here; a
    // tile past the last one reads tile 0's, which are finite, and loads nothing)
    const float2* cg0 = reinterpret_cast<const float2*>(a.coords) + ((t < a.ntiles ? t : 0) / tpe) * (long)HW +
                        ((t < a.ntiles ? t : 0) % tpe) * kCeTP + half * 64;
    const float2* cg1 = reinterpret_cast<const float2*>(a.coords) + ((t + g < a.ntiles ? t + g : 0) / tpe) * (long)HW +
                        ((t + g < a.ntiles ? t + g : 0) % tpe) * kCeTP + half * 64;
    float cx0 = 0.f, cy0 = 0.f, cx1 = 0.f, cy1 = 0.f;
    load_coords(t, cx0, cy0);
    load_coords(t + g, cx1, cy1);
    if (lvl == 0) {
      *reinterpret_cast<float2*>(&As[px * kCeKS + 224]) = make_float2(cx0, cy0);
      *reinterpret_cast<float2*>(&As[px * kCeKS + 228]) = make_float2(cx1, cy1);
    }
    stage_coords(0, t + 2 * g);
    issue_co(0, t, cg0);
    stage_coords(1, t + 3 * g);
    issue_co(1, t + g, cg1);
  } else {
    float cx0 = 0.f, cy0 = 0.f, cx1 = 0.f, cy1 = 0.f;
    load_coords(t, cx0, cy0);
    load_coords(t + g, cx1, cy1);
    stage_coords(0, t + 2 * g);
    issue(0, t, cx0, cy0);
    stage_coords(1, t + 3 * g);
    issue(1, t + g, cx1, cy1);
  }
  __syncthreads();  // weights and pad columns are in LDS
  // two tiles in flight per lane (16 window rows each): slot 0 holds the even
  // steps, slot 1 the odd ones.  Both steps run unconditionally (a guarded
  // second step would make the loop-carried coordinates a phi whose copy waits
  // for the loads in flight); a step past the last tile loads and stores nothing.
  for (; t < a.ntiles; t += 2 * g) {
    process(0, t);
    process(1, t + g);
  }
}

}  // namespace droid
}  // extern "C++"

// Fused CorrBlock lookup + corr_encoder[0] (see corr_ce0_kernel).
static int corr_lookup_ce0_impl(const void* const* levels, const int* H2s, const int* W2s, const float* coords,
                                const void* w, const float* bias, void* out, int E, int H, int W, bool tiled,
                                const int* slot, hipStream_t stream) {
  using namespace droid;
  if ((H * W) % kCeTP)
    return fail(kUnsupported, "corr_lookup_ce0: H*W must be a multiple of 128");
  CorrCe0Args a{};
  for (int l = 0; l < 4; ++l) {
    if (H2s[l] <= 0 || W2s[l] <= 0) return fail(kInvalidArgument, "corr_lookup_ce0: empty level");
    const bool aligned = W2s[l] % 8 == 0 && (reinterpret_cast<uintptr_t>(levels[l]) & 15) == 0;
    if (tiled && !aligned) return fail(kUnsupported, "corr_lookup_ce0_tiled: W2 % 8 != 0 or unaligned level");
    if (aligned) a.fast |= 1 << l;
    if (tiled) a.tiled |= 1 << l;
    a.vol[l] = (const __half*)levels[l];
    a.H2[l] = H2s[l];
    a.W2[l] = W2s[l];
  }
  if (!w || !bias || !out || !coords) return fail(kInvalidArgument, "corr_lookup_ce0: null pointer");
  a.coords = coords;
  a.w = (const __half*)w;
  a.bias = bias;
  a.out = (__half*)out;
  a.HW = H * W;
  a.slot = slot;
  a.ntiles = (long)E * (H * W / kCeTP);
  if (a.ntiles == 0) return kOk;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_ce0_kernel<true>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kCeLds));
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_ce0_kernel<false>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kCeLds));
    attr = true;
  }
  const long grid = std::min<long>(a.ntiles, device_cu_count());
  if (a.fast == 15)
    corr_ce0_kernel<true><<<dim3((unsigned)grid), 512, kCeLds, stream>>>(a);
  else
    corr_ce0_kernel<false><<<dim3((unsigned)grid), 512, kCeLds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_corr_lookup_ce0(const void* const* levels, const int* H2s, const int* W2s, const float* coords,
                          const void* w, const float* bias, void* out, int E, int H, int W, hipStream_t stream) {
  return corr_lookup_ce0_impl(levels, H2s, W2s, coords, w, bias, out, E, H, W, false, nullptr, stream);
}

int droid_corr_lookup_ce0_tiled(const void* const* levels, const int* H2s, const int* W2s, const float* coords,
                                const void* w, const float* bias, void* out, int E, int H, int W,
                                hipStream_t stream) {
  return corr_lookup_ce0_impl(levels, H2s, W2s, coords, w, bias, out, E, H, W, true, nullptr, stream);
}

// The same on a slot pool: edge e's volume is row slot[e] of the levels (device
// int32 (E)); the frontend's edge edits then move no volume bytes.
int droid_corr_lookup_ce0_tiled_slots(const void* const* levels, const int* H2s, const int* W2s, const int* slot,
                                      const float* coords, const void* w, const float* bias, void* out, int E, int H,
                                      int W, hipStream_t stream) {
  if (!slot) return fail(kInvalidArgument, "corr_lookup_ce0_tiled_slots: null slot map");
  return corr_lookup_ce0_impl(levels, H2s, W2s, coords, w, bias, out, E, H, W, true, slot, stream);
}

int droid_altcorr_forward(int dtype, const void* fmap1, const void* fmap2, const float* coords,
                          void* corr, int B, int S, int H, int W, int H2, int W2, int C,
                          int radius, hipStream_t stream) {
  if (radius != 3) return fail(kUnsupported, "altcorr_forward: only radius 3 is implemented");
  if (B < 0 || S <= 0 || H <= 0 || W <= 0 || H2 <= 0 || W2 <= 0 || C <= 0)
    return fail(kInvalidArgument, "altcorr_forward: bad shape");
  if (B == 0) return kOk;
  dim3 grid(ceil_div(H * W, 64), S, B);
  switch (dtype) {
    case 0: altcorr_fwd_kernel<__half><<<grid, 64, 0, stream>>>((const __half*)fmap1, (const __half*)fmap2, coords, (__half*)corr, B, S, H, W, H2, W2, C); break;
    case 1: altcorr_fwd_kernel<float><<<grid, 64, 0, stream>>>((const float*)fmap1, (const float*)fmap2, coords, (float*)corr, B, S, H, W, H2, W2, C); break;
    default: return fail(kUnsupported, "altcorr_forward: dtype must be fp16/fp32");
  }
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_altcorr_backward(const float* fmap1, const float* fmap2, const float* coords,
                           const float* corr_grad, float* fmap1_grad, float* fmap2_grad,
                           int B, int S, int H, int W, int H2, int W2, int C, int radius,
                           hipStream_t stream) {
  if (radius != 3) return fail(kUnsupported, "altcorr_backward: only radius 3 is implemented");
  if (B == 0) return kOk;
  dim3 grid(ceil_div(H * W, 64), 1, B);
  altcorr_bwd_kernel<<<grid, 64, 0, stream>>>(fmap1, fmap2, coords, corr_grad, fmap1_grad, fmap2_grad,
                                             B, S, H, W, H2, W2, C);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
