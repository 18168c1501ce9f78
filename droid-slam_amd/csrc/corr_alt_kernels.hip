// On-the-fly correlation pyramid lookup fused with corr_encoder[0], gfx950.
//
// The reference's CorrBlock (modules/corr.py:23-71) materialises, per edge, the
// all-pairs volume  V0[p][q] = <f1(p)/4, f2(q)/4>  (fp16, HW x HW) and its 2x2
// average-pooled levels, and the update reads a bilinear 8x8 window of every
// level at coords(p)/2^l (correlation_kernels.cu:19-70).  By linearity level l
// equals <f1(p)/4, avgpool^l(f2/4)(q)> - the reference's own AltCorrBlock
// (corr.py:91-139) - so the windows can be computed when they are needed from
// a feature pyramid of the frames (NHWC fp16, a few hundred MB) instead of
// gathered from a 51 GB volume whose 16-B window rows make the lookup
// DRAM-burst bound.
//
// corr_alt_ce0_kernel: persistent, one 8-wave workgroup per CU.  Work unit =
// an 8x8-pixel query tile of one edge.  Per level:
//   * the union of the 64 windows (their bounding box, clipped to the map) is
//     DMA'd from the f2 pyramid level into LDS (NHWC rows are contiguous, one
//     16-B piece per lane, XOR-swizzled slots);
//   * C = F1 (64 px x 128) x box^T on MFMA (f32 accumulate), rounded to fp16 -
//     the values the volume would hold at those taps;
//   * each pixel's 7x7 bilinear outputs are formed from its 8x8 taps of C with
//     the volume lookup's at::Half arithmetic (rnd16 after every op).
// A tile whose box exceeds the LDS capacity (incoherent coordinates) is split
// into its four 4x4 quadrants, and a quadrant still too wide into single
// pixels (box = the pixel's own window); correctness never depends on
// coherence, only speed does.  The 196 lookup channels of the tile then go
// through corr_encoder[0] (1x1 196 -> 128, bias, ReLU) on MFMA with the
// weights held in registers (wave w owns output channels 16w .. 16w+15), and
// only the 128-channel result is written.
//
// Numerics vs the volume path: level 0 differs only in the fp32 summation order
// of the dot products before their fp16 rounding; levels >= 1 pool the
// features instead of the correlations (both fp16), a difference at the fp16
// rounding level.  The bilinear arithmetic and the corr_encoder[0] GEMM are
// the same.
#include "common.hpp"
#include "lds_dma.hpp"

#include <algorithm>

// the bilinear at::Half arithmetic needs every product and sum rounded separately
#pragma clang fp contract(off)

namespace droid {

struct AltArgs {
  const __half* pyr[4];  // level l: (NF, H_l, W_l, 128) fp16 = avgpool^l(fmap / 4)
  int Hl[4], Wl[4];
  const int* f1;         // (E) frame (pyramid row) of the query features
  const int* f2;         // (E) frame of the target features
  const float* coords;   // (E, H, W, 2)
  const __half* w;       // [128][224] corr_encoder[0] weights (columns >= 196 zero)
  const float* bias;     // [128]
  __half* out;           // (E, H, W, 128)
  int H, W;
  long ntiles;           // E * (H / 8) * (W / 8)
};

constexpr int kAltCap = 240;   // box taps held in LDS
constexpr int kAltCS = 248;    // C row stride (halves)
constexpr int kAltAS = 232;    // lookup tile row stride (halves)
constexpr int kAltOS = 136;    // output staging row stride (halves)
constexpr int kAltMaxGroups = 1 + 4 + 64;
// LDS map (bytes)
constexpr int kAltF1 = 0;                                  // [64 px][256 B] query features
constexpr int kAltBox = kAltF1 + 64 * 256;                 // [kAltCap taps][256 B]  (output staging aliases it)
constexpr int kAltC = kAltBox + kAltCap * 256;             // [64 px][kAltCS] fp16
constexpr int kAltA = kAltC + 64 * kAltCS * 2;             // [64 px][kAltAS] fp16 lookup tile
constexpr int kAltMeta = kAltA + 64 * kAltAS * 2;          // per px: cx, cy, box x0, y0, bw (5 x 4 B)
constexpr int kAltGrp = kAltMeta + 64 * 5 * 4;             // groups: x0, y0, bw, bh, mmask, pix (6 x 4 B)
constexpr int kAltLds = kAltGrp + (kAltMaxGroups * 6 + 4) * 4;

// tile pixel p = 16 q + r: quadrant q = (qy, qx) = (q >> 1, q & 1), r = (ry, rx)
__device__ __forceinline__ int alt_py(int p) { return 4 * ((p >> 4) >> 1) + ((p & 15) >> 2); }
__device__ __forceinline__ int alt_px(int p) { return 4 * ((p >> 4) & 1) + (p & 3); }

__global__ void __launch_bounds__(512) corr_alt_ce0_kernel(AltArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* meta = reinterpret_cast<float*>(lds + kAltMeta);
  int* imeta = reinterpret_cast<int*>(lds + kAltMeta);
  int* grp = reinterpret_cast<int*>(lds + kAltGrp);
  _Float16* Cs = reinterpret_cast<_Float16*>(lds + kAltC);
  _Float16* As = reinterpret_cast<_Float16*>(lds + kAltA);
  _Float16* Os = reinterpret_cast<_Float16*>(lds + kAltBox);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int H = a.H, W = a.W, HW = H * W;
  const int tcols = W / 8, tpe = (H / 8) * tcols;
  const unsigned lds_a = lds_addr(lds);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  // corr_encoder[0] B fragments of this wave's 16 output channels, all 7 K-steps
  half8 wb[7];
#pragma unroll
  for (int ks = 0; ks < 7; ++ks)
    wb[ks] = *reinterpret_cast<const half8*>(a.w + (wave * 16 + fr) * 224 + ks * 32 + fq * 8);
  const float bias = a.bias[wave * 16 + fr];
  // lookup-tile pad columns 196..231 stay zero
  for (int idx = tid; idx < 64 * 36; idx += 512) As[(idx / 36) * kAltAS + 196 + idx % 36] = (_Float16)0.f;

  for (long t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const long e = t / tpe;
    const int tt = (int)(t - e * tpe);
    const int ty0 = (tt / tcols) * 8, tx0 = (tt % tcols) * 8;
    const int f1 = a.f1[e], f2 = a.f2[e];

    // query features of the 64 pixels -> LDS (16 x 1 KB DMA, 2 per wave)
    {
      const rsrc_t rs = make_rsrc(a.pyr[0] + (long)f1 * HW * 128, (unsigned)HW * 256);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ins = wave_u + 8 * q;
        const int p = ins * 4 + (lane >> 4);
        const int piece = (lane & 15) ^ (p & 15);
        const unsigned off = (unsigned)((((ty0 + alt_py(p)) * W + tx0 + alt_px(p)) * 128 + piece * 8) * 2);
        dma16(rs, lds_a + kAltF1 + ins * 1024, off);
      }
    }
    if (tid < 64) {
      const float2 c = *reinterpret_cast<const float2*>(a.coords + ((e * H + ty0 + alt_py(tid)) * (long)W + tx0 + alt_px(tid)) * 2);
      meta[tid * 5 + 0] = c.x;
      meta[tid * 5 + 1] = c.y;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // query A fragments stay in registers for all four levels
    half8 af[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int row = q * 16 + fr, piece = ks * 4 + fq;
        af[q][ks] = *reinterpret_cast<const half8*>(lds + kAltF1 + row * 256 + ((piece ^ (row & 15)) << 4));
      }

    for (int lvl = 0; lvl < 4; ++lvl) {
      const int Hl = a.Hl[lvl], Wl = a.Wl[lvl];
      const float scl = 1.0f / (float)(1 << lvl);
      // ---- groups: wave 0, one lane per pixel ----
      if (wave == 0) {
        const float x0 = meta[lane * 5 + 0] * scl, y0 = meta[lane * 5 + 1] * scl;
        const int ox = (int)fminf(fmaxf(floorf(x0), -1e6f), 1e6f) - 3;
        const int oy = (int)fminf(fmaxf(floorf(y0), -1e6f), 1e6f) - 3;
        // bounding boxes of the windows (tile, quadrant), clipped to the map
        int bx0 = ox, bx1 = ox + 7, by0 = oy, by1 = oy + 7;
        int qx0 = bx0, qx1 = bx1, qy0 = by0, qy1 = by1;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
          bx0 = min(bx0, __shfl_xor(bx0, m)); bx1 = max(bx1, __shfl_xor(bx1, m));
          by0 = min(by0, __shfl_xor(by0, m)); by1 = max(by1, __shfl_xor(by1, m));
          if (m < 16) {
            qx0 = min(qx0, __shfl_xor(qx0, m)); qx1 = max(qx1, __shfl_xor(qx1, m));
            qy0 = min(qy0, __shfl_xor(qy0, m)); qy1 = max(qy1, __shfl_xor(qy1, m));
          }
        }
        auto clip = [&](int& x0c, int& x1c, int& y0c, int& y1c) {
          x0c = max(x0c, 0); x1c = min(x1c, Wl - 1); y0c = max(y0c, 0); y1c = min(y1c, Hl - 1);
          return (x1c >= x0c && y1c >= y0c) ? (x1c - x0c + 1) * (y1c - y0c + 1) : 0;
        };
        const int tn = clip(bx0, bx1, by0, by1);
        const int qn = clip(qx0, qx1, qy0, qy1);
        int px0 = ox, px1 = ox + 7, py0 = oy, py1 = oy + 7;
        const int pn = clip(px0, px1, py0, py1);
        // lane's group box (its pixel's C row is indexed in it)
        int gx0, gy0, gbw;
        if (tn <= kAltCap) { gx0 = bx0; gy0 = by0; gbw = bx1 - bx0 + 1; }
        else if (qn <= kAltCap) { gx0 = qx0; gy0 = qy0; gbw = qx1 - qx0 + 1; }
        else { gx0 = px0; gy0 = py0; gbw = px1 - px0 + 1; }
        imeta[lane * 5 + 2] = gx0;
        imeta[lane * 5 + 3] = gy0;
        imeta[lane * 5 + 4] = gbw;
        // group list: the tile if its box fits; else per quadrant q (in order) the
        // quadrant if its box fits, or its 16 pixels one by one
        if (tn <= kAltCap) {
          if (lane == 0) {
            int* g = grp + 4;
            g[0] = bx0; g[1] = by0; g[2] = tn ? bx1 - bx0 + 1 : 0; g[3] = tn ? by1 - by0 + 1 : 0;
            g[4] = 15; g[5] = -1;
            grp[0] = 1;
          }
        } else {
          const unsigned long long narrow = __ballot(qn <= kAltCap);  // bit 16 q: quadrant q fits
          const int q = lane >> 4;
          int base = 0, ng = 0;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int cnt = ((narrow >> (16 * qq)) & 1ull) ? 1 : 16;
            if (qq < q) base += cnt;
            ng += cnt;
          }
          if (qn <= kAltCap) {
            if ((lane & 15) == 0) {
              int* g = grp + 4 + 6 * base;
              g[0] = qx0; g[1] = qy0; g[2] = qn ? qx1 - qx0 + 1 : 0; g[3] = qn ? qy1 - qy0 + 1 : 0;
              g[4] = 1 << q; g[5] = -1;
            }
          } else {
            int* g = grp + 4 + 6 * (base + (lane & 15));
            g[0] = px0; g[1] = py0; g[2] = pn ? px1 - px0 + 1 : 0; g[3] = pn ? py1 - py0 + 1 : 0;
            g[4] = 1 << q; g[5] = lane;
          }
          if (lane == 0) grp[0] = ng;
        }
      }
      __syncthreads();
      const int ng = grp[0];
      const rsrc_t rs = make_rsrc(a.pyr[lvl] + (long)f2 * Hl * Wl * 128, (unsigned)(Hl * Wl * 256));
      // ---- per group: box -> LDS, C = F1 x box^T ----
      for (int gi = 0; gi < ng; ++gi) {
        const int* g = grp + 4 + 6 * gi;
        const int gx0 = g[0], gy0 = g[1], gbw = g[2], gbh = g[3], mmask = g[4], gpix = g[5];
        const int tn = gbw * gbh;
        if (tn > 0) {
          const int nins = (tn + 3) >> 2;
          for (int ins = wave_u; ins < nins; ins += 8) {
            const int tap = ins * 4 + (lane >> 4);
            const int piece = (lane & 15) ^ (tap & 15);
            const int ry = tap / gbw, rx = tap - ry * gbw;
            const unsigned off = tap < tn ? (unsigned)((((gy0 + ry) * Wl + gx0 + rx) * 128 + piece * 8) * 2) : kOob;
            dma16(rs, lds_a + kAltBox + ins * 1024, off);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int nb = (tn + 15) >> 4;
        for (int b = wave_u; b < nb; b += 8) {
          half8 bf[4];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const int row = b * 16 + fr, piece = ks * 4 + fq;
            bf[ks] = *reinterpret_cast<const half8*>(lds + kAltBox + row * 256 + ((piece ^ (row & 15)) << 4));
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!((mmask >> q) & 1)) continue;
            floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[q][ks], bf[ks], c, 0, 0, 0);
            const int tap = b * 16 + fr;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int p = q * 16 + fq * 4 + k;
              if (tap < tn && (gpix < 0 || gpix == p)) Cs[p * kAltCS + tap] = (_Float16)c[k];
            }
          }
        }
        __syncthreads();  // box free for the next group, C complete
      }
      // ---- bilinear windows (volume-lookup arithmetic): thread (px, a) -> 7 outputs ----
      if (tid < 64 * 7) {
        const int p = tid / 7, ac = tid - p * 7;
        const float x0 = meta[p * 5 + 0] * scl, y0 = meta[p * 5 + 1] * scl;
        const float fx0 = floorf(x0), fy0 = floorf(y0);
        const float dx = x0 - fx0, dy = y0 - fy0;
        const int xi0 = (int)fminf(fmaxf(fx0, -1e6f), 1e6f), yi0 = (int)fminf(fmaxf(fy0, -1e6f), 1e6f);
        const float w11 = rnd16(dx * dy);
        const float w10 = rnd16(dx * (1.0f - dy));
        const float w01 = rnd16((1.0f - dx) * dy);
        const float w00 = rnd16((1.0f - dx) * (1.0f - dy));
        const int gx0 = imeta[p * 5 + 2], gy0 = imeta[p * 5 + 3], gbw = imeta[p * 5 + 4];
        const _Float16* crow = Cs + p * kAltCS;
        auto tapv = [&](int x, int y) -> float {
          return (x >= 0 && x < Wl && y >= 0 && y < Hl) ? (float)crow[(y - gy0) * gbw + (x - gx0)] : 0.f;
        };
        const int xa = xi0 - 3 + ac;
        float pa = 0.f, pb = 0.f;
        _Float16* arow = As + p * kAltAS + lvl * 49 + ac * 7;
#pragma unroll
        for (int j = 0; j <= 7; ++j) {
          const int y = yi0 - 3 + j;
          const float ca = tapv(xa, y), cb = tapv(xa + 1, y);
          if (j > 0) {
            float acc = 0.f + rnd16(pa * w00);
            acc = rnd16(acc + rnd16(ca * w01));
            acc = rnd16(acc + rnd16(pb * w10));
            acc = rnd16(acc + rnd16(cb * w11));
            arow[j - 1] = (_Float16)acc;
          }
          pa = ca;
          pb = cb;
        }
      }
      __syncthreads();  // C and the per-pixel group boxes are reused by the next level
    }

    // ---- corr_encoder[0]: 64 px x 16 co per wave, K = 224 ----
    floatx4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const half8 x = *reinterpret_cast<const half8*>(&As[(q * 16 + fr) * kAltAS + ks * 32 + fq * 8]);
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, wb[ks], acc[q], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        Os[(q * 16 + fq * 4 + k) * kAltOS + wave * 16 + fr] = (_Float16)fmaxf(acc[q][k] + bias, 0.f);
    __syncthreads();
    for (int idx = tid; idx < 64 * 16; idx += 512) {
      const int p = idx >> 4, pc = idx & 15;
      const long m = (e * H + ty0 + alt_py(p)) * (long)W + tx0 + alt_px(p);
      *reinterpret_cast<uint4*>(a.out + m * 128 + pc * 8) = *reinterpret_cast<const uint4*>(&Os[p * kAltOS + pc * 8]);
    }
    __syncthreads();  // output staging (box region) and meta free for the next tile
  }
}

}  // namespace droid

using namespace droid;

extern "C" {

// On-the-fly CorrBlock lookup fused with corr_encoder[0] (corr_alt_ce0_kernel).
int droid_corr_alt_ce0(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                       const float* coords, const void* w, const float* bias, void* out, int E, int H, int W,
                       hipStream_t stream) {
  if (E < 0 || H <= 0 || W <= 0 || !coords || !w || !bias || !out || !f1 || !f2)
    return fail(kInvalidArgument, "corr_alt_ce0: bad arguments");
  if (H % 8 || W % 8) return fail(kUnsupported, "corr_alt_ce0: H and W must be multiples of 8");
  AltArgs a{};
  for (int l = 0; l < 4; ++l) {
    if (!pyr[l] || Hl[l] <= 0 || Wl[l] <= 0 || (reinterpret_cast<uintptr_t>(pyr[l]) & 15))
      return fail(kInvalidArgument, "corr_alt_ce0: bad pyramid level");
    if ((long)Hl[l] * Wl[l] * 256 > 0x7fffffffL) return fail(kUnsupported, "corr_alt_ce0: level too large");
    a.pyr[l] = (const __half*)pyr[l];
    a.Hl[l] = Hl[l];
    a.Wl[l] = Wl[l];
  }
  if (Hl[0] != H || Wl[0] != W) return fail(kInvalidArgument, "corr_alt_ce0: level 0 must be H x W");
  a.f1 = f1; a.f2 = f2; a.coords = coords;
  a.w = (const __half*)w; a.bias = bias; a.out = (__half*)out;
  a.H = H; a.W = W;
  a.ntiles = (long)E * (H / 8) * (W / 8);
  if (a.ntiles == 0) return kOk;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt_ce0_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kAltLds));
    attr = true;
  }
  const long grid = std::min<long>(a.ntiles, device_cu_count());
  corr_alt_ce0_kernel<<<dim3((unsigned)grid), 512, kAltLds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
