// Implicit-GEMM convolution for the update operator (droid_net.py:78-143,
// modules/gru.py:19-32) on gfx950 MFMA, NHWC fp16 in / fp32 accumulate.
//
//   out[b,y,x,co] = epilogue( sum_{tap,ci} in[b, y+ty, x+tx, ci] * W[co, tap, ci] )
//
// GEMM view: M = B*H*W pixels, N = Cout, K = taps * Cin.  A workgroup (4
// waves) owns a 128-pixel x TN-channel output tile (TN = 128, 64 or 16, so the
// narrow heads do not pay for 128 columns of MFMA work); each wave holds FMxFN
// tiles of v_mfma_f32_16x16x32_f16.  K is consumed in 64-wide stages (two MFMA
// K-steps per barrier):
//   CHUNKED : stage = (source, 64-channel chunk, tap) - the A tile is gathered
//             straight from up to 4 NHWC sources (the reference's channel
//             concatenations never materialise), shifted per tap, zero padded;
//   IM2COL8 : one 8-channel source, stage = 8 consecutive taps x 8 channels
//             (the 7x7 flow-encoder conv: 7 stages instead of 49 mostly-zero ones).
// Stage t+1 sits in registers while stage t is multiplied; it is written into
// the other LDS buffer right after the barrier and stage t+2 is issued at once
// (one barrier per stage).  The stage decode is wave-uniform (scalar).
// 3x3 convs (CHUNKED, Cout % 128 == 0) run the LDS-halo variant instead: a
// 256-pixel x 128-channel tile on 8 waves that loads each 64-channel chunk of
// its pixels plus a +-(W+1) halo once and serves all 9 taps from LDS (the A
// operand crosses L2->CU once per chunk, not once per tap).
// Tiles are mapped XCD-major so each XCD's L2 sees contiguous pixel rows (3x3
// halos) and both N tiles of a pixel tile.
//
// Epilogues fuse what the reference runs as separate elementwise kernels;
// inputs (h, z) and outputs go through LDS so every global access is a
// coalesced 16-B row piece:
//   EPI_ACT   : act(acc + bias[co] + bbias[b,co]), act in {none, relu}
//   EPI_GRU_ZR: co <  Ch: z = sigmoid(.)            -> zout
//               co >= Ch: r = sigmoid(.); r*h       -> rnet
//   EPI_GRU_Q : q = tanh(.); h' = (1-z) h + z q     -> out (the new hidden state)
//   EPI_HEAD  : fp32 out, co < 2 raw (delta), co >= 2 sigmoid (weight)
//   EPI_GLO   : sigmoid(.) * h summed over the tile's pixels, atomically added
//               (scaled by 1/HW) into glo[b][co]: the GRU global-context mean
//   EPI_GRU_ZRP / EPI_GRU_QP (band tiles, droid_conv_gru_pre_f16): EPI_GRU_ZR /
//               EPI_GRU_Q with a per-source-frame term added before the gate:
//               gate(acc + bias + bbias[b] + pre[pre_idx[b], pixel, pre_coff + co])
#include "common.hpp"
#include "lds_dma.hpp"
#include <algorithm>
#include <type_traits>

#ifndef DROID_CONV_PROFILE
#define DROID_CONV_PROFILE 0
#endif
#ifndef DROID_CONV_ABLATE
#define DROID_CONV_ABLATE 0
#endif
#if DROID_CONV_ABLATE && !DROID_CONV_PROFILE
#error "DROID_CONV_ABLATE is for profiling builds only"
#endif

namespace droid {
typedef unsigned u32x4nt __attribute__((ext_vector_type(4)));  // non-temporal 16-B stores


enum ConvEpi : int { EPI_ACT = 0, EPI_GRU_ZR = 1, EPI_GRU_Q = 2, EPI_HEAD = 3, EPI_GLO = 4, EPI_DWHEAD = 5,
                     EPI_GRU_ZRP = 6, EPI_GRU_QP = 7 };
constexpr int kEpiPreShift = EPI_GRU_ZRP - EPI_GRU_ZR;  // EPI_GRU_*P -> its base epilogue

struct ConvSrc {
  const __half* ptr;
  int C;        // channels used (multiple of 8)
  int cstride;  // pixel stride in elements (>= C, multiple of 8)
};

struct ConvArgs {
  ConvSrc src[4];
  int nsrc;
  int chunk_end[4];  // cumulative 64-channel chunk counts per source (within one tap)
  int cpt;           // chunks per tap
  int nstage;        // K / 64
  int im2col;        // IM2COL8 loader
  const __half* wp;  // [Cout][nstage][64]
  const float* bias;   // [Cout] or null
  const float* bbias;  // [B][Cout] or null (per-image bias, e.g. the GRU global branch)
  int B, H, W, Cout, ks, act;
  int epi;
  int n_tiles;  // Cout tiles
  long m_tiles;
  __half* out;
  int out_cstride, out_coff;
  int stage_out;  // fp16 output rows can be written as 16-B pieces
  // GRU
  const __half* h;  // hidden state, NHWC
  int h_cstride;
  const __half* z;  // z gates from the ZR pass
  int z_cstride;
  __half* zout;
  __half* rnet;
  int gru_ch;  // hidden channels (128)
  float* out32;  // EPI_HEAD / EPI_GLO fp32 output
  // band kernel
  int nslot;  // band pixels ((TMX/W + 2) * W)
  int nhi;    // halo DMA instructions per wave per chunk
  const __half* hw;  // EPI_DWHEAD: head weights [48][256] (row = tap*4 + out channel)
  long long* prof;   // band kernel timeline (droid_conv_set_profile): 4 stamps per workgroup, or null
  // EPI_GRU_ZRP / EPI_GRU_QP: per-source-frame pre-activation term, NHWC fp16
  // (frames, H, W, pre_cstride); image b reads frame pre_idx[b]
  const __half* pre;
  const long long* pre_idx;
  int pre_cstride, pre_coff;
  int ab_no_h;   // A/B build only (DROID_ZR_NO_H): the z|r epilogue skips its h re-read (a timing bound)
};

constexpr int TM = 128, BK = 64;
constexpr int LDA = BK;  // LDS row = 128 B; 16-B slot q of row r is stored at q ^ (r & 7)
// (conflict-free for the gfx950 ds_read_b128 lane groups at any row offset)
__device__ __forceinline__ int swz(int row, int slot) { return ((slot ^ (row & 7)) << 3); }

template <int TN>
struct Tile;
template <>
struct Tile<128> { static constexpr int WM = 2, WN = 2, FM = 4, FN = 4; };
template <>
struct Tile<64> { static constexpr int WM = 2, WN = 2, FM = 4, FN = 2; };
template <>
struct Tile<16> { static constexpr int WM = 4, WN = 1, FM = 2, FN = 1; };

template <int TN>
constexpr int conv_lds_bytes() {
  constexpr int main_b = (2 * TM * LDA + 2 * TN * LDA) * 2;
  constexpr int epi_b = 2 * TM * (TN + 8) * 2;
  return main_b > epi_b ? main_b : epi_b;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// ---------------------------------------------------------------------------
// Shared epilogue.  Lane holds rows row0 + i*16 + k (k < 4), column col0 + j*16
// of the workgroup's TMx x TN tile.  `smem` must hold 2*TMx*(TN+8) halves.
template <int TMx, int TN, int FM, int FN, int NT>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, floatx4 (&acc)[FM][FN], _Float16* smem, long m0,
                                              int n0, int row0, int col0, int lane, int tid) {
  const int HW = a.H * a.W;
  const long Mtot = (long)a.B * HW;
  const int epi = a.epi;
  constexpr int ER = TN + 8;  // epilogue LDS row stride (halves)
  _Float16* Hs = smem;            // [TMx][ER] h tile, then the output tile (in place)
  _Float16* Zs = smem + TMx * ER; // [TMx][ER] z tile
  const int b_tile = (int)(m0 / HW);

  // bias (+ per-image bias) into the accumulators
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int co = n0 + col0 + j * 16;
    const float bv = (a.bias && co < a.Cout) ? a.bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = acc[i][j][k] + bv;
        if (a.bbias && co < a.Cout) {
          const long m = m0 + row0 + i * 16 + k;
          int b = b_tile;
          if (HW >= TMx) b += (m >= (long)(b_tile + 1) * HW) ? 1 : 0;
          else b = (int)(m / HW);
          if (m >= Mtot) b = 0;
          v += a.bbias[(long)b * a.Cout + co];
        }
        acc[i][j][k] = v;
      }
  }

  if (epi == EPI_HEAD || (epi == EPI_ACT && !a.stage_out)) {
    // narrow outputs: direct element stores
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long m = m0 + row0 + i * 16 + k;
        if (m >= Mtot) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int co = n0 + col0 + j * 16;
          if (co >= a.Cout) continue;
          float v = acc[i][j][k];
          if (epi == EPI_HEAD) {
            a.out32[m * a.out_cstride + co] = (co >= 2) ? sigmoidf_(v) : v;
          } else {
            if (a.act == 1) v = fmaxf(v, 0.f);
            a.out[m * a.out_cstride + a.out_coff + co] = __float2half(v);
          }
        }
      }
    return;
  }

  // stage the h (and z) tiles through LDS with coalesced 16-B loads
  const bool zr_r = (epi == EPI_GRU_ZR) && n0 >= a.gru_ch;
  const bool need_h = zr_r || epi == EPI_GRU_Q || epi == EPI_GLO;
  const bool need_z = epi == EPI_GRU_Q;
  constexpr int PPR = TN / 8;  // 16-B pieces per tile row
  __syncthreads();             // main-loop LDS reads are done
  if (need_h || need_z) {
    const int hc0 = zr_r ? n0 - a.gru_ch : n0;
    for (int idx = tid; idx < TMx * PPR; idx += NT) {
      const int r = idx / PPR, p = idx - r * PPR;
      const long m = m0 + r;
      if (m >= Mtot) continue;
      if (need_h)
        *reinterpret_cast<uint4*>(&Hs[r * ER + p * 8]) =
            *reinterpret_cast<const uint4*>(a.h + m * a.h_cstride + hc0 + p * 8);
      if (need_z)
        *reinterpret_cast<uint4*>(&Zs[r * ER + p * 8]) =
            *reinterpret_cast<const uint4*>(a.z + m * a.z_cstride + n0 + p * 8);
    }
    __syncthreads();
  }

  if (epi == EPI_GLO) {
    // all pixels of the tile belong to one image (HW % TMx == 0, checked by
    // the host): sum each column over rows, then one atomic per column.
    const int b = b_tile;
    const float inv = 1.0f / (float)HW;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float sacc = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int r = row0 + i * 16 + k;
          const float hv = (float)Hs[r * ER + col0 + j * 16];
          sacc += (m0 + r < Mtot) ? sigmoidf_(acc[i][j][k]) * hv : 0.f;
        }
      sacc += __shfl_xor(sacc, 16);
      sacc += __shfl_xor(sacc, 32);
      const int co = n0 + col0 + j * 16;
      if (lane < 16 && co < a.Cout) atomicAdd(a.out32 + (long)b * a.Cout + co, sacc * inv);
    }
    return;
  }

  // elementwise epilogue into the LDS output tile (in place over Hs)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = row0 + i * 16 + k;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = col0 + j * 16;
        const float v = acc[i][j][k];
        float o;
        if (epi == EPI_ACT) {
          o = (a.act == 1) ? fmaxf(v, 0.f) : v;
        } else if (epi == EPI_GRU_ZR) {
          const float g = sigmoidf_(v);
          o = zr_r ? g * (float)Hs[r * ER + c] : g;
        } else {  // EPI_GRU_Q
          const float q = tanhf(v);
          const float zv = (float)Zs[r * ER + c];
          const float hv = (float)Hs[r * ER + c];
          o = (1.0f - zv) * hv + zv * q;
        }
        Hs[r * ER + c] = (_Float16)o;
      }
    }
  __syncthreads();
  __half* dst;
  int dcs, dco;
  if (epi == EPI_GRU_ZR) {
    dst = zr_r ? a.rnet : a.zout;
    dcs = a.gru_ch;
    dco = zr_r ? n0 - a.gru_ch : n0;
  } else {
    dst = a.out;
    dcs = a.out_cstride;
    dco = a.out_coff + n0;
  }
  const int ncol = min(TN, a.Cout - n0);
  for (int idx = tid; idx < TMx * PPR; idx += NT) {
    const int r = idx / PPR, p = idx - r * PPR;
    const long m = m0 + r;
    if (m >= Mtot || p * 8 >= ncol) continue;
    *reinterpret_cast<uint4*>(dst + m * dcs + dco + p * 8) = *reinterpret_cast<const uint4*>(&Hs[r * ER + p * 8]);
  }
}

// XCD-major work id: consecutive ids share an XCD (bijective remap)
__device__ __forceinline__ long xcd_work_id(long nwg) {
  const long orig = blockIdx.x;
  const long xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// ---------------------------------------------------------------------------
// Generic kernel: 128 x TN tile, 4 waves, A and B staged per 64-wide K stage.
template <int TN>
__global__ void __launch_bounds__(256) conv_nhwc_f16_kernel(ConvArgs a) {
  using T = Tile<TN>;
  constexpr int FM = T::FM, FN = T::FN;
  constexpr int BROWS = TN * 8 / 256 > 0 ? TN * 8 / 256 : 1;  // B pieces per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  _Float16* As = smem;                  // [2][TM][LDA]
  _Float16* Bs = smem + 2 * TM * LDA;   // [2][TN][LDA]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WN, wn = wave % T::WN;
  const int HW = a.H * a.W;
  const long Mtot = (long)a.B * HW;

  const long wgid = xcd_work_id(a.m_tiles * a.n_tiles);
  const long mt = wgid / a.n_tiles;
  const int nt = (int)(wgid - mt * a.n_tiles);
  const long m0 = mt * TM;
  const int n0 = nt * TN;
  const int pad = a.ks >> 1;

  // this thread's 4 A rows and 8-channel piece
  const int piece = tid & 7;
  int am[4], ay[4], ax[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long m = m0 + (tid >> 3) + 32 * r;
    if (m < Mtot) {
      am[r] = (int)m;
      const int p = (int)(m % HW);
      ay[r] = p / a.W;
      ax[r] = p - ay[r] * a.W;
    } else {
      am[r] = 0;
      ay[r] = -100000;  // never inside the image
      ax[r] = 0;
    }
  }
  const int brow = (tid >> 3);
  const bool bthread = TN * 8 >= 256 || tid < TN * 8;

  // wave-uniform stage cursor (CHUNKED, K order (chunk, tap)): tap (ty,tx), chunk
  int cur_ty = -pad, cur_tx = -pad, cur_ci = 0;
  // per-thread tap cursor (IM2COL8)
  int i2_tap = piece, i2_ty = 0, i2_tx = piece;
  if (a.im2col) {
    i2_ty = piece / a.ks;
    i2_tx = piece - i2_ty * a.ks;
  }
  const int taps = a.ks * a.ks;

  uint4 ra[4], rb[BROWS];
  auto load_stage = [&](int st) {
    // A operand
    int dy, dx, c, cs;
    const __half* base;
    bool ok_k;
    if (a.im2col) {
      dy = i2_ty - pad;
      dx = i2_tx - pad;
      c = 0;
      cs = a.src[0].cstride;
      base = a.src[0].ptr;
      ok_k = i2_tap < taps;
      // advance to the next stage's tap (8 further)
      i2_tap += 8;
      i2_tx += 8;
      while (i2_tx >= a.ks) { i2_tx -= a.ks; ++i2_ty; }
    } else {
      int s = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q + 1 < a.nsrc && cur_ci >= a.chunk_end[q]) s = q + 1;
      const int cstart = s ? a.chunk_end[s - 1] : 0;
      const ConvSrc src = a.src[s];
      dy = cur_ty;
      dx = cur_tx;
      c = (cur_ci - cstart) * BK + piece * 8;
      cs = src.cstride;
      base = src.ptr;
      ok_k = c < src.C;
      if (++cur_tx > pad) {
        cur_tx = -pad;
        if (++cur_ty > pad) { cur_ty = -pad; ++cur_ci; }
      }
    }
    const int doff = dy * a.W + dx;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int y = ay[r] + dy, x = ax[r] + dx;
      const bool ok = ok_k && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W;
      ra[r] = ok ? *reinterpret_cast<const uint4*>(base + (long)(am[r] + doff) * cs + c) : make_uint4(0, 0, 0, 0);
    }
    // B operand (packed weights)
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      const int co = n0 + brow + 32 * r;
      rb[r] = (bthread && co < a.Cout)
                  ? *reinterpret_cast<const uint4*>(a.wp + ((long)co * a.nstage + st) * BK + piece * 8)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_stage = [&](int buf) {
    _Float16* A = As + buf * TM * LDA;
    _Float16* Bm = Bs + buf * TN * LDA;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<uint4*>(&A[((tid >> 3) + 32 * r) * LDA + swz(tid >> 3, piece)]) = ra[r];
    if (bthread) {
#pragma unroll
      for (int r = 0; r < BROWS; ++r)
        *reinterpret_cast<uint4*>(&Bm[(brow + 32 * r) * LDA + swz(brow, piece)]) = rb[r];
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nst = a.nstage;
  load_stage(0);
  store_stage(0);
  if (nst > 1) load_stage(1);
  const int fr = lane & 15;
  for (int st = 0; st < nst; ++st) {
    __syncthreads();
    if (st + 1 < nst) {
      store_stage((st + 1) & 1);
      if (st + 2 < nst) load_stage(st + 2);
    }
    const _Float16* A = As + (st & 1) * TM * LDA + (wm * FM * 16 + fr) * LDA;
    const _Float16* Bm = Bs + (st & 1) * TN * LDA + (wn * FN * 16 + fr) * LDA;
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
      const int ko = swz(fr, (lane >> 4) + hk * 4);
      half8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const half8*>(A + i * 16 * LDA + ko);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const half8*>(Bm + j * 16 * LDA + ko);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  conv_epilogue<TM, TN, FM, FN, 256>(a, acc, smem, m0, n0, wm * FM * 16 + (lane >> 4) * 4, wn * FN * 16 + fr,
                                     lane, tid);
}

// ---------------------------------------------------------------------------
// Halo kernel (ks > 1, CHUNKED): HTM-pixel x 128-channel tile, NW waves
// ((NW/2) x 2, 64x64 per wave).  For each 64-channel chunk the tile's pixels
// plus a +-pad*(W+1) halo are loaded ONCE into LDS and all ks*ks taps read
// their shifted A fragments from it (rows whose shifted pixel leaves the image
// are masked to zero), so the A operand crosses L2->CU once per chunk instead
// of once per tap.  B (weights) is double-buffered per (chunk, tap) stage.
constexpr int kHaloMax = 192;  // max pad*(W+1) supported by the register-staged halo loader
#ifndef DROID_HALO_ISSUE_TAP
#define DROID_HALO_ISSUE_TAP 0
#endif
constexpr int kHaloIssueTap = DROID_HALO_ISSUE_TAP;
constexpr int kRowsSlotsMax = 448;  // padded band pixels the row-band kernel's loader covers

template <int NW>
struct Halo {
  static constexpr int NT = NW * 64;
  static constexpr int HTM = (NW / 2) * 64;
  static constexpr int NP = ((HTM + 2 * kHaloMax) * 8 + NT - 1) / NT;  // halo pieces per thread
  static constexpr int NB = 128 * 8 / NT;                              // B pieces per thread
};

template <int NW>
__host__ __device__ constexpr int halo_lds_bytes_max() {
  return ((Halo<NW>::HTM + 2 * kHaloMax) * LDA + 2 * 128 * LDA) * 2 > 2 * Halo<NW>::HTM * 136 * 2
             ? ((Halo<NW>::HTM + 2 * kHaloMax) * LDA + 2 * 128 * LDA) * 2
             : 2 * Halo<NW>::HTM * 136 * 2;
}

template <int NW>
__global__ void __launch_bounds__(NW * 64) conv_halo_kernel(ConvArgs a) {
  using HP = Halo<NW>;
  constexpr int TN = 128, FM = 4, FN = 4, NT = HP::NT, HTM = HP::HTM;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = a.H * a.W;
  const long Mtot = (long)a.B * HW;
  const long wgid = xcd_work_id(a.m_tiles * a.n_tiles);
  const long mt = wgid / a.n_tiles;
  const int nt = (int)(wgid - mt * a.n_tiles);
  const long m0 = mt * HTM;
  const int n0 = nt * TN;
  const int pad = a.ks >> 1;
  const int hal = pad * (a.W + 1);
  const int HR = HTM + 2 * hal;
  _Float16* Ah = smem;              // [HR][LDA]
  _Float16* Bs = smem + HR * LDA;   // [2][TN][LDA]

  const int piece = tid & 7;
  const int prow = tid >> 3;        // NT/8 rows per pass
  uint4 rh[HP::NP], rb[HP::NB];

  auto load_halo = [&](int chunk) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q + 1 < a.nsrc && chunk >= a.chunk_end[q]) s = q + 1;
    const int cstart = s ? a.chunk_end[s - 1] : 0;
    const ConvSrc src = a.src[s];
    const int c = (chunk - cstart) * BK + piece * 8;
    const bool okc = c < src.C;
#pragma unroll
    for (int q = 0; q < HP::NP; ++q) {
      const int r = prow + (NT / 8) * q;
      const long m = m0 - hal + r;
      const bool ok = okc && r < HR && m >= 0 && m < Mtot;
      rh[q] = ok ? *reinterpret_cast<const uint4*>(src.ptr + m * src.cstride + c) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int q = 0; q < HP::NP; ++q) {
      const int r = prow + (NT / 8) * q;
      if (r < HR) *reinterpret_cast<uint4*>(&Ah[r * LDA + swz(r, piece)]) = rh[q];
    }
  };
  auto load_b = [&](int st) {
#pragma unroll
    for (int q = 0; q < HP::NB; ++q) {
      const int co = n0 + prow + (NT / 8) * q;
      rb[q] = co < a.Cout ? *reinterpret_cast<const uint4*>(a.wp + ((long)co * a.nstage + st) * BK + piece * 8)
                          : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < HP::NB; ++q)
      *reinterpret_cast<uint4*>(&Bs[buf * TN * LDA + (prow + (NT / 8) * q) * LDA + swz(prow, piece)]) = rb[q];
  };

  // the lane's fragment rows: pixel m0 + wm*64 + i*16 + fr
  const int fr = lane & 15;
  int fy[FM], fx[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long m = m0 + wm * 64 + i * 16 + fr;
    if (m < Mtot) {
      const int p = (int)(m % HW);
      fy[i] = p / a.W;
      fx[i] = p - fy[i] * a.W;
    } else {
      fy[i] = -100000;
      fx[i] = 0;
    }
  }

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int taps = a.ks * a.ks;
  const int nch = a.cpt;
  const int nst = a.nstage;  // nch * taps
  load_halo(0);
  load_b(0);
  store_b(0);
  if (nst > 1) load_b(1);
  int st = 0;
  for (int ch = 0; ch < nch; ++ch) {
    __syncthreads();  // every wave is done reading the previous chunk's halo
    store_halo();
    int ty = -pad, tx = -pad;
    for (int t = 0; t < taps; ++t, ++st) {
      __syncthreads();
      if (st + 1 < nst) {
        store_b((st + 1) & 1);
        if (st + 2 < nst) load_b(st + 2);
      }
      // the next chunk's halo is issued behind this stage's B loads: loads
      // retire in order, so it is first waited for two stages later
      if (t == min(kHaloIssueTap, taps - 1) && ch + 1 < nch) load_halo(ch + 1);
      unsigned msk[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        msk[i] = ((unsigned)(fy[i] + ty) < (unsigned)a.H && (unsigned)(fx[i] + tx) < (unsigned)a.W) ? ~0u : 0u;
      const int arow = wm * 64 + fr + hal + ty * a.W + tx;
      const _Float16* A = Ah + arow * LDA;
      const _Float16* Bm = Bs + (st & 1) * TN * LDA + (wn * 64 + fr) * LDA;
#pragma unroll
      for (int hk = 0; hk < 2; ++hk) {
        const int ka = swz(arow, (lane >> 4) + hk * 4), kb = swz(fr, (lane >> 4) + hk * 4);
        half8 af[FM], bf[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          uint4 v = *reinterpret_cast<const uint4*>(A + i * 16 * LDA + ka);
          v.x &= msk[i]; v.y &= msk[i]; v.z &= msk[i]; v.w &= msk[i];
          af[i] = __builtin_bit_cast(half8, v);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const half8*>(Bm + j * 16 * LDA + kb);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      if (++tx > pad) { tx = -pad; ++ty; }
    }
  }
  conv_epilogue<HTM, TN, FM, FN, NT>(a, acc, smem, m0, n0, wm * 64 + (lane >> 4) * 4, wn * 64 + fr, lane, tid);
}

// ---------------------------------------------------------------------------
// Row-band kernel (ks > 1, CHUNKED, 256 % W == 0, 16 | W, H*W % 256 == 0):
// the 256-pixel tile is R = 256/W whole image rows, so the halo is held in LDS
// as a zero-padded (R+2*pad) x (W+2*pad) pixel image and every tap is a pure
// row shift of it - no wrap-around, no masks.  All global loads are buffer
// loads with per-thread offsets fixed for the whole kernel (zero VALU address
// math in the loop); padding / out-of-image pixels use an out-of-range offset,
// which the buffer unit returns as zeros.

__device__ __forceinline__ uint4 buf_load16(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0));
}

template <int NW>
__global__ void __launch_bounds__(NW * 64) conv_rows_kernel(ConvArgs a) {
  constexpr int TN = 128, FM = 4, FN = 4, NT = NW * 64, HTM = (NW / 2) * 64;
  constexpr int NP = (kRowsSlotsMax * 8 + NT - 1) / NT;  // halo pieces per thread
  constexpr int NB = TN * 8 / NT;                        // B pieces per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int W = a.W, H = a.H, HW = H * W;
  const long wgid = xcd_work_id(a.m_tiles * a.n_tiles);
  const long mt = wgid / a.n_tiles;
  const int nt = (int)(wgid - mt * a.n_tiles);
  const long m0 = mt * HTM;
  const int n0 = nt * TN;
  const int pad = a.ks >> 1;
  const int R = HTM / W;            // image rows in the tile
  const int PW = W + 2 * pad;       // padded row length (pixels)
  const int nslot = (R + 2 * pad) * PW;
  const int y0 = (int)((m0 % HW) / W);
  _Float16* Ah = smem;                  // [nslot][64]
  _Float16* Bs = smem + nslot * LDA;    // [2][TN][64]

  const int piece = tid & 7;
  const int prow = tid >> 3;
  // halo slot -> pixel offset relative to the band's first row (y0 - pad), or -1
  int hpix[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int slot = prow + (NT / 8) * q;
    const int ry = slot / PW, rx = slot - (slot / PW) * PW;
    const int y = y0 + ry - pad, x = rx - pad;
    hpix[q] = (slot < nslot && y >= 0 && y < H && x >= 0 && x < W) ? ry * W + x : -1;
  }
  const long band0 = m0 - (long)pad * W;  // pixel index of the band's first row
  const int band_rows = R + 2 * pad;

  // lane fragment slots (tap (0,0)) for i < FM
  const int fr = lane & 15;
  int fslot[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int p = wm * 64 + i * 16 + fr;
    fslot[i] = (p / W + pad) * PW + (p % W) + pad;
  }

  // B: weights of this tile's 128 output channels
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.wp + (long)n0 * a.nstage * BK), (short)0, TN * a.nstage * BK * 2, kBufFlags);
  unsigned boff[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) boff[q] = (unsigned)(((prow + (NT / 8) * q) * a.nstage * BK + piece * 8) * 2);

  uint4 rh[NP], rb[NB];
  auto load_halo = [&](int chunk) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q + 1 < a.nsrc && chunk >= a.chunk_end[q]) s = q + 1;
    const int cstart = s ? a.chunk_end[s - 1] : 0;
    const ConvSrc src = a.src[s];
    const int c0 = (chunk - cstart) * BK;
    const bool okc = c0 + piece * 8 < src.C;
    // the band may start before the tensor (first image rows): only valid
    // slots ever read, and those lie inside it
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(src.ptr + band0 * src.cstride + c0), (short)0, band_rows * W * src.cstride * 2, kBufFlags);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const unsigned off = (okc && hpix[q] >= 0) ? (unsigned)((hpix[q] * src.cstride + piece * 8) * 2) : kOob;
      rh[q] = buf_load16(rs, off, 0);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int slot = prow + (NT / 8) * q;
      if (slot < nslot) *reinterpret_cast<uint4*>(&Ah[slot * LDA + swz(slot, piece)]) = rh[q];
    }
  };
  auto load_b = [&](int st) {
#pragma unroll
    for (int q = 0; q < NB; ++q) rb[q] = buf_load16(rsb, boff[q], st * BK * 2);
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NB; ++q)
      *reinterpret_cast<uint4*>(&Bs[buf * TN * LDA + (prow + (NT / 8) * q) * LDA + swz(prow, piece)]) = rb[q];
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int taps = a.ks * a.ks;
  const int nch = a.cpt;
  const int nst = a.nstage;
  load_halo(0);
  load_b(0);
  store_b(0);
  if (nst > 1) load_b(1);
  int st = 0;
  for (int ch = 0; ch < nch; ++ch) {
    __syncthreads();  // every wave is done reading the previous chunk's halo
    store_halo();
    int ty = -pad, tx = -pad;
    for (int t = 0; t < taps; ++t, ++st) {
      __syncthreads();
      if (st + 1 < nst) {
        store_b((st + 1) & 1);
        if (st + 2 < nst) load_b(st + 2);
      }
      if (t == min(kHaloIssueTap, taps - 1) && ch + 1 < nch) load_halo(ch + 1);
      const int sh = ty * PW + tx;
      const _Float16* Bm = Bs + (st & 1) * TN * LDA + (wn * 64 + fr) * LDA;
#pragma unroll
      for (int hk = 0; hk < 2; ++hk) {
        const int kq = (lane >> 4) + hk * 4;
        const int kb = swz(fr, kq);
        half8 af[FM], bf[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int sl = fslot[i] + sh;
          af[i] = *reinterpret_cast<const half8*>(Ah + sl * LDA + swz(sl, kq));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const half8*>(Bm + j * 16 * LDA + kb);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      if (++tx > pad) { tx = -pad; ++ty; }
    }
  }
  conv_epilogue<HTM, TN, FM, FN, NT>(a, acc, smem, m0, n0, wm * 64 + (lane >> 4) * 4, wn * 64 + fr, lane, tid);
}

template <int NW>
static int launch_rows(const ConvArgs& a0, hipStream_t stream) {
  constexpr int HTM = (NW / 2) * 64;
  ConvArgs a = a0;
  a.n_tiles = a.Cout / 128;
  const long M = (long)a.B * a.H * a.W;
  a.m_tiles = M / HTM;
  const int pad = a.ks >> 1;
  const int nslot = (HTM / a.W + 2 * pad) * (a.W + 2 * pad);
  const int main_b = (nslot * LDA + 2 * 128 * LDA) * 2;
  const int epi_b = 2 * HTM * 136 * 2;
  const int lds = main_b > epi_b ? main_b : epi_b;
  constexpr int lds_max = (kRowsSlotsMax * LDA + 2 * 128 * LDA) * 2 > 2 * HTM * 136 * 2
                              ? (kRowsSlotsMax * LDA + 2 * 128 * LDA) * 2
                              : 2 * HTM * 136 * 2;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_rows_kernel<NW>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
    attr = true;
  }
  if (a.m_tiles * a.n_tiles > 0x7fffffffL) return fail(kUnsupported, "conv_nhwc_f16: problem too large");
  conv_rows_kernel<NW><<<dim3((unsigned)(a.m_tiles * a.n_tiles)), NW * 64, lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

template <int TN>
static int launch_conv(const ConvArgs& a0, hipStream_t stream) {
  ConvArgs a = a0;
  a.n_tiles = ceil_div(a.Cout, TN);
  const long M = (long)a.B * a.H * a.W;
  a.m_tiles = (M + TM - 1) / TM;
  constexpr int lds = conv_lds_bytes<TN>();
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_nhwc_f16_kernel<TN>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = true;
  }
  const long nwg = a.m_tiles * a.n_tiles;
  if (nwg > 0x7fffffffL) return fail(kUnsupported, "conv_nhwc_f16: problem too large");
  conv_nhwc_f16_kernel<TN><<<dim3((unsigned)nwg), 256, lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

template <int NW>
static int launch_halo(const ConvArgs& a0, hipStream_t stream) {
  using HP = Halo<NW>;
  ConvArgs a = a0;
  a.n_tiles = ceil_div(a.Cout, 128);
  const long M = (long)a.B * a.H * a.W;
  a.m_tiles = (M + HP::HTM - 1) / HP::HTM;
  const int hal = (a.ks >> 1) * (a.W + 1);
  const int main_b = ((HP::HTM + 2 * hal) * LDA + 2 * 128 * LDA) * 2;
  const int epi_b = 2 * HP::HTM * 136 * 2;
  const int lds = main_b > epi_b ? main_b : epi_b;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_halo_kernel<NW>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, halo_lds_bytes_max<NW>()));
    attr = true;
  }
  const long nwg = a.m_tiles * a.n_tiles;
  if (nwg > 0x7fffffffL) return fail(kUnsupported, "conv_nhwc_f16: problem too large");
  conv_halo_kernel<NW><<<dim3((unsigned)nwg), HP::NT, lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

// ---------------------------------------------------------------------------
// Band kernel (3x3, CHUNKED; W in {16, 32, 64}, TMX | H*W, TN | Cout): a
// TMX-pixel x TN-channel tile on 8 waves (4 along pixels x 2 along channels),
// each wave 64x128 (TN = 256) or 96x64 (TN = 128) - the whole Cout = 256 of
// the ConvGRU z|r gates in one workgroup, so the A operand crosses L2->CU once
// per chunk for all outputs.  A wave's 16-pixel fragments are interleaved with
// the other pixel waves' (fragment i of wave wm = tile pixels 16 (wm + 4i) ..),
// so with W | 64 every fragment of a wave starts at the same image column.
// Both operands reach LDS by LDS-DMA (buffer_load ... lds, no VGPR staging,
// no ds_write):
//   * the tile's R = TMX/W image rows plus one halo row above and below, an
//     (R+2) x W pixel band of one 64-channel chunk, double buffered: the next
//     chunk's band is in flight during the 9 taps of the current one;
//   * the weights of one (chunk, tap) stage, double buffered, one stage ahead.
// A tap is a row shift of the band (compile-time ds_read offsets; taps are
// unrolled).  The x = -1 / x = W neighbours of the image's edge columns would
// land on the adjacent row's edge pixel: those lanes (only lane 0 / 15 of the
// waves whose fragments start at column 0 / W-16) read through a base address
// past the LDS allocation instead, which the LDS returns as zeros - no masks.  Rows outside
// the image and channels past a source's end are out-of-range buffer offsets,
// which the DMA fills with zeros.  One raw s_barrier per stage with counted
// vmcnt waits: a wave waits only for its own DMA of the stage about to be
// read, the barrier then publishes every wave's.
// NW = 8: 4 x 2 waves of 64 x TN/2 (the default); NW = 4: 2 x 2 waves of 128 x
// 128 at TMX = TN = 256 (one wave per SIMD, its 256 accumulators in AGPRs; a
// third fewer LDS read bytes per MFMA).  With WM = 2 a wave's fragments are 32
// pixels apart, so at W = 64 consecutive fragments alternate between two image
// columns: NPAR per-parity A base addresses.
template <int TMX, int TN, int NW = 8>
struct Band {
  static constexpr int WM = NW / 2, WN = 2, FM = TMX / (WM * 16), FN = TN / (WN * 16);
  static constexpr int NT = NW * 64;
  static constexpr int NBI = TN / (8 * NW);              // weight DMA instructions per wave per stage
  static constexpr int MAX_NHI = 64 / NW;
  static constexpr int NPAR = WM == 2 ? 2 : 1;
  static_assert(WM * WN == NW && FM * 16 * WM == TMX && (NW == 8 || NW == 4), "band tile");
};
constexpr int kLdsMax = 163840;
// profiling builds: int64 slots per workgroup (hw id, entry, loop start, loop end,
// epilogue stores issued, drained (wave 0), pass 1 written, pass-2 loads issued,
// staging barrier passed, last wave drained)
constexpr int kProfSlots = 12;   // [10] / [11]: s_memrealtime at loop start / end (in-kernel clock)

__device__ __forceinline__ void wait_vmcnt(int n) {
  // n is wave-uniform; s_waitcnt takes an immediate
  switch (n) {
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}


// Band epilogue in two passes through one fp16 LDS tile [TMX][TN + 8]:
// (1) each wave writes act(acc + bias + bbias) of its fragments (act = relu /
//     none, sigmoid for z|r, tanh for q - rounded to fp16 as the reference's
//     autocast rounds the gate before using it);
// (2) coalesced 16-B row pieces: r * h for the r half, the GRU blend
//     (1 - z) h + z q for q (h, z read as 16-B pieces), then the store.
// tile row of accumulator row (i, fq, k): pixel fragments are interleaved across
// the WM pixel waves (fragment i of wave wm = pixels 16 (wm + WM i) ..) or
// contiguous (wave wm owns pixels wm*FM*16 .. + FM*16)
template <int FM, int WM, bool CONTIG>
__device__ __forceinline__ int frag_row(int wm, int i) {
  return CONTIG ? wm * FM * 16 + 16 * i : 16 * (wm + WM * i);
}

// The epilogue type is a template parameter (EPI < 0: runtime a.epi, for the
// kernels that still dispatch at run time): with a runtime switch every one of
// the FM*FN*4 unrolled elements carried a 3-way branch and tanhf's divergent
// range reduction, ~50 KB of straight-line code fetched cold once per tile
// (the timeline measured 20k clocks per 384x128 epilogue).
__device__ __forceinline__ float tanh_fast(float x) {
  // 1 - 2 / (1 + e^(2x)) with the hardware reciprocal (v_rcp_f32, 1 ulp) in
  // place of the IEEE division sequence (10 VALU ops, the band epilogue's
  // largest cost): branch-free, saturates to +-1; abs error ~1e-7, far below
  // the fp16 rounding of the gate that follows
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x));
}
// sigmoid for fp16-rounded gates: 1 / (1 + e^-x) with the hardware reciprocal
__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// Pass-1 staging of a pixels x weights fragment: lane (fr, fq) holds 4
// consecutive pixels (rows row0 .. row0 + 3) of one channel c as two fp16 pairs
// (lo = pixels 0, 1; hi = pixels 2, 3).  Written as they are that is four 2-B
// LDS stores.  Instead the two lanes of adjacent channels trade one pair (DPP
// quad_perm [1,0,3,2]): the even lane then holds channels c, c + 1 of pixels 0
// and 1, the odd lane those of pixels 2 and 3, and each writes two 4-B words
// (half the LDS store instructions; conflict-free with the ER = TN + 8 row pitch).
__device__ __forceinline__ void stage_pixel_pairs(_Float16* smem, int row0, int c, int ER, int fr, unsigned lo,
                                                  unsigned hi) {
  const bool odd = fr & 1;
  const unsigned x = odd ? lo : hi;
  const unsigned r = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
  const unsigned ca = odd ? r : lo;   // channel c & ~1
  const unsigned cb = odd ? hi : r;   // channel (c & ~1) + 1
  unsigned* d = reinterpret_cast<unsigned*>(&smem[(row0 + (odd ? 2 : 0)) * ER + (c & ~1)]);
  d[0] = (ca & 0xFFFFu) | (cb << 16);
  d[ER / 2] = (ca >> 16) | (cb & 0xFFFF0000u);
}
__device__ __forceinline__ unsigned pack_f16x2(float a, float b) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const h2_t h = __builtin_convertvector(f2_t{a, b}, h2_t);
  return __builtin_bit_cast(unsigned, h);
}

// kBandSwap: the main loop multiplies weights x pixels (MFMA A = weight
// fragment), so a lane's accumulators are 4 consecutive channels of one pixel
// and the epilogue's LDS staging writes 8 B per fragment instead of four 2-B
// writes (pass 1 1.6-2x faster).  The 256x256 tile keeps pixels x weights: with
// the operands swapped its register allocation spills (256 VGPRs + scratch).
template <int TN>
constexpr bool kBandSwap = TN != 256;

// (1 - z) h + z q on packed fp16, every op rounded (no contraction into an
// fma): the reference's autocast evaluates the GRU blend as fp16 tensor ops
__device__ __forceinline__ half8 gru_blend_f16(half8 z, half8 h, half8 q) {
#pragma clang fp contract(off)
  const half8 one = {(_Float16)1.f, (_Float16)1.f, (_Float16)1.f, (_Float16)1.f,
                     (_Float16)1.f, (_Float16)1.f, (_Float16)1.f, (_Float16)1.f};
  const half8 a = (one - z) * h;
  const half8 b = z * q;
  return a + b;
}

// DROID_BAND_A_NT (A/B builds): the band kernel's input bands by non-temporal LDS-DMA
#ifndef DROID_BAND_A_NT
#define DROID_BAND_A_NT 0
#endif
// DROID_EPI_NT (A/B builds): the band epilogue's output rows as non-temporal
// stores (the maps are 0.8-1.6 GB at C3, far past L2 and the Infinity Cache)
#ifndef DROID_EPI_NT
#define DROID_EPI_NT 0
#endif

// The band epilogue around a caller-supplied pass 1: stage1(bl, act) writes
// act(acc + column bias) of the caller's accumulators into the fp16 staging
// tile smem[TMX][TN + 8] (bl = the tile's column biases in LDS, act = the
// epilogue's pass-1 activation); pass 2 below is shared by the band tile and
// the Winograd tile.  EARLY: the per-frame term may be loaded before pass 1.
template <int TMX, int TN, int NT, int EPI, bool EARLY, class Stage1>
__device__ __forceinline__ void band_epilogue_core(const ConvArgs& a, _Float16* smem, long m0, int n0, int tid,
                                                   float bcol, long long* prof, Stage1 stage1);

template <int TMX, int TN, int FM, int FN, int WM = 4, bool CONTIG = false, int NT = 512, int EPI = -1,
          bool EARLY = true, bool SWAP = kBandSwap<TN>>
__device__ __forceinline__ void band_epilogue(const ConvArgs& a, floatx4 (&acc)[FM][FN], _Float16* smem, long m0,
                                              int n0, int wm, int wn, int lane, int tid, float bcol,
                                              long long* prof = nullptr) {
  constexpr int ER = TN + 8;
  constexpr bool kPre = EPI == EPI_GRU_ZRP || EPI == EPI_GRU_QP;
  const int fr = lane & 15, fq = lane >> 4;
  band_epilogue_core<TMX, TN, NT, EPI, EARLY>(a, smem, m0, n0, tid, bcol, prof, [&](const float* bl, auto act) {
  if constexpr (SWAP) {
    // (1) lane (fr, fq) of fragment (i, j) holds channels 16 j + 4 fq .. + 3 of
    // pixel row frag_row(i) + fr: one 8-B LDS write per fragment
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * FN * 16 + j * 16 + fq * 4;
      const floatx4 bv = *reinterpret_cast<const floatx4*>(bl + c);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        half4_t o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = (_Float16)act(acc[i][j][k] + bv[k]);
        *reinterpret_cast<half4_t*>(&smem[(frag_row<FM, WM, CONTIG>(wm, i) + fr) * ER + c]) = o;
      }
    }
  } else {
    // (1) lane (fr, fq) of fragment (i, j) holds pixel rows frag_row(i) + 4 fq .. + 3
    // of channel 16 j + fr
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * FN * 16 + j * 16 + fr;
      const float bv = bl[c];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (kPre) {
          // the staged pre-activation: bias added two values at a time (v_pk_add_f32)
          // and rounded two at a time (v_cvt_pk_f16_f32); the halves go to their rows
          typedef float f2_t __attribute__((ext_vector_type(2)));
          typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
          const f2_t b2 = {bv, bv};
          const f2_t lo = f2_t{acc[i][j][0], acc[i][j][1]} + b2, hi = f2_t{acc[i][j][2], acc[i][j][3]} + b2;
          const h2_t l16 = __builtin_convertvector(lo, h2_t), h16 = __builtin_convertvector(hi, h2_t);
          stage_pixel_pairs(smem, frag_row<FM, WM, CONTIG>(wm, i) + fq * 4, c, ER, fr,
                            __builtin_bit_cast(unsigned, l16), __builtin_bit_cast(unsigned, h16));
        } else {
          stage_pixel_pairs(smem, frag_row<FM, WM, CONTIG>(wm, i) + fq * 4, c, ER, fr,
                            pack_f16x2(act(acc[i][j][0] + bv), act(acc[i][j][1] + bv)),
                            pack_f16x2(act(acc[i][j][2] + bv), act(acc[i][j][3] + bv)));
        }
      }
    }
  }
  });
}

template <int TMX, int TN, int NT, int EPI, bool EARLY, class Stage1>
__device__ __forceinline__ void band_epilogue_core(const ConvArgs& a, _Float16* smem, long m0, int n0, int tid,
                                                   float bcol, long long* prof, Stage1 stage1) {
  constexpr int ER = TN + 8, PPR = TN / 8;
  const int HW = a.H * a.W;
  const int b = (int)(m0 / HW);  // a tile never straddles two images
  // kPre: the gate's argument gets the per-source term in pass (2), so pass (1)
  // stages the pre-activation acc + bias (fp16, as the reference's autocast
  // conv output is) and the gate is applied after the sum
  constexpr bool kPre = EPI == EPI_GRU_ZRP || EPI == EPI_GRU_QP;
  constexpr int EB = kPre ? EPI - kEpiPreShift : EPI;
  const int epi = EB >= 0 ? EB : a.epi;
  const bool relu = a.act == 1;
  // the tile's column biases (bias + per-image bias, loaded by thread t < TN
  // before the main loop) go through LDS: with kBandSwap a lane's accumulators
  // are 4 consecutive channels of one pixel, so each lane needs 4 x FN of them
  float* const bl = reinterpret_cast<float*>(smem + TMX * ER);
  static_assert((TMX * PPR) % NT == 0, "band epilogue: whole store rounds");
  constexpr int RND = TMX * PPR / NT;
  // GRU epilogues: every round's h (and z) pieces are loaded after pass 1, all
  // in flight together while the staging barrier waits (issued inside the store
  // loop they were serialised behind the previous round's store)
  constexpr bool kPreH = EB == EPI_GRU_ZR || EB == EPI_GRU_Q;
  // round q of thread tid: tile row r0 + q*RQ, 16-B piece p (NT % PPR == 0), so
  // every global address is a per-thread base plus q times a uniform row step
  static_assert(NT % PPR == 0, "band epilogue: rounds are whole rows");
  constexpr int RQ = NT / PPR;
  const int r0 = tid / PPR, p = tid % PPR;
  const int c = n0 + p * 8;
  const long mrow = m0 + r0;
  const bool rhalf = epi == EPI_GRU_ZR && c >= a.gru_ch;
  // pass (2) in batches of RB rounds (the 4-wave tile has 32 rounds per thread:
  // all of them in flight would need 3 x 128 VGPRs; with its accumulators in
  // the AGPR file its VGPRs are free here, so it takes batches of 16)
  constexpr int RBMAX = (NT >= 512 || TN == 256) ? 16 : 8;
  constexpr int RB = RND > RBMAX ? RBMAX : RND;
  static_assert(RND % RB == 0, "band epilogue: whole batches");
  half8 hpre[kPreH ? RB : 1], zpre[EB == EPI_GRU_Q ? RB : 1], ppre[kPre ? RB : 1];
  // the per-frame term's pieces (pixel m of image b -> pixel of its source
  // frame): on the 384-row tiles they go out before pass 1 - the accumulators
  // leave room for them there - so their latency and L1 bandwidth overlap the
  // staging writes; the 256x256 tile (2 VGPRs short) issues them after pass 1
  constexpr bool kEarlyPre = kPre && TN != 256 && RB == RND && EARLY;
  auto load_pre = [&](int q0) {
    const long pshift = ((long)a.pre_idx[b] - b) * HW;
    const __half* const pp = a.pre + (mrow + (long)q0 * RQ + pshift) * a.pre_cstride + a.pre_coff + c;
    const long pstep = (long)RQ * a.pre_cstride;
#pragma unroll
    for (int q = 0; q < RB; ++q) ppre[q] = *reinterpret_cast<const half8*>(pp + q * pstep);
  };
  if constexpr (kEarlyPre) load_pre(0);
  __syncthreads();  // main-loop LDS reads are done
  if (tid < TN) bl[tid] = bcol;
  __syncthreads();
  auto act = [&](float v) -> float {
    if constexpr (kPre) return v;
    else if constexpr (EPI == EPI_GRU_ZR) return sigmoid_fast(v);
    else if constexpr (EPI == EPI_GRU_Q) return tanh_fast(v);
    else if constexpr (EPI == EPI_ACT) return relu ? fmaxf(v, 0.f) : v;
    else if (epi == EPI_GRU_ZR) return sigmoidf_(v);
    else if (epi == EPI_GRU_Q) return tanhf(v);
    else return (a.act == 1) ? fmaxf(v, 0.f) : v;
  };
  stage1(static_cast<const float*>(bl), act);
  if (prof && tid == 0) prof[6] = (long long)__builtin_amdgcn_s_memtime();  // pass 1 written
  // h (and z) pieces of rounds [q0, q0 + RB)
#if DROID_AB
  // A/B timing bound only (wrong r*h): DROID_ZR_NO_H=1 skips the z|r epilogue's
  // global re-read of h - what serving h from LDS could at most save
  const bool no_h = a.ab_no_h != 0;
#else
  constexpr bool no_h = false;
#endif
  auto load_h = [&](int q0) {
    if constexpr (kPreH) {
      const __half* const hp = a.h + (mrow + (long)q0 * RQ) * a.h_cstride + c - (EB == EPI_GRU_ZR ? a.gru_ch : 0);
      const __half* const zp = EB == EPI_GRU_Q ? a.z + (mrow + (long)q0 * RQ) * a.z_cstride + c : nullptr;
      const long hstep = (long)RQ * a.h_cstride, zstep = (long)RQ * a.z_cstride;
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        if constexpr (EB == EPI_GRU_Q) {
          hpre[q] = *reinterpret_cast<const half8*>(hp + q * hstep);
          zpre[q] = *reinterpret_cast<const half8*>(zp + q * zstep);
        } else if (rhalf && !no_h) {
          hpre[q] = *reinterpret_cast<const half8*>(hp + q * hstep);
        }
      }
    }
  };
  if constexpr (kPre && !kEarlyPre) load_pre(0);
  load_h(0);
  if (prof && tid == 0) prof[7] = (long long)__builtin_amdgcn_s_memtime();  // pass-2 loads issued
  __syncthreads();
  if (prof && tid == 0) prof[8] = (long long)__builtin_amdgcn_s_memtime();  // staging barrier passed
  __half* dst0;
  long dstep;
  if (epi == EPI_GRU_ZR) {
    dst0 = rhalf ? a.rnet + mrow * a.gru_ch + c - a.gru_ch : a.zout + mrow * a.gru_ch + c;
    dstep = (long)RQ * a.gru_ch;
  } else {
    dst0 = a.out + mrow * a.out_cstride + a.out_coff + c;
    dstep = (long)RQ * a.out_cstride;
  }
#pragma unroll
  for (int q0 = 0; q0 < RND; q0 += RB) {
    if (q0 > 0) {   // the next batch's pieces (the first batch's went out before the barrier)
      if constexpr (kPre) load_pre(q0);
      load_h(q0);
    }
    // (2a) every round's output piece computed first, (2b) then all stores: with
    // a store inside each round, the in-order vmcnt wait for round q+1's h / z /
    // pre pieces also drained round q's stores (gfx9 counts stores in vmcnt) -
    // one store round trip per round
    half8 outv[RB];
#pragma unroll  // all rounds' LDS reads in flight together
    for (int q = 0; q < RB; ++q) {
      const long m = mrow + (q0 + q) * RQ;
      half8 v = *reinterpret_cast<const half8*>(&smem[(r0 + (q0 + q) * RQ) * ER + p * 8]);
      // The gate algebra runs on packed fp16 (v_pk_add / v_pk_mul_f16, no f32
      // round trips), each op rounded as the reference's autocast fp16 tensor ops
      // round it (gru.py:27-32: conv + glo, r * h, (1 - z) * h + z * q); only the
      // sigmoid / tanh go through f32 (torch evaluates them in f32 and rounds).
      if constexpr (kPre) {
        const half8 x = v + ppre[q];   // the gate argument: per-edge conv + per-frame term
        // sigmoid / tanh two at a time: the exp argument scaling and the "+ 1" on
        // packed f32 (v_pk_mul_f32 / v_pk_add_f32), exp and rcp per value
        typedef float f2_t __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f2_t xf = {(float)x[e], (float)x[e + 1]};
          const f2_t t = xf * (EB == EPI_GRU_ZR ? f2_t{-1.4426950408889634f, -1.4426950408889634f}
                                                : f2_t{2.8853900817779268f, 2.8853900817779268f});
          const f2_t den = f2_t{__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])} + f2_t{1.0f, 1.0f};
          const f2_t r = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
          if constexpr (EB == EPI_GRU_ZR) {   // sigmoid(x) = 1 / (1 + 2^(-x log2 e))
            v[e] = (_Float16)r[0];
            v[e + 1] = (_Float16)r[1];
          } else {                            // tanh(x) = 1 - 2 / (1 + 2^(2x log2 e))
            const f2_t th = f2_t{1.0f, 1.0f} - f2_t{2.0f, 2.0f} * r;
            v[e] = (_Float16)th[0];
            v[e + 1] = (_Float16)th[1];
          }
        }
      }
      if (epi == EPI_GRU_ZR) {
        if (rhalf && !no_h) {
          half8 h;
          if constexpr (kPreH) h = hpre[q];
          else h = *reinterpret_cast<const half8*>(a.h + m * a.h_cstride + c - a.gru_ch);
          v = v * h;   // exact products rounded once: the same bits as the f32 product rounded
        }
      } else if (epi == EPI_GRU_Q) {
        half8 h, z;
        if constexpr (EB == EPI_GRU_Q) {
          h = hpre[q];
          z = zpre[q];
        } else {
          h = *reinterpret_cast<const half8*>(a.h + m * a.h_cstride + c);
          z = *reinterpret_cast<const half8*>(a.z + m * a.z_cstride + c);
        }
        v = gru_blend_f16(z, h, v);
      }
      outv[q] = v;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      if constexpr (DROID_EPI_NT) __builtin_nontemporal_store(outv[q], reinterpret_cast<half8*>(dst0 + (q0 + q) * dstep));
      else *reinterpret_cast<half8*>(dst0 + (q0 + q) * dstep) = outv[q];
    }
  }
}

// EPI_DWHEAD (band <256,256> only): the delta/weight heads (droid_net.py:
// 95-103: conv3x3 128->256 + ReLU, then conv3x3 256->2 per head) in one launch.
// The 256-channel hidden map dw of the tile's R image rows never leaves the CU:
//   (1) T = relu(acc + bias) -> LDS fp16, stored channel-major [256 ch][256 px]
//       (see dwh_t_off): a lane's accumulators are 4 consecutive pixels of one
//       channel, so each fragment is ONE 8-B store with no lane exchange;
//   (2) Y[p][tap*4 + c] = sum_ch T[p][ch] Wh[c][ch][tap] for all 9 taps at once
//       (one 256 x 48 x 256 MFMA GEMM: the taps ride on the N dimension, so the
//       tile needs no halo); its pixel operand comes back channel-contiguous by
//       ds_read_b64_tr_b16 (cdna_hip_programming.md T10);
//   (3) out[o][c] = sum over taps of Y[o + shift(tap)][tap*4 + c] for the output
//       rows y0-1 .. y0+R that this tile's rows feed, atomically added into the
//       zero-initialised fp32 out32 (E,H,W,4).  Each output pixel receives at most
//       two contributions (this tile and one neighbour), so the result does not
//       depend on their order.  Head bias and the weight sigmoid are applied by
//       the caller.
// Byte offset of the 4-pixel chunk ch (pixels 4 ch .. + 3, 8 B) of channel row r
// in the channel-major T image: 512-B rows, the chunk index XORed with a
// function of r & 15.  Bits 0-1 of the XOR are (r >> 2) & 3 and bits 2-4 are
// (r & 3) | ((r >> 3) & 1) << 2, which makes both accesses conflict-free:
//   pass-1 ds_write_b64 (banks mod 32, 16-lane groups): one chunk of 16
//     consecutive rows -> (chunk ^ x) mod 16 takes 16 distinct values;
//   ds_read_b64_tr_b16 (banks mod 64, 32-lane halves): rows r0 + {0..3, 8..11}
//     (+4), chunks 4F .. 4F+3 -> (chunk ^ x) mod 32 takes 32 distinct values.
__device__ __forceinline__ int dwh_t_off(int r, int ch) {
  const int x = ((r >> 2) & 3) | ((r & 3) << 2) | (((r >> 3) & 1) << 4);
  return r * 512 + ((ch ^ x) << 3);
}

template <int FM, int FN, int WM = 4, bool CONTIG = false>
__device__ __forceinline__ void dwhead_epilogue(const ConvArgs& a, floatx4 (&acc)[FM][FN], _Float16* smem, long m0,
                                                int wm, int wn, int lane, int tid, float bcol,
                                                long long* prof = nullptr) {
  constexpr int TMX = 256, YS = 37, NT = 512;
  const int W = a.W, H = a.H, HW = H * W;
  const int R = TMX / W;
  const int b = (int)(m0 / HW);
  const int y0 = (int)((m0 % HW) / W);
  const int fr = lane & 15, fq = lane >> 4;
  char* const T = reinterpret_cast<char*>(smem);   // [256 ch][256 px] fp16, dwh_t_off
  // head weights [48][256] fp16, unpadded 512-B rows with the 16-B piece p of
  // row r stored at slot p ^ (r & 15) (the 16 rows of a B fragment read one
  // piece each: 16 distinct 16-B slots of one 256-B span, conflict-free)
  _Float16* Bh = smem + TMX * 256;
  float* const bl = reinterpret_cast<float*>(smem + TMX * 256 + 48 * 256);  // [256] column biases
  __syncthreads();  // main-loop LDS reads are done
  {
    // the head weights (24 KB) by LDS-DMA now, so they land during pass 1 and
    // take no VGPRs (loaded after pass 1 they cost ~4k of the epilogue's 16k
    // clk, profiles/r05/r05k_*): instruction q of wave w fills rows
    // 2 (w + 8 q) .. + 1, lane l the slot l & 31 of row 2 (w + 8 q) + (l >> 5)
    static_assert(48 * 32 == 3 * NT, "dwhead: three 16-B weight pieces per thread");
    const rsrc_t rs = make_rsrc(a.hw, 48 * 256 * 2);
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int ins = wv + 8 * q, row = 2 * ins + (l >> 5), piece = (l & 31) ^ (row & 15);
      dma16(rs, lds_addr(Bh) + ins * 1024, (unsigned)((row * 256 + piece * 8) * 2));
    }
  }
  if (tid < 256) bl[tid] = bcol;
  __syncthreads();
  // lane (fr, fq) of fragment (i, j): pixels frag_row(i) + 4 fq .. + 3 of
  // channel 16 j + fr = one 8-B chunk of channel row c.  ReLU after the fp16
  // rounding: round(max(x, 0)) == max(round(x), 0) (rounding is monotone and
  // keeps 0), up to the sign of a zero, which no later sum can see.
  {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    const h2_t zero2 = {(_Float16)0.f, (_Float16)0.f};
    // every column bias read before the first store (lgkmcnt counts both: a read
    // issued between stores waits for them), and one address per pixel fragment:
    // dwh_t_off(c + 16 j, ch) = dwh_t_off(c, ch) + 16 j * 512 (the XOR depends on
    // c & 15 only), so the channel blocks are immediate offsets
    float bv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) bv[j] = bl[wn * FN * 16 + j * 16 + fr];
    char* tb[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) tb[i] = T + dwh_t_off(wn * FN * 16 + fr, (frag_row<FM, WM, CONTIG>(wm, i) >> 2) + fq);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const f2_t b2 = {bv[j], bv[j]};
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const h2_t lo = __builtin_elementwise_max(
            __builtin_convertvector(f2_t{acc[i][j][0], acc[i][j][1]} + b2, h2_t), zero2);
        const h2_t hi = __builtin_elementwise_max(
            __builtin_convertvector(f2_t{acc[i][j][2], acc[i][j][3]} + b2, h2_t), zero2);
        const half4_t o = {lo.x, lo.y, hi.x, hi.y};
        *reinterpret_cast<half4_t*>(tb[i] + j * 16 * 512) = o;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's head-weight DMAs landed
  __syncthreads();
  if (prof && tid == 0) prof[6] = (long long)__builtin_amdgcn_s_memtime();  // pass 1 + head weights in LDS
  // (2) wave w: pixel fragments 2w, 2w+1; all 3 tap-channel fragments; K = 256
  const int wave = tid >> 6;
  floatx4 y[2][3];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int n = 0; n < 3; ++n) y[f][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // A operand of pixel fragment F = 2 wave + f, k-step s, by two transposed
  // reads: lane (i = fr, g = fq) gets channels 32 s + 8 g + 4 t .. + 3 (t = 0, 1)
  // of pixel 16 F + i; as the address-supplying lane 4 q + p of its 16-lane
  // group it points at channel row 32 s + 8 g + 4 t + q, pixels 16 F + 4 p .. + 3
  typedef short s4_t __attribute__((vector_size(8)));
  int toff[2][2];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < 2; ++t) toff[f][t] = dwh_t_off(8 * fq + 4 * t + (fr >> 2), 4 * (2 * wave + f) + (fr & 3));
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    half8 af[2], bf[3];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const s4_t r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s4_t*)(T + toff[f][0] + s * 32 * 512));
      const s4_t r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s4_t*)(T + toff[f][1] + s * 32 * 512));
      const half4_t h0 = __builtin_bit_cast(half4_t, r0), h1 = __builtin_bit_cast(half4_t, r1);
      af[f] = half8{h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    }
#pragma unroll
    for (int n = 0; n < 3; ++n) {
      const int row = n * 16 + fr;
      bf[n] = *reinterpret_cast<const half8*>(&Bh[row * 256 + (((4 * s + fq) ^ (row & 15)) << 3)]);
    }
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int n = 0; n < 3; ++n) y[f][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[f], bf[n], y[f][n], 0, 0, 0);
  }
  if (prof && tid == 0) prof[7] = (long long)__builtin_amdgcn_s_memtime();  // wave 0's head GEMM issued
  __syncthreads();  // T and Bh reads done: Y overwrites them
  float* Y = reinterpret_cast<float*>(smem);  // [256][YS]
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int n = 0; n < 3; ++n)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = n * 16 + fr;
        if (col < 36) Y[((2 * wave + f) * 16 + fq * 4 + k) * YS + col] = y[f][n][k];
      }
  __syncthreads();
  if (prof && tid == 0) prof[8] = (long long)__builtin_amdgcn_s_memtime();  // Y in LDS
  // (3) output rows y0-1 .. y0+R
  for (int idx = tid; idx < (R + 2) * W * 4; idx += NT) {
    const int c = idx & 3, px = idx >> 2;
    const int orow = px / W - 1, x = px - (px / W) * W;
    const int oy = y0 + orow;
    if (oy < 0 || oy >= H) continue;
    // all nine taps read first (clamped in-tile addresses), the out-of-tile ones
    // then summed as +0: the same sum in the same order as skipping them (the
    // running sum starts at +0 and so is never -0)
    float v[9];
#pragma unroll
    for (int ty = -1; ty <= 1; ++ty) {
      const int sr = min(max(orow + ty, 0), R - 1);
#pragma unroll
      for (int tx = -1; tx <= 1; ++tx) {
        const int sx = min(max(x + tx, 0), W - 1);
        v[(ty + 1) * 3 + tx + 1] = Y[(sr * W + sx) * YS + ((ty + 1) * 3 + tx + 1) * 4 + c];
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int ty = -1; ty <= 1; ++ty) {
      const bool rok = orow + ty >= 0 && orow + ty < R;
#pragma unroll
      for (int tx = -1; tx <= 1; ++tx) {
        const bool ok = rok && x + tx >= 0 && x + tx < W;
        sum += ok ? v[(ty + 1) * 3 + tx + 1] : 0.f;
      }
    }
    atomicAdd(a.out32 + ((long)b * HW + (long)oy * W + x) * 4 + c, sum);
  }
}

// acc += a x b (v_mfma_f32_16x16x32_f16) with the accumulator pinned in the
// AGPR file ("+a"): the 4-wave tile's 256 accumulators per lane fill the AGPRs
// exactly, and with the builtin the register allocator moved some of them to
// VGPRs and back (v_accvgpr_read / write in every stage and ~512 at each chunk's
// back edge).  Hazards the compiler no longer pads (cdna_hip_programming.md
// §5.7 item 2): operands come from ds_read (LDS loads, counted by hipcc's
// lgkmcnt waits, no VALU wait states); consecutive MFMAs on the same
// accumulator take it whole as C (0 states); the accumulators' zero fill is
// separated from the first MFMA by the stage prologue; and mfma_acc_drain()
// pads the 12 states an 8-pass MFMA's D needs before any other reader.
__device__ __forceinline__ void mfma_acc(floatx4& acc, const half8& a, const half8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc_drain() { asm volatile("s_nop 7\n\ts_nop 4" ::: "memory"); }

// one MFMA then one LDS read, R times (sched_group_barrier sequence)
template <int R>
struct MfmaReadPairs {
  static __device__ __forceinline__ void emit() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    MfmaReadPairs<R - 1>::emit();
  }
};
template <>
struct MfmaReadPairs<0> {
  static __device__ __forceinline__ void emit() {}
};

template <int TMX, int TN, bool DWHEAD, bool ILV, int EPI, int NW = 8, bool PAIR = false>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 4 ? 1 : 2, NW == 4 ? 1 : 2)))
conv_band_kernel(ConvArgs a) {
  using BP = Band<TMX, TN, NW>;
  constexpr int FM = BP::FM, FN = BP::FN, WN = BP::WN, NBI = BP::NBI, NPAR = BP::NPAR;
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  char* lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int W = a.W, H = a.H, HW = H * W;
  const long wgid = xcd_work_id(a.m_tiles * a.n_tiles);
  const long mt = wgid / a.n_tiles;
  const int nt = (int)(wgid - mt * a.n_tiles);
  const long m0 = mt * TMX;
  const int n0 = nt * TN;
  const int y0 = (int)((m0 % HW) / W);
  const long band0 = m0 - W;  // pixel index of the band's first (halo) row
  const int nslot = a.nslot, nhi = a.nhi;
  const int hbytes = nhi * NW * 1024;  // one band buffer
  char* Bl = lds;                     // [2][TN][128 B]  (PAIR: [2][2 taps][TN][128 B])
  char* Hl = lds + (PAIR ? 4 : 2) * TN * 128;      // [2][nhi * 64 slots][128 B]

  // ---- DMA lane geometry: instruction q of this wave covers 8 LDS rows of
  // 128 B; lane l writes row 8*(wave + 8q) + (l >> 3), 16-B slot l & 7, which
  // holds logical piece (l & 7) ^ (row & 7) (the XOR swizzle)
  const int lrow = lane >> 3;
  const int lpiece = (lane & 7) ^ lrow;
  // halo slot -> pixel offset within the band, or -1 (outside the image / padding)
  int hpix[BP::MAX_NHI];
#pragma unroll
  for (int q = 0; q < BP::MAX_NHI; ++q) {
    const int slot = (wave + NW * q) * 8 + lrow;
    const int ry = slot / W;
    const int y = y0 - 1 + ry;
    hpix[q] = (q < nhi && slot < nslot && y >= 0 && y < H) ? slot : -1;
  }
  const rsrc_t rsb = make_rsrc(a.wp + (long)n0 * a.nstage * BK, TN * a.nstage * BK * 2);
  const unsigned Bl_a = lds_addr(Bl), Hl_a = lds_addr(Hl);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  unsigned boff[NBI];
#pragma unroll
  for (int q = 0; q < NBI; ++q) boff[q] = (unsigned)((((wave + NW * q) * 8 + lrow) * a.nstage * BK + lpiece * 8) * 2);

  auto issue_b = [&](int st) {
    const unsigned dst = Bl_a + (st & 1) * TN * 128;
#pragma unroll
    for (int q = 0; q < NBI; ++q) dma16(rsb, dst + (wave_u + NW * q) * 1024, boff[q] + st * BK * 2);
  };
  auto issue_halo = [&](int chunk) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q + 1 < a.nsrc && chunk >= a.chunk_end[q]) s = q + 1;
    const int cstart = s ? a.chunk_end[s - 1] : 0;
    const ConvSrc src = a.src[s];
    const int c = (chunk - cstart) * BK + lpiece * 8;
    const bool okc = c < src.C;
    const rsrc_t rs = make_rsrc(src.ptr + band0 * src.cstride, nslot * src.cstride * 2);
    const unsigned dst = Hl_a + (chunk & 1) * hbytes;
#pragma unroll
    for (int q = 0; q < BP::MAX_NHI; ++q) {
      if (q < nhi) {
        const unsigned off = (okc && hpix[q] >= 0) ? (unsigned)((hpix[q] * src.cstride + c) * 2) : kOob;
        if constexpr (DROID_BAND_A_NT) dma16_nt(rs, dst + (wave_u + NW * q) * 1024, off);
        else dma16(rs, dst + (wave_u + NW * q) * 1024, off);
      }
    }
  };

  // ---- fragment addresses.  Lane (fr, kq): A row = tile pixel p = 16 (wm + 4i) + fr,
  // band slot W + p + ty*W + tx; B row wn*TN/2 + 16j + fr.  Since W % 16 == 0 the
  // slot's low 3 bits are (fr + tx) & 7, so the swizzled byte offset splits into a
  // per-lane base (by tx, K half) plus compile-time i*8192 and a uniform ty*W*128.
  // Column of the lane's pixels: (16 wm + fr) % W for every i (W | 64).
  const int fr = lane & 15;
  constexpr int kLdsZero = 0x100000;  // base past the LDS allocation: reads return 0
  // fragment i of the wave: tile pixels 16 (wm + WM i) + fr = the parity-(i % NPAR)
  // base plus (i / NPAR) x 64 pixels (8192 B): the same image column for every i
  // of one parity (W | 64)
  int abase[NPAR][3][2], bbase[2];
#pragma unroll
  for (int hk = 0; hk < 2; ++hk) {
    const int kq = (lane >> 4) + hk * 4;
#pragma unroll
    for (int par = 0; par < NPAR; ++par) {
      const int px0 = 16 * wm + 16 * BP::WM * par + fr;
      const int xcol = px0 % W;
#pragma unroll
      for (int tx = -1; tx <= 1; ++tx) {
        const int sl = W + px0 + tx;
        const bool off_image = (tx < 0 && xcol == 0) || (tx > 0 && xcol == W - 1);
        abase[par][tx + 1][hk] = off_image ? kLdsZero : sl * 128 + ((kq ^ ((fr + tx) & 7)) << 4);
      }
    }
    bbase[hk] = (wn * (TN / 2) + fr) * 128 + ((kq ^ (fr & 7)) << 4);
  }

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nch = a.cpt;
  const int nst = a.nstage;  // nch * 9
  const int rowb = W * 128;

  // timeline (profiling builds of the call only): s_memtime at entry, loop
  // start (first stage's operands landed), loop end and exit, plus the CU id
#if DROID_CONV_PROFILE
  long long* const prof = a.prof ? a.prof + kProfSlots * blockIdx.x : nullptr;
#else
  long long* const prof = nullptr;  // the hooks cost the 256x256 tile registers: profiling builds only
#endif
  if (prof && tid == 0) {
    const unsigned hwid = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
    prof[0] = (long long)hwid | ((long long)(xcc & 15) << 32);
    prof[1] = (long long)__builtin_amdgcn_s_memtime();
  }
  // PAIR: the weights of two-tap stage (ch, u) - taps 2u and 2u + 1 (u = 4: tap
  // 8 alone) - into tap blocks 0 / 1 of the double buffer of stage position sp
  auto issue_pair = [&](int ch, int u, int sp) {
    const unsigned dst = Bl_a + (sp & 1) * 2 * TN * 128;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int tap = 2 * u + k;
      if (tap < 9) {
#pragma unroll
        for (int q = 0; q < NBI; ++q)
          dma16(rsb, dst + k * TN * 128 + (wave_u + NW * q) * 1024, boff[q] + (ch * 9 + tap) * BK * 2);
      }
    }
  };
  issue_halo(0);
  if constexpr (PAIR) issue_pair(0, 0, 0);
  else issue_b(0);
  // column tid's bias (+ per-image bias), loaded now so the latency hides under
  // the main loop; the epilogue shares them through LDS
  float bcol = 0.f;
  if (tid < TN) {
    const int co = n0 + tid;
    if (a.bias) bcol = a.bias[co];
    if (a.bbias) bcol += a.bbias[(long)(m0 / HW) * a.Cout + co];
  }
  if (prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) {
      prof[2] = (long long)__builtin_amdgcn_s_memtime();
      prof[10] = (long long)__builtin_amdgcn_s_memrealtime();   // 100 MHz: the in-kernel clock over the loop
    }
  }
  if constexpr (NW == 4) {
    // One wave per SIMD: nothing else on the SIMD hides this wave's LDS
    // latency, so each stage is software pipelined in program order (every
    // group fenced by sched_barrier), the tap t a compile-time constant (a
    // generic lambda per tap: the nine stages of a chunk exceed the unroller's
    // budget).  The stage's first four K-half-0 A fragments were read before
    // its barrier (same band, t > 0), so after the barrier the B fragments are
    // the only reads outstanding, and half 0 runs column by column over A_0..A_3
    // (B_j, then B_j+1, ...: the first four MFMAs need B_0 alone while the other
    // B reads - the four waves' reads land in one burst after the barrier -
    // still arrive), then over A_4..A_7 (read behind B); half 1's fragments are
    // read under half 0's MFMAs, the next stage's first four A fragments under
    // half 1's.  Every accumulator still sees the same products in the same
    // order: bitwise the sums of the 8-wave tile.
    half8 apf[4];
    for (int ch = 0; ch < nch; ++ch) {
      const char* Hb = Hl + (ch & 1) * hbytes;
      auto stage = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        constexpr int ty = t / 3 - 1, tx = t % 3 - 1;
        const int st = ch * 9 + t;
        if (!(DROID_CONV_ABLATE & 4) || st == 0) wait_vmcnt((t == 1 && ch + 1 < nch) ? nhi : 0);
        if (!(DROID_CONV_ABLATE & 1)) __builtin_amdgcn_s_barrier();
        const char* Bb = Bl + (st & 1) * TN * 128;
        auto ald = [&](int hk, int i, int tyy, int txx) {
          return *reinterpret_cast<const half8*>(Hb + abase[i % NPAR][txx + 1][hk] + tyy * rowb + (i / NPAR) * 8192);
        };
        auto bld = [&](int hk, int j) { return *reinterpret_cast<const half8*>(Bb + bbase[hk] + j * 2048); };
        half8 a0[FM], a1[FM], b0[FN], b1[FN];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j) b0[j] = bld(0, j);
#pragma unroll
        for (int i = 0; i < 4; ++i) a0[i] = t == 0 ? ald(0, i, ty, tx) : apf[i];
#pragma unroll
        for (int i = 4; i < FM; ++i) a0[i] = ald(0, i, ty, tx);
        __builtin_amdgcn_sched_barrier(0);
        // half 0: columns over A_0..A_3, then over A_4..A_7; half 1's 16
        // fragments read one per 4 MFMAs; the next stage's DMA issued once the
        // first MFMAs are under way
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
              const int i = 4 * ih + ii;
              mfma_acc(acc[i][j], a0[i], b0[j]);
              const int m = (ih * FN + j) * 4 + ii;
              if (m % 4 == 3) {
                const int r = m / 4;   // 0 .. 15
                if (r < FN) b1[r] = bld(1, r);
                else a1[r - FN] = ald(1, r - FN, ty, tx);
              }
              __builtin_amdgcn_sched_barrier(0);
              if (m == 1 && (!(DROID_CONV_ABLATE & 2) || st == 0)) {
                if (st + 1 < nst) issue_b(st + 1);
                if (t == 0 && ch + 1 < nch) issue_halo(ch + 1);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
          }
        }
        // half 1; the next stage's first four half-0 A fragments (same band,
        // t < 8) read one per 16 MFMAs
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            mfma_acc(acc[i][j], a1[i], b1[j]);
            if constexpr (t < 8) {
              if (j == 3 && i % 2 == 1) {
                constexpr int tn = t + 1;
                apf[i / 2] = ald(0, i / 2, tn / 3 - 1, tn % 3 - 1);
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      };
      stage(std::integral_constant<int, 0>{});
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      stage(std::integral_constant<int, 4>{});
      stage(std::integral_constant<int, 5>{});
      stage(std::integral_constant<int, 6>{});
      stage(std::integral_constant<int, 7>{});
      stage(std::integral_constant<int, 8>{});
    }
  } else if constexpr (PAIR) {
    // Two-tap stages (the 64-channel 384-row tile, flow_encoder[2]): 5 barriers
    // per chunk instead of 9, each over 2 x 24 MFMAs per wave (the one-tap
    // stage's fixed costs - barrier, waits, DMA issue - were a third of its
    // time); the double-buffered weights are two tap blocks per stage, which
    // fills the LDS exactly (32 + 128 KB).  Same products in the same order per
    // accumulator: bitwise the one-tap kernel.
    static_assert(ILV && NW == 8 && TN == 64, "two-tap stages: the 64-channel interleaved tile");
    auto tap_mfma = [&](const char* Hb, const char* Bb, int ty, int tx) {
      __builtin_amdgcn_sched_barrier(0);
      half8 af[2][FM], bf[2][FN];
#pragma unroll
      for (int hk = 0; hk < 2; ++hk) {
        auto aptr = [&](int i) { return Hb + abase[i % NPAR][tx + 1][hk] + ty * rowb + (i / NPAR) * 8192; };
        af[hk][0] = *reinterpret_cast<const half8*>(aptr(0));
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[hk][j] = *reinterpret_cast<const half8*>(Bb + bbase[hk] + j * 2048);
#pragma unroll
        for (int i = 1; i < FM; ++i) af[hk][i] = *reinterpret_cast<const half8*>(aptr(i));
      }
#pragma unroll
      for (int hk = 0; hk < 2; ++hk)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[hk][j], af[hk][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, FM + FN, 0);
      MfmaReadPairs<FM + FN>::emit();
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * FM * FN - (FM + FN), 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    const int nsp = nch * 5;
    int sp = 0;
    for (int ch = 0; ch < nch; ++ch) {
      const char* Hb = Hl + (ch & 1) * hbytes;
#pragma unroll
      for (int u = 0; u < 5; ++u, ++sp) {
        // this stage's weights (and at u == 0 this chunk's band) must have
        // landed; at u == 1 the next chunk's band (issued after them) may stay in flight
        wait_vmcnt((u == 1 && ch + 1 < nch) ? nhi : 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (sp + 1 < nsp) issue_pair(u < 4 ? ch : ch + 1, u < 4 ? u + 1 : 0, sp + 1);
        if (u == 0 && ch + 1 < nch) issue_halo(ch + 1);
        const char* Bb = Bl + (sp & 1) * 2 * TN * 128;
        tap_mfma(Hb, Bb, (2 * u) / 3 - 1, (2 * u) % 3 - 1);
        if (u < 4) tap_mfma(Hb, Bb + TN * 128, (2 * u + 1) / 3 - 1, (2 * u + 1) % 3 - 1);
      }
    }
  } else {
  int st = 0;
  for (int ch = 0; ch < nch; ++ch) {
    const char* Hb = Hl + (ch & 1) * hbytes;
#pragma unroll
    for (int t = 0; t < 9; ++t, ++st) {
      const int ty = t / 3 - 1, tx = t % 3 - 1;
      // this stage's weights (and at t == 0 this chunk's band) must have landed;
      // at t == 1 the next chunk's band (issued after them) may stay in flight
      if (!(DROID_CONV_ABLATE & 4) || st == 0) wait_vmcnt((t == 1 && ch + 1 < nch) ? nhi : 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // DROID_CONV_ABLATE (profiling experiments only, results invalid):
      // bit 0 drops the stage barrier, bit 1 the DMA after the first stage,
      // bit 2 the DMA waits after the first stage
      if (!(DROID_CONV_ABLATE & 1)) __builtin_amdgcn_s_barrier();
      if (!(DROID_CONV_ABLATE & 2) || st == 0) {
        if (st + 1 < nst) issue_b(st + 1);
        if (t == 0 && ch + 1 < nch) issue_halo(ch + 1);
      }
      const char* Bb = Bl + (st & 1) * TN * 128;
      if constexpr (ILV) {
        // all fragments of the stage read up front (A0, B0..B7 first, so the
        // first MFMA waits for two reads only); the K-half-1 reads interleave
        // one per MFMA with the K-half-0 multiplies (sched_group_barrier), so
        // they land long before their use and the MFMA pipe is not paced by
        // the LDS latency
        static_assert(kBandSwap<TN> || NW == 4, "the interleaved body: the swapped 384-row tiles, the 4-wave tile");
        __builtin_amdgcn_sched_barrier(0);
        half8 af[2][FM], bf[2][FN];
#pragma unroll
        for (int hk = 0; hk < 2; ++hk) {
          auto aptr = [&](int i) {
            return Hb + abase[i % NPAR][tx + 1][hk] + ty * rowb + (i / NPAR) * 8192;
          };
          af[hk][0] = *reinterpret_cast<const half8*>(aptr(0));
#pragma unroll
          for (int j = 0; j < FN; ++j) bf[hk][j] = *reinterpret_cast<const half8*>(Bb + bbase[hk] + j * 2048);
#pragma unroll
          for (int i = 1; i < FM; ++i) af[hk][i] = *reinterpret_cast<const half8*>(aptr(i));
        }
#pragma unroll
        for (int hk = 0; hk < 2; ++hk)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = kBandSwap<TN> ? __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[hk][j], af[hk][i], acc[i][j], 0, 0, 0)
                                        : __builtin_amdgcn_mfma_f32_16x16x32_f16(af[hk][i], bf[hk][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, FM + FN, 0);
        MfmaReadPairs<FM + FN>::emit();
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * FM * FN - (FM + FN), 0);
        __builtin_amdgcn_sched_barrier(0);
      } else {
#pragma unroll
        for (int hk = 0; hk < 2; ++hk) {
          half8 af[FM], bf[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[i] = *reinterpret_cast<const half8*>(Hb + abase[i % NPAR][tx + 1][hk] + ty * rowb + (i / NPAR) * 8192);
#pragma unroll
          for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const half8*>(Bb + bbase[hk] + j * 2048);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = kBandSwap<TN> ? __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0)
                                        : __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  }   // NW == 4
  if constexpr (NW == 4) mfma_acc_drain();
  if (prof && tid == 0) {
    prof[3] = (long long)__builtin_amdgcn_s_memtime();
    prof[11] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  if constexpr (DWHEAD) {
    static_assert(TMX == 256 && TN == 256 && NW == 8, "dw/head fusion runs on the 8-wave 256x256 tile");
    dwhead_epilogue<FM, FN>(a, acc, smem, m0, wm, wn, lane, tid, bcol, prof);
  } else {
    band_epilogue<TMX, TN, FM, FN, BP::WM, false, BP::NT, EPI>(a, acc, smem, m0, n0, wm, wn, lane, tid, bcol, prof);
  }
  if (prof) {
    if (tid == 0) prof[4] = (long long)__builtin_amdgcn_s_memtime();  // stores issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) prof[5] = (long long)__builtin_amdgcn_s_memtime();  // stores drained
    // the last wave's drain (the workgroup's resources free only then)
    if (lane == 0) atomicMax(reinterpret_cast<unsigned long long*>(prof + 9),
                             (unsigned long long)__builtin_amdgcn_s_memtime());
  }
}

// DROID_CONV_ILV=0 selects the compiler-scheduled stage body (A/B runs)
static bool band_interleaved() {
  static const bool on = ab_knob("DROID_CONV_ILV", 1) != 0;
  return on;
}

template <int TMX, int TN, int NW = 8>
static bool band_fits(int W, int* nslot, int* nhi) {
  const int ns = (TMX / W + 2) * W;
  const int nh = ceil_div(ns, 8 * NW);
  if (nh > Band<TMX, TN, NW>::MAX_NHI) return false;
  const int lds = 2 * TN * 128 + 2 * nh * NW * 1024;
  const int epi = TMX * (TN + 8) * 2 + TN * 4;  // staging tile + column biases
  if (lds > kLdsMax || epi > kLdsMax) return false;
  *nslot = ns;
  *nhi = nh;
  return true;
}

template <int TMX, int TN, bool DWHEAD, bool ILV, int EPI, int NW = 8, bool PAIR = false>
static int launch_band_kernel(const ConvArgs& a, long nwg, int lds, hipStream_t stream) {
  static bool attr = false;  // one per instantiation
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_band_kernel<TMX, TN, DWHEAD, ILV, EPI, NW, PAIR>),
        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    attr = true;
  }
  conv_band_kernel<TMX, TN, DWHEAD, ILV, EPI, NW, PAIR><<<dim3((unsigned)nwg), NW * 64, lds, stream>>>(a);
  return kOk;
}

// the 64-channel 384-row tile's two-tap stages (flow_encoder[2]); DROID_CONV_PAIR=0
// (A/B build) keeps the one-tap stages
static int& band_pair() {
  static int on = ab_knob("DROID_CONV_PAIR", 1);
  return on;
}

static int& band2_mode();
#if DROID_AB
// A/B build: the z|r gates (256x256, per-frame term) on the 4-wave tile, tile
// policy 2 (droid_conv_set_tile) or DROID_CONV_NW4=1.  Measured (round 5,
// profiles/r05/): 7.85 vs 7.45 ms for the 8-wave tile at C3 - a single wave
// per SIMD pays every ds_read_b128's issue (~18 clk, scripts/probe/
// mfma_1wave.hip) on its own MFMA stream: 2818 vs 2564 clk per stage.
static bool band_nw4() {
  static const bool env = ab_knob("DROID_CONV_NW4", 0) == 1;
  return env || band2_mode() == 2;
}

template <int TMX, int TN>
static int launch_band_nw4(const ConvArgs& a0, hipStream_t stream) {
  ConvArgs a = a0;
  if (!band_fits<TMX, TN, 4>(a.W, &a.nslot, &a.nhi)) return fail(kUnsupported, "conv band: shape");
  a.n_tiles = a.Cout / TN;
  a.m_tiles = (long)a.B * a.H * a.W / TMX;
  const int main_b = 2 * TN * 128 + 2 * a.nhi * 4 * 1024;
  const int epi_b = TMX * (TN + 8) * 2 + TN * 4;
  const int lds = main_b > epi_b ? main_b : epi_b;
  if (lds > kLdsMax) return fail(kUnsupported, "conv band: LDS");
  const long nwg = a.m_tiles * a.n_tiles;
  const int st = launch_band_kernel<TMX, TN, false, false, EPI_GRU_ZRP, 4>(a, nwg, lds, stream);
  if (st != kOk) return st;
  DROID_LAUNCH_CHECK();
  return kOk;
}
#else
static bool band_nw4() { return false; }
template <int TMX, int TN>
static int launch_band_nw4(const ConvArgs&, hipStream_t) {
  return fail(kUnsupported, "conv band: the 4-wave z|r tile ships in the A/B build only (make ab)");
}
#endif

template <int TMX, int TN, bool DWHEAD = false>
static int launch_band(const ConvArgs& a0, hipStream_t stream) {
  ConvArgs a = a0;
  if (!band_fits<TMX, TN>(a.W, &a.nslot, &a.nhi)) return fail(kUnsupported, "conv band: shape");
  a.n_tiles = a.Cout / TN;
  a.m_tiles = (long)a.B * a.H * a.W / TMX;
  const int main_b = 2 * TN * 128 + 2 * a.nhi * 8 * 1024;
  // EPI_DWHEAD keeps the head weights [48][264] beside the hidden-map tile
  const int epi_b = TMX * (TN + 8) * 2 + TN * 4 + (DWHEAD ? 48 * 256 * 2 : 0);
  const int lds = main_b > epi_b ? main_b : epi_b;
  if (lds > kLdsMax) return fail(kUnsupported, "conv band: LDS");
  const long nwg = a.m_tiles * a.n_tiles;
  if (nwg > 0x7fffffffL) return fail(kUnsupported, "conv_nhwc_f16: problem too large");
  // interleaved stage body: +2-5 % on the 384-row tiles; the 256x256 tile has
  // no registers for it (it spills), so it keeps the compiler's schedule
  bool ilv = false;
  if constexpr (TN != 256) ilv = band_interleaved();
  int st = kOk;
  if constexpr (DWHEAD) {
    st = launch_band_kernel<TMX, TN, true, false, EPI_DWHEAD>(a, nwg, lds, stream);
  } else {
    int epi = a.epi == EPI_GRU_ZR ? EPI_GRU_ZR : a.epi == EPI_GRU_Q ? EPI_GRU_Q : EPI_ACT;
    if (a.pre && epi != EPI_ACT) epi += kEpiPreShift;
    // the instantiations the update operator's shapes take: z|r on 256x256,
    // q and the plain convs on the 384-row tiles
    if constexpr (TN != 256) {
      if (ilv) {
        if (epi == EPI_GRU_Q) st = launch_band_kernel<TMX, TN, false, true, EPI_GRU_Q>(a, nwg, lds, stream);
        else if (epi == EPI_GRU_QP) st = launch_band_kernel<TMX, TN, false, true, EPI_GRU_QP>(a, nwg, lds, stream);
        else if (epi == EPI_GRU_ZR) st = launch_band_kernel<TMX, TN, false, true, EPI_GRU_ZR>(a, nwg, lds, stream);
        else if (epi == EPI_GRU_ZRP) st = launch_band_kernel<TMX, TN, false, true, EPI_GRU_ZRP>(a, nwg, lds, stream);
        else if constexpr (TN == 64) {
          // two-tap stages when the doubled weight buffer still fits (W == 64: exactly)
          const int main_p = 4 * TN * 128 + 2 * a.nhi * 8 * 1024;
          if (band_pair() && main_p <= kLdsMax)
            st = launch_band_kernel<TMX, TN, false, true, EPI_ACT, 8, true>(a, nwg, main_p > epi_b ? main_p : epi_b,
                                                                           stream);
          else
            st = launch_band_kernel<TMX, TN, false, true, EPI_ACT>(a, nwg, lds, stream);
        } else {
          st = launch_band_kernel<TMX, TN, false, true, EPI_ACT>(a, nwg, lds, stream);
        }
      }
    }
    if (!ilv) {
      if (epi == EPI_GRU_ZR) st = launch_band_kernel<TMX, TN, false, false, EPI_GRU_ZR>(a, nwg, lds, stream);
      else if (epi == EPI_GRU_ZRP) st = launch_band_kernel<TMX, TN, false, false, EPI_GRU_ZRP>(a, nwg, lds, stream);
      else if (epi == EPI_GRU_Q) st = launch_band_kernel<TMX, TN, false, false, EPI_GRU_Q>(a, nwg, lds, stream);
      else if (epi == EPI_GRU_QP) st = launch_band_kernel<TMX, TN, false, false, EPI_GRU_QP>(a, nwg, lds, stream);
      else st = launch_band_kernel<TMX, TN, false, false, EPI_ACT>(a, nwg, lds, stream);
    }
  }
  if (st != kOk) return st;
  DROID_LAUNCH_CHECK();
  return kOk;
}

// ---------------------------------------------------------------------------
// Two-workgroups-per-CU band kernel (3x3, CHUNKED, W == 64): the direct conv
// of conv_band_kernel on a 4-wave 256-pixel x 128-channel tile in 72 KB of
// LDS, so two workgroups share a CU and one's epilogue, barriers and DMA
// waits run under the other's MFMAs (with one 8-wave workgroup per CU the
// SQ counters put 28 % of the z|r wave time in s_waitcnt / s_barrier and the
// MFMA pipe idles through every tile's epilogue; profiles/r03/wino_r03bg.txt).
// Wave (wm, wn): image rows 2 wm, 2 wm + 1 of the tile (8 pixel fragments of
// 16, contiguous) x channels wn*64 .. +63, pixels x weights on MFMA (a lane's
// accumulators are 4 pixels of one channel; swapped, the allocation spills, as
// on the 256x256 band tile), 128 accumulators.
// Stage = (32-channel half chunk, tap): one K-step, 32 MFMAs, 8 + 4
// ds_read_b128 per wave.  LDS: the 6-row band of one half chunk (6 x 64 px x
// 64 B = 24 KB, double buffered, issued 9 stages ahead) and the weights of one
// stage (128 rows x 64 B = 8 KB, triple buffered, issued 2 stages ahead).
// 64-B rows: 16-B slot kq of row r stored at kq ^ (2 * ((r >> 2) & 1)) - no
// bank conflict for a 16-row ds_read_b128 fragment at any row offset, so the
// taps' +-1 pixel shifts stay conflict-free (searched exhaustively over the
// four ds_read_b128 lane groups).  Weights: the direct conv's packed layout
// [Cout][chunks*9][64] (pack_conv), read half a stage row at a time.
constexpr int kB2TM = 256, kB2TN = 128;
constexpr int kB2Band = 6 * 64 * 64;     // one half-chunk band buffer (bytes)
constexpr int kB2Wst = kB2TN * 64;       // one weight stage buffer (bytes)
constexpr int kB2Lds = 2 * kB2Band + 3 * kB2Wst;
static_assert(kB2Lds >= kB2TM * (kB2TN + 8) * 2 + kB2TN * 4, "band2: epilogue staging fits the loop's LDS");
__device__ __forceinline__ int b2_slot(int r, int kq) { return kq ^ (((r >> 2) & 1) << 1); }
// pixels x weights on MFMA; weights x pixels (DROID_B2_SWAP=1) measured the same
#ifndef DROID_B2_SWAP
#define DROID_B2_SWAP 0
#endif
constexpr bool kB2Swap = DROID_B2_SWAP != 0;

// REUSE (round 4): the taps run column-major (tx outer, ty inner) and a wave
// reads the A fragments of a tap column once: fragment i of tap (ty, tx) is band
// row 2 wm + (i >> 2) + ty + 1, column group i & 3, so the three ty taps of one
// tx use band rows 2 wm .. 2 wm + 3 - 16 fragments for 96 MFMAs instead of 24.
// LDS reads per MFMA fall from 12 KB / 32 to 28 KB / 96 (-22 %); the weights
// stay one (half chunk, tap) stage per DMA step, issued in the same tap order.
template <int EPI, bool REUSE = true>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) conv_band2_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = a.H * 64;
  const long wgid = xcd_work_id(a.m_tiles * a.n_tiles);
  const long mt = wgid / a.n_tiles;
  const int nt = (int)(wgid - mt * a.n_tiles);
  const long m0 = mt * kB2TM;
  const int n0 = nt * kB2TN;
  const int y0 = (int)((m0 % HW) >> 6);
  const long band0 = m0 - 64;
  char* Hl = lds;                     // [2][6 rows][64 px][64 B]
  char* Bl = lds + 2 * kB2Band;       // [3][128 ch][64 B]
  const unsigned Hl_a = lds_addr(Hl), Bl_a = lds_addr(Bl);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  float bcol = 0.f;   // column tid's bias (+ per-image bias), loaded before any DMA
  if (tid < kB2TN) {
    const int co = n0 + tid;
    if (a.bias) bcol = a.bias[co];
    if (a.bbias) bcol += a.bbias[(long)(m0 / HW) * a.Cout + co];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // DMA lane geometry (band and weights): instruction block b fills LDS rows
  // 16 b .. + 15; lane l writes row 16 b + (l >> 2), physical slot l & 3 =
  // logical K piece (l & 3) ^ (2 * ((l >> 4) & 1))
  const int lpiece = b2_slot(lane >> 2, lane & 3);
  // band instruction q of wave w covers band row q, pixels 16 w + (l >> 2): the
  // row's validity is wave-uniform
  const int bpix = wave * 16 + (lane >> 2);
  auto issue_band = [&](int bg) {
    const int chunk = bg >> 1;
    int s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q + 1 < a.nsrc && chunk >= a.chunk_end[q]) s = q + 1;
    const int cstart = s ? a.chunk_end[s - 1] : 0;
    const ConvSrc src = a.src[s];
    const int c = (chunk - cstart) * BK + (bg & 1) * 32 + lpiece * 8;
    const bool okc = c < src.C;
    const rsrc_t rs = make_rsrc(src.ptr + band0 * src.cstride, 6 * 64 * src.cstride * 2);
    const unsigned dst = Hl_a + (bg & 1) * kB2Band;
    const unsigned off0 = okc ? (unsigned)((bpix * src.cstride + c) * 2) : kOob;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int y = y0 - 1 + q;
      const unsigned off = (y >= 0 && y < a.H && okc) ? off0 + (unsigned)(q * 64 * src.cstride * 2) : kOob;
      dma16(rs, dst + (wave_u + 4 * q) * 1024, off);
    }
  };
  const int nst9 = a.nstage;   // chunks * 9 (the packed layout's stages)
  const rsrc_t rsw = make_rsrc(a.wp + (long)n0 * nst9 * BK, kB2TN * nst9 * BK * 2);
  unsigned woff[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) woff[q] = (unsigned)((((wave + 4 * q) * 16 + (lane >> 2)) * nst9 * BK + lpiece * 8) * 2);
  // loop stage s = (half chunk bg = s / 9, step u = s % 9) -> tap t = tap_of(u): packed
  // stage (bg >> 1) * 9 + t, K half bg & 1 (REUSE: column-major tap order)
  auto tap_of = [](int u) { return REUSE ? (u % 3) * 3 + u / 3 : u; };
  auto issue_w = [&](int s, int buf) {
    const int bg = s / 9, t = tap_of(s - 9 * bg);
    const unsigned sb = (unsigned)((((bg >> 1) * 9 + t) * BK + (bg & 1) * 32) * 2);
    const unsigned dst = Bl_a + buf * kB2Wst;
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16(rsw, dst + (wave_u + 4 * q) * 1024, woff[q] + sb);
  };

  // fragment addresses: A fragment i = tile pixels 128 wm + 16 i + fr = image
  // row 2 wm + (i >> 2), column x = 16 (i & 3) + fr; tap (ty, tx) reads band row
  // 2 wm + (i >> 2) + ty + 1, column x + tx (a base past the LDS allocation,
  // which reads as zeros, where x + tx leaves the image)
  const int fr = lane & 15, kq = lane >> 4;
  constexpr int kLdsZero = 0x100000;
  // column x = 16 c4 + fr + tx: bit 2 of x (the slot swizzle) does not depend on
  // c4, so a tap's base is one per-lane value plus c4 * 1024; only (c4 = 0, tx =
  // -1, fr = 0) and (c4 = 3, tx = 1, fr = 15) leave the image
  int abase[3];
#pragma unroll
  for (int tx = -1; tx <= 1; ++tx) abase[tx + 1] = (fr + tx) * 64 + (b2_slot(fr + tx + 16, kq) << 4);
  const int aedge_l = fr == 0 ? kLdsZero : abase[0];
  const int aedge_r = fr == 15 ? kLdsZero : abase[2] + 3 * 1024;
  auto aoff = [&](int c4, int tx) {
    return (c4 == 0 && tx < 0) ? aedge_l : (c4 == 3 && tx > 0) ? aedge_r : abase[tx + 1] + c4 * 1024;
  };
  const int bbase = (wn * 64 + fr) * 64 + (b2_slot(fr, kq) << 4);

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nb = 2 * a.cpt;
  const int nst = 9 * nb;
  issue_band(0);
  issue_w(0, 0);
  issue_w(1, 1);
  int s = 0, wbuf = 0;
  for (int bg = 0; bg < nb; ++bg) {
    const char* Hb = Hl + (bg & 1) * kB2Band + wm * 2 * 4096;
    half8 a16[REUSE ? 16 : 1];   // REUSE: band rows 2 wm .. + 3 x 4 column groups of this tap column
#pragma unroll
    for (int t = 0; t < 9; ++t, ++s) {
      // t = step within the half chunk; tap = tap_of(t)
      const int tap = tap_of(t);
      const int ty = tap / 3 - 1, tx = tap % 3 - 1;
      // this wave's DMAs issued after W(s): W(s+1) (2, one stage ago) and the
      // bands issued at stages s-1 / s-2 (6 each, at the first stage of a group)
      const int nafter = (s + 1 < nst ? 2 : 0) + ((t == 1 && bg + 1 < nb) ? 6 : 0) + ((t == 2 && bg + 1 < nb) ? 6 : 0);
      wait_vmcnt(nafter);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (s + 2 < nst) issue_w(s + 2, wbuf == 0 ? 2 : wbuf - 1);
      if (t == 0 && bg + 1 < nb) issue_band(bg + 1);
      const char* Bb = Bl + wbuf * kB2Wst + bbase;
      half8 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const half8*>(Bb + j * 1024);
      if constexpr (REUSE) {
        if (t % 3 == 0) {   // a new tap column: its 16 A fragments
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4)
              a16[r * 4 + c4] = *reinterpret_cast<const half8*>(Hb + r * 4096 + aoff(c4, tx));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const half8 af = a16[((i >> 2) + ty + 1) * 4 + (i & 3)];
            acc[i][j] = kB2Swap ? __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af, acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
          }
      } else {
        const char* Ab = Hb + (ty + 1) * 4096;
        half8 af[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const half8*>(Ab + aoff(i & 3, tx) + (i >> 2) * 4096);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = kB2Swap ? __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      wbuf = wbuf == 2 ? 0 : wbuf + 1;
    }
  }
  band_epilogue<kB2TM, kB2TN, 8, 4, 2, true, 256, EPI, false, kB2Swap>(a, acc, smem, m0, n0, wm, wn, lane, tid, bcol);
}

// Which convs take the two-workgroups-per-CU tile (profiles/r03/band2_r03bh.txt,
// band2_c2_r03bl.txt; round 4 with the tap-column A reuse, profiles/r04/
// gate_tiles_r04b.txt): the plain 128-channel-tile convs (EPI_ACT:
// corr_encoder[2], GraphAgg conv1 / conv2, the per-frame gate term) and the q
// gate always (C3: 128->128 1.57 vs 1.67 ms, q 4.08 vs 4.43); the z|r gates
// only on small grids - at C3 the two tiles tie (7.42 / 7.42 ms), and on the
// frontend window (C2, 96 edges: 1152 z|r tiles = 4.5 rounds of the 8-wave tile
// over 256 CUs) the finer tiles fill the last round: update() 1.252 vs 1.308 ms.
// DROID_CONV_BAND2=0 / 1: none / every shape it takes (A/B runs), read at load;
// droid_conv_set_tile changes it per call (tests compare both tiles in one process).
static int& band2_mode() {
  static int mode = ab_knob("DROID_CONV_BAND2", -1);
  return mode;
}
static bool band2_for(int epi, long px) {
  const int mode = band2_mode();
  return mode == 1 || ((mode < 0 || mode == 2) && (epi == EPI_ACT || epi == EPI_GRU_Q || px / 256 <= 8L * device_cu_count()));
}
// a band-eligible 3x3 conv of this shape runs on the two-workgroup tile
static bool band2_shape(int epi, int B, int H, int W, int Cout, int gru_ch) {
  return band2_for(epi, (long)B * H * W) && W == 64 && H % 4 == 0 && Cout % kB2TN == 0 &&
         (epi != EPI_GRU_ZR || gru_ch % kB2TN == 0);
}

template <int EPI>
static int launch_band2_kernel(const ConvArgs& a0, hipStream_t stream) {
  ConvArgs a = a0;
  a.n_tiles = a.Cout / kB2TN;
  a.m_tiles = (long)a.B * a.H * a.W / kB2TM;
  const long nwg = a.m_tiles * a.n_tiles;
  if (nwg > 0x7fffffffL) return fail(kUnsupported, "conv band2: problem too large");
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_band2_kernel<EPI>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
    attr = true;
  }
  conv_band2_kernel<EPI><<<dim3((unsigned)nwg), 256, kB2Lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

#if DROID_AB
#include "ab/conv_wino_ab.inc"
#endif

// ---------------------------------------------------------------------------
// ConvGRU global context (modules/gru.py:19-32, the glo branch):
//   glo[e][co] = mean over the edge's pixels of sigmoid(w . h + b)[co] * h[co]
// for a 1x1 128 -> 128 conv w on the hidden state h itself.  One workgroup per
// edge streams its pixels in 64-pixel tiles by LDS-DMA through a ring of tile
// buffers (kGloRingProd = 3: two tiles in flight per workgroup, three
// workgroups per CU - round 5; the round-4 ring of 5 held four in flight with
// two workgroups per CU); wave w keeps the weight fragments of its output
// columns 32w .. 32w+31 in registers (32 VGPRs), so the LDS holds only the ring.
// The per-column sums stay in registers and the mean is a plain store - no
// atomics, deterministic.
// DROID_GLO_NT (A/B builds): the hidden-state stream by non-temporal LDS-DMA
#ifndef DROID_GLO_NT
#define DROID_GLO_NT 0
#endif
constexpr int kGloTP = 64;
// the tile ring: kGloRing buffers of 16 KB (kGloRingProd below)
constexpr int glo_lds(int ring) { return ring * 2 * kGloTP * 128; }

// split: blockIdx.y of gridDim.y pixel ranges of the edge (whole 64-pixel tiles);
// range y writes its share of the mean to glo + y * E * 128 (the caller adds
// the ranges in order; one range = the plain mean)
// PK (the product, kGloPkProd): sigmoid(y + b) * h on packed fp32 (v_pk_fma_f32
// / v_pk_add_f32, two values per instruction; the exp argument as one fma of y
// with the scaled bias) - the kernel is VALU-bound on this (2 transcendentals
// per value); 0.3835 vs 0.4249 ms at C3 for the scalar form, which the A/B
// build keeps (droid_glo_set_pk; profiles/r05/r05pk_glo_pk_ab.txt)
template <int kGloRing, bool PK>
__global__ void __launch_bounds__(256) gru_glo_kernel(const __half* __restrict__ h, const __half* __restrict__ w,
                                                      const float* __restrict__ bias, float* __restrict__ glo,
                                                      int HW) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem_glo[];
  char* lds = reinterpret_cast<char*>(smem_glo);
  char* Al = lds;                     // [kGloRing buf][2 k-chunks][64 px][128 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e = blockIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntot = HW / kGloTP, S = gridDim.y, sp = blockIdx.y;
  const int tbeg = (int)((long)ntot * sp / S), ntile = (int)((long)ntot * (sp + 1) / S) - tbeg;
  // this wave's weight fragments (B operand of K-step ks, column block j)
  half8 wf[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = wave * 32 + j * 16 + fr, k = (ks >> 1) * 64 + ((ks & 1) * 4 + fq) * 8;
      wf[ks][j] = *reinterpret_cast<const half8*>(w + co * 128 + k);
    }
  const __half* he = h + ((long)e * HW + (long)tbeg * kGloTP) * 128;
  const rsrc_t rs = make_rsrc(he, (unsigned)(ntile * kGloTP * 256));
  const unsigned Al_a = lds_addr(Al);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  // DMA: 16 instructions of 8 pixel rows (one k-chunk) per tile, 4 per wave:
  // instruction q = wave + 4*i: chunk q & 1, pixels 8 (q >> 1) .. +8
  const int lrow = lane >> 3, lpiece = (lane & 7) ^ lrow;
  auto issue = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wave_u + 4 * i, c = q & 1, pr = (q >> 1) * 8;
      const unsigned off = (unsigned)(((t * kGloTP + pr + lrow) * 128 + c * 64 + lpiece * 8) * 2);
      if constexpr (DROID_GLO_NT) dma16_nt(rs, Al_a + (t % kGloRing) * 16384 + c * 8192 + pr * 128, off);
      else dma16(rs, Al_a + (t % kGloRing) * 16384 + c * 8192 + pr * 128, off);
    }
  };
  // the MFMA multiplies weights x pixels: lane (fr, fq) of block (i, j) holds
  // channels wave*32 + 16 j + 4 fq .. + 3 of pixel 16 i + fr, so its h values
  // are one 8-B LDS read and its column sums 4 per j
  floatx4 bj[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bj[j] = *reinterpret_cast<const floatx4*>(bias + wave * 32 + j * 16 + fq * 4);
  floatx4 colsum[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  typedef float f2_t __attribute__((ext_vector_type(2)));
  f2_t nb[2][2], cs2[2][2];   // PK: -log2(e) b and the column sums, in pairs
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      nb[j][k] = f2_t{bj[j][2 * k], bj[j][2 * k + 1]} * f2_t{-1.4426950408889634f, -1.4426950408889634f};
      cs2[j][k] = f2_t{0.f, 0.f};
    }
  // the weight and bias loads land before the ring starts (the counted vmcnt
  // waits below assume only DMAs are outstanding)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int t = 0; t < kGloRing - 1 && t < ntile; ++t) issue(t);
  for (int t = 0; t < ntile; ++t) {
    // tile t landed: each later tile in flight is 4 DMA instructions of this wave
    const int later = min(kGloRing - 2, ntile - 1 - t);
    if (later >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (later == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // tile t landed (all waves); tile t-1's reads done
    if (t + kGloRing - 1 < ntile) issue(t + kGloRing - 1);  // into tile t-1's buffer
    const char* At = Al + (t % kGloRing) * 16384;
    floatx4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = ks >> 1, kq = (ks & 1) * 4 + fq;
      half8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 16 + fr;
        af[i] = *reinterpret_cast<const half8*>(At + c * 8192 + r * 128 + ((kq ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][j], af[i], acc[i][j], 0, 0, 0);
    }
    // sigmoid(. + b) * h summed over the tile's pixels (h = the tile itself: k == co)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = wave * 32 + j * 16 + fq * 4, c = co >> 6, kk = co & 63;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 16 + fr;
        const half4_t hv = *reinterpret_cast<const half4_t*>(
            At + c * 8192 + r * 128 + ((((kk >> 3) ^ (r & 7)) << 4) | ((kk & 7) << 1)));
        if constexpr (PK) {
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const f2_t tt = __builtin_elementwise_fma(
                f2_t{acc[i][j][2 * k], acc[i][j][2 * k + 1]},
                f2_t{-1.4426950408889634f, -1.4426950408889634f}, nb[j][k]);
            const f2_t den = f2_t{__builtin_amdgcn_exp2f(tt[0]), __builtin_amdgcn_exp2f(tt[1])} + f2_t{1.f, 1.f};
            const f2_t sg = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
            cs2[j][k] = __builtin_elementwise_fma(sg, f2_t{(float)hv[2 * k], (float)hv[2 * k + 1]}, cs2[j][k]);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)  // v_rcp_f32 sigmoid: no IEEE division
            colsum[j][k] += sigmoid_fast(acc[i][j][k] + bj[j][k]) * (float)hv[k];
        }
      }
    }
  }
  if constexpr (PK) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      colsum[j] = floatx4{cs2[j][0][0], cs2[j][0][1], cs2[j][1][0], cs2[j][1][1]};
  }
  // sum over the 16 pixel lanes (fr) of each channel quadruple
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = colsum[j][k];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      if (fr == 0) glo[((long)sp * gridDim.x + e) * 128 + wave * 32 + j * 16 + fq * 4 + k] = v / (float)HW;
    }
}

// ---------------------------------------------------------------------------
// flow_encoder[0] (droid_net.py:88-90: conv7x7 4 -> 128, ReLU) straight from the
// motion features motn (E,4,H,W) fp32 (the conv input cast to fp16 as under
// autocast).  Persistent: one 8-wave workgroup per CU keeps the packed weights
// (K = 52 taps x 8 channels, 4 real) in LDS and walks 128-pixel tiles; a tile's
// input band (its rows +-3, fp16, 8 channels per pixel with zero padding) is a
// few KB of LDS, built from registers loaded during the previous tile.  The
// band holds 4 channels per pixel (8 B), so the 8 K values of an A fragment are
// two horizontally adjacent taps x 4 channels - two neighbouring band pixels,
// one 16-B LDS piece: a K-step of 32 is one kernel row (4 tap pairs, the
// eighth tap of the row has zero weights) and the 7x7 conv takes 7 K-steps,
// not the 13 of the 8-channel packing (half of whose K was zero padding).
// The weights keep the ABI layout w[co][tap*8 + c] (K = 52 x 8) and are
// re-packed to [co][7 rows x 4 pairs x 8] while staged into LDS.
// Round 4: TP = 256-pixel tiles on 16 waves where the shape allows (C3's 48x64:
// twice the bytes in flight per CU and four waves per SIMD to cover the
// tile's barriers; the 128-pixel, 8-wave tile measured 2.6 TB/s of output).
constexpr int kFeK = 416, kFeK2 = 224, kFeKS = kFeK2 + 8, kFeOS = 136;

__host__ __device__ constexpr int fe_lds_bytes(int W, int TP) {
  return 128 * kFeKS * 2 + (TP / W + 6) * (W + 8) * 8 + TP * kFeOS * 2;
}

template <int TP>
__global__ void __launch_bounds__(4 * TP) flow_enc0_kernel(const float* __restrict__ motn, const __half* __restrict__ w,
                                                        const float* __restrict__ bias, __half* __restrict__ out,
                                                        int H, int W, long ntiles) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem_fe[];
  // band rows; padded row length: 3 columns left, 5 right (the pair (6, 7) of
  // a row reads column x + 7, whose weights are zero)
  constexpr int NT = 4 * TP;
  const int RB = TP / W + 6, PW = W + 8;
  _Float16* Ws = smem_fe;                    // [128][kFeKS]: [row 7][pair 4][tap 2][ch 4]
  _Float16* In = Ws + 128 * kFeKS;           // [RB][PW][4]
  _Float16* Os = In + RB * PW * 4;           // [128][kFeOS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int HW = H * W, tpe = HW / TP;
  for (int idx = tid; idx < 128 * 28 * 2; idx += NT) {  // (co, row, pair, tap of the pair)
    const int co = idx / 56, q = idx - co * 56, kb = q >> 1, h2 = q & 1;
    const int ty = kb >> 2, tx = 2 * (kb & 3) + h2;
    const uint2 v = tx < 7 ? *reinterpret_cast<const uint2*>(w + co * kFeK + (ty * 7 + tx) * 8) : make_uint2(0, 0);
    *reinterpret_cast<uint2*>(&Ws[co * kFeKS + kb * 8 + h2 * 4]) = v;
  }
  for (int idx = tid; idx < RB * PW; idx += NT)
    *reinterpret_cast<uint2*>(&In[idx * 4]) = make_uint2(0, 0);  // padding columns stay zero
  // input staging: thread -> band pixel (row idx / W, column idx % W), several per thread
  const int nin = (RB * W + NT - 1) / NT;  // <= 2 for W <= 128
  float v[2][4];
  auto load_in = [&](long t) {
    const long e = t / tpe;
    const int y0 = (int)(t - e * tpe) * (TP / W);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + NT * u;
      const int ry = idx / W, x = idx - ry * W, y = y0 - 3 + ry;
      const bool ok = u < nin && ry < RB && t < ntiles && y >= 0 && y < H;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = ok ? motn[(e * 4 + c) * HW + (long)y * W + x] : 0.f;
    }
  };
  auto store_in = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + NT * u;
      const int ry = idx / W, x = idx - ry * W;
      if (u < nin && ry < RB) {
        half4_t h;
#pragma unroll
        for (int c = 0; c < 4; ++c) h[c] = (_Float16)v[u][c];
        *reinterpret_cast<half4_t*>(&In[(ry * PW + x + 3) * 4]) = h;
      }
    }
  };
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fq = lane >> 4;
  // weights x pixels: lane (fr, fq) of block (f, j) holds channels
  // wn*64 + 16 j + 4 fq .. + 3 of pixel wm*32 + 16 f + fr (one 8-B LDS write)
  floatx4 bj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bj[j] = *reinterpret_cast<const floatx4*>(bias + wn * 64 + j * 16 + fq * 4);
  int pyx[2];  // band slot of the lane's pixel in fragment f, at tap (-3,-3)
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int p = wm * 32 + f * 16 + fr;
    pyx[f] = (p / W) * PW + (p % W);
  }
  long t = blockIdx.x;
  load_in(t);
  __syncthreads();
  for (; t < ntiles; t += gridDim.x) {
    store_in();
    __syncthreads();
    load_in(t + gridDim.x);
    floatx4 acc[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[f][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < kFeK2 / 32; ++ks) {  // K-step = kernel row ks, lane group fq = tap pair
      half8 af[2], bf[4];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        // band pixels (x + 2 fq, x + 2 fq + 1) of row ks: 16 B at an 8-B boundary
        const uint2* src = reinterpret_cast<const uint2*>(&In[(pyx[f] + ks * PW + 2 * fq) * 4]);
        const uint2 lo = src[0], hi = src[1];
        af[f] = __builtin_bit_cast(half8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const half8*>(&Ws[(wn * 64 + j * 16 + fr) * kFeKS + ks * 32 + fq * 8]);
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[f], acc[f][j], 0, 0, 0);
    }
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        half4_t o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = (_Float16)fmaxf(acc[f][j][k] + bj[j][k], 0.f);
        *reinterpret_cast<half4_t*>(&Os[(wm * 32 + f * 16 + fr) * kFeOS + wn * 64 + j * 16 + fq * 4]) = o;
      }
    __syncthreads();
    const long e = t / tpe;
    const long pix0 = e * HW + (t - e * tpe) * TP;
    for (int idx = tid; idx < TP * 16; idx += NT) {
      const int r = idx >> 4, q = idx & 15;
      const uint4 ov = *reinterpret_cast<const uint4*>(&Os[r * kFeOS + q * 8]);
      if constexpr (DROID_EPI_NT) __builtin_nontemporal_store(__builtin_bit_cast(u32x4nt, ov), reinterpret_cast<u32x4nt*>(out + (pix0 + r) * 128 + q * 8));
      else *reinterpret_cast<uint4*>(out + (pix0 + r) * 128 + q * 8) = ov;
    }
  }
}

// Round 5: the same conv with the weights resident in VGPRs - the product's
// 256-pixel tile (flow_enc0_kernel<256>, above, stays in the A/B build as
// droid_fe_set_variant(0)).  There every one of the 16 waves re-reads its half
// of the weights (64 channels x K 224, 28 KB) from LDS for every tile, ~700 KB
// of LDS reads per 256-pixel tile with the A fragments for 896 MFMAs.  Here 8
// waves, wave (wm, wn) = 128 pixels x 32 channels (WN = 4), hold their 14 B
// fragments (56 VGPRs, loaded once per workgroup straight from the ABI
// layout), so a tile's LDS traffic is the A fragments and the output staging.
// C3: 0.440-0.444 vs 0.490-0.498 ms (profiles/r05/r05ac_fe_ab.txt); WN = 2
// (64 x 64 per wave, half the A reads) needs 254 VGPRs and measured 0.484.  The
// K order, the operands and the epilogue are those of flow_enc0_kernel: the
// outputs are bitwise the same (test_flow_encoder0_resident_weights_bitwise).
template <int TP, int WN>
__global__ void __launch_bounds__(512) flow_enc0_rw_kernel(const float* __restrict__ motn,
                                                           const __half* __restrict__ w,
                                                           const float* __restrict__ bias, __half* __restrict__ out,
                                                           int H, int W, long ntiles) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem_fe[];
  // WN channel waves x WM pixel waves: wave (wm, wn) = TP / WM pixels (FP fragments) x 128 / WN channels (NJ)
  constexpr int NT = 512, WM = 8 / WN, FP = TP / (16 * WM), NJ = 128 / (16 * WN), CW = 128 / WN;
  static_assert(WM * WN == 8 && FP * 16 * WM == TP && NJ >= 1, "flow_enc0_rw: wave grid");
  const int RB = TP / W + 6, PW = W + 8;
  _Float16* In = smem_fe;                    // [RB][PW][4]
  _Float16* Os = In + RB * PW * 4;           // [TP][kFeOS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int HW = H * W, tpe = HW / TP;
  const int wm = wave / WN, wn = wave % WN, fr = lane & 15, fq = lane >> 4;
  // B fragment (ks, j): channel wn*64 + 16 j + fr, kernel row ks, taps 2 fq and
  // 2 fq + 1 (4 channels each; the row's eighth tap is zero)
  half8 wf[7][NJ];
#pragma unroll
  for (int ks = 0; ks < 7; ++ks)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const __half* wr = w + (wn * CW + j * 16 + fr) * kFeK + (ks * 7 + 2 * fq) * 8;
      const uint2 lo = *reinterpret_cast<const uint2*>(wr);
      const uint2 hi = fq < 3 ? *reinterpret_cast<const uint2*>(wr + 8) : make_uint2(0, 0);
      wf[ks][j] = __builtin_bit_cast(half8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
  for (int idx = tid; idx < RB * PW; idx += NT)
    *reinterpret_cast<uint2*>(&In[idx * 4]) = make_uint2(0, 0);  // padding columns stay zero
  const int nin = (RB * W + NT - 1) / NT;  // <= 2 for TP = 256, W <= 128
  float v[2][4];
  auto load_in = [&](long t) {
    const long e = t / tpe;
    const int y0 = (int)(t - e * tpe) * (TP / W);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + NT * u;
      const int ry = idx / W, x = idx - ry * W, y = y0 - 3 + ry;
      const bool ok = u < nin && ry < RB && t < ntiles && y >= 0 && y < H;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = ok ? motn[(e * 4 + c) * HW + (long)y * W + x] : 0.f;
    }
  };
  auto store_in = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + NT * u;
      const int ry = idx / W, x = idx - ry * W;
      if (u < nin && ry < RB) {
        half4_t h;
#pragma unroll
        for (int c = 0; c < 4; ++c) h[c] = (_Float16)v[u][c];
        *reinterpret_cast<half4_t*>(&In[(ry * PW + x + 3) * 4]) = h;
      }
    }
  };
  floatx4 bj[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bj[j] = *reinterpret_cast<const floatx4*>(bias + wn * CW + j * 16 + fq * 4);
  int pyx[FP];  // band slot of the lane's pixel in fragment f, at tap (-3,-3)
#pragma unroll
  for (int f = 0; f < FP; ++f) {
    const int p = wm * 16 * FP + f * 16 + fr;
    pyx[f] = (p / W) * PW + (p % W);
  }
  long t = blockIdx.x;
  load_in(t);
  __syncthreads();
  for (; t < ntiles; t += gridDim.x) {
    store_in();
    __syncthreads();
    load_in(t + gridDim.x);
    floatx4 acc[FP][NJ];
#pragma unroll
    for (int f = 0; f < FP; ++f)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[f][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) {
      half8 af[FP];
#pragma unroll
      for (int f = 0; f < FP; ++f) {
        const uint2* src = reinterpret_cast<const uint2*>(&In[(pyx[f] + ks * PW + 2 * fq) * 4]);
        const uint2 lo = src[0], hi = src[1];
        af[f] = __builtin_bit_cast(half8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
#pragma unroll
      for (int f = 0; f < FP; ++f)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[ks][j], af[f], acc[f][j], 0, 0, 0);
      // one kernel row's A fragments live at a time (hoisting all seven rows'
      // loads ahead of the MFMAs spilled the resident weights)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int f = 0; f < FP; ++f)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        half4_t o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = (_Float16)fmaxf(acc[f][j][k] + bj[j][k], 0.f);
        *reinterpret_cast<half4_t*>(&Os[(wm * 16 * FP + f * 16 + fr) * kFeOS + wn * CW + j * 16 + fq * 4]) = o;
      }
    __syncthreads();
    const long e = t / tpe;
    const long pix0 = e * HW + (t - e * tpe) * TP;
    for (int idx = tid; idx < TP * 16; idx += NT) {
      const int r = idx >> 4, q = idx & 15;
      const uint4 ov = *reinterpret_cast<const uint4*>(&Os[r * kFeOS + q * 8]);
      *reinterpret_cast<uint4*>(out + (pix0 + r) * 128 + q * 8) = ov;
    }
  }
}

constexpr int kFeRwWN = 4;   // channel waves of flow_enc0_rw_kernel (2: 254 VGPRs and slower)
__host__ __device__ constexpr int fe_rw_lds_bytes(int W, int TP) {
  return (TP / W + 6) * (W + 8) * 8 + TP * kFeOS * 2;
}
template <int WN>
static int launch_fe_rw(const float* motn, const void* w, const float* bias, void* out, int H, int W, long ntiles,
                         long grid, hipStream_t stream) {
  static bool attr = false;  // one per instantiation
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&flow_enc0_rw_kernel<256, WN>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    attr = true;
  }
  flow_enc0_rw_kernel<256, WN><<<dim3((unsigned)grid), 512, fe_rw_lds_bytes(W, 256), stream>>>(
      motn, (const __half*)w, bias, (__half*)out, H, W, ntiles);
  return kOk;
}

// GraphAgg's eta head (droid_net.py:48-50: a 3x3 conv 128 -> 1 on the
// aggregated map; the conv_nhwc_f16 entry with Cout == 1 at W == 64).  The
// generic 128 x 16 tile spends 18 barrier-separated K stages on one output
// channel (0.17 ms per update at C3, latency-bound).  Here the conv is the 1x1
// projection onto the nine taps, Y(q, t) = w_t . x(q) (MFMA, K = 128, N = 16 with
// taps 9..15 zero), over the band of rows y0 - 1 .. y0 + R of one frame, loaded
// straight from global memory into the A fragments; then each output pixel
// sums its nine shifted taps from LDS (zero outside the image) and adds the
// bias.  One pass over the input (+2/R for the halo rows), fp32 sums, one fp16
// rounding - as the generic tile, in another order.
constexpr int kEtaR = 4, kEtaYS = 17;
__global__ void __launch_bounds__(256) eta_conv_kernel(const __half* __restrict__ x, int cstride,
                                                       const __half* __restrict__ wp, const float* __restrict__ bias,
                                                       __half* __restrict__ out, int out_cstride, int out_coff, int H) {
  constexpr int W = 64, NF = (kEtaR + 2) * W / 16;   // band fragments of 16 pixels (24)
  __shared__ float Ys[(kEtaR + 2) * W * kEtaYS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int bands = H / kEtaR;
  const int b = blockIdx.x / bands, y0 = (blockIdx.x - b * bands) * kEtaR;
  // B fragment s: tap fr (zero past 8) x channels 32 s + 8 fq .. + 7 (packed
  // weights: [chunk][tap][64], pack_conv)
  half8 wf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    wf[s] = fr < 9 ? *reinterpret_cast<const half8*>(wp + ((s >> 1) * 9 + fr) * 64 + (s & 1) * 32 + 8 * fq)
                   : half8{};
#pragma unroll
  for (int i = 0; i < NF / 4; ++i) {
    const int fgi = wave + 4 * i;
    const int bp = fgi * 16 + fr;               // band pixel of the lane's A row
    const int y = y0 - 1 + bp / W;
    const bool ok = y >= 0 && y < H;
    const __half* src = x + ((long)(b * H + (ok ? y : 0)) * W + (bp % W)) * cstride + 8 * fq;
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half8 af = ok ? *reinterpret_cast<const half8*>(src + 32 * s) : half8{};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, wf[s], acc, 0, 0, 0);
    }
    // D: column fr = tap, rows 4 fq .. + 3 = the fragment's pixels
    if (fr < 9) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Ys[(fgi * 16 + 4 * fq + k) * kEtaYS + fr] = acc[k];
    }
  }
  __syncthreads();
  const int r = tid / W, xx = tid - r * W;     // output pixel (row y0 + r)
  float sum = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int xs = xx + dx;
      if (xs >= 0 && xs < W) sum += Ys[((r + 1 + dy) * W + xs) * kEtaYS + (dy + 1) * 3 + dx + 1];
    }
  if (bias) sum += bias[0];
  out[((long)(b * H + y0 + r) * W + xx) * out_cstride + out_coff] = (__half)sum;
}

// The delta / weight heads' finish (droid_net.py:128-132 + factor_graph.py:
// 209-211) in one pass over the fused head output: head (E,HW,4) f32 = the raw
// 3x3 head sums [du, dv, wu, wv] (droid_conv_dw_head_f16), b [4]:
//   target (E,HW,2) = base + (head[0:2] + b[0:2])     (coords1 + delta)
//   weight (E,HW,2) = sigmoid(head[2:4] + b[2:4])
// and, when target_ba is given, the same two maps in the BA's (rows,2,HW)
// layout at row row0 + e (the bundle adjustment's input, so no transposing
// copies and no concatenation with the stored inactive edges per update).
__global__ void __launch_bounds__(256) head_finish_kernel(const float4* __restrict__ head, const float* __restrict__ b,
                                                          const float2* __restrict__ base, float2* __restrict__ target,
                                                          float2* __restrict__ weight, float* __restrict__ target_ba,
                                                          float* __restrict__ weight_ba, int row0, long n, int HW) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float4 h = head[i];
  float du = h.x + b[0], dv = h.y + b[1];
  const float wu = 1.0f / (1.0f + expf(-(h.z + b[2]))), wv = 1.0f / (1.0f + expf(-(h.w + b[3])));
  if (base) {
    const float2 c = base[i];
    du = c.x + du;
    dv = c.y + dv;
  }
  target[i] = make_float2(du, dv);
  weight[i] = make_float2(wu, wv);
  if (target_ba) {
    const long e = i / HW, p = i - e * HW;
    const long o = ((long)(row0 + e) * 2) * HW + p;
    target_ba[o] = du;
    target_ba[o + HW] = dv;
    weight_ba[o] = wu;
    weight_ba[o + HW] = wv;
  }
}

// GraphAgg's damping (droid_net.py:73: eta = 0.01 softplus(eta conv), factor_graph.py:
// 211 / 221): for the BA's frames frames[k] (k < nba), map[k] = the frame's row of
// er (U,HW) fp16 (the raw eta conv output) or -1 (a frame only the stored
// inactive edges touch): state[frame] = 0.01 softplus(er[map]) where map >= 0,
// and out[k] = 0.2 state[frame] + ep (the BA's eta) - fp32, each op rounded as
// the torch ops it replaces (softplus: log1p(exp(x)), x itself above 20).
__global__ void __launch_bounds__(256) eta_damping_kernel(const __half* __restrict__ er, const int* __restrict__ map,
                                                          const int* __restrict__ frames, float* __restrict__ state,
                                                          float* __restrict__ out, long n, int HW, float ep) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long k = i / HW, p = i - k * HW;
  const int f = frames[k], u = map[k];
  float v;
  if (u >= 0) {
    const float x = __half2float(er[(long)u * HW + p]);
    v = 0.01f * (x > 20.0f ? x : log1pf(expf(x)));
    state[(long)f * HW + p] = v;
  } else {
    v = state[(long)f * HW + p];
  }
  out[i] = 0.2f * v + ep;
}

}  // namespace droid

using namespace droid;

static int band_version() {
  static const int v = ab_knob("DROID_CONV_BAND", 1);
  return v;
}

static bool rows_enabled() {
  static const bool on = ab_knob("DROID_CONV_ROWS", 1) != 0;
  return on;
}

extern "C" {

// srcs/C/cstride: nsrc NHWC fp16 inputs concatenated along channels.
// wp: packed weights [Cout][nstage][64] fp16 (see droid_mi355x.fused.pack_conv):
//   nsrc == 1 && C == 8 && ks > 1: IM2COL8, nstage = ceil(ks*ks/8), stage = 8 taps x 8 channels;
//   otherwise CHUNKED, nstage = ks*ks * sum_s ceil(C_s/64), stage = (source, 64-ch chunk, tap).
// epi: 0 act (act 0 none / 1 relu) -> out fp16 NHWC slice; 1 GRU z|r; 2 GRU q;
// 3 head (fp32 out32, sigmoid on co >= 2); 4 GRU global mean (atomic fp32 out32, zeroed by caller).
static long long* g_conv_prof = nullptr;

#if DROID_TESTING
// Timeline of the next band-kernel launches (debug/profiling): buf receives 6
// int64 per workgroup (hardware id, s_memtime at entry / loop start / loop end /
// epilogue stores issued / stores drained); null turns it off.  Only the profiling build (make prof ->
// lib/prof/libdroid_hip.so, -DDROID_CONV_PROFILE=1) writes them; the regular
// library reports DROID_UNSUPPORTED.  Not thread-safe by design.
int droid_conv_set_profile(void* buf) {
#if DROID_CONV_PROFILE
  g_conv_prof = static_cast<long long*>(buf);
  return droid::kOk;
#else
  (void)buf;
  return droid::fail(droid::kUnsupported, "conv_set_profile: build with make prof (DROID_CONV_PROFILE=1)");
#endif
}
#endif  // DROID_TESTING

static int conv_nhwc_impl(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                          const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                          int Cout, int ks, int act, int epi, void* out, int out_cstride, int out_coff,
                          const void* h, int h_cstride, const void* z, int z_cstride, void* zout,
                          void* rnet, int gru_ch, void* out32, const void* pre, const long long* pre_idx,
                          int pre_cstride, int pre_coff, hipStream_t stream, const void* wt = nullptr) {
  if (nsrc < 1 || nsrc > 4 || B < 0 || H <= 0 || W <= 0 || Cout <= 0 || ks < 1 || ks > 7 || !(ks & 1) ||
      epi < EPI_ACT || epi > EPI_GLO)
    return fail(kInvalidArgument, "conv_nhwc_f16: bad arguments");
  if ((long)B * H * W * 8 > 0x7fffffffL)
    return fail(kUnsupported, "conv_nhwc_f16: pixel count too large for 32-bit row indices");
  if (epi == EPI_GLO && (H * W) % TM != 0)
    return fail(kUnsupported, "conv_nhwc_f16: global-context epilogue needs H*W % 128 == 0");
  ConvArgs a{};
  a.prof = g_conv_prof;
  a.ab_no_h = ab_knob("DROID_ZR_NO_H", 0);
  int chunks = 0;
  for (int s = 0; s < nsrc; ++s) {
    if (C[s] % 8 || cstride[s] % 8 || cstride[s] < C[s] || (reinterpret_cast<uintptr_t>(srcs[s]) & 15))
      return fail(kInvalidArgument, "conv_nhwc_f16: channels/strides must be multiples of 8, 16-B aligned");
    a.src[s].ptr = (const __half*)srcs[s];
    a.src[s].C = C[s];
    a.src[s].cstride = cstride[s];
    chunks += ceil_div(C[s], BK);
    a.chunk_end[s] = chunks;
  }
  a.nsrc = nsrc;
  a.cpt = chunks;
  a.im2col = (nsrc == 1 && C[0] == 8 && ks > 1) ? 1 : 0;
  a.nstage = a.im2col ? ceil_div(ks * ks, 8) : ks * ks * chunks;
  a.wp = (const __half*)wp;
  a.bias = bias;
  a.bbias = bbias;
  a.B = B; a.H = H; a.W = W; a.Cout = Cout; a.ks = ks; a.act = act; a.epi = epi;
  a.out = (__half*)out; a.out_cstride = out_cstride; a.out_coff = out_coff;
  a.h = (const __half*)h; a.h_cstride = h_cstride;
  a.z = (const __half*)z; a.z_cstride = z_cstride;
  a.zout = (__half*)zout; a.rnet = (__half*)rnet; a.gru_ch = gru_ch;
  a.out32 = (float*)out32;
  a.pre = (const __half*)pre; a.pre_idx = pre_idx; a.pre_cstride = pre_cstride; a.pre_coff = pre_coff;
  const int TN = Cout >= 128 ? 128 : (Cout > 16 ? 64 : 16);
  a.stage_out = (Cout % 8 == 0 && out_cstride % 8 == 0 && out_coff % 8 == 0) ? 1 : 0;
  if (epi == EPI_ACT && !out) return fail(kInvalidArgument, "conv_nhwc_f16: out is null");
  if ((epi == EPI_GRU_ZR || epi == EPI_GRU_Q || epi == EPI_GLO) &&
      (!h || h_cstride % 8 || Cout % 8 || (reinterpret_cast<uintptr_t>(h) & 15)))
    return fail(kInvalidArgument, "conv_nhwc_f16: GRU epilogues need h with 16-B aligned rows");
  if (epi == EPI_GRU_ZR && (gru_ch % TN || Cout != 2 * gru_ch || !zout || !rnet))
    return fail(kInvalidArgument, "conv_nhwc_f16: z|r epilogue needs Cout == 2*gru_ch, gru_ch % tile == 0");
  if (epi == EPI_GRU_Q && (!z || z_cstride % 8 || !out || !a.stage_out || (reinterpret_cast<uintptr_t>(z) & 15)))
    return fail(kInvalidArgument, "conv_nhwc_f16: q epilogue needs z and a 16-B aligned out");
  if ((epi == EPI_HEAD || epi == EPI_GLO) && !out32)
    return fail(kInvalidArgument, "conv_nhwc_f16: out32 is null");
  if (a.stage_out && out && (reinterpret_cast<uintptr_t>(out) & 15)) a.stage_out = 0;
  if (B == 0) return kOk;
  // the one-output-channel 3x3 conv (GraphAgg's eta head) at W == 64
  if (!wt && ks == 3 && Cout == 1 && nsrc == 1 && C[0] == 128 && epi == EPI_ACT && act == 0 && !bbias && W == 64 &&
      H % kEtaR == 0 && (cstride[0] % 8) == 0) {
    const long nwg = (long)B * (H / kEtaR);
    if (nwg > 0x7fffffffL) return fail(kUnsupported, "conv_nhwc_f16: problem too large");
    eta_conv_kernel<<<dim3((unsigned)nwg), 256, 0, stream>>>((const __half*)srcs[0], cstride[0], (const __half*)wp,
                                                            bias, (__half*)out, out_cstride, out_coff, H);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  // 3x3 (and larger) convs over wide-enough outputs take the LDS-halo kernel;
  // DROID_CONV_HALO=0 / 4 / 8 (default) selects none / 4-wave / 8-wave tiles;
  // DROID_CONV_ROWS=0 disables the row-band variant.
  static const int halo_nw = ab_knob("DROID_CONV_HALO", 8);
  const bool halo_ok = !a.im2col && ks > 1 && Cout % 128 == 0 && (ks >> 1) * (W + 1) <= kHaloMax &&
                       epi != EPI_GLO && epi != EPI_HEAD;
  // LDS-DMA band kernel (3x3, whole-row tiles); DROID_CONV_BAND=0 disables it
  const bool band_on = band_version() > 0;
  const bool band_ok = band_on && !a.im2col && ks == 3 && W % 16 == 0 && 64 % W == 0 &&
                       (epi == EPI_GRU_ZR || epi == EPI_GRU_Q || (epi == EPI_ACT && a.stage_out)) &&
                       (epi != EPI_GRU_ZR || gru_ch % 128 == 0);
  int ns_, nh_;
  if (wt) {  // Winograd tile (droid_conv_wino_f16): W == 64, whole 4-row tiles, 128-channel N tiles
#if !DROID_AB
    return fail(kUnsupported, "conv_wino_f16: the Winograd tile ships in the A/B build only (make ab)");
#else
    if (a.im2col || ks != 3 || W != 64 || H % 4 || Cout % kWinoTN ||
        !(epi == EPI_ACT ? a.stage_out != 0 : (pre && (epi == EPI_GRU_ZR || epi == EPI_GRU_Q))) ||
        (epi == EPI_GRU_ZR && gru_ch % kWinoTN))
      return fail(kUnsupported, "conv_wino_f16: needs a 3x3 conv, W == 64, H % 4 == 0, Cout % 128 == 0");
    a.wp = (const __half*)wt;
    a.nstage = 6 * chunks;
    a.n_tiles = Cout / kWinoTN;
    a.m_tiles = (long)B * H * W / kWinoTM;
    const long nwg = a.m_tiles * a.n_tiles;
    if (nwg > 0x7fffffffL || (long)4 * Cout * 64 * a.nstage > 0x7fffffffL)
      return fail(kUnsupported, "conv_wino_f16: problem too large");
    int st;
    if (epi == EPI_GRU_ZR) st = launch_wino_kernel<EPI_GRU_ZRP>(a, nwg, stream);
    else if (epi == EPI_GRU_Q) st = launch_wino_kernel<EPI_GRU_QP>(a, nwg, stream);
    else st = launch_wino_kernel<EPI_ACT>(a, nwg, stream);
    if (st != kOk) return st;
    DROID_LAUNCH_CHECK();
    return kOk;
#endif
  }
  // two-workgroups-per-CU tile: W == 64, 128-channel N tiles
  if (band_ok && band2_shape(epi, B, H, W, Cout, gru_ch)) {
    if (epi == EPI_GRU_ZR) return pre ? launch_band2_kernel<EPI_GRU_ZRP>(a, stream) : launch_band2_kernel<EPI_GRU_ZR>(a, stream);
    if (epi == EPI_GRU_Q) return pre ? launch_band2_kernel<EPI_GRU_QP>(a, stream) : launch_band2_kernel<EPI_GRU_Q>(a, stream);
    return launch_band2_kernel<EPI_ACT>(a, stream);
  }
  if (pre) {  // the per-source term exists on the band tiles only
    if (band_ok && epi == EPI_GRU_ZR && Cout == 256 && 256 % W == 0 && (H * W) % 256 == 0 && band_nw4() &&
        band_fits<256, 256, 4>(W, &ns_, &nh_))
      return launch_band_nw4<256, 256>(a, stream);
    if (band_ok && epi == EPI_GRU_ZR && Cout == 256 && 256 % W == 0 && (H * W) % 256 == 0 &&
        band_fits<256, 256>(W, &ns_, &nh_))
      return launch_band<256, 256>(a, stream);
    if (band_ok && epi == EPI_GRU_Q && Cout == 128 && 384 % W == 0 && (H * W) % 384 == 0 &&
        band_fits<384, 128>(W, &ns_, &nh_))
      return launch_band<384, 128>(a, stream);
    return fail(kUnsupported, "conv_gru_pre_f16: shape has no band tile");
  }
  if (band_ok && Cout % 256 == 0 && 256 % W == 0 && (H * W) % 256 == 0 && band_fits<256, 256>(W, &ns_, &nh_))
    return launch_band<256, 256>(a, stream);
  if (band_ok && Cout % 128 == 0 && 384 % W == 0 && (H * W) % 384 == 0 && band_fits<384, 128>(W, &ns_, &nh_))
    return launch_band<384, 128>(a, stream);
  if (band_ok && Cout == 64 && 384 % W == 0 && (H * W) % 384 == 0 && band_fits<384, 64>(W, &ns_, &nh_))
    return launch_band<384, 64>(a, stream);
  // row-band variant: tile = whole image rows, zero-padded halo, no masks
  const int pad = ks >> 1;
  const bool rows_ok = halo_ok && halo_nw == 8 && 256 % W == 0 && W % 16 == 0 && (H * W) % 256 == 0 &&
                       (256 / W + 2 * pad) * (W + 2 * pad) <= kRowsSlotsMax &&
                       (long)(256 / W + 2 * pad) * W * 256 * 2 < 0x7fffffffL && rows_enabled();
  if (rows_ok) return launch_rows<8>(a, stream);
  if (halo_ok && halo_nw == 8) return launch_halo<8>(a, stream);
  if (halo_ok && halo_nw == 4) return launch_halo<4>(a, stream);
  if (TN == 128) return launch_conv<128>(a, stream);
  if (TN == 64) return launch_conv<64>(a, stream);
  return launch_conv<16>(a, stream);
}

#if DROID_TESTING
// Tile policy of the W == 64 3x3 convs: -1 = default (plain convs and small
// gate-conv grids on the two-workgroups-per-CU tile, C3-sized gate convs on the
// 8-wave band tiles), 0 = 8-wave band tiles only, 1 = the two-workgroup tile
// wherever it applies, 2 (A/B build only) = the default with the factored z|r
// gates of the 8-wave-tile grids on the 4-wave 256x256 tile.  Returns the previous policy.
// Process-wide, not thread-safe by design (tests and A/B runs).
int droid_conv_set_tile(int mode) {
  if (mode < -1 || mode > (DROID_AB ? 2 : 1)) return -2;
  const int prev = band2_mode();
  band2_mode() = mode;
  return prev;
}
#endif  // DROID_TESTING

#if DROID_AB
// A/B build only (not in include/droid_backends.h): the 64-channel band tile's
// two-tap stages (1, the product's) or one-tap stages (0); returns the previous
int droid_conv_set_pair(int on) {
  const int prev = band_pair();
  band_pair() = on ? 1 : 0;
  return prev;
}
#endif

#if DROID_TESTING
// Which kernel droid_conv_gru_pre_f16 runs for a ConvGRU gate conv (epi 1: z|r,
// Cout 256; epi 2: q, Cout 128) over B images of H x W under the current tile
// policy: 1 = conv_band2_kernel, 0 = the 8-wave band tile (<256,256> for z|r,
// <384,128> for q), 2 = the 4-wave z|r tile (A/B build, DROID_CONV_NW4=1), -1 = no
// band tile for the shape.
int droid_conv_gate_tile(int epi, int B, int H, int W) {
  if ((epi != EPI_GRU_ZR && epi != EPI_GRU_Q) || B < 0 || H <= 0 || W <= 0) return -1;
  if (band_version() <= 0 || W % 16 || 64 % W) return -1;
  const int Cout = epi == EPI_GRU_ZR ? 256 : 128;
  if (band2_shape(epi, B, H, W, Cout, 128)) return 1;
  int ns_, nh_;
  if (epi == EPI_GRU_ZR && band_nw4() && (H * W) % 256 == 0 && band_fits<256, 256, 4>(W, &ns_, &nh_)) return 2;
  if (epi == EPI_GRU_ZR) return ((H * W) % 256 == 0 && band_fits<256, 256>(W, &ns_, &nh_)) ? 0 : -1;
  return ((H * W) % 384 == 0 && band_fits<384, 128>(W, &ns_, &nh_)) ? 0 : -1;
}
#endif  // DROID_TESTING

int droid_conv_nhwc_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                        const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                        int Cout, int ks, int act, int epi, void* out, int out_cstride, int out_coff,
                        const void* h, int h_cstride, const void* z, int z_cstride, void* zout,
                        void* rnet, int gru_ch, void* out32, hipStream_t stream) {
  return conv_nhwc_impl(srcs, C, cstride, nsrc, wp, bias, bbias, B, H, W, Cout, ks, act, epi, out, out_cstride,
                        out_coff, h, h_cstride, z, z_cstride, zout, rnet, gru_ch, out32, nullptr, nullptr, 0, 0,
                        stream);
}

// ConvGRU gates with the per-source-frame term factored out (EPI_GRU_ZRP /
// EPI_GRU_QP): the srcs conv excludes the context features inp, whose part of
// the gate argument, conv3x3(inp[frame]), is the same for every edge leaving
// that frame and arrives precomputed in pre (frames, H, W, pre_cstride) fp16;
// image b adds frame pre_idx[b] at channel offset pre_coff.
int droid_conv_gru_pre_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                           const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                           int Cout, int epi, void* out, int out_cstride, int out_coff, const void* h,
                           int h_cstride, const void* z, int z_cstride, void* zout, void* rnet, int gru_ch,
                           const void* pre, const long long* pre_idx, int pre_cstride, int pre_coff,
                           hipStream_t stream) {
  if ((epi != EPI_GRU_ZR && epi != EPI_GRU_Q) || !pre || !pre_idx || pre_cstride % 8 || pre_coff % 8 ||
      pre_coff + Cout > pre_cstride || (reinterpret_cast<uintptr_t>(pre) & 15))
    return fail(kInvalidArgument, "conv_gru_pre_f16: needs a z|r or q epilogue and a 16-B aligned pre map");
  return conv_nhwc_impl(srcs, C, cstride, nsrc, wp, bias, bbias, B, H, W, Cout, 3, 0, epi, out, out_cstride,
                        out_coff, h, h_cstride, z, z_cstride, zout, rnet, gru_ch, nullptr, pre, pre_idx,
                        pre_cstride, pre_coff, stream);
}

// 3x3 conv as Winograd F(2,3) along x (conv_wino_kernel): same operands as
// droid_conv_nhwc_f16 / droid_conv_gru_pre_f16 with the weights pre-transformed
// (wt: droid_mi355x.fused.pack_conv_wino); epi EPI_ACT (act 0 / 1) or, with a
// per-source-frame term pre (else null), EPI_GRU_ZR / EPI_GRU_Q.  W == 64,
// H % 4 == 0, Cout % 128 == 0; DROID_UNSUPPORTED otherwise (the caller then runs
// the direct conv).
int droid_conv_wino_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc, const void* wt,
                        const float* bias, const float* bbias, int B, int H, int W, int Cout, int act, int epi,
                        void* out, int out_cstride, int out_coff, const void* h, int h_cstride, const void* z,
                        int z_cstride, void* zout, void* rnet, int gru_ch, const void* pre,
                        const long long* pre_idx, int pre_cstride, int pre_coff, hipStream_t stream) {
  if (!wt || (epi != EPI_ACT && epi != EPI_GRU_ZR && epi != EPI_GRU_Q) ||
      (epi != EPI_ACT && (!pre || !pre_idx || pre_cstride % 8 || pre_coff % 8 || pre_coff + Cout > pre_cstride ||
                          (reinterpret_cast<uintptr_t>(pre) & 15))) ||
      (reinterpret_cast<uintptr_t>(wt) & 15))
    return fail(kInvalidArgument, "conv_wino_f16: bad arguments");
  return conv_nhwc_impl(srcs, C, cstride, nsrc, nullptr, bias, bbias, B, H, W, Cout, 3, act, epi, out, out_cstride,
                        out_coff, h, h_cstride, z, z_cstride, zout, rnet, gru_ch, nullptr,
                        epi == EPI_ACT ? nullptr : pre, epi == EPI_ACT ? nullptr : pre_idx, pre_cstride, pre_coff,
                        stream, wt);
}

// Fused delta/weight heads (EPI_DWHEAD): conv3x3 (srcs -> 256, bias, ReLU) feeding
// conv3x3 256 -> 4 (hw: [48][256] fp16, row tap*4 + c, rows 36..47 zero); raw head
// sums are atomically added into out32 (B,H,W,4) fp32, which the caller zeroes.
// Needs the band tile: Cout == 256, ks == 3, W in {16,32,64}, H*W % 256 == 0;
// returns kUnsupported otherwise (the caller then runs the two convs).
int droid_conv_dw_head_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc, const void* wp,
                           const float* bias, int B, int H, int W, const void* hw, void* out32,
                           hipStream_t stream) {
  if (nsrc < 1 || nsrc > 4 || B < 0 || H <= 0 || W <= 0 || !wp || !hw || !out32)
    return fail(kInvalidArgument, "conv_dw_head_f16: bad arguments");
  int ns_, nh_;
  if (W % 16 || 64 % W || (H * W) % 256 || !band_fits<256, 256>(W, &ns_, &nh_))
    return fail(kUnsupported, "conv_dw_head_f16: shape needs the band tile (W in {16,32,64}, H*W % 256 == 0)");
  if ((long)B * H * W * 8 > 0x7fffffffL) return fail(kUnsupported, "conv_dw_head_f16: too many pixels");
  ConvArgs a{};
  a.prof = g_conv_prof;
  a.ab_no_h = ab_knob("DROID_ZR_NO_H", 0);
  int chunks = 0;
  for (int s = 0; s < nsrc; ++s) {
    if (C[s] % 8 || cstride[s] % 8 || cstride[s] < C[s] || (reinterpret_cast<uintptr_t>(srcs[s]) & 15))
      return fail(kInvalidArgument, "conv_dw_head_f16: channels/strides must be multiples of 8, 16-B aligned");
    a.src[s].ptr = (const __half*)srcs[s];
    a.src[s].C = C[s];
    a.src[s].cstride = cstride[s];
    chunks += ceil_div(C[s], BK);
    a.chunk_end[s] = chunks;
  }
  a.nsrc = nsrc;
  a.cpt = chunks;
  a.nstage = 9 * chunks;
  a.wp = (const __half*)wp;
  a.bias = bias;
  a.B = B; a.H = H; a.W = W; a.Cout = 256; a.ks = 3; a.act = 1; a.epi = EPI_DWHEAD;
  a.hw = (const __half*)hw;
  a.out32 = (float*)out32;
  if (B == 0) return kOk;
  return launch_band<256, 256, true>(a, stream);
}

// ConvGRU global context (gru_glo_kernel): h (E, HW, 128) fp16, w [128][128]
// fp16 (the 1x1 conv weight, [co][ci]), bias [128] f32 -> glo (E, 128) f32.
__global__ void __launch_bounds__(384) glo_gates_kernel(const float* __restrict__ part, int splits,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float* __restrict__ out_zr, float* __restrict__ out_q, int E) {
  __shared__ float g[128];
  const int e = blockIdx.x, t = threadIdx.x;
  if (t < 128) {
    float s = 0.f;
    for (int r = 0; r < splits; ++r) s += part[((long)r * E + e) * 128 + t];
    g[t] = s;
  }
  __syncthreads();
  const float4* wr = reinterpret_cast<const float4*>(w + (long)t * 128);
  float acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < 32; ++k) {
    const float4 v = wr[k];
    acc = fmaf(g[4 * k], v.x, acc);
    acc = fmaf(g[4 * k + 1], v.y, acc);
    acc = fmaf(g[4 * k + 2], v.z, acc);
    acc = fmaf(g[4 * k + 3], v.w, acc);
  }
  // z | r terms and q terms as the two gate convs' per-image biases (contiguous rows)
  if (t < 256) out_zr[(long)e * 256 + t] = acc + b[t];
  else out_q[(long)e * 128 + t - 256] = acc + b[t];
}

// Tile ring of gru_glo_kernel: 3 buffers (48 KB, three workgroups per CU) in the
// product - 0.386 vs 0.426 ms for the round-4 ring of 5 (80 KB, two per CU) at
// C3, bitwise the same sums (profiles/r05/r05al_glo_ab*.txt); the A/B build
// keeps rings 5 and 2 (five per CU: 0.389 ms) behind droid_glo_set_ring.
constexpr int kGloRingProd = 3;
constexpr bool kGloPkProd = true;
#if DROID_AB
static int& glo_ring() {
  static int r = ab_knob("DROID_GLO_RING", kGloRingProd);
  return r;
}
int droid_glo_set_ring(int r) {
  const int prev = glo_ring();
  glo_ring() = (r == 2 || r == 3 || r == 5) ? r : kGloRingProd;
  return prev;
}
static int& glo_pk() {
  static int v = ab_knob("DROID_GLO_PK", kGloPkProd ? 1 : 0);
  return v;
}
// A/B: the packed-fp32 sigmoid sum of gru_glo_kernel (1, the product) or the
// scalar one (0, round 5 until its last commits)
int droid_glo_set_pk(int v) {
  const int prev = glo_pk();
  glo_pk() = v ? 1 : 0;
  return prev;
}
#endif
}  // extern "C"
template <int R, bool PK = kGloPkProd>
static int launch_glo_ring(dim3 grid, const void* h, const void* w, const float* bias, float* out, int HW,
                           hipStream_t stream) {
  static bool attr = false;  // one per instantiation
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&gru_glo_kernel<R, PK>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, glo_lds(R)));
    attr = true;
  }
  gru_glo_kernel<R, PK><<<grid, 256, glo_lds(R), stream>>>((const __half*)h, (const __half*)w, bias, out, HW);
  return kOk;
}
extern "C" {
static int launch_glo(dim3 grid, const void* h, const void* w, const float* bias, float* out, int HW,
                      hipStream_t stream) {
#if DROID_AB
  if (glo_pk() != (kGloPkProd ? 1 : 0)) {
    if (glo_ring() == 5) return launch_glo_ring<5, !kGloPkProd>(grid, h, w, bias, out, HW, stream);
    if (glo_ring() == 2) return launch_glo_ring<2, !kGloPkProd>(grid, h, w, bias, out, HW, stream);
    return launch_glo_ring<kGloRingProd, !kGloPkProd>(grid, h, w, bias, out, HW, stream);
  }
  if (glo_ring() == 5) return launch_glo_ring<5>(grid, h, w, bias, out, HW, stream);
  if (glo_ring() == 2) return launch_glo_ring<2>(grid, h, w, bias, out, HW, stream);
#endif
  return launch_glo_ring<kGloRingProd>(grid, h, w, bias, out, HW, stream);
}

int droid_gru_global_f16(const void* h, const void* w, const float* bias, float* glo, int E, int HW,
                         hipStream_t stream) {
  if (E < 0 || HW <= 0 || !h || !w || !bias || !glo) return fail(kInvalidArgument, "gru_global_f16: bad arguments");
  if (HW % kGloTP || (long)HW * 256 > 0x7fffffffL || (reinterpret_cast<uintptr_t>(h) & 15) ||
      (reinterpret_cast<uintptr_t>(w) & 15) || (reinterpret_cast<uintptr_t>(bias) & 15))
    return fail(kUnsupported, "gru_global_f16: needs H*W % 64 == 0 and 16-B aligned operands");
  if (E == 0) return kOk;
  { const int st = launch_glo(dim3(E, 1), h, w, bias, glo, HW, stream); if (st != kOk) return st; }
  DROID_LAUNCH_CHECK();
  return kOk;
}

// ... split into `splits` pixel ranges per edge (few edges: more workgroups than
// edges): part (splits, E, 128) f32, range y = its share of the mean; the caller
// sums the ranges in order (glo = part.sum(0)).
int droid_gru_global_split_f16(const void* h, const void* w, const float* bias, float* part, int splits, int E,
                               int HW, hipStream_t stream) {
  if (E < 0 || HW <= 0 || splits < 1 || !h || !w || !bias || !part)
    return fail(kInvalidArgument, "gru_global_split_f16: bad arguments");
  if (HW % kGloTP || splits > HW / kGloTP || (long)HW * 256 > 0x7fffffffL || (reinterpret_cast<uintptr_t>(h) & 15) ||
      (reinterpret_cast<uintptr_t>(w) & 15) || (reinterpret_cast<uintptr_t>(bias) & 15))
    return fail(kUnsupported, "gru_global_split_f16: needs H*W % 64 == 0, splits <= H*W/64, 16-B aligned operands");
  if (E == 0) return kOk;
  { const int st = launch_glo(dim3(E, splits), h, w, bias, part, HW, stream); if (st != kOk) return st; }
  DROID_LAUNCH_CHECK();
  return kOk;
}

// The GRU's global-context gate terms (gru.py:29-32, convz_glo | convr_glo |
// convq_glo on glo): out[e][o] = b[o] + sum_k glo[e][k] w[o][k], o < 384, with glo
// the in-order sum of the `splits` per-range partial means (gru_global_split).
// One workgroup per edge; a plain fp32 dot per output (no BLAS library call in
// the update path - it keeps update() capturable as one HIP graph).
int droid_head_finish_f32(const float* head, const float* b, const float* base, float* target, float* weight,
                          float* target_ba, float* weight_ba, int row0, int E, int HW, hipStream_t stream) {
  if (E < 0 || HW <= 0 || row0 < 0 || !head || !b || !target || !weight || (!target_ba != !weight_ba))
    return fail(kInvalidArgument, "head_finish_f32: bad arguments");
  const long n = (long)E * HW;
  if (n == 0) return kOk;
  droid::head_finish_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(
      reinterpret_cast<const float4*>(head), b, reinterpret_cast<const float2*>(base),
      reinterpret_cast<float2*>(target), reinterpret_cast<float2*>(weight), target_ba, weight_ba, row0, n, HW);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_eta_damping_f32(const void* er, const int* map, const int* frames, float* state, float* out, int nba,
                          int HW, float ep, hipStream_t stream) {
  if (nba < 0 || HW <= 0 || !er || !map || !frames || !state || !out)
    return fail(kInvalidArgument, "eta_damping_f32: bad arguments");
  const long n = (long)nba * HW;
  if (n == 0) return kOk;
  droid::eta_damping_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(
      static_cast<const __half*>(er), map, frames, state, out, n, HW, ep);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_glo_gates_f32(const float* part, int splits, const float* w, const float* b, float* out_zr, float* out_q,
                        int E, hipStream_t stream) {
  if (E < 0 || splits < 1 || !part || !w || !b || !out_zr || !out_q)
    return fail(kInvalidArgument, "glo_gates_f32: bad arguments");
  if (E == 0) return kOk;
  glo_gates_kernel<<<dim3(E), 384, 0, stream>>>(part, splits, w, b, out_zr, out_q, E);
  DROID_LAUNCH_CHECK();
  return kOk;
}

// flow_encoder[0] (flow_enc0_kernel): motn (E,4,H,W) f32, w [128][416] fp16
// (column t*8 + c = weight[co][c][t/7][t%7] for t < 49, c < 4; else zero), bias
// [128] f32 -> out (E,H,W,128) fp16 = relu(conv7x7(motn) + bias).
#if DROID_AB
// A/B build only: the 256-pixel flow_enc0 tile, 1 = flow_enc0_rw_kernel (the
// product's, weights in VGPRs), 0 = flow_enc0_kernel<256> (weights in LDS)
static int& fe_variant() {
  static int v = ab_knob("DROID_FE_VARIANT", 1);
  return v;
}
int droid_fe_set_variant(int v) {
  const int prev = fe_variant();
  fe_variant() = v ? 1 : 0;
  return prev;
}
#endif

int droid_flow_enc0_f16(const float* motn, const void* w, const float* bias, void* out, int E, int H, int W,
                        hipStream_t stream) {
  if (E < 0 || H <= 0 || W <= 0 || !motn || !w || !bias || !out || (reinterpret_cast<uintptr_t>(bias) & 15))
    return fail(kInvalidArgument, "flow_enc0_f16: bad arguments (bias must be 16-B aligned)");
  if (W % 16 || 128 % W || (H * W) % 128 || (long)E * H * W * 4 > 0x7fffffffL)
    return fail(kUnsupported, "flow_enc0_f16: needs W in {16,32,64,128} and H*W % 128 == 0");
  if (E == 0) return kOk;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&flow_enc0_kernel<128>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
#if DROID_AB
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&flow_enc0_kernel<256>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
#endif
    attr = true;
  }
  // DROID_FE_TP=128: the 128-pixel tile on a shape that allows 256 (A/B runs)
  static const int tp_env = ab_knob("DROID_FE_TP", 256);
  if (tp_env == 256 && (H * W) % 256 == 0 && fe_rw_lds_bytes(W, 256) <= kLdsMax) {
    const long ntiles = (long)E * H * W / 256;
    const long grid = std::min<long>(ntiles, device_cu_count());
#if DROID_AB
    if (fe_variant() == 0)   // the round-4 tile: 16 waves, weights in LDS
      flow_enc0_kernel<256><<<dim3((unsigned)grid), 1024, fe_lds_bytes(W, 256), stream>>>(
          motn, (const __half*)w, bias, (__half*)out, H, W, ntiles);
    else
#endif
      launch_fe_rw<kFeRwWN>(motn, w, bias, out, H, W, ntiles, grid, stream);
  } else {
    const long ntiles = (long)E * H * W / 128;
    const long grid = std::min<long>(ntiles, device_cu_count());
    flow_enc0_kernel<128><<<dim3((unsigned)grid), 512, fe_lds_bytes(W, 128), stream>>>(
        motn, (const __half*)w, bias, (__half*)out, H, W, ntiles);
  }
  DROID_LAUNCH_CHECK();
  return kOk;
}
}  // extern "C"

namespace droid {

// GraphAgg's scatter_mean over edges sharing a source frame (droid_net.py:
// 27-45): out[u] = mean_{e in segment u} src[e], rows of `row` fp16 values
// (H*W*C), fp32 accumulation.  One thread per 16-B piece of a row.
__global__ void __launch_bounds__(256) segment_mean_f16_kernel(const __half* __restrict__ src,
                                                               const int64_t* __restrict__ seg_ptr,
                                                               const int64_t* __restrict__ seg_idx,
                                                               __half* __restrict__ out, long row) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  const int u = blockIdx.y;
  if (q * 8 >= row) return;
  const long e0 = seg_ptr[u], e1 = seg_ptr[u + 1];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  long e = e0;
  // four rows in flight per thread; summed in edge order (same rounding)
  for (; e + 4 <= e1; e += 4) {
    half8 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __builtin_nontemporal_load(reinterpret_cast<const half8*>(src + seg_idx[e + i] * row + q * 8));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += (float)v[i][k];
  }
  for (; e < e1; ++e) {
    const half8 v = __builtin_nontemporal_load(reinterpret_cast<const half8*>(src + seg_idx[e] * row + q * 8));
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += (float)v[k];
  }
  const float inv = 1.0f / (float)max(e1 - e0, 1L);
  half8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = (_Float16)(acc[k] * inv);
  *reinterpret_cast<half8*>(out + (long)u * row + q * 8) = o;
}

}  // namespace droid

extern "C" int droid_segment_mean_f16(const void* src, const int64_t* seg_ptr, const int64_t* seg_idx,
                                      void* out, int num_segments, long row, hipStream_t stream) {
  if (num_segments < 0 || row <= 0 || row % 8 || (reinterpret_cast<uintptr_t>(src) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 15))
    return fail(kInvalidArgument, "segment_mean_f16: rows must be multiples of 8 halves, 16-B aligned");
  if (num_segments == 0) return kOk;
  const long pieces = row / 8;
  if ((pieces + 255) / 256 > 0x7fffffffL) return fail(kUnsupported, "segment_mean_f16: row too long");
  segment_mean_f16_kernel<<<dim3((unsigned)((pieces + 255) / 256), num_segments), 256, 0, stream>>>(
      (const __half*)src, seg_ptr, seg_idx, (__half*)out, row);
  DROID_LAUNCH_CHECK();
  return kOk;
}
