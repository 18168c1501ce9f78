// CorrBlock pyramid construction (modules/corr.py:24-38, 63-71) in one pass,
// gfx950.
//
// The reference builds, per edge, the all-pairs volume V0 = (f1/4)^T (f2/4)
// with an autocast fp16 GEMM (fp32 accumulation, fp16 result, HW x HW) and then
// three F.avg_pool2d(2) levels over the target dimensions, each from the
// previous level's fp16 values (float sum in (h, w) order / 4, rounded).  Every
// level is written to HBM and read back by the next; at 2048 edges that is
// 51 GB written + 70 GB re-read, plus the tile8 copy for the fused lookup.
//
// Here every level is written exactly once and never re-read by the build
// itself, in two launches (the design history - the round-3 one-pass kernel
// and two other variants, all writing the same bytes - is in ab/, built only
// by `make ab`):
//   * corr_volume_pyramid2_kernel: a workgroup owns 256 query pixels of one
//     edge and walks the target map in 8x8 patches (Z order); each patch's 64
//     target feature rows (16 KB) reach LDS by LDS-DMA one patch ahead; the
//     level-0 values are an MFMA GEMM (v_mfma_f32_16x16x32_f16, fp32
//     accumulation) with the patch's target rows as A, so a lane's four
//     accumulators are a 2x2 target window, rounded to fp16; level 1 is pooled
//     in the lane with the reference's arithmetic (the window's four fp16
//     values summed in float in (h, w) order, / 4, rounded) and, in the tiled
//     layout, held in registers until the 2x2 patch group completes one
//     level-1 tile; levels 0 and 1 leave as whole 128-B tiles (non-temporal
//     stores: the volume is read by a later kernel, never by this one);
//   * corr_volume_pool23_kernel: levels 2 and 3 pooled from the stored level 1
//     in storage order, one 128-B line per wave-instruction.
// Query features come from the frames' NHWC level-0 feature maps (the
// AltCorrBlock pyramid level 0, i.e. fmap / 4) indexed per edge, so no
// per-edge feature copy exists either.
#include "common.hpp"
#include "lds_dma.hpp"

#include <algorithm>
#include <type_traits>

#pragma clang fp contract(off)

namespace droid {

struct VolArgs {
  const __half* f;   // (NF, H, W, 128) fp16 = fmap / 4
  const int* f1;     // (E) query frame of each edge
  const int* f2;     // (E) target frame
  __half* lvl[4];    // outputs
  int H, W;          // query and target maps are H x W
  int tiled;         // 1: (E,H,W,ceil(H_l/8),W_l/8,8,8) 8x8 tiles; 0: (E,H,W,H_l,W_l)
  int qblocks;       // ceil(HW / 256)
  int ablate;        // timing experiments only (DROID_VOL_ABLATE, results invalid): bit 0 no stores, bit 1 no DMA after the first patch, (v2) bit 2 no level 1-3 stores, bit 3 no level-0 stores
};

constexpr int kVolQ = 256;                 // query pixels per workgroup
constexpr int kVolB = 0;                   // 2 x [64 target px][256 B] patch buffers
constexpr int kVolStage = 2 * 64 * 256;    // per wave: [32 q][64] V0 | [32][16] L1 | [32][4] L2 | [32] L3 fp16
constexpr int kVolStageWave = 32 * 64 * 2 + 32 * 16 * 2 + 32 * 4 * 2 + 32 * 2;
constexpr int kVolLds = kVolStage + 8 * kVolStageWave;

// target pixel of N-block b, column c inside an 8x8 patch at (ty0, tx0)
__device__ __forceinline__ int vol_ty(int b, int c) { return 4 * (b >> 1) + (c >> 2); }
__device__ __forceinline__ int vol_tx(int b, int c) { return 4 * (b & 1) + (c & 3); }

__device__ __forceinline__ float vol_pool4(float a, float b, float c, float d) {
  // F.avg_pool2d(2) on half: float accumulation over the window in (h, w) order, / 4, rounded
  float s = 0.0f;
  s += a;
  s += b;
  s += c;
  s += d;
  return rnd16(s / 4.0f);
}


// ---------------------------------------------------------------------------
// Round 4: corr_volume_pyramid2_kernel, the same pyramid with the MFMA operands
// swapped so that pooling is (mostly) register-local, and no store drain per
// patch.  Measured cost of the kernel above (34.4 ms at 2048 edges, 1.5 TB/s
// of writes): per patch and wave 192 cross-lane shuffles (ds_bpermute on the
// LDS pipe) for the two lower pooling levels, 64 two-byte LDS staging writes,
// and a vmcnt(0) wait at every patch that drains the previous patch's 8 global
// stores (gfx9 counts stores in vmcnt, in order with the LDS-DMA) before the
// next patch may start.
//   * D = target x query (A = the patch's target rows from LDS, B = the wave's
//     query rows in registers): lane (fq, fr) holds targets 4 fq + i (i < 4) of
//     an N-block for query fr, and the patch buffer orders an N-block's 16
//     target rows so that those four are a 2x2 window (row c = 4 fq + i ->
//     sub-patch (2 (fq >> 1) + (i >> 1), 2 (fq & 1) + (i & 1))): level 1 is
//     pooled inside the lane, level 2 takes 3 shuffles per (row block, N-block)
//     (lanes l ^ 16, ^ 32, ^ 48), level 3 is register-local across N-blocks -
//     24 shuffles per patch instead of 192; same arithmetic and summation order.
//   * level 0 is staged as 4-byte pairs (16 ds_write_b32 instead of 32
//     ds_write_b16), the 16-B tile rows of query q XOR-swizzled by q & 7
//     (2-way bank conflicts instead of 8), so that two workgroups fit a CU
//     (80.5 KB of LDS each, 108 VGPRs: 4 waves per SIMD instead of 2).
//   * every store is an unconditional buffer store (an out-of-range offset is
//     dropped), so each wave issues exactly kVol2Stores per patch and the patch
//     hand-off waits with vmcnt(kVol2Stores): the LDS-DMA of the next patch,
//     issued before this patch's stores, is awaited without draining them.
// ---------------------------------------------------------------------------
constexpr int kVol2S0 = 64;    // staging row (halves): level 0, one 8x8 tile, 16-B row pieces XOR-swizzled by q & 7
constexpr int kVol2S1 = 20;    // level 1, 4x4 + pad (8-B aligned rows)
constexpr int kVol2StageWave = 32 * kVol2S0 * 2 + 32 * kVol2S1 * 2 + 32 * 4 * 2 + 32 * 2;
constexpr int kVol2Lds = kVolStage + 8 * kVol2StageWave;
static_assert(2 * kVol2Lds <= 160 * 1024, "corr_volume_pyramid2: two workgroups per CU");
constexpr int kVol2Stores = 8;  // per wave and patch: 4 (level 0) + 2 (level 1) + 1 + 1

// target pixel of N-block b, row c (= 4 fq + i) inside an 8x8 patch
__device__ __forceinline__ int vol2_ty(int b, int c) { return 4 * (b >> 1) + 2 * (c >> 3) + ((c >> 1) & 1); }
__device__ __forceinline__ int vol2_tx(int b, int c) { return 4 * (b & 1) + 2 * ((c >> 2) & 1) + (c & 1); }

// cache policy of the level-0 / level-1 tile stores (buffer-op aux bits; A/B
// builds: 2 = nt, streamed past the caches - the volume is read back only by
// the next update()'s lookups, long after it has left L2 and the Infinity Cache)
#ifndef DROID_VOL_STORE_AUX
#define DROID_VOL_STORE_AUX 2
#endif
// the same for the pooling pass's level-1 loads and level-2/3 stores (A/B)
#ifndef DROID_POOL_AUX
#define DROID_POOL_AUX 2
#endif
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack2h(float lo, float hi) {
  return (unsigned)__half_as_ushort(__float2half(lo)) | ((unsigned)__half_as_ushort(__float2half(hi)) << 16);
}

// L23 = false (round 4, variant 4): levels 2 and 3 are neither pooled nor
// stored here - corr_volume_pool23_kernel forms them from the stored level 1
// MODE 0: every level stored per patch.  MODE 1 (tiled layout): a 2x2 patch
// group is one level-1 tile, so the group's level-1 values are held in
// registers (16 VGPRs of packed pairs) and stored as whole tiles when the group
// ends; MODE 2: level 1 per patch.  MODEs 1 and 2 leave levels 2 and 3 to
// corr_volume_pool23_kernel.
template <int MODE>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) corr_volume_pyramid2_kernel(VolArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr bool L23 = MODE == 0, GRP = MODE == 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int H = a.H, W = a.W, HW = H * W;
  // XCD-aware order: the hardware deals consecutive workgroups to the 8 XCDs in
  // turn, so an edge's workgroups (its query blocks, which all read the same
  // target frame's patches) would land on 8 different L2s and fetch that frame
  // from HBM up to 8 times; remapped, each XCD takes a contiguous run of edges
  const int G = (int)gridDim.x;
  const int bid = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int e = __builtin_amdgcn_readfirstlane(bid / a.qblocks);
  const int qb = bid % a.qblocks;
  const int fa = __builtin_amdgcn_readfirstlane(a.f1[e]);
  const int fb = __builtin_amdgcn_readfirstlane(a.f2[e]);
  const unsigned lds_a = lds_addr(lds);
  char* stage = lds + kVolStage + wave * kVol2StageWave;
  _Float16* s0 = reinterpret_cast<_Float16*>(stage);                   // [32][kVol2S0]
  _Float16* s1 = s0 + 32 * kVol2S0;                                    // [32][kVol2S1]
  _Float16* s2 = s1 + 32 * kVol2S1;                                    // [32][4]
  _Float16* s3 = s2 + 32 * 4;                                          // [32]

  // this wave's 32 query rows: B fragments (lane: query fr, channels 8 fq ..) x 4 K-steps
  const int q0 = qb * kVolQ + wave * 32;
  half8 qf[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = min(q0 + 16 * r + fr, HW - 1);
    const __half* row = a.f + ((long)fa * HW + q) * 128;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[r][ks] = *reinterpret_cast<const half8*>(row + ks * 32 + fq * 8);
  }

  // level geometry and this edge's output slices (one descriptor per level:
  // offsets past a query pixel that does not exist are dropped)
  int Hl[4], Wl[4], TR[4];
  long slice[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    Hl[l] = H >> l;
    Wl[l] = W >> l;
    TR[l] = (Hl[l] + 7) / 8;  // tile rows (tiled layout)
    slice[l] = a.tiled ? (long)TR[l] * (Wl[l] / 8) * 64 : (long)Hl[l] * Wl[l];
  }
  __amdgpu_buffer_rsrc_t ro[4];
#pragma unroll
  for (int l = 0; l < 4; ++l)
    ro[l] = __builtin_amdgcn_make_buffer_rsrc(a.lvl[l] + (long)e * HW * slice[l], (short)0,
                                              (int)(HW * slice[l] * 2), kBufFlags);

  const rsrc_t rsb = make_rsrc(a.f + (long)fb * HW * 128, (unsigned)(HW * 256));
  const int pcols = W / 8, npatch = (H / 8) * pcols;
  (void)npatch;
  auto patch_yx = [&](int p, int& py, int& px) {
    const int gcols = (pcols + 1) / 2;
    const int g = p >> 2, k = p & 3;
    int gy = g / gcols, gx = g - gy * gcols;
    py = 2 * gy + (k >> 1);
    px = 2 * gx + (k & 1);
  };
  const int gslots = ((H / 8 + 1) / 2) * ((pcols + 1) / 2) * 4;
  auto patch_dma = [&](int p, int buf) {
    int py, px;
    patch_yx(p, py, px);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ins = wave_u + 8 * k;
      const int row = ins * 4 + (lane >> 4);
      const int b = row >> 4, c = row & 15;
      const int t = (8 * py + vol2_ty(b, c)) * W + 8 * px + vol2_tx(b, c);
      const int piece = (lane & 15) ^ (row & 15);
      dma16(rsb, lds_a + kVolB + buf * 16384 + ins * 1024, (unsigned)((t * 128 + piece * 8) * 2));
    }
  };
  auto valid = [&](int p) {
    int py, px;
    patch_yx(p, py, px);
    return py < H / 8 && px < pcols;
  };
  int first = 0;
  while (first < gslots && !valid(first)) ++first;
  if (first < gslots) patch_dma(first, 0);
  unsigned l1g[4][2][2];   // MODE 1: the group's level-1 values, [patch k][row block r][pair (b, b + 1)]
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) l1g[kk][0][0] = l1g[kk][0][1] = l1g[kk][1][0] = l1g[kk][1][1] = 0u;
  int buf = 0;
  bool stores_out = false;   // this wave has kVol2Stores stores in flight after the last DMA
  for (int p = first; p < gslots;) {
    int nxt = p + 1;
    while (nxt < gslots && !valid(nxt)) ++nxt;
    if (stores_out) {
      // the stores issued after the next patch's DMA: MODE 0 4 + 2 + 1 + 1, MODE 1
      // 4 + 4 (the group's level-1 rows, out of range but at its last patch), MODE 2 4 + 2
      if (MODE != 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();   // patch p landed in buf; every wave done with buf ^ 1
    if (nxt < gslots && !(a.ablate & 2)) patch_dma(nxt, buf ^ 1);
    int py, px;
    patch_yx(p, py, px);
    const int ty0 = 8 * py, tx0 = 8 * px;

    // per N-block b and row block r: V0 = targets (4 fq + i) for query 16 r + fr,
    // rounded to fp16, staged as the lane's 2x2 window (two 4-B pairs of the 8x8
    // tile, row-major), and its level-1 value pooled in place ((h, w) order;
    // level-1 pixel (2 (b >> 1) + (fq >> 1), 2 (b & 1) + (fq & 1)) of the patch's
    // 4x4 block) - only four V0 values are live at a time
    float u[2][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      half8 tf[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int row = b * 16 + fr, piece = ks * 4 + fq;
        tf[ks] = *reinterpret_cast<const half8*>(lds + kVolB + buf * 16384 + row * 256 + ((piece ^ (row & 15)) << 4));
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(tf[ks], qf[r][ks], c, 0, 0, 0);
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = rnd16(c[i]);
        const int q = 16 * r + fr;
        const int y = 4 * (b >> 1) + 2 * (fq >> 1), x = 4 * (b & 1) + 2 * (fq & 1);
        *reinterpret_cast<unsigned*>(s0 + q * kVol2S0 + ((y ^ (q & 7)) << 3) + x) = pack2h(v[0], v[1]);
        *reinterpret_cast<unsigned*>(s0 + q * kVol2S0 + (((y + 1) ^ (q & 7)) << 3) + x) = pack2h(v[2], v[3]);
        u[r][b] = vol_pool4(v[0], v[1], v[2], v[3]);
        if (!GRP) s1[q * kVol2S1 + (2 * (b >> 1) + (fq >> 1)) * 4 + 2 * (b & 1) + (fq & 1)] = (_Float16)u[r][b];
        if (GRP && (b & 1)) {   // the pair (b - 1, b) into the group's registers (select chain: k is a runtime value)
          const unsigned pk = pack2h(u[r][b - 1], u[r][b]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) l1g[kk][r][b >> 1] = ((p & 3) == kk) ? pk : l1g[kk][r][b >> 1];
        }
      }
    }
    // level 2: the four level-1 values of an N-block sit in lanes fq = 0..3 ((h, w)
    // order = fq order); level 3: the four N-blocks of a lane
#pragma unroll
    for (int r = 0; r < (L23 ? 2 : 0); ++r) {
      float w2[4];
#pragma unroll
      for (int b = 0; b < 4; ++b)
        w2[b] = vol_pool4(u[r][b], __shfl_xor(u[r][b], 16), __shfl_xor(u[r][b], 32), __shfl_xor(u[r][b], 48));
      if (fq == 0) {
        const int q = 16 * r + fr;
#pragma unroll
        for (int b = 0; b < 4; ++b) s2[q * 4 + b] = (_Float16)w2[b];
        s3[q] = (_Float16)vol_pool4(w2[0], w2[1], w2[2], w2[3]);
      }
    }
    // stores (the staging area is this wave's own: a wave barrier suffices)
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ablations: every offset out of range (no bytes written) - bit 0 all levels,
    // bit 2 levels 1..3 only, bit 3 level 0 only
    const int qlim0 = (a.ablate & 9) ? 0 : HW;
    const int qlim = (a.ablate & 5) ? 0 : HW;
    // level 0: 32 q x 128 B, 8 lanes per query pixel
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = 8 * k + (lane >> 3), seg = lane & 7;   // seg = tile row
      const int qg = q0 + q;
      const u32x4_t val = *reinterpret_cast<const u32x4_t*>(s0 + q * kVol2S0 + ((seg ^ (q & 7)) << 3));
      const long off = a.tiled ? ((long)qg * TR[0] * (Wl[0] / 8) + py * (Wl[0] / 8) + px) * 64 + seg * 8
                               : (long)qg * HW + (long)(ty0 + seg) * W + tx0;
      __builtin_amdgcn_raw_buffer_store_b128(val, ro[0], qg < qlim0 ? (int)(off * 2) : (int)kOob, 0, DROID_VOL_STORE_AUX);
    }
    // level 1: 32 q x 4 rows x 8 B (the patch's 4x4 level-1 block)
#pragma unroll
    for (int k = 0; k < (GRP ? 0 : 2); ++k) {
      const int q = 16 * k + (lane >> 2), rr = lane & 3;
      const int qg = q0 + q;
      const u32x2_t val = *reinterpret_cast<const u32x2_t*>(s1 + q * kVol2S1 + rr * 4);
      const int y = ty0 / 2 + rr, x = tx0 / 2;
      const long off = a.tiled ? ((long)qg * TR[1] * (Wl[1] / 8) + (y >> 3) * (Wl[1] / 8) + (x >> 3)) * 64 +
                                     (y & 7) * 8 + (x & 7)
                               : (long)qg * (Hl[1] * Wl[1]) + (long)y * Wl[1] + x;
      __builtin_amdgcn_raw_buffer_store_b64(val, ro[1], qg < qlim ? (int)(off * 2) : (int)kOob, 0, 0);
    }
    if (GRP) {
      // at the group's last patch: its 8x8 level-1 tile per query through the
      // level-0 staging rows (free once the level-0 stores above have read
      // them), then 4 x 16-B row pieces per lane = whole 128-B tiles
      const bool flush = nxt >= gslots || (nxt >> 2) != (p >> 2);
      if (flush) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const int q = 16 * r + fr;
              const int y1 = 4 * (kk >> 1) + 2 * (b >> 1) + (fq >> 1), x1 = 4 * (kk & 1) + 2 * (b & 1) + (fq & 1);
              const unsigned pk = l1g[kk][r][b >> 1];
              s0[q * kVol2S0 + ((y1 ^ (q & 7)) << 3) + x1] =
                  __builtin_bit_cast(_Float16, (unsigned short)((b & 1) ? (pk >> 16) : (pk & 0xffffu)));
            }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      const int g = p >> 2, gcols = (pcols + 1) / 2;
      const int gy = g / gcols, gx = g - gy * gcols;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = 8 * k + (lane >> 3), seg = lane & 7;
        const int qg = q0 + q;
        const u32x4_t val = flush ? *reinterpret_cast<const u32x4_t*>(s0 + q * kVol2S0 + ((seg ^ (q & 7)) << 3))
                                  : u32x4_t{0u, 0u, 0u, 0u};
        const long off = ((long)qg * TR[1] * (Wl[1] / 8) + gy * (Wl[1] / 8) + gx) * 64 + seg * 8;
        __builtin_amdgcn_raw_buffer_store_b128(val, ro[1], (flush && qg < qlim) ? (int)(off * 2) : (int)kOob, 0,
                                               DROID_VOL_STORE_AUX);
      }
      if (flush) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) l1g[kk][0][0] = l1g[kk][0][1] = l1g[kk][1][0] = l1g[kk][1][1] = 0u;
      }
    }
    // level 2: 32 q x 2 rows x 4 B; level 3: 32 q x 2 B
    if (L23) {
      const int q = lane >> 1, rr = lane & 1;
      const int qg = q0 + q;
      const unsigned val = *reinterpret_cast<const unsigned*>(s2 + q * 4 + rr * 2);
      const int y = ty0 / 4 + rr, x = tx0 / 4;
      const long off = a.tiled ? ((long)qg * TR[2] * (Wl[2] / 8) + (y >> 3) * (Wl[2] / 8) + (x >> 3)) * 64 +
                                     (y & 7) * 8 + (x & 7)
                               : (long)qg * (Hl[2] * Wl[2]) + (long)y * Wl[2] + x;
      __builtin_amdgcn_raw_buffer_store_b32(val, ro[2], qg < qlim ? (int)(off * 2) : (int)kOob, 0, 0);
    }
    if (L23) {
      const int qg = q0 + (lane & 31);
      const int y = ty0 / 8, x = tx0 / 8;
      const long off = a.tiled ? ((long)qg * TR[3] * (Wl[3] / 8) + (y >> 3) * (Wl[3] / 8) + (x >> 3)) * 64 +
                                     (y & 7) * 8 + (x & 7)
                               : (long)qg * (Hl[3] * Wl[3]) + (long)y * Wl[3] + x;
      const short val = (short)__half_as_ushort(*reinterpret_cast<const __half*>(s3 + (lane & 31)));
      __builtin_amdgcn_raw_buffer_store_b16(val, ro[3], (lane < 32 && qg < qlim) ? (int)(off * 2) : (int)kOob, 0, 0);
    }
    stores_out = true;
    buf ^= 1;
    p = nxt;
  }
  // tiled layout: rows of the last tile row past H_l are zero (levels whose height is not a multiple of 8)
  if (a.tiled) {
#pragma unroll
    for (int l = 1; l < (L23 ? 4 : 2); ++l) {
      const int pad = TR[l] * 8 - Hl[l];
      if (pad == 0) continue;
      const int tcols = Wl[l] / 8;
      const int pieces = tcols * pad;
      for (int idx = lane; idx < 32 * pieces; idx += 64) {
        const int q = idx / pieces, k = idx - q * pieces;
        const int tc = k / pad, rr = Hl[l] - (TR[l] - 1) * 8 + (k - tc * pad);
        const int qg = q0 + q;
        if (qg < HW) {
          const long off = (((long)e * HW + qg) * TR[l] * tcols + (TR[l] - 1) * tcols + tc) * 64 + rr * 8;
          *reinterpret_cast<uint4*>(a.lvl[l] + off) = uint4{0u, 0u, 0u, 0u};
        }
      }
    }
  }
}

#if DROID_AB
#include "ab/corr_volume_ab.inc"
#endif

// ---------------------------------------------------------------------------
// corr_volume_pool23_kernel (round 4, variant 4): levels 2 and 3 of every
// (edge, query pixel) from its stored level 1, with the pyramid kernel's
// arithmetic (vol_pool4 over the four fp16 values in (h, w) order - the same
// values in the same order, so the bytes are those of variant 2).  Written
// this way because the per-patch level-2/3 pieces (2-8 B of lines completed
// over 16-48 patches) left the L2 partial and cost more than the whole level-0
// stream (profiles/r04/r04f_vol2_ablate*.txt).  One wave per query pixel: a
// level is walked in its storage order, so each wave-instruction stores 128
// contiguous bytes (one tiled-layout tile or a 64-element row run) and the
// padding rows of the tiled layout are written as zeros; level 2 is kept in
// LDS for level 3.
// ---------------------------------------------------------------------------
__device__ __forceinline__ long vol_elem(bool tiled, int tcols, int W, int y, int x) {
  return tiled ? ((long)((y >> 3) * tcols + (x >> 3)) << 6) + ((y & 7) << 3) + (x & 7) : (long)y * W + x;
}

__global__ void __launch_bounds__(256) corr_volume_pool23_kernel(VolArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // wave-uniform in an SGPR: the per-query buffer descriptors below stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int H = a.H, W = a.W, HW = H * W;
  const long nq = a.qblocks;   // = E * H * W (set by the launcher)
  const bool tiled = a.tiled != 0;
  int Hl[4], Wl[4], TR[4], TC[4];
  long slice[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    Hl[l] = H >> l;
    Wl[l] = W >> l;
    TR[l] = (Hl[l] + 7) / 8;
    TC[l] = Wl[l] / 8;
    slice[l] = tiled ? (long)TR[l] * TC[l] * 64 : (long)Hl[l] * Wl[l];
  }
  const int n2 = (int)slice[2], n3 = (int)slice[3], n1 = (int)slice[1];
  if (n2 <= 8 * 64 && n3 <= 64) {
    // the common shapes (C3's 48x64: 256 + 64 halves): two query pixels per wave
    // step with every level-1 load of both in flight before the first use (the
    // generic loop below waits for each 64-element run's loads in turn), all
    // through per-query buffer descriptors with out-of-range offsets for the
    // elements a query does not have - branch-free, fixed instruction counts
    constexpr int QPW = 2;
    _Float16* s2q = reinterpret_cast<_Float16*>(lds) + (long)wave * QPW * Hl[2] * Wl[2];
    // each lane forms two horizontally adjacent level-2 values (x even): their
    // 2x2 level-1 sources are one 8-B load per row (four consecutive halves of a
    // tile row / a row run) and the pair is one 4-B store, so a wave-instruction
    // moves 512 / 256 B instead of 256 / 128; NI pair rounds cover the slice
    // (C3's 256 halves: 2 rounds, no out-of-range rounds issued)
    auto run = [&](auto nic) {
      constexpr int NI = decltype(nic)::value;
      for (long qp0 = ((long)blockIdx.x * 4 + wave) * QPW; qp0 < nq; qp0 += 4L * QPW * gridDim.x) {
        u32x2_t top[QPW][NI], bot[QPW][NI];
#pragma unroll
        for (int k = 0; k < QPW; ++k) {
          const long qp = qp0 + k;
          const bool qok = qp < nq;
          const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<__half*>(a.lvl[1] + (qok ? qp : 0) * slice[1]), (short)0, qok ? n1 * 2 : 0, kBufFlags);
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const int s = 2 * (lane + 64 * i);
            int y, x;
            if (tiled) {
              const int t = s >> 6, r = s & 63;
              y = (t / TC[2]) * 8 + (r >> 3);
              x = (t % TC[2]) * 8 + (r & 7);
            } else {
              y = s / Wl[2];
              x = s % Wl[2];
            }
            const bool ok = s < n2 && y < Hl[2];
            const unsigned ot = ok ? (unsigned)vol_elem(tiled, TC[1], Wl[1], 2 * y, 2 * x) * 2u : kOob;
            const unsigned ob = ok ? (unsigned)vol_elem(tiled, TC[1], Wl[1], 2 * y + 1, 2 * x) * 2u : kOob;
            top[k][i] = __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r1, (int)ot, 0, DROID_POOL_AUX));
            bot[k][i] = __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r1, (int)ob, 0, DROID_POOL_AUX));
          }
        }
#pragma unroll
        for (int k = 0; k < QPW; ++k) {
          const long qp = qp0 + k;
          const bool qok = qp < nq;
          const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
              a.lvl[2] + (qok ? qp : 0) * slice[2], (short)0, qok ? n2 * 2 : 0, kBufFlags);
          _Float16* s2 = s2q + k * Hl[2] * Wl[2];
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const int s = 2 * (lane + 64 * i);
            int y, x;
            if (tiled) {
              const int t = s >> 6, r = s & 63;
              y = (t / TC[2]) * 8 + (r >> 3);
              x = (t % TC[2]) * 8 + (r & 7);
            } else {
              y = s / Wl[2];
              x = s % Wl[2];
            }
            float v0 = 0.0f, v1 = 0.0f;
            if (s < n2 && y < Hl[2]) {
              const u32x2_t t0 = top[k][i], b0 = bot[k][i];
              v0 = vol_pool4(__half2float(__ushort_as_half((unsigned short)(t0[0] & 0xffffu))),
                             __half2float(__ushort_as_half((unsigned short)(t0[0] >> 16))),
                             __half2float(__ushort_as_half((unsigned short)(b0[0] & 0xffffu))),
                             __half2float(__ushort_as_half((unsigned short)(b0[0] >> 16))));
              v1 = vol_pool4(__half2float(__ushort_as_half((unsigned short)(t0[1] & 0xffffu))),
                             __half2float(__ushort_as_half((unsigned short)(t0[1] >> 16))),
                             __half2float(__ushort_as_half((unsigned short)(b0[1] & 0xffffu))),
                             __half2float(__ushort_as_half((unsigned short)(b0[1] >> 16))));
              s2[y * Wl[2] + x] = (_Float16)v0;
              s2[y * Wl[2] + x + 1] = (_Float16)v1;
            }
            const unsigned pk = (unsigned)__half_as_ushort(__float2half(v0)) |
                                ((unsigned)__half_as_ushort(__float2half(v1)) << 16);
            __builtin_amdgcn_raw_buffer_store_b32(pk, r2, s < n2 ? s * 2 : (int)kOob, 0, DROID_POOL_AUX);
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < QPW; ++k) {
          const long qp = qp0 + k;
          const bool qok = qp < nq;
          const __amdgpu_buffer_rsrc_t r3 = __builtin_amdgcn_make_buffer_rsrc(
              a.lvl[3] + (qok ? qp : 0) * slice[3], (short)0, qok ? n3 * 2 : 0, kBufFlags);
          const _Float16* s2 = s2q + k * Hl[2] * Wl[2];
          const int s = lane;
          int y, x;
          if (tiled) {
            const int t = s >> 6, r = s & 63;
            y = (t / TC[3]) * 8 + (r >> 3);
            x = (t % TC[3]) * 8 + (r & 7);
          } else {
            y = s / Wl[3];
            x = s % Wl[3];
          }
          float v = 0.0f;
          if (s < n3 && y < Hl[3]) {
            const _Float16* r0 = s2 + (2 * y) * Wl[2] + 2 * x;
            v = vol_pool4((float)r0[0], (float)r0[1], (float)r0[Wl[2]], (float)r0[Wl[2] + 1]);
          }
          __builtin_amdgcn_raw_buffer_store_b16((short)__half_as_ushort(__float2half(v)), r3,
                                                s < n3 ? s * 2 : (int)kOob, 0, DROID_POOL_AUX);
        }
        __builtin_amdgcn_wave_barrier();   // s2 is rewritten by the next step's level 2
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    };
    if (n2 <= 2 * 128) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 4>{});
    return;
  }
  _Float16* s2 = reinterpret_cast<_Float16*>(lds) + (long)wave * Hl[2] * Wl[2];
  // persistent: wave w of the grid takes (edge, query pixel) w, w + 4 G, ..
  for (long qp = (long)blockIdx.x * 4 + wave; qp < nq; qp += 4L * gridDim.x) {
  const __half* l1 = a.lvl[1] + qp * slice[1];
  __half* l2 = a.lvl[2] + qp * slice[2];
  __half* l3 = a.lvl[3] + qp * slice[3];
  // level 2, in storage order
  for (long s = lane; s < slice[2]; s += 64) {
    int y, x;
    if (tiled) {
      const int t = (int)(s >> 6), r = (int)(s & 63);
      y = (t / TC[2]) * 8 + (r >> 3);
      x = (t % TC[2]) * 8 + (r & 7);
    } else {
      y = (int)(s / Wl[2]);
      x = (int)(s % Wl[2]);
    }
    float v = 0.0f;
    if (y < Hl[2]) {
      const unsigned top = *reinterpret_cast<const unsigned*>(l1 + vol_elem(tiled, TC[1], Wl[1], 2 * y, 2 * x));
      const unsigned bot = *reinterpret_cast<const unsigned*>(l1 + vol_elem(tiled, TC[1], Wl[1], 2 * y + 1, 2 * x));
      v = vol_pool4(__half2float(__ushort_as_half((unsigned short)(top & 0xffffu))),
                    __half2float(__ushort_as_half((unsigned short)(top >> 16))),
                    __half2float(__ushort_as_half((unsigned short)(bot & 0xffffu))),
                    __half2float(__ushort_as_half((unsigned short)(bot >> 16))));
      s2[y * Wl[2] + x] = (_Float16)v;
    }
    l2[s] = __float2half(v);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // level 3 from level 2
  for (long s = lane; s < slice[3]; s += 64) {
    int y, x;
    if (tiled) {
      const int t = (int)(s >> 6), r = (int)(s & 63);
      y = (t / TC[3]) * 8 + (r >> 3);
      x = (t % TC[3]) * 8 + (r & 7);
    } else {
      y = (int)(s / Wl[3]);
      x = (int)(s % Wl[3]);
    }
    float v = 0.0f;
    if (y < Hl[3]) {
      const _Float16* r0 = s2 + (2 * y) * Wl[2] + 2 * x;
      v = vol_pool4((float)r0[0], (float)r0[1], (float)r0[Wl[2]], (float)r0[Wl[2] + 1]);
    }
    l3[s] = __float2half(v);
  }
  __builtin_amdgcn_wave_barrier();   // s2 is rewritten by the next query's level 2
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

}  // namespace droid

using namespace droid;

extern "C" {

// CorrBlock pyramid (modules/corr.py:24-38,63-71) of E edges from the frames'
// NHWC feature maps divided by 4 (fmaps (NF,H,W,128) fp16, the AltCorrBlock
// level 0): level l of edge e = avgpool^l(<fmaps[f1[e]], fmaps[f2[e]]>) as
// fp16, written to levels[l]: (E,H,W,ceil(H_l/8),W_l/8,8,8) when tiled (the
// layout of droid_corr_lookup_ce0_tiled) or (E,H,W,H_l,W_l).  H, W multiples of 8.
int droid_corr_volume_pyramid(const void* fmaps, const int* f1, const int* f2, int E, int NF, int H, int W,
                              void* const* levels, int tiled, hipStream_t stream) {
  if (!fmaps || !f1 || !f2 || !levels || E < 0 || NF <= 0 || H <= 0 || W <= 0)
    return fail(kInvalidArgument, "corr_volume_pyramid: bad arguments");
  if (H % 8 || W % 8) return fail(kUnsupported, "corr_volume_pyramid: H and W must be multiples of 8");
  if (tiled && (W >> 3) % 8) return fail(kUnsupported, "corr_volume_pyramid: tiled levels need W / 8 % 8 == 0");
  if ((long)H * W * 256 > 0x7fffffffL) return fail(kUnsupported, "corr_volume_pyramid: frames too large");
  VolArgs a{};
  a.f = (const __half*)fmaps;
  a.f1 = f1;
  a.f2 = f2;
  for (int l = 0; l < 4; ++l) {
    if (!levels[l]) return fail(kInvalidArgument, "corr_volume_pyramid: null level");
    a.lvl[l] = (__half*)levels[l];
  }
  a.H = H;
  a.W = W;
  a.tiled = tiled ? 1 : 0;
  a.qblocks = ceil_div(H * W, kVolQ);
  a.ablate = ab_knob("DROID_VOL_ABLATE", 0);   // timing experiments (A/B build only)
  const long grid = (long)E * a.qblocks;
  if (grid == 0) return kOk;
  if (grid > 0x7fffffffL) return fail(kUnsupported, "corr_volume_pyramid: too many edges");
  // The product kernel is variant 4: corr_volume_pyramid2_kernel<1 / 2> writes
  // levels 0 and 1, corr_volume_pool23_kernel pools levels 2 and 3 from the
  // stored level 1.  The A/B build keeps DROID_VOL_VARIANT 1 (the round-3
  // kernel), 2 (corr_volume_pyramid2_kernel<0>, every level per patch) and 3
  // (the ring variant).  C3, 2048 edges, identical bytes (hash64): v1 33.3 ms,
  // v2 19.9-23.2, v3 23.6, v4 15.6-16.1 then 12.0-12.8 with non-temporal
  // stores (profiles/r04/vol_v*.txt, r04g_vol_v*.txt, r04x_vol_store_aux.txt)
  static const int variant = ab_knob("DROID_VOL_VARIANT", 4);
  if ((long)H * W * H * W * 2 >= 0x7fffffffL && variant != 1)
    return fail(kUnsupported, "corr_volume_pyramid: an edge's level-0 volume must stay below 2 GB");
#if DROID_AB
  if (variant == 3) {
    static bool attr3 = false;
    if (!attr3) {
      DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_volume_pyramid3_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kVol3Lds));
      attr3 = true;
    }
    corr_volume_pyramid3_kernel<<<dim3((unsigned)grid), 512, kVol3Lds, stream>>>(a);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  if (variant == 1) {
    static bool attr = false;
    if (!attr) {
      DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_volume_pyramid_kernel),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kVolLds));
      attr = true;
    }
    corr_volume_pyramid_kernel<<<dim3((unsigned)grid), 512, kVolLds, stream>>>(a);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
  if (variant == 2) {
    static bool attr0 = false;
    if (!attr0) {
      DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_volume_pyramid2_kernel<0>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kVol2Lds));
      attr0 = true;
    }
    corr_volume_pyramid2_kernel<0><<<dim3((unsigned)grid), 512, kVol2Lds, stream>>>(a);
    DROID_LAUNCH_CHECK();
    return kOk;
  }
#endif
  static bool attr2 = false;
  if (!attr2) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_volume_pyramid2_kernel<1>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kVol2Lds));
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_volume_pyramid2_kernel<2>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kVol2Lds));
    attr2 = true;
  }
  if (tiled) corr_volume_pyramid2_kernel<1><<<dim3((unsigned)grid), 512, kVol2Lds, stream>>>(a);
  else corr_volume_pyramid2_kernel<2><<<dim3((unsigned)grid), 512, kVol2Lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  VolArgs b = a;
  const long nq = (long)E * H * W;
  b.qblocks = (int)nq;   // the pooling pass reads its (edge, pixel) count from qblocks
  const long g2 = std::min<long>((nq + 3) / 4, 16L * device_cu_count());
  if (g2 > 0x7fffffffL || nq > 0x7fffffffL) return fail(kUnsupported, "corr_volume_pyramid: too many pixels");
  const int lds2 = 2 * 4 * (H / 4) * (W / 4) * 2;   // two query pixels' level 2 per wave
  corr_volume_pool23_kernel<<<dim3((unsigned)g2), 256, lds2, stream>>>(b);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
