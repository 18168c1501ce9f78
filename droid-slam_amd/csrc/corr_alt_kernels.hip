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
// The product kernel is corr_alt2_kernel<kAltProdCV> (two 4-wave workgroups
// per CU, its design note below; round 5: C pixel-major, row-K lookup tile).  It refines the round-2 kernel described here,
// corr_alt_ce0_kernel (now in ab/, the A/B build only; bitwise-equal outputs):
// persistent, one 8-wave workgroup per CU, software pipelined over "stages" =
// (8x8-pixel query tile of one edge, pyramid level):
//   * the union of the tile's 64 windows at that level (their bounding box,
//     clipped to the map) reaches LDS by LDS-DMA (NHWC rows are contiguous, one
//     16-B piece per lane, XOR-swizzled slots) ONE STAGE AHEAD, into the other
//     of two box buffers, while the current stage computes;
//   * C = F1 (64 px x 128, in registers for the tile's four levels) x box^T on
//     MFMA (f32 accumulate), rounded to fp16 - the values the volume would hold
//     at those taps;
//   * each pixel's 7x7 bilinear outputs come from its 8x8 taps of C with the
//     volume lookup's at::Half arithmetic (rnd16 after every op);
//   * the level's 49 lookup channels go straight through their slice of
//     corr_encoder[0] (1x1 196 -> 128) on MFMA into fp32 accumulators (K = 49
//     padded to 64 per level; the weights live in registers, wave w owns output
//     channels 16w .. 16w+15), so the 196-channel lookup never exists;
//   * after level 3: bias, ReLU, fp16, one coalesced 128-channel row per pixel.
// The next tile's coordinates arrive by LDS-DMA and its window boxes are
// computed during the current tile, so the pipeline never drains between
// tiles.  A box larger than a buffer (incoherent coordinates) runs that stage
// synchronously: its four 4x4 quadrants, a quadrant still too wide pixel by
// pixel (box = the pixel's own window); correctness never depends on
// coherence, only speed does.
//
// Numerics vs the volume path: level 0 differs only in the fp32 summation order
// of the dot products before their fp16 rounding; levels >= 1 pool the
// features instead of the correlations (both fp16), a difference at the fp16
// rounding level.  The bilinear arithmetic is the same; corr_encoder[0] sums
// its 196 products level by level in fp32.
#include "common.hpp"
#include "lds_dma.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

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
  long long* prof;       // profiling builds: s_memtime per (workgroup, stage < 32, phase < 8), or null
  const int* order;      // (E) edge processed in the k-th slot of the tile walk (edges grouped by target frame), or null
  int chunk;             // corr_alt2_kernel: tiles per XCD chunk (0 = the plain interleaved walk)
};

#ifndef DROID_CONV_PROFILE
#define DROID_CONV_PROFILE 0
#endif
#if DROID_CONV_PROFILE
#define ALT_STAMP(ph, v)                                                                            \
  do {                                                                                            \
    if (a.prof && tid == 0 && stage < 32)                                                         \
      a.prof[((long)blockIdx.x * 32 + stage) * 8 + (ph)] = (v);                                    \
  } while (0)
#else
#define ALT_STAMP(ph, v) do { } while (0)
#endif
#define ALT_NOW() ((long long)__builtin_amdgcn_s_memtime())
// DROID_ALT_CSTAMP=1 (timing builds): stamps 3/4/5 split the C phase instead
// (next-box DMA issued / box MFMA done / pixel boxes written)
#ifndef DROID_ALT_CSTAMP
#define DROID_ALT_CSTAMP 0
#endif
#define ALT_CSTAMP(ph) do { if (DROID_ALT_CSTAMP) ALT_STAMP(ph, ALT_NOW()); } while (0)
#define ALT_LSTAMP(ph) do { if (!DROID_ALT_CSTAMP) ALT_STAMP(ph, ALT_NOW()); } while (0)
// timing ablations (scripts only; results are wrong): bit 0 skips the box MFMA,
// bit 1 the bilinear, bit 2 the encoder MFMA, bit 3 the next-box DMA, bit 4 the
// output stores, bit 5 the next tile's boxes, bit 6 the frame-index loads, bit 7
// the slow path, bit 8 the lookup tile's K-padding zeroes
#ifndef DROID_ALT_ABL
#define DROID_ALT_ABL 0
#endif


// Box buffer 0 holds the boxes of levels 3 and 1, buffer 1 those of levels 2 and
// 0, so buffer 1 is the larger: on the C3 trajectory the level-0 box of a tile
// is 210 taps at the median and exceeds 288 for ~7 % of the tiles, the level-1
// box exceeds 191 for ~1.5 %.
constexpr int kAltCap0 = 191;  // box taps in buffer 0
constexpr int kAltCap1 = 288;  // box taps in buffer 1
constexpr int kAltCS = 292;    // C row stride (halves): >= 16 * ceil(kAltCap1 / 16), 8-B aligned rows
constexpr int kAltAS = 72;     // per-level lookup tile row stride (halves): 49 used, 64 multiplied
constexpr int kAltOS = 136;    // output staging row stride (halves)
constexpr int kAltMaxGroups = 1 + 2 + 4 + 64;
constexpr int kAltF1 = 20 * 1024;   // next tile's query features, inside box 1 past the output staging
constexpr int kAltA1 = kAltF1 + 64 * 256;   // the lookup tile of the stages on box 1, past the features
// LDS map (bytes)
// The per-level lookup tile [64 px][kAltAS] fp16 lives in the stage's own box
// buffer (dead once C is computed): at offset 0 of box 0, at kAltA1 of box 1.
constexpr int kAltBox0 = 0;                                  // [kAltCap0 taps][256 B]
constexpr int kAltBox1 = kAltBox0 + kAltCap0 * 256;          // [kAltCap1 taps][256 B] (+ output staging, F1)
constexpr int kAltC = kAltBox1 + kAltCap1 * 256;             // [64 px][kAltCS] fp16
constexpr int kAltCoord = kAltC + 64 * kAltCS * 2;           // [2 tiles][64 px] float2 (by LDS-DMA)
constexpr int kAltLvl = kAltCoord + 2 * 64 * 8;              // [2 tiles][4 levels] box x0, y0, w, h (int)
constexpr int kAltPix = kAltLvl + 2 * 4 * 4 * 4;             // slow path: per px group box x0, y0, w (int)
constexpr int kAltGrp = kAltPix + 64 * 3 * 4;                // slow path: count + groups (x0, y0, w, h, mmask, pix)
constexpr int kAltLds = kAltGrp + (kAltMaxGroups * 6 + 4) * 4;
static_assert(kAltLds <= 160 * 1024, "corr_alt_ce0 LDS budget");
static_assert(64 * kAltOS * 2 <= kAltF1 && kAltA1 + 64 * kAltAS * 2 <= kAltCap1 * 256,
              "output staging + F1 + lookup tile fit box 1");
static_assert(64 * kAltAS * 2 <= kAltCap0 * 256 && kAltBox1 % 16 == 0 && kAltAS == 72, "lookup tile fits box 0, 16-B aligned rows");
static_assert(kAltCS >= 16 * ((kAltCap1 + 15) / 16) && kAltCap0 <= kAltCap1, "C rows hold a box's taps");
__host__ __device__ constexpr int alt_cap(int l) { return (l & 1) ? kAltCap0 : kAltCap1; }

// tile pixel p = 16 q + r: quadrant q = (qy, qx) = (q >> 1, q & 1), r = (ry, rx)
__device__ __forceinline__ int alt_py(int p) { return 4 * ((p >> 4) >> 1) + ((p & 15) >> 2); }
__device__ __forceinline__ int alt_px(int p) { return 4 * ((p >> 4) & 1) + (p & 3); }

__device__ __forceinline__ int alt_floor(float v) { return (int)fminf(fmaxf(floorf(v), -1e6f), 1e6f); }

// clipped box [x0,x1] x [y0,y1] of the map -> tap count (0 when empty)
__device__ __forceinline__ int alt_clip(int& x0, int& x1, int& y0, int& y1, int Wl, int Hl) {
  x0 = max(x0, 0); x1 = min(x1, Wl - 1); y0 = max(y0, 0); y1 = min(y1, Hl - 1);
  return (x1 >= x0 && y1 >= y0) ? (x1 - x0 + 1) * (y1 - y0 + 1) : 0;
}

// one wave: level boxes [l0, l1) of a tile from its coordinates in LDS (lane = pixel)
__device__ __forceinline__ void alt_tile_boxes(const AltArgs& a, const float* cxy, int* lvl, int lane, int l0 = 0,
                                               int l1 = 4) {
#pragma unroll
  for (int l = l0; l < l1; ++l) {
    const float scl = 1.0f / (float)(1 << l);
    const int ox = alt_floor(cxy[2 * lane] * scl) - 3, oy = alt_floor(cxy[2 * lane + 1] * scl) - 3;
    // wave reductions on DPP (ockl), not LDS-routed shuffles
    int x0 = __ockl_wfred_min_i32(ox), x1 = __ockl_wfred_max_i32(ox) + 7;
    int y0 = __ockl_wfred_min_i32(oy), y1 = __ockl_wfred_max_i32(oy) + 7;
    const int tn = alt_clip(x0, x1, y0, y1, a.Wl[l], a.Hl[l]);
    if (lane == 0) {
      lvl[4 * l + 0] = x0;
      lvl[4 * l + 1] = y0;
      lvl[4 * l + 2] = tn ? x1 - x0 + 1 : 0;
      lvl[4 * l + 3] = tn ? y1 - y0 + 1 : 0;
    }
  }
}

// all waves: LDS-DMA of a gbw x gbh box of level `l` of frame f2 into `box`
__device__ __forceinline__ void alt_box_dma(const AltArgs& a, int l, int f2, int gx0, int gy0, int gbw, int gbh,
                                            unsigned box, int wave_u, int lane) {
  const int tn = gbw * gbh;
  if (tn <= 0) return;
  const int Hl = a.Hl[l], Wl = a.Wl[l];
  const rsrc_t rs = make_rsrc(a.pyr[l] + (long)__builtin_amdgcn_readfirstlane(f2) * Hl * Wl * 128,
                              (unsigned)(Hl * Wl * 256));
  const int nins = (tn + 3) >> 2;
  // tap / gbw by a float reciprocal: (tap + 0.5) / gbw is >= 0.5 / gbw >= 2^-8 from
  // an integer and tap < 2^12, so the v_rcp_f32 product (~2^-22 relative) floors exactly
  const float inv = __builtin_amdgcn_rcpf((float)gbw);
  for (int ins = wave_u; ins < nins; ins += 8) {
    const int tap = ins * 4 + (lane >> 4);
    const int piece = (lane & 15) ^ (tap & 15);
    const int ry = (int)(((float)tap + 0.5f) * inv), rx = tap - ry * gbw;
    const unsigned off = tap < tn ? (unsigned)((((gy0 + ry) * Wl + gx0 + rx) * 128 + piece * 8) * 2) : kOob;
    dma16(rs, box + ins * 1024, off);
  }
}

// C[p][tap] = <F1(p), box tap> for the taps of one box (nb blocks of 16), pixels
// restricted to the quadrants in mmask (and to pixel `gpix` when >= 0)
__device__ __forceinline__ void alt_box_mfma(const char* lds, int box, _Float16* Cs, const half8 (&af)[4][4], int tn,
                                             int mmask, int gpix, int wave_u, int fr, int fq) {
  const int nb = (tn + 15) >> 4;
  for (int b = wave_u; b < nb; b += 8) {
    half8 bf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int row = b * 16 + fr, piece = ks * 4 + fq;
      bf[ks] = *reinterpret_cast<const half8*>(lds + box + row * 256 + ((piece ^ (row & 15)) << 4));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!((mmask >> q) & 1)) continue;
      // taps x pixels: lane (fr, fq) gets taps b*16 + 4 fq + k (k < 4) of pixel q*16 + fr
      floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[ks], af[q][ks], c, 0, 0, 0);
      const int p = q * 16 + fr;
      if (gpix < 0 || gpix == p) {
        half4_t h = {(_Float16)c[0], (_Float16)c[1], (_Float16)c[2], (_Float16)c[3]};
        // taps past tn land in the row's slack (kAltCS >= 16 * ceil(kAltCap1 / 16)) and are never read
        *reinterpret_cast<half4_t*>(Cs + p * kAltCS + b * 16 + 4 * fq) = h;
      }
    }
  }
}

#if DROID_AB
#include "ab/corr_alt_v1_ab.inc"
#endif


// ===========================================================================
// corr_alt2_kernel: the same lookup with TWO 4-wave workgroups per CU, so one
// workgroup's DMA waits and barriers overlap the other's MFMA / VALU work (the
// one-workgroup kernel above spends ~2 ms of its 4.4 ms at C3 in barrier-phased
// stage skeletons).  LDS per workgroup <= 80 KB - one region of 304 tap rows x
// 256 B, used three ways:
//   * box: tap row t = the 128 fp16 features of box tap t (16-B pieces XOR
//     swizzled by t & 15, as the LDS-DMA lands them);
//   * C in place: C(p, t) = <F1(p), tap t> (fp16) overwrites the FIRST 128 B of
//     tap row t once every wave has read the box (wave w multiplies all blocks
//     by its own 16 query pixels and keeps its C in registers until then); the
//     bilinear then addresses C(p, t) = 256 t + 2 p - linear in t, one base per
//     window row plus immediate offsets;
//   * the lookup tile of level slot s, [64 px][64 k] (49 used), in the SECOND
//     halves: As(s, p, k) at row 64 s + p, byte 128 + 16 ((k / 8) ^ (p & 7)) +
//     2 (k % 8); the padding columns are zeroed in registers, not in LDS;
//   * the finished tile's output rows staged in the first halves of rows 64..191.
// Per tile: levels 3, 2, 1 in one stage (boxes packed at 4-aligned tap
// offsets, 292 taps at the C3 trajectory's p95), then level 0 (296 at p95).  A
// box set that does not fit runs one level at a time, a level box that does not
// fit runs as halves / quadrants / single pixels, each group with its own
// encoder pass over its M-block(s) (rows of pixels outside the group are zero,
// so the pass adds exactly 0 to them).  Every value is computed by the same
// operations in the same order as corr_alt_ce0_kernel: the outputs are
// bitwise equal (tests/test_gpu_fused.py).
// The layout above is the round-4 kernel's (A/B variant 4).  The round-5
// product (kCvRowK | kCvPm, see kAltProdCV) keeps the box rows but stores C
// pixel-major past the box's use - C(p, t) at byte p S + 2 t (b2_cstride) -
// puts the lookup tiles in a dense 128-B-per-pixel area from kB2Lk (k = 8 iy +
// ix order, one 16-B store per window row) and the per-pixel window table at
// kB2Win; see the notes at b2_corr and b2_bl_prep and DESIGN.md §3.
// ===========================================================================
constexpr int kB2Rows = 304;
constexpr int kB2Coord = kB2Rows * 256;       // [2 slots][64 px] float2
constexpr int kB2Lvl = kB2Coord + 2 * 512;    // [2 slots][4 levels] x0, y0, w, h
constexpr int kB2Grp = kB2Lvl + 2 * 16 * 4;   // fallback groups: count, then (x0, y0, w, h, qmask, gpix)
constexpr int kB2Bias = kB2Grp + (4 + kAltMaxGroups * 6) * 4;   // [128] f32 corr_encoder[0] bias
constexpr int kB2Lds = kB2Bias + 128 * 4;
static_assert(kB2Lds <= 80 * 1024, "two workgroups per CU");
static_assert(3 * 64 <= kB2Rows && 64 + 128 <= kB2Rows, "lookup tiles and output staging fit the region");
constexpr unsigned kB2Zero = 0x100000u;       // past the LDS allocation: ds reads return 0
#if DROID_CONV_PROFILE
// profiling builds: s_memtime per (workgroup, tile < 8, phase < 16), wave 0's view
#define B2_STAMP(k)                                                                                     \
  do {                                                                                                \
    if (a.prof && tid == 0 && tile_i < 8) a.prof[((long)blockIdx.x * 8 + tile_i) * 16 + (k)] = ALT_NOW(); \
  } while (0)
#else
#define B2_STAMP(k) do { } while (0)
#endif

__device__ __forceinline__ _Float16 b2_ldh(const char* lds, unsigned addr) {
  return *reinterpret_cast<const _Float16*>(lds + addr);
}

// LDS-DMA of a gbw x gbh box of level l of frame f2 to tap rows [toff, toff + taps), 4 waves
__device__ __forceinline__ void b2_box_dma(const AltArgs& a, int l, int f2, int gx0, int gy0, int gbw, int gbh,
                                           int toff, unsigned lds_a, int wave_u, int lane) {
  const int tn = gbw * gbh;
  if (tn <= 0) return;
  const int Hl = a.Hl[l], Wl = a.Wl[l];
  const rsrc_t rs = make_rsrc(a.pyr[l] + (long)__builtin_amdgcn_readfirstlane(f2) * Hl * Wl * 128,
                              (unsigned)(Hl * Wl * 256));
  const int nins = (tn + 3) >> 2;
  const float inv = __builtin_amdgcn_rcpf((float)gbw);   // exact floor: see alt_box_dma
  for (int ins = wave_u; ins < nins; ins += 4) {
    const int tap = ins * 4 + (lane >> 4);
    const int piece = (lane & 15) ^ ((toff + tap) & 15);
    const int ry = (int)(((float)tap + 0.5f) * inv), rx = tap - ry * gbw;
    const unsigned off = tap < tn ? (unsigned)((((gy0 + ry) * Wl + gx0 + rx) * 128 + piece * 8) * 2) : kOob;
    dma16(rs, lds_a + (unsigned)(toff + ins * 4) * 256u, off);
  }
}

// C of tap rows [0, T) for the pixels of M-block `wave` (if in qmask), written in
// place.  Each wave multiplies every 16-tap block by its own 16 query pixels, so
// a wave holds only its M-block's query features (4 fragments: the tile's 16 KB
// of query rows cross L2 -> CU once, not once per wave), at 4x the LDS reads of
// the box.  Since every wave reads every block, the C values (packed fp16, 2
// VGPRs per block) are written only after a barrier.
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// Round 5, PM (the product layout): C pixel-major - C(p, t) at byte p S + 2 t
// of the region, S = the stage's per-pixel stride (b2_cstride: the T taps
// rounded up to whole 16-tap blocks, S = 8 mod 16) - instead of in place over the box rows (C(p, t) at 256 t + 2 p).  A
// lane's 4 consecutive taps of one pixel are then ONE aligned 8-B store per
// block (conflict-free: S / 4 = 2 mod 4 spreads the 16 lanes of a store group
// over all 32 banks) instead of four 2-B stores, and a window row - 8
// consecutive taps of one pixel - comes back as 5 aligned dwords (b2_crow)
// instead of 8 2-B reads that the compiler had to pack pairwise, with an LDS
// round trip per pair.  The lookup tiles move to their own area (b2_lk) past
// the C region.  Same products, same fp16 rounding: C is bitwise the same.
constexpr int kB2Lk = 160 * 256;   // PM: lookup tiles, 3 slots x 64 px x 128 B
static_assert(kB2Lk >= 64 * (32 * ((kB2Rows + 15) / 16) + 8) && kB2Lk + 3 * 64 * 128 <= kB2Rows * 256, "PM C region and lookup tiles");
// S covers whole 16-tap blocks (b2_corr stores every tap of its last block)
__device__ __forceinline__ int b2_cstride(int T) { return 32 * ((T + 15) >> 4) + 8; }
template <bool PM>
__device__ __forceinline__ unsigned b2_lk(int as, int p) {
  return PM ? (unsigned)(kB2Lk + (as * 64 + p) * 128) : (unsigned)((as * 64 + p) * 256 + 128);
}
template <bool PM, typename Post>
__device__ __forceinline__ void b2_corr(char* lds, int T, int S, int qmask, const half8 (&af)[4], int wave_u, int fr,
                                        int fq, Post post) {
  constexpr int NB = kB2Rows / 16;
  const bool on = (qmask >> wave_u) & 1;
  const int nb = (T + 15) >> 4;
  half2_t cv[NB][2];
  auto ldb = [&](int b, half8 (&bf)[4]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      bf[ks] = *reinterpret_cast<const half8*>(lds + (b * 16 + fr) * 256 + (((ks * 4 + fq) ^ fr) << 4));
  };
  if (on && PM) {
    // software-pipelined (round 5): block b + 1's box fragments are loaded
    // before block b's MFMAs and block b - 1's fp16 conversion is deferred into
    // block b, so the LDS latency and the MFMA result latency overlap work
    // instead of serialising every block (rows past nb are loaded and dropped)
    half8 bb[2][4];   // ping-pong by block parity (a compile-time index: no copies)
    floatx4 cp = floatx4{0.f, 0.f, 0.f, 0.f};
    ldb(0, bb[0]);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b < nb) {
        if (b + 1 < NB) ldb(b + 1, bb[(b + 1) & 1]);
        floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bb[b & 1][ks], af[ks], c, 0, 0, 0);
        if (b > 0) {
          cv[b - 1][0] = half2_t{(_Float16)cp[0], (_Float16)cp[1]};
          cv[b - 1][1] = half2_t{(_Float16)cp[2], (_Float16)cp[3]};
        }
        cp = c;
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (b == nb - 1) {
        cv[b][0] = half2_t{(_Float16)cp[0], (_Float16)cp[1]};
        cv[b][1] = half2_t{(_Float16)cp[2], (_Float16)cp[3]};
      }
  } else if (on) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b < nb) {
        half8 bf[4];
        ldb(b, bf);
        floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[ks], af[ks], c, 0, 0, 0);
        cv[b][0] = half2_t{(_Float16)c[0], (_Float16)c[1]};
        cv[b][1] = half2_t{(_Float16)c[2], (_Float16)c[3]};
      }
    }
  }
  __syncthreads();   // every wave is done reading the box
  if (on) {
    const int q = wave_u;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b < nb) {
        // lane (fr, fq): C[tap b*16 + 4 fq + k][pixel q*16 + fr]
        if (PM) {
          const u32x2_t v = {__builtin_bit_cast(unsigned, cv[b][0]), __builtin_bit_cast(unsigned, cv[b][1])};
          *reinterpret_cast<u32x2_t*>(lds + (q * 16 + fr) * S + 2 * (b * 16 + 4 * fq)) = v;
        } else {
          char* base = lds + (b * 16 + 4 * fq) * 256 + (q * 16 + fr) * 2;
          *reinterpret_cast<_Float16*>(base) = cv[b][0][0];
          *reinterpret_cast<_Float16*>(base + 256) = cv[b][0][1];
          *reinterpret_cast<_Float16*>(base + 512) = cv[b][1][0];
          *reinterpret_cast<_Float16*>(base + 768) = cv[b][1][1];
        }
      }
    }
  }
  post();   // PM: the bilinear's per-pixel window table (b2_win_table), in the dead box past C
}

// The 8 window-row taps tr + i (i < 8) of pixel p of the 4 window rows a thread
// needs (rows (r, ab): output row r, its upper / lower tap row) as 4 packed
// pairs (2q, 2q + 1); a row outside the map (ok false) reads past the
// allocation, i.e. zeros.  PM: 5 aligned dwords over each row's 16 bytes - all
// 20 loads issued before the first funnel shift, one LDS round trip for the
// four rows - then a shift by 0 or 16 bits.
template <bool PM>
__device__ __forceinline__ void b2_crows(const char* lds, const int (&tr)[2][2], const bool (&ok)[2][2], int p, int S,
                                         unsigned (&pe)[2][2][4]) {
  if (PM) {
    unsigned d[2][2][5], sh[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int ab = 0; ab < 2; ++ab) {
        const unsigned rb = ok[r][ab] ? (unsigned)(p * S + 2 * tr[r][ab]) : kB2Zero;
        sh[r][ab] = (rb & 2u) * 8u;
#pragma unroll
        for (int i = 0; i < 5; ++i) d[r][ab][i] = *reinterpret_cast<const unsigned*>(lds + (rb & ~3u) + 4 * i);
      }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int ab = 0; ab < 2; ++ab)
#pragma unroll
        for (int q = 0; q < 4; ++q) pe[r][ab][q] = __builtin_amdgcn_alignbit(d[r][ab][q + 1], d[r][ab][q], sh[r][ab]);
  } else {
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int ab = 0; ab < 2; ++ab) {
        const unsigned rb = ok[r][ab] ? (unsigned)(tr[r][ab] * 256 + 2 * p) : kB2Zero;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          pe[r][ab][q] = __builtin_bit_cast(unsigned, h2_t{b2_ldh(lds, rb + (2 * q) * 256), b2_ldh(lds, rb + (2 * q + 1) * 256)});
      }
  }
}

// Round 4 (V3): C of tap rows [0, T) with the blocks split over the waves
// instead of the query pixels: wave w takes blocks w, w + 4, .. and multiplies
// each by all 64 query pixels (the tile's query rows in registers four times,
// from L2), so every box row is read from LDS ONCE per workgroup instead of
// once per wave (the C phase was LDS-read bound: 4 x 54 KB per level-0 box).
// The MFMA runs transposed (query pixels as rows), so a lane holds 4
// consecutive pixels of one tap: one 8-B LDS write per (block, M-block) instead
// of four 2-B writes.  A wave overwrites only rows it alone has read, so no
// barrier is needed before the writes.  Same products, same fp16 rounding: C is
// bitwise the V2 values.
__device__ __forceinline__ void b2_corr3(char* lds, int T, int qmask, const half8 (&af)[4][4], int wave_u, int fr,
                                         int fq) {
  constexpr int NBW = (kB2Rows / 16 + 3) / 4;
  const int nb = (T + 15) >> 4;
#pragma unroll 1
  for (int j = 0; j < NBW; ++j) {
    const int b = wave_u + 4 * j;
    if (b < nb) {
      half8 bf[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        bf[ks] = *reinterpret_cast<const half8*>(lds + (b * 16 + fr) * 256 + (((ks * 4 + fq) ^ fr) << 4));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if ((qmask >> q) & 1) {
          floatx4 c = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[q][ks], bf[ks], c, 0, 0, 0);
          // lane (fr, fq): C[pixel q*16 + 4 fq + k][tap b*16 + fr], k < 4
          half4_t h;
          h[0] = (_Float16)c[0];
          h[1] = (_Float16)c[1];
          h[2] = (_Float16)c[2];
          h[3] = (_Float16)c[3];
          *reinterpret_cast<half4_t*>(lds + (b * 16 + fr) * 256 + (q * 16 + 4 * fq) * 2) = h;
        }
      }
    }
  }
}

// bilinear windows of level l for the pixels of the M-blocks in qmask (only
// pixel gpix when >= 0; the others' rows are zeroed) -> lookup tile slot `as`.
// Thread = (wave w, pixel lane): window rows w and w + 4 (< 7) with the
// volume-lookup at::Half arithmetic in corr_alt_ce0_kernel's order.  Both
// rows' 32 taps are read before any arithmetic (one LDS round trip; wave 3's
// second row is read and dropped).
template <bool PM>
__device__ __forceinline__ void b2_bilinear(char* lds, const float* cxy, int l, int Hl, int Wl, int bx0, int by0,
                                            int bw, int toff, int S, int as, int qmask, int gpix, int wave_u, int lane) {
  const int p = lane;
  if (!((qmask >> (p >> 4)) & 1)) return;
  char* arow = lds + b2_lk<PM>(as, p);
  const int sw = p & 7;
  const int nr = wave_u == 3 ? 1 : 2;
  const _Float16 z = (_Float16)0.f;
  auto put = [&](int k, _Float16 v) { *reinterpret_cast<_Float16*>(arow + (((k >> 3) ^ sw) << 4) + (k & 7) * 2) = v; };
  if (gpix >= 0 && gpix != p) {   // a single-pixel group: the M-block's other rows are zero
    for (int r = 0; r < nr; ++r)
#pragma unroll
      for (int ix = 0; ix < 7; ++ix) put(ix * 7 + wave_u + 4 * r, z);
    return;
  }
  const float scl = 1.0f / (float)(1 << l);
  const float x0 = cxy[2 * p] * scl, y0 = cxy[2 * p + 1] * scl;
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xi0 = alt_floor(x0), yi0 = alt_floor(y0);
  const _Float16 w11 = (_Float16)rnd16(dx * dy);
  const _Float16 w10 = (_Float16)rnd16(dx * (1.0f - dy));
  const _Float16 w01 = (_Float16)rnd16((1.0f - dx) * dy);
  const _Float16 w00 = (_Float16)rnd16((1.0f - dx) * (1.0f - dy));
  const int xs = xi0 - 3;
  // columns xs + i inside the map: i in [lo, hi); rows outside read the zero address
  const int lo = min(max(-xs, 0), 8), hi = max(min(Wl - xs, 8), 0);
  const unsigned cmask = hi > lo ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u;
  const bool any_partial = __builtin_amdgcn_ballot_w64(cmask != 0xffu) != 0;
  // window rows (ya, ya + 1) of both output rows as packed tap pairs (2j, 2j + 1):
  // the arithmetic below runs two outputs per instruction (v_pk_mul / v_pk_add
  // _f16, each op rounded exactly as the scalar half op)
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  unsigned pe[2][2][4];
  int tr[2][2];
  bool okr[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int ya = yi0 - 3 + wave_u + 4 * r;
#pragma unroll
    for (int ab = 0; ab < 2; ++ab) {
      const int y = ya + ab;
      tr[r][ab] = toff + (y - by0) * bw + xs - bx0;
      okr[r][ab] = y >= 0 && y < Hl;
    }
  }
  b2_crows<PM>(lds, tr, okr, p, S, pe);
  if (any_partial) {   // columns outside the map read zeros
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned m = (((cmask >> (2 * q)) & 1) ? 0xffffu : 0u) | (((cmask >> (2 * q + 1)) & 1) ? 0xffff0000u : 0u);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        pe[r][0][q] &= m;
        pe[r][1][q] &= m;
      }
    }
  }
  const h2_t W00 = {w00, w00}, W01 = {w01, w01}, W10 = {w10, w10}, W11 = {w11, w11}, Z2 = {z, z};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (r >= nr) break;
    const int iy = wave_u + 4 * r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // outputs 2q, 2q + 1 (output 7 does not exist)
      const h2_t ae = __builtin_bit_cast(h2_t, pe[r][0][q]), be = __builtin_bit_cast(h2_t, pe[r][1][q]);
      const unsigned an = q < 3 ? pe[r][0][q + 1] : 0u, bn = q < 3 ? pe[r][1][q + 1] : 0u;
      const h2_t ao = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(an, pe[r][0][q], 16));
      const h2_t bo = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(bn, pe[r][1][q], 16));
      h2_t v = Z2 + ae * W00;
      v = v + be * W01;
      v = v + ao * W10;
      v = v + bo * W11;
      put(2 * q * 7 + iy, v[0]);
      if (q < 3) put((2 * q + 1) * 7 + iy, v[1]);
    }
  }
}

// V3: the same windows with the lookup tile's K order changed to k = 8 iy + ix
// (ix < 7; k = 8 iy + 7 and the row iy = 7 are zero, the encoder weights of
// build_wl3 zero there too): a thread's 7 outputs of window row iy are one
// 16-B piece, so a level costs a lane 2 ds_write_b128 instead of 14
// ds_write_b16.  Every piece of every pixel in qmask is written (wave 3 writes
// the zero row 7), so the encoder needs no padding mask.  Same arithmetic as
// b2_bilinear, value for value.
template <bool PM>
__device__ __forceinline__ void b2_bilinear3(char* lds, const float* cxy, int l, int Hl, int Wl, int bx0, int by0,
                                             int bw, int toff, int S, int as, int qmask, int gpix, int wave_u, int lane) {
  const int p = lane;
  if (!((qmask >> (p >> 4)) & 1)) return;
  char* arow = lds + b2_lk<PM>(as, p);
  const int sw = p & 7;
  auto put_row = [&](int iy, uint4 v) { *reinterpret_cast<uint4*>(arow + ((iy ^ sw) << 4)) = v; };
  const uint4 zero4 = uint4{0u, 0u, 0u, 0u};
  if (gpix >= 0 && gpix != p) {   // a single-pixel group: the M-block's other rows are zero
    put_row(wave_u, zero4);
    put_row(wave_u + 4, zero4);
    return;
  }
  const float scl = 1.0f / (float)(1 << l);
  const float x0 = cxy[2 * p] * scl, y0 = cxy[2 * p + 1] * scl;
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xi0 = alt_floor(x0), yi0 = alt_floor(y0);
  const _Float16 w11 = (_Float16)rnd16(dx * dy);
  const _Float16 w10 = (_Float16)rnd16(dx * (1.0f - dy));
  const _Float16 w01 = (_Float16)rnd16((1.0f - dx) * dy);
  const _Float16 w00 = (_Float16)rnd16((1.0f - dx) * (1.0f - dy));
  const int xs = xi0 - 3;
  const int lo = min(max(-xs, 0), 8), hi = max(min(Wl - xs, 8), 0);
  const unsigned cmask = hi > lo ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u;
  const bool any_partial = __builtin_amdgcn_ballot_w64(cmask != 0xffu) != 0;
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const int nr = wave_u == 3 ? 1 : 2;
  unsigned pe[2][2][4];
  int tr[2][2];
  bool okr[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int ya = yi0 - 3 + wave_u + 4 * r;
#pragma unroll
    for (int ab = 0; ab < 2; ++ab) {
      const int y = ya + ab;
      tr[r][ab] = toff + (y - by0) * bw + xs - bx0;
      okr[r][ab] = y >= 0 && y < Hl;
    }
  }
  b2_crows<PM>(lds, tr, okr, p, S, pe);
  if (any_partial) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned m = (((cmask >> (2 * q)) & 1) ? 0xffffu : 0u) | (((cmask >> (2 * q + 1)) & 1) ? 0xffff0000u : 0u);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        pe[r][0][q] &= m;
        pe[r][1][q] &= m;
      }
    }
  }
  const _Float16 z = (_Float16)0.f;
  const h2_t W00 = {w00, w00}, W01 = {w01, w01}, W10 = {w10, w10}, W11 = {w11, w11}, Z2 = {z, z};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (r >= nr) {   // wave 3: window row 7 does not exist - its piece is zero
      put_row(7, zero4);
      break;
    }
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // outputs 2q, 2q + 1 (output 7 is the zero pad)
      const h2_t ae = __builtin_bit_cast(h2_t, pe[r][0][q]), be = __builtin_bit_cast(h2_t, pe[r][1][q]);
      const unsigned an = q < 3 ? pe[r][0][q + 1] : 0u, bn = q < 3 ? pe[r][1][q + 1] : 0u;
      const h2_t ao = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(an, pe[r][0][q], 16));
      const h2_t bo = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(bn, pe[r][1][q], 16));
      h2_t v = Z2 + ae * W00;
      v = v + be * W01;
      v = v + ao * W10;
      v = v + bo * W11;
      o[q] = __builtin_bit_cast(unsigned, v);
    }
    o[3] &= 0xffffu;
    put_row(wave_u + 4 * r, uint4{o[0], o[1], o[2], o[3]});
  }
}

// Round 5, the product's bilinear (PM + row-K), in two halves so the merged
// level-3/2/1 stage can issue the next level's C reads before this level's
// lookup-tile stores (LDS stores the compiler cannot reorder loads across).
// Thread = (wave w, pixel lane): ADJACENT output rows 2w, 2w + 1 (wave 3: row
// 6 and the zero row 7), so 3 tap rows (15 aligned dwords) instead of 4 per
// thread.  The arithmetic is b2_bilinear3's, value for value.
struct B2Bl {
  unsigned d[3][5];
  unsigned bits;   // column mask (bits 0..7) | 16-bit shift of tap row j (bit 8 + j)
};
// the pixel's window origin and bilinear weights at level l (fp32 -> fp16 as
// the volume lookup's at::Half arithmetic), computed ONCE per pixel and level
// into a 16-B LDS entry - {xs (24 bits) | column mask << 24, yi0, w00 | w01 << 16,
// w10 | w11 << 16} - instead of by every wave in every bilinear pass (the
// bilinear phase is VALU-issue bound)
constexpr int kB2Win = 256 * 256;   // PM: [4 levels][64 px] uint4, past the lookup tiles
static_assert(kB2Win >= kB2Lk + 3 * 64 * 128 && kB2Win + 4 * 64 * 16 <= kB2Rows * 256, "PM window table");
__device__ __forceinline__ void b2_win_table(char* lds, const float* cxy, int l, int Wl, int p) {
  const float scl = 1.0f / (float)(1 << l);
  const float x0 = cxy[2 * p] * scl, y0 = cxy[2 * p + 1] * scl;
  const float fx0 = floorf(x0), fy0 = floorf(y0);
  const float dx = x0 - fx0, dy = y0 - fy0;
  const int xs = alt_floor(x0) - 3;
  const int lo = min(max(-xs, 0), 8), hi = max(min(Wl - xs, 8), 0);
  const unsigned cmask = hi > lo ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u;
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t wa = {(_Float16)rnd16((1.0f - dx) * (1.0f - dy)), (_Float16)rnd16((1.0f - dx) * dy)};   // w00, w01
  const h2_t wb = {(_Float16)rnd16(dx * (1.0f - dy)), (_Float16)rnd16(dx * dy)};                      // w10, w11
  *reinterpret_cast<uint4*>(lds + kB2Win + (l * 64 + p) * 16) =
      uint4{((unsigned)xs & 0xffffffu) | (cmask << 24), (unsigned)alt_floor(y0), __builtin_bit_cast(unsigned, wa),
            __builtin_bit_cast(unsigned, wb)};
}
__device__ __forceinline__ B2Bl b2_bl_prep(const char* lds, int l, int Hl, int bx0, int by0, int bw, int toff, int S,
                                           int qmask, int wave_u, int lane) {
  B2Bl st;
  const int p = lane;
  const bool on = (qmask >> (p >> 4)) & 1;
  const uint4 e = *reinterpret_cast<const uint4*>(lds + kB2Win + (l * 64 + p) * 16);
  const int xs = (int)(e.x << 8) >> 8, yi0 = (int)e.y;
  st.bits = e.x >> 24;
  const int nrow = wave_u == 3 ? 2 : 3;   // wave 3: tap rows 6, 7 (output row 6 only)
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= nrow) break;
    const int y = yi0 - 3 + 2 * wave_u + j;
    const unsigned rb = (on && y >= 0 && y < Hl) ? (unsigned)(p * S + 2 * (toff + (y - by0) * bw + xs - bx0)) : kB2Zero;
    st.bits |= (rb & 2u) << (7 + j);
#pragma unroll
    for (int i = 0; i < 5; ++i) st.d[j][i] = *reinterpret_cast<const unsigned*>(lds + (rb & ~3u) + 4 * i);
  }
  return st;
}
__device__ __forceinline__ void b2_bl_fin(char* lds, const B2Bl& st, int l, int as, int qmask, int gpix, int wave_u,
                                          int lane) {
  const int p = lane;
  if (!((qmask >> (p >> 4)) & 1)) return;
  char* arow = lds + b2_lk<true>(as, p);
  const int sw = p & 7;
  auto put_row = [&](int iy, uint4 v) { *reinterpret_cast<uint4*>(arow + ((iy ^ sw) << 4)) = v; };
  const uint4 zero4 = uint4{0u, 0u, 0u, 0u};
  if (gpix >= 0 && gpix != p) {   // a single-pixel group: the M-block's other rows are zero
    put_row(2 * wave_u, zero4);
    put_row(2 * wave_u + 1, zero4);
    return;
  }
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const int nrow = wave_u == 3 ? 2 : 3;
  unsigned pe[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j >= nrow) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) pe[j][q] = __builtin_amdgcn_alignbit(st.d[j][q + 1], st.d[j][q], ((st.bits >> (8 + j)) & 1u) * 16u);
  }
  const unsigned cmask = st.bits & 0xffu;
  if (__builtin_amdgcn_ballot_w64(cmask != 0xffu) != 0) {   // columns outside the map read zeros
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned m = (((cmask >> (2 * q)) & 1) ? 0xffffu : 0u) | (((cmask >> (2 * q + 1)) & 1) ? 0xffff0000u : 0u);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (j >= nrow) break;
        pe[j][q] &= m;
      }
    }
  }
  const _Float16 z = (_Float16)0.f;
  // the weights as two named scalars: hipcc (ROCm 7.2) miscompiles
  // __builtin_bit_cast of an ext_vector element (v[i], v.y) to element 0
  const unsigned* we = reinterpret_cast<const unsigned*>(lds + kB2Win + (l * 64 + p) * 16 + 8);
  const unsigned we0 = we[0], we1 = we[1];
  const h2_t wa = __builtin_bit_cast(h2_t, we0), wb = __builtin_bit_cast(h2_t, we1);
  const h2_t W00 = {wa[0], wa[0]}, W01 = {wa[1], wa[1]}, W10 = {wb[0], wb[0]}, W11 = {wb[1], wb[1]}, Z2 = {z, z};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (r == 1 && wave_u == 3) {   // window row 7 does not exist - its piece is zero
      put_row(7, zero4);
      break;
    }
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // outputs 2q, 2q + 1 (output 7 is the zero pad)
      const h2_t ae = __builtin_bit_cast(h2_t, pe[r][q]), be = __builtin_bit_cast(h2_t, pe[r + 1][q]);
      const unsigned an = q < 3 ? pe[r][q + 1] : 0u, bn = q < 3 ? pe[r + 1][q + 1] : 0u;
      const h2_t ao = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(an, pe[r][q], 16));
      const h2_t bo = __builtin_bit_cast(h2_t, __builtin_amdgcn_alignbit(bn, pe[r + 1][q], 16));
      h2_t v = Z2 + ae * W00;
      v = v + be * W01;
      v = v + ao * W10;
      v = v + bo * W11;
      o[q] = __builtin_bit_cast(unsigned, v);
    }
    o[3] &= 0xffffu;
    put_row(2 * wave_u + r, uint4{o[0], o[1], o[2], o[3]});
  }
}

// corr_encoder[0] slice of level L for the M-blocks in qmask from lookup tile slot `as`;
// acc[q][n] = out^T: lane (fr, fq) holds out[pixel q*16 + fr][co 32 w + 16 n + 4 fq + k]
template <int L, bool V3, bool PM>
__device__ __forceinline__ void b2_encode(const char* lds, int as, int qmask, const half8 (&wl)[4][2][2],
                                          floatx4 (&acc)[4][2], int fq, const int (&eoff)[2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!((qmask >> q) & 1)) continue;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 x = *reinterpret_cast<const half8*>(lds + b2_lk<PM>(as, q * 16) - (PM ? 0 : 128) + eoff[s]);
      if (!V3 && s == 1) {   // columns 49..63 (lanes fq 2: k 48..55, fq 3: k 56..63) are padding
        uint4 u = __builtin_bit_cast(uint4, x);
        u.x &= fq == 3 ? 0u : fq == 2 ? 0xffffu : 0xffffffffu;
        u.y = fq >= 2 ? 0u : u.y;
        u.z = fq >= 2 ? 0u : u.z;
        u.w = fq >= 2 ? 0u : u.w;
        x = __builtin_bit_cast(half8, u);
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[q][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[L][n][s], x, acc[q][n], 0, 0, 0);
    }
  }
}

// wave 0: the fallback groups of level l of a tile whose level box does not fit
// (halves, else quadrants, else the quadrant's 16 pixels' own windows) -> grp
__device__ __forceinline__ void b2_plan_groups(const AltArgs& a, const float* cxy, int l, int* grp, int lane) {
  const int Hl = a.Hl[l], Wl = a.Wl[l];
  const float scl = 1.0f / (float)(1 << l);
  const int ox = alt_floor(cxy[2 * lane] * scl) - 3, oy = alt_floor(cxy[2 * lane + 1] * scl) - 3;
  int qx0 = ox, qx1 = ox + 7, qy0 = oy, qy1 = oy + 7;
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) {
    qx0 = min(qx0, __shfl_xor(qx0, m)); qx1 = max(qx1, __shfl_xor(qx1, m));
    qy0 = min(qy0, __shfl_xor(qy0, m)); qy1 = max(qy1, __shfl_xor(qy1, m));
  }
  int hx0 = min(qx0, __shfl_xor(qx0, 16)), hx1 = max(qx1, __shfl_xor(qx1, 16));
  int hy0 = min(qy0, __shfl_xor(qy0, 16)), hy1 = max(qy1, __shfl_xor(qy1, 16));
  const int hn = alt_clip(hx0, hx1, hy0, hy1, Wl, Hl);
  const int qn = alt_clip(qx0, qx1, qy0, qy1, Wl, Hl);
  int px0 = ox, px1 = ox + 7, py0 = oy, py1 = oy + 7;
  const int pn = alt_clip(px0, px1, py0, py1, Wl, Hl);
  const bool hfit = hn <= kB2Rows, qfit = qn <= kB2Rows;
  const unsigned long long hb = __ballot(hfit), qb = __ballot(qfit);
  const int q = lane >> 4, h = lane >> 5;
  auto qcnt = [&](int qq) { return ((qb >> (16 * qq)) & 1ull) ? 1 : 16; };
  auto hcnt = [&](int hh) { return ((hb >> (32 * hh)) & 1ull) ? 1 : qcnt(2 * hh) + qcnt(2 * hh + 1); };
  const int hbase = h ? hcnt(0) : 0;
  const int qbase = hbase + ((q & 1) ? qcnt(q - 1) : 0);
  if (hfit) {
    if ((lane & 31) == 0) {
      int* g = grp + 4 + 6 * hbase;
      g[0] = hx0; g[1] = hy0; g[2] = hn ? hx1 - hx0 + 1 : 0; g[3] = hn ? hy1 - hy0 + 1 : 0;
      g[4] = 3 << (2 * h); g[5] = -1;
    }
  } else if (qfit) {
    if ((lane & 15) == 0) {
      int* g = grp + 4 + 6 * qbase;
      g[0] = qx0; g[1] = qy0; g[2] = qn ? qx1 - qx0 + 1 : 0; g[3] = qn ? qy1 - qy0 + 1 : 0;
      g[4] = 1 << q; g[5] = -1;
    }
  } else {
    int* g = grp + 4 + 6 * (qbase + (lane & 15));
    g[0] = px0; g[1] = py0; g[2] = pn ? px1 - px0 + 1 : 0; g[3] = pn ? py1 - py0 + 1 : 0;
    g[4] = 1 << q; g[5] = lane;
  }
  if (lane == 0) grp[0] = hcnt(0) + hcnt(1);
}

// corr_alt2_kernel variants (CV bits): kCvSplit - the C phase with the box
// blocks split over the waves (all four M-blocks' query rows per wave, b2_corr3);
// kCvRowK - the lookup tile in the k = 8 iy + ix order (b2_bilinear3: one 16-B
// store per window row) with corr_encoder[0]'s weights permuted to match;
// kCvPm - C pixel-major with 8-B C stores and dword window-row reads, the
// lookup tiles in their own area (b2_corr<true>, b2_crow<true>, b2_lk<true>).
// V2 = 0, V3 = kCvSplit | kCvRowK, the round-5 product = kCvRowK | kCvPm.
constexpr int kCvSplit = 1, kCvRowK = 2, kCvPm = 4;
constexpr int kAltProdCV = kCvRowK | kCvPm;
template <int CV>
__global__ void __launch_bounds__(256, 2) corr_alt2_kernel(AltArgs a) {
  constexpr bool V3 = (CV & kCvSplit) != 0;        // C split over the waves
  constexpr bool RK = (CV & kCvRowK) != 0;         // k = 8 iy + ix lookup tile
  constexpr bool PM = (CV & kCvPm) != 0;           // pixel-major C, lookup tiles apart
  static_assert(!(V3 && PM), "the split C phase writes the tap-major layout");
  static_assert(!V3 || RK, "the split C phase ships with the row-K tile only (V3)");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int* grp = reinterpret_cast<int*>(lds + kB2Grp);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int fr = lane & 15, fq = lane >> 4;
  const int H = a.H, W = a.W, HW = H * W;
  const int tcols = W / 8, tpe = (H / 8) * tcols;
  const unsigned lds_a = lds_addr(lds);

  // XCD-aware walk: the tile walk is cut into chunks of a.chunk tiles (a few
  // edges), dealt round-robin to the 8 XCDs (the workgroups blockIdx % 8 == x);
  // an XCD's workgroups interleave inside its chunks.  The edges of a chunk -
  // grouped by target frame when a.order is given - then share one L2, and all
  // XCDs still progress through the walk together (per-edge costs differ with
  // the motion, so contiguous per-XCD eighths finish unevenly).  Local step j of
  // XCD x is tile ((j / C) * 8 + x) * C + j % C, increasing in j.
  const int G = gridDim.x;
  const bool chunked = (G % 8 == 0) && a.chunk > 0;
  const int nx = chunked ? 8 : 1, xcd = (int)blockIdx.x % nx, step = G / nx;
  const int C = chunked ? a.chunk : 1;
  auto walk = [&](int j) -> int {
    return chunked ? ((j / C) * 8 + xcd) * C + j % C : j;
  };
  int j = (int)blockIdx.x / nx;
  const int b0 = walk(j);
  if (b0 >= a.ntiles) return;

  // corr_encoder[0] B fragments of this wave's 32 output channels (2 N-blocks):
  // per level K = 49 real columns padded to 64 (2 K-steps of 32)
  half8 wl[4][2][2];
#pragma unroll
  for (int l = 0; l < 4; ++l)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        half8 v;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = 32 * s + 8 * fq + i;
          // V3 lookup-tile order k = 8 iy + ix <-> the reference channel 7 ix + iy
          const int iy = k >> 3, ix = k & 7;
          const bool ok = RK ? (ix < 7 && iy < 7) : k < 49;
          const int ch = RK ? 7 * ix + iy : k;
          v[i] = ok ? (_Float16)a.w[(wave * 32 + 16 * n + fr) * 224 + 49 * l + ch] : (_Float16)0.f;
        }
        wl[l][n][s] = v;
      }
  if (tid < 128) reinterpret_cast<float*>(lds + kB2Bias)[tid] = a.bias[tid];   // read at the output staging
  int eoff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) eoff[s] = (PM ? fr * 128 : fr * 256 + 128) + (((s * 4 + fq) ^ (fr & 7)) << 4);

  struct Tile { int e, ty0, tx0, f1, f2; };
  auto tile_of = [&](int t) {
    Tile r;
    const int slot = t / tpe;   // the walk's edge slot; the tile inside the edge is the same either way
    r.e = __builtin_amdgcn_readfirstlane(a.order ? a.order[slot] : slot);
    const int tt = t - slot * tpe;
    r.ty0 = (tt / tcols) * 8;
    r.tx0 = (tt - (tt / tcols) * tcols) * 8;
    r.f1 = a.f1[r.e];
    r.f2 = a.f2[r.e];
    return r;
  };
  auto coords_dma = [&](const Tile& T, int slot) {
    if (wave_u == 0) {
      const rsrc_t rs = make_rsrc(a.coords + (long)T.e * HW * 2, (unsigned)(HW * 8));
      const int p = 2 * (lane & 31);
      if (lane < 32)
        dma16(rs, lds_a + kB2Coord + slot * 512, (unsigned)((((T.ty0 + alt_py(p)) * W + T.tx0 + alt_px(p)) * 2) * 4));
    }
  };
  // this wave's 16 query feature rows (M-block `wave`) straight into the MFMA B fragments
  // V2: M-block `wave` into af[0]; V3: all four M-blocks
  auto load_f1 = [&](const Tile& T, half8 (&af)[4][4]) {
    const unsigned long long pa =
        (unsigned long long)(a.pyr[0] + (long)__builtin_amdgcn_readfirstlane(T.f1) * HW * 128);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(pa), (short)0, HW * 256, 0x00020000);
#pragma unroll
    for (int m = 0; m < (V3 ? 4 : 1); ++m) {
      const int p = (V3 ? m : wave) * 16 + fr;
      const int pix = (T.ty0 + alt_py(p)) * W + T.tx0 + alt_px(p);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        af[m][ks] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rs, (int)((pix * 128 + (ks * 4 + fq) * 8) * 2), 0, 0));
    }
  };

  half8 af[4][4];
  floatx4 acc[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q][0] = acc[q][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  int tile_i = 0;   // profiling stamps only
  (void)tile_i;

  // one group: DMA its box, C, bilinear, encoder; ends with a barrier (the
  // region is free for the next DMA).  The level is a runtime value except in
  // the encoder (static register operands): one copy of the group code.
  auto wait_bar = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto encode = [&](int L, int as, int qmask) {
    switch (L) {
      case 3: b2_encode<3, RK, PM>(lds, as, qmask, wl, acc, fq, eoff); break;
      case 2: b2_encode<2, RK, PM>(lds, as, qmask, wl, acc, fq, eoff); break;
      case 1: b2_encode<1, RK, PM>(lds, as, qmask, wl, acc, fq, eoff); break;
      default: b2_encode<0, RK, PM>(lds, as, qmask, wl, acc, fq, eoff); break;
    }
  };
  // level L of tile T: its tile box if it fits the region, else the fallback groups
  auto run_level = [&](int L, const Tile& T, const Tile& nxt, const float* cxy, const int* lv, bool side, bool more,
                       int nslot) {
    const int Hl = a.Hl[L], Wl = a.Wl[L];
    const int bw0 = __builtin_amdgcn_readfirstlane(lv[4 * L + 2]), bh0 = __builtin_amdgcn_readfirstlane(lv[4 * L + 3]);
    const bool fits = bw0 * bh0 <= kB2Rows;
    if (!fits) {
      if (wave_u == 0) b2_plan_groups(a, cxy, L, grp, lane);
      __syncthreads();
    }
    const int ng = fits ? 1 : __builtin_amdgcn_readfirstlane(grp[0]);
    for (int gi = 0; gi < ng; ++gi) {
      const int* g = fits ? lv + 4 * L : grp + 4 + 6 * gi;
      const int gx0 = __builtin_amdgcn_readfirstlane(g[0]), gy0 = __builtin_amdgcn_readfirstlane(g[1]);
      const int gw = __builtin_amdgcn_readfirstlane(g[2]), gh = __builtin_amdgcn_readfirstlane(g[3]);
      const int qmask = fits ? 15 : __builtin_amdgcn_readfirstlane(g[4]);
      const int gpix = fits ? -1 : __builtin_amdgcn_readfirstlane(g[5]);
      b2_box_dma(a, L, T.f2, gx0, gy0, gw, gh, 0, lds_a, wave_u, lane);
      if (L == 0) B2_STAMP(8);
      wait_bar();
      if (L == 0) B2_STAMP(9);
      if (V3) b2_corr3(lds, gw * gh, qmask, af, wave_u, fr, fq);
      else b2_corr<PM>(lds, gw * gh, b2_cstride(gw * gh), qmask, af[0], wave_u, fr, fq, [&] {
          if (RK && PM && wave_u == 0) b2_win_table(lds, cxy, L, Wl, lane);   // this group's level
        });
      if (L == 0) B2_STAMP(10);
      __syncthreads();
      if (RK && PM) {
        const B2Bl bl = b2_bl_prep(lds, L, Hl, gx0, gy0, gw, 0, b2_cstride(gw * gh), qmask, wave_u, lane);
        b2_bl_fin(lds, bl, L, 0, qmask, gpix, wave_u, lane);
      } else if (RK) {
        b2_bilinear3<PM>(lds, cxy, L, Hl, Wl, gx0, gy0, gw, 0, b2_cstride(gw * gh), 0, qmask, gpix, wave_u, lane);
      } else {
        b2_bilinear<PM>(lds, cxy, L, Hl, Wl, gx0, gy0, gw, 0, b2_cstride(gw * gh), 0, qmask, gpix, wave_u, lane);
      }
      if (side && gi == ng - 1 && wave_u == 3 && more)   // the next tile's boxes, on the wave with one window row
        alt_tile_boxes(a, reinterpret_cast<const float*>(lds + kB2Coord + nslot * 512),
                       reinterpret_cast<int*>(lds + kB2Lvl) + nslot * 16, lane);
      __syncthreads();
      if (L == 0) B2_STAMP(11);
      // af for the next C phase: this level's next group, the next level, or the next tile
      encode(L, 0, qmask);
      __syncthreads();
      if (L == 0) B2_STAMP(12);
    }
  };

  // ---- prologue: tile b0's coordinates, boxes and query features ----
  int t = b0;
  int slot = 0;
  Tile cur = tile_of(t);
  coords_dma(cur, 0);
  load_f1(cur, af);
  wait_bar();
  if (wave_u == 0)
    alt_tile_boxes(a, reinterpret_cast<const float*>(lds + kB2Coord), reinterpret_cast<int*>(lds + kB2Lvl), lane);
  __syncthreads();

  for (;;) {
    j += step;
    const int tn_ = walk(j);
    const bool more = tn_ < a.ntiles;
    const Tile nxt = more ? tile_of(tn_) : cur;
    const float* cxy = reinterpret_cast<const float*>(lds + kB2Coord + slot * 512);
    const int* lv = reinterpret_cast<const int*>(lds + kB2Lvl) + slot * 16;
    // ---- levels 3, 2, 1 ----
    const int tn3 = __builtin_amdgcn_readfirstlane(lv[14] * lv[15]);
    const int tn2 = __builtin_amdgcn_readfirstlane(lv[10] * lv[11]);
    const int tn1 = __builtin_amdgcn_readfirstlane(lv[6] * lv[7]);
    const int o2 = (tn3 + 3) & ~3, o1 = o2 + ((tn2 + 3) & ~3), T321 = o1 + tn1;
    B2_STAMP(0);
    if (more) coords_dma(nxt, slot ^ 1);
    if (T321 <= kB2Rows) {
      const int toffs[3] = {0, o2, o1};
      for (int i = 0; i < 3; ++i) {
        const int L = 3 - i;
        b2_box_dma(a, L, cur.f2, __builtin_amdgcn_readfirstlane(lv[4 * L]), __builtin_amdgcn_readfirstlane(lv[4 * L + 1]),
                   __builtin_amdgcn_readfirstlane(lv[4 * L + 2]), __builtin_amdgcn_readfirstlane(lv[4 * L + 3]),
                   toffs[i], lds_a, wave_u, lane);
      }
      B2_STAMP(1);
      wait_bar();
      B2_STAMP(2);
      if (V3) b2_corr3(lds, T321, 15, af, wave_u, fr, fq);
      else b2_corr<PM>(lds, T321, b2_cstride(T321), 15, af[0], wave_u, fr, fq, [&] {
          if (RK && PM && wave_u >= 1)   // levels 1, 2, 3
            b2_win_table(lds, cxy, wave_u, wave_u == 1 ? a.Wl[1] : wave_u == 2 ? a.Wl[2] : a.Wl[3], lane);
        });
      B2_STAMP(3);
      __syncthreads();
      B2_STAMP(4);
      if (RK && PM) {   // levels 3, 2, 1 pipelined: level i + 1's C reads before level i's stores
        auto prep = [&](int L, int i) {
          return b2_bl_prep(lds, L, a.Hl[L], __builtin_amdgcn_readfirstlane(lv[4 * L]),
                            __builtin_amdgcn_readfirstlane(lv[4 * L + 1]), __builtin_amdgcn_readfirstlane(lv[4 * L + 2]),
                            toffs[i], b2_cstride(T321), 15, wave_u, lane);
        };
        const B2Bl s3 = prep(3, 0);
        const B2Bl s2 = prep(2, 1);
        b2_bl_fin(lds, s3, 3, 0, 15, -1, wave_u, lane);
        const B2Bl s1 = prep(1, 2);
        b2_bl_fin(lds, s2, 2, 1, 15, -1, wave_u, lane);
        b2_bl_fin(lds, s1, 1, 2, 15, -1, wave_u, lane);
      } else {
        for (int i = 0; i < 3; ++i) {
          const int L = 3 - i;
          if (RK)
            b2_bilinear3<PM>(lds, cxy, L, a.Hl[L], a.Wl[L], __builtin_amdgcn_readfirstlane(lv[4 * L]),
                         __builtin_amdgcn_readfirstlane(lv[4 * L + 1]), __builtin_amdgcn_readfirstlane(lv[4 * L + 2]),
                         toffs[i], b2_cstride(T321), i, 15, -1, wave_u, lane);
          else
            b2_bilinear<PM>(lds, cxy, L, a.Hl[L], a.Wl[L], __builtin_amdgcn_readfirstlane(lv[4 * L]),
                        __builtin_amdgcn_readfirstlane(lv[4 * L + 1]), __builtin_amdgcn_readfirstlane(lv[4 * L + 2]),
                        toffs[i], b2_cstride(T321), i, 15, -1, wave_u, lane);
        }
      }
      B2_STAMP(5);
      __syncthreads();
      B2_STAMP(6);
      b2_encode<3, RK, PM>(lds, 0, 15, wl, acc, fq, eoff);
      b2_encode<2, RK, PM>(lds, 1, 15, wl, acc, fq, eoff);
      b2_encode<1, RK, PM>(lds, 2, 15, wl, acc, fq, eoff);
      __syncthreads();
      B2_STAMP(7);
    } else {
      for (int L = 3; L >= 1; --L) run_level(L, cur, nxt, cxy, lv, false, more, slot ^ 1);
    }
    // ---- level 0 (its last group computes the next tile's boxes on the side) ----
    run_level(0, cur, nxt, cxy, lv, true, more, slot ^ 1);
    // ---- output: bias, ReLU -> rows staged in the first halves of rows 64..191
    // (pixel p: rows 64 + 2p, 64 + 2p + 1 = channels 0..63, 64..127; 16-B pieces
    // XOR swizzled by p & 7) -> coalesced 16-B pieces to HBM
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int px = q * 16 + fr, co0 = wave * 32 + 16 * n + 4 * fq;
        half4_t h;
        const float4 bv = *reinterpret_cast<const float4*>(lds + kB2Bias + co0 * 4);
        h[0] = (_Float16)fmaxf(acc[q][n][0] + bv.x, 0.f);
        h[1] = (_Float16)fmaxf(acc[q][n][1] + bv.y, 0.f);
        h[2] = (_Float16)fmaxf(acc[q][n][2] + bv.z, 0.f);
        h[3] = (_Float16)fmaxf(acc[q][n][3] + bv.w, 0.f);
        *reinterpret_cast<half4_t*>(lds + (64 + 2 * px + (co0 >> 6)) * 256 + (((co0 & 63) * 2) ^ ((px & 7) << 4))) = h;
        acc[q][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    __syncthreads();
    B2_STAMP(13);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + 256 * r;
      const int p = idx >> 4, pc = idx & 15;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + (64 + 2 * p + (pc >> 3)) * 256 + (((pc & 7) ^ (p & 7)) << 4));
      const long m = ((long)cur.e * H + cur.ty0 + alt_py(p)) * W + cur.tx0 + alt_px(p);
      *reinterpret_cast<uint4*>(a.out + m * 128 + pc * 8) = v;
    }
    if (more) load_f1(nxt, af);   // behind the stores: in flight during the next tile's DMA issue
    B2_STAMP(14);
    if (!more) break;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();   // staging read out before the next DMA overwrites it
    B2_STAMP(15);
    ++tile_i;
    t = tn_;
    cur = nxt;
    slot ^= 1;
  }
}
}  // namespace droid

using namespace droid;

static long long* g_alt_prof = nullptr;
static int& alt_chunk_edges() {
  static int v = std::max(0, ab_knob("DROID_ALT_CHUNK", 0));
  return v;
}
// 2 = corr_alt2_kernel (the product kernel); the A/B build adds 1 (the round-2
// one-workgroup-per-CU kernel) and 3 (corr_alt2_kernel<V3>)
static int& alt_variant() {
  static int v = [] {
    const int e = ab_knob("DROID_ALT_VARIANT", 2);
    return (e == 1 || e == 3) ? e : 2;
  }();
  return v;
}

#if DROID_AB
// the A/B build's corr_alt2_kernel variant for alt variant 2 (DROID_ALT2_CV: 0, 2, 4, 6)
static int& alt2_cv() {
  static int v = [] {
    const int e = ab_knob("DROID_ALT2_CV", kAltProdCV);
    return (e == 0 || e == kCvRowK || e == kCvPm) ? e : kAltProdCV;
  }();
  return v;
}
#endif

extern "C" {

#if DROID_TESTING
// Profiling builds (make prof): per workgroup, for its first 32 stages, 8 int64:
// s_memtime at stage start / box landed / C done / C barrier / bilinear done /
// lookup barrier / stage end, then (box taps * 2 + slow-path flag).
int droid_alt_set_profile(void* buf) {
#if DROID_CONV_PROFILE
  g_alt_prof = static_cast<long long*>(buf);
  return kOk;
#else
  (void)buf;
  return fail(kUnsupported, "alt_set_profile: build with make prof (DROID_CONV_PROFILE=1)");
#endif
}
#endif  // DROID_TESTING

int droid_corr_alt_ce0_ordered(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                               const int* order, const float* coords, const void* w, const float* bias, void* out,
                               int E, int H, int W, hipStream_t stream);

// On-the-fly CorrBlock lookup fused with corr_encoder[0] (corr_alt_ce0_kernel).
int droid_corr_alt_ce0(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                       const float* coords, const void* w, const float* bias, void* out, int E, int H, int W,
                       hipStream_t stream) {
  return droid_corr_alt_ce0_ordered(pyr, Hl, Wl, f1, f2, nullptr, coords, w, bias, out, E, H, W, stream);
}

// The same with the edges walked in `order` (a permutation of 0..E-1, device
// int32; null = 0..E-1): grouping the edges that share a target frame keeps
// that frame's pyramid rows in the XCD's L2 across their tiles' box DMAs.
// Outputs are the same bytes in the same places whatever the order.
int droid_corr_alt_ce0_ordered(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                               const int* order, const float* coords, const void* w, const float* bias, void* out,
                               int E, int H, int W, hipStream_t stream) {
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
  if ((long)H * W * 8 > 0x7fffffffL) return fail(kUnsupported, "corr_alt_ce0: coordinate plane too large");
  a.f1 = f1; a.f2 = f2; a.coords = coords; a.order = order;
  a.w = (const __half*)w; a.bias = bias; a.out = (__half*)out;
  a.H = H; a.W = W;
  a.ntiles = (long)E * (H / 8) * (W / 8);
  if (a.ntiles + device_cu_count() >= 0x7fffffffL) return fail(kUnsupported, "corr_alt_ce0: too many tiles");
  a.prof = g_alt_prof;
  // corr_alt2_kernel's XCD chunks: DROID_ALT_CHUNK edges' tiles (0, the default:
  // the plain interleaved walk - chunks of 1-32 edges measured 0-12 % slower at
  // C3, with or without the target-frame order, profiles/r04/r04n_alt_time.txt)
  const long chunk = (long)alt_chunk_edges() * (H / 8) * (W / 8);
  a.chunk = (chunk > 0 && 8 * chunk + a.ntiles < 0x7fffffffL) ? (int)chunk : 0;
  if (a.ntiles == 0) return kOk;
#if DROID_AB
  if (alt_variant() == 1) {
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
#endif
  static bool attr2 = false;
  if (!attr2) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt2_kernel<kAltProdCV>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
#if DROID_AB
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt2_kernel<kCvSplit | kCvRowK>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt2_kernel<0>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt2_kernel<kCvRowK>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_alt2_kernel<kCvPm>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds));
#endif
    attr2 = true;
  }
  // two workgroups per CU (A/B: DROID_ALT2_WG_PER_CU=1 for one)
  static const int per_cu = ab_knob("DROID_ALT2_WG_PER_CU", 2) == 1 ? 1 : 2;
  const long grid = std::min<long>(a.ntiles, (long)per_cu * device_cu_count());
#if DROID_AB
  // variant 3 = V3; variant 2 runs DROID_ALT2_CV's kernel (0 = the round-4
  // V2, 2 = row-K only, 4 = pixel-major C only, 6 = the product)
  const int cv = alt_variant() == 3 ? (kCvSplit | kCvRowK) : alt2_cv();
  if (cv != kAltProdCV) {
    const dim3 g((unsigned)grid);
    switch (cv) {
      case kCvSplit | kCvRowK: corr_alt2_kernel<kCvSplit | kCvRowK><<<g, 256, kB2Lds, stream>>>(a); break;
      case 0: corr_alt2_kernel<0><<<g, 256, kB2Lds, stream>>>(a); break;
      case kCvRowK: corr_alt2_kernel<kCvRowK><<<g, 256, kB2Lds, stream>>>(a); break;
      default: corr_alt2_kernel<kCvPm><<<g, 256, kB2Lds, stream>>>(a); break;
    }
    DROID_LAUNCH_CHECK();
    return kOk;
  }
#endif
  corr_alt2_kernel<kAltProdCV><<<dim3((unsigned)grid), 256, kB2Lds, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

#if DROID_TESTING
// A/B hook: corr_alt2_kernel's XCD chunk in edges (0, the default = the plain
// interleaved walk; in the A/B build env DROID_ALT_CHUNK sets the initial value)
int droid_alt_set_chunk(int edges) {
  if (edges < 0) return fail(kInvalidArgument, "alt_set_chunk: edges >= 0");
  alt_chunk_edges() = edges;
  return kOk;
}
#endif  // DROID_TESTING

#if DROID_TESTING
// A/B hook: 2 = corr_alt2_kernel (the product kernel); in the A/B build only:
// 1 = the one-workgroup-per-CU kernel, 3 = corr_alt2_kernel<V3>, and the
// round-5 pieces apart - 4 = the round-4 V2 (CV 0), 5 = row-K lookup tile only
// (CV 2), 6 = pixel-major C only (CV 4); env DROID_ALT_VARIANT / DROID_ALT2_CV
// set the initial values there
int droid_alt_set_variant(int v) {
  if (v < 1 || v > 6) return fail(kInvalidArgument, "alt_set_variant: 1 .. 6");
  if (!DROID_AB && v != 2) return fail(kUnsupported, "alt_set_variant: variants other than 2 ship in the A/B build only (make ab)");
#if DROID_AB
  static const int cvs[7] = {0, 0, kAltProdCV, 0, 0, kCvRowK, kCvPm};
  alt2_cv() = v == 2 || v >= 4 ? cvs[v] : alt2_cv();
  alt_variant() = v >= 4 ? 2 : v;
#else
  alt_variant() = v;
#endif
  return kOk;
}
#endif  // DROID_TESTING

}  // extern "C"
