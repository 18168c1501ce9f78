// Implicit-GEMM convolution for the update operator (droid_net.py:78-143,
// modules/gru.py:19-32) on gfx950 MFMA, NHWC fp16 in / fp32 accumulate.
//
//   out[b,y,x,co] = epilogue( sum_{tap,ci} in[b, y+ty, x+tx, ci] * W[co, tap, ci] )
//
// GEMM view: M = B*H*W pixels, N = Cout, K = taps * Cin.  A workgroup owns a
// 128-pixel x 128-channel output tile; 4 waves (2x2) each hold 4x4 tiles of
// v_mfma_f32_16x16x32_f16.  K is walked as (source, 32-channel chunk, tap):
// the A tile is gathered straight from up to 4 NHWC source tensors (the
// channel concatenations of the reference never materialise), shifted per tap
// with zero padding; the B tile is the packed weight [Cout][kstep][32].
// Both are double-buffered through LDS with one barrier per k-step.
//
// Epilogues fuse what the reference runs as separate elementwise kernels:
//   EPI_ACT   : act(acc + bias[co] + bbias[b,co]), act in {none, relu}
//   EPI_GRU_ZR: co <  Ch: z = sigmoid(.)            -> zout
//               co >= Ch: r = sigmoid(.); r*h       -> rnet
//   EPI_GRU_Q : q = tanh(.); h' = (1-z) h + z q     -> out (the new hidden state)
//   EPI_HEAD  : fp32 out, co < 2 raw (delta), co >= 2 sigmoid (weight)
//   EPI_GLO   : sigmoid(.) * h summed over the tile's pixels, atomically added
//               (scaled by 1/HW) into glo[b][co]: the GRU global-context mean
#include "common.hpp"

namespace droid {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

enum ConvEpi : int { EPI_ACT = 0, EPI_GRU_ZR = 1, EPI_GRU_Q = 2, EPI_HEAD = 3, EPI_GLO = 4 };

struct ConvSrc {
  const __half* ptr;
  int C;        // channels used (multiple of 8)
  int cstride;  // pixel stride in elements (>= C, multiple of 8)
};

struct ConvArgs {
  ConvSrc src[4];
  int nsrc;
  int chunk_end[4];  // cumulative 32-channel chunk counts per source
  int nchunk;
  const __half* wp;  // [Cout][nchunk*taps][32]
  const float* bias;   // [Cout] or null
  const float* bbias;  // [B][Cout] or null (per-image bias, e.g. the GRU global branch)
  int B, H, W, Cout, ks, act;
  int epi;
  __half* out;
  int out_cstride, out_coff;
  // GRU
  const __half* h;  // hidden state, NHWC
  int h_cstride;
  const __half* z;  // z gates from the ZR pass
  int z_cstride;
  __half* zout;
  __half* rnet;
  int gru_ch;  // hidden channels (128)
  float* out32;  // EPI_HEAD / EPI_GLO fp32 output
};

constexpr int TM = 128, TN = 128, TK = 32;
constexpr int LROW = 40;  // LDS row stride in halves (80 B: 16-B aligned, spreads banks)

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

__global__ void __launch_bounds__(256) conv_nhwc_f16_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 As[2][TM * LROW];
  __shared__ __attribute__((aligned(16))) _Float16 Bs[2][TN * LROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = a.H * a.W;
  const long Mtot = (long)a.B * HW;
  const long m0 = (long)blockIdx.x * TM;
  const int n0 = blockIdx.y * TN;
  const int taps = a.ks * a.ks;
  const int pad = a.ks >> 1;
  const int nk = a.nchunk * taps;

  // this thread's two A rows / B rows and its 8-channel piece
  const int piece = tid & 3;
  int arow[2], ab[2], ay[2], ax[2];
  bool avalid[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    arow[r] = (tid >> 2) + 64 * r;
    const long m = m0 + arow[r];
    avalid[r] = m < Mtot;
    const long mm = avalid[r] ? m : 0;
    ab[r] = (int)(mm / HW);
    const int p = (int)(mm % HW);
    ay[r] = p / a.W;
    ax[r] = p % a.W;
  }

  auto load_tiles = [&](int ks, uint4* ra, uint4* rb) {
    const int chunk = ks / taps;
    const int tap = ks - chunk * taps;
    const int ty = tap / a.ks - pad, tx = tap % a.ks - pad;
    int s = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q + 1 < a.nsrc && chunk >= a.chunk_end[q]) s = q + 1;
    const int cc = chunk - (s ? a.chunk_end[s - 1] : 0);
    const ConvSrc src = a.src[s];
    const int c = cc * TK + piece * 8;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int y = ay[r] + ty, x = ax[r] + tx;
      const bool ok = avalid[r] && c < src.C && y >= 0 && y < a.H && x >= 0 && x < a.W;
      ra[r] = ok ? *reinterpret_cast<const uint4*>(src.ptr + ((long)ab[r] * HW + (long)y * a.W + x) * src.cstride + c)
                 : make_uint4(0, 0, 0, 0);
      const int co = n0 + arow[r];
      rb[r] = (co < a.Cout) ? *reinterpret_cast<const uint4*>(a.wp + ((long)co * nk + ks) * TK + piece * 8)
                            : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tiles = [&](int buf, const uint4* ra, const uint4* rb) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      *reinterpret_cast<uint4*>(&As[buf][arow[r] * LROW + piece * 8]) = ra[r];
      *reinterpret_cast<uint4*>(&Bs[buf][arow[r] * LROW + piece * 8]) = rb[r];
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[2], rb[2];
  load_tiles(0, ra, rb);
  store_tiles(0, ra, rb);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  int cur = 0;
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) load_tiles(ks + 1, ra, rb);
    half8 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = *reinterpret_cast<const half8*>(&As[cur][(wm * 64 + i * 16 + fr) * LROW + fk]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bf[j] = *reinterpret_cast<const half8*>(&Bs[cur][(wn * 64 + j * 16 + fr) * LROW + fk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    if (more) store_tiles(cur ^ 1, ra, rb);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: lane holds rows 4*(lane>>4)+k, column lane&15 of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + k;
      if (m >= Mtot) continue;
      const int b = (int)(m / HW);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = n0 + wn * 64 + j * 16 + fr;
        if (co >= a.Cout) continue;
        float v = acc[i][j][k];
        if (a.bias) v += a.bias[co];
        if (a.bbias) v += a.bbias[(long)b * a.Cout + co];
        if (a.epi == EPI_ACT) {
          if (a.act == 1) v = fmaxf(v, 0.f);
          a.out[m * a.out_cstride + a.out_coff + co] = __float2half(v);
        } else if (a.epi == EPI_GRU_ZR) {
          const float g = sigmoidf_(v);
          if (co < a.gru_ch) {
            a.zout[m * a.gru_ch + co] = __float2half(g);
          } else {
            const int c = co - a.gru_ch;
            const float hv = __half2float(a.h[m * a.h_cstride + c]);
            a.rnet[m * a.gru_ch + c] = __float2half(g * hv);
          }
        } else if (a.epi == EPI_HEAD) {
          a.out32[m * a.out_cstride + co] = (co >= 2) ? sigmoidf_(v) : v;
        } else if (a.epi == EPI_GLO) {
          acc[i][j][k] = sigmoidf_(v) * __half2float(a.h[m * a.h_cstride + co]);
        } else {  // EPI_GRU_Q
          const float q = tanhf(v);
          const float zv = __half2float(a.z[m * a.z_cstride + co]);
          const float hv = __half2float(a.h[m * a.h_cstride + co]);
          a.out[m * a.out_cstride + a.out_coff + co] = __float2half((1.0f - zv) * hv + zv * q);
        }
      }
    }
  }
  if (a.epi == EPI_GLO) {
    // all 128 pixels of the tile belong to one image (HW % 128 == 0, checked
    // by the host): sum each column over rows, then one atomic per column.
    const long mrow = m0 + wm * 64;
    if (mrow < Mtot) {
      const int b = (int)(mrow / HW);
      const float inv = 1.0f / (float)HW;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sacc = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const long m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + k;
            sacc += (m < Mtot) ? acc[i][j][k] : 0.f;
          }
        sacc += __shfl_xor(sacc, 16);
        sacc += __shfl_xor(sacc, 32);
        const int co = n0 + wn * 64 + j * 16 + fr;
        if (lane < 16 && co < a.Cout) atomicAdd(a.out32 + (long)b * a.Cout + co, sacc * inv);
      }
    }
  }
}

}  // namespace droid

using namespace droid;

extern "C" {

// srcs/C/cstride: nsrc NHWC fp16 inputs concatenated along channels.
// wp: packed weights [Cout][sum_s ceil(C_s/32) * ks*ks][32] fp16 (see droid_mi355x.fused).
// epi: 0 act (act 0 none / 1 relu) -> out fp16 NHWC slice; 1 GRU z|r; 2 GRU q;
// 3 head (fp32 out32, sigmoid on co >= 2); 4 GRU global mean (atomic fp32 out32, zeroed by caller).
int droid_conv_nhwc_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                        const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                        int Cout, int ks, int act, int epi, void* out, int out_cstride, int out_coff,
                        const void* h, int h_cstride, const void* z, int z_cstride, void* zout,
                        void* rnet, int gru_ch, void* out32, hipStream_t stream) {
  if (nsrc < 1 || nsrc > 4 || B < 0 || H <= 0 || W <= 0 || Cout <= 0 || ks < 1 || ks > 7 || !(ks & 1))
    return fail(kInvalidArgument, "conv_nhwc_f16: bad arguments");
  if (epi == EPI_GLO && (H * W) % TM != 0)
    return fail(kUnsupported, "conv_nhwc_f16: global-context epilogue needs H*W % 128 == 0");
  ConvArgs a{};
  int chunks = 0;
  for (int s = 0; s < nsrc; ++s) {
    if (C[s] % 8 || cstride[s] % 8 || cstride[s] < C[s] || (reinterpret_cast<uintptr_t>(srcs[s]) & 15))
      return fail(kInvalidArgument, "conv_nhwc_f16: channels/strides must be multiples of 8, 16-B aligned");
    a.src[s].ptr = (const __half*)srcs[s];
    a.src[s].C = C[s];
    a.src[s].cstride = cstride[s];
    chunks += ceil_div(C[s], TK);
    a.chunk_end[s] = chunks;
  }
  a.nsrc = nsrc;
  a.nchunk = chunks;
  a.wp = (const __half*)wp;
  a.bias = bias;
  a.bbias = bbias;
  a.B = B; a.H = H; a.W = W; a.Cout = Cout; a.ks = ks; a.act = act; a.epi = epi;
  a.out = (__half*)out; a.out_cstride = out_cstride; a.out_coff = out_coff;
  a.h = (const __half*)h; a.h_cstride = h_cstride;
  a.z = (const __half*)z; a.z_cstride = z_cstride;
  a.zout = (__half*)zout; a.rnet = (__half*)rnet; a.gru_ch = gru_ch;
  a.out32 = (float*)out32;
  if (B == 0) return kOk;
  const long M = (long)B * H * W;
  dim3 grid((unsigned)ceil_div((int)((M + TM - 1) / TM), 1), ceil_div(Cout, TN));
  conv_nhwc_f16_kernel<<<grid, 256, 0, stream>>>(a);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
