// Dense bundle adjustment kernels for gfx950 (see ba.hpp for the pipeline).
// Numerics follow ba_cuda (droid_kernels.cu:176-424, 854-1434): fp32
// linearisation and Schur products, fp64 reduced system and Cholesky.
#include <cstring>
#include <string>

#include "ba.hpp"
#include "common.hpp"

namespace droid {

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct BaDev {
  // problem data
  float* poses;             // (N,7), updated in place
  float* disps;             // (N,H,W), updated in place
  const float* intr;        // (4)
  const float* disps_sens;  // (N,H,W)
  const float* targets;     // (E,2,H,W)
  const float* weights;     // (E,2,H,W)
  const float* eta;         // (eta_rows,H,W)
  float* dx;                // (P,6) out
  float* dz;                // (K,HW) out
  // plan
  const int *ii, *jj, *kx, *feptr, *fedges, *frptr, *rpose, *redge, *fnb, *fgoff;
  const int *blka, *blkb, *blkcptr, *rhscptr, *rhspos;
  const int4 *contrib, *rhscontrib;
  const int *widef, *wideeoff, *widetasks;  // wide-path frames, their Ei image offsets, (w, IB, JB) tasks
  const int* slot;                          // tile slot map of the factor [nbr*nbc]
  float* hpart;
  float* gram;
  float* qw;
  float* ei;                                // Ei images of the wide-path frames (6 x HW each)
  double* M;                                // factor tiles, slot s at M + kTile*s
  double* x;
  int* flag;
  int E, N, H, W, HW, t0, t1, P, K, n, nbc, eta_rows, nsplit, nchunk, gpw, nblk, nwide;
  float lm, ep;
};

// ---------------------------------------------------------------------------
// Per-pixel linearisation of one edge (projective_transform_kernel :281-378).
// ---------------------------------------------------------------------------
struct PixLin {
  float wu, wv, ru, rv, Jzu, Jzv;
  float Jju[6], Jjv[6];
  float C, bz;  // wu*Jzu^2 + wv*Jzv^2, wu*ru*Jzu + wv*rv*Jzv (before the stereo zeroing)
};

__device__ __forceinline__ void linearize_pixel(const SE3f& T, bool stereo, float fx, float fy,
                                                float cx, float cy, float u, float v, float disp,
                                                float tu, float tv, float wtu, float wtv,
                                                PixLin& L) {
  const float Xi[4] = {(u - cx) / fx, (v - cy) / fy, 1.0f, disp};
  float Xj[4];
  act_se3(T, Xi, Xj);
  const float x = Xj[0], y = Xj[1], h = Xj[3];
  const bool bad = Xj[2] < kMinDepth;
  const float d = bad ? 0.0f : 1.0f / Xj[2];
  const float d2 = d * d;
  float wu = bad ? 0.0f : 0.001f * wtu;
  float wv = bad ? 0.0f : 0.001f * wtv;
  L.ru = tu - (fx * d * x + cx);
  L.rv = tv - (fy * d * y + cy);
  L.Jju[0] = fx * (h * d);
  L.Jju[1] = fx * 0.0f;
  L.Jju[2] = fx * (-x * h * d2);
  L.Jju[3] = fx * (-x * y * d2);
  L.Jju[4] = fx * (1 + x * x * d2);
  L.Jju[5] = fx * (-y * d);
  L.Jzu = fx * (T.t[0] * d - T.t[2] * (x * d2));
  L.Jjv[0] = fy * 0.0f;
  L.Jjv[1] = fy * (h * d);
  L.Jjv[2] = fy * (-y * h * d2);
  L.Jjv[3] = fy * (-1 - y * y * d2);
  L.Jjv[4] = fy * (x * y * d2);
  L.Jjv[5] = fy * (x * d);
  L.Jzv = fy * (T.t[1] * d - T.t[2] * (y * d2));
  L.C = wu * L.Jzu * L.Jzu;
  L.bz = wu * L.ru * L.Jzu;
  L.C += wv * L.Jzv * L.Jzv;
  L.bz += wv * L.rv * L.Jzv;
  if (stereo) { wu = 0.0f; wv = 0.0f; }
  L.wu = wu;
  L.wv = wv;
}

__device__ __forceinline__ void ji_from_jj(const SE3f& T, const float* Jj, float* Ji) {
  adj_se3(T, Jj, Ji);
#pragma unroll
  for (int n = 0; n < 6; ++n) Ji[n] = -Ji[n];
}

// ---------------------------------------------------------------------------
// Wave64 transpose-reduction of 128 per-lane values: after it, lane l holds the
// wave totals of values 2l and 2l+1 in v[0], v[1] (126 shuffles, not 128*6).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_transpose_reduce128(float* v, int lane) {
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int off = 32 >> s;
    const int n = 64 >> s;
    const bool upper = (lane & off) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const float send = upper ? v[k] : v[k + n];
      const float keep = upper ? v[k + n] : v[k];
      v[k] = keep + __shfl_xor(send, off);
    }
  }
}

// ---------------------------------------------------------------------------
// Kernel A: per-edge 12x12 Hessian (upper triangle, reference order) and
// gradient, reduced over a pixel split.  grid = (nsplit, E), 256 threads.
// ---------------------------------------------------------------------------
// Zero-fill of a workspace region as a kernel (16-B stores; sizes and offsets
// here are multiples of 16 B): in a captured HIP graph the solve's resets are
// then kernel nodes like the rest of the chain, not runtime memset nodes.
__global__ void __launch_bounds__(256) ba_zero_kernel(uint4* __restrict__ p, long n16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) p[i] = uint4{0u, 0u, 0u, 0u};
}

// Every region it is given is a 16-B aligned multiple of 16 B by the plan's
// workspace layout (ba_plan.cpp aligns each section); anything else is a
// layout bug and is rejected - there is no runtime-memset fallback, so no
// memset node can enter a captured solve.
static int ba_zero(void* p, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return kOk;
  if ((reinterpret_cast<uintptr_t>(p) & 15u) || (bytes & 15u))
    return fail(kInvalidArgument, "ba: workspace region not 16-B aligned (layout bug)");
  const long n16 = (long)(bytes / 16);
  const long grid = std::min<long>((n16 + 255) / 256, 1024);
  ba_zero_kernel<<<dim3((unsigned)grid), 256, 0, stream>>>(static_cast<uint4*>(p), n16);
  DROID_LAUNCH_CHECK();
  return kOk;
}

__global__ void __launch_bounds__(256) ba_edge_hessian_kernel(BaDev d) {
  __shared__ float red[4][128];
  const int e = blockIdx.y, split = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = d.ii[e], j = d.jj[e];
  const bool stereo = (i == j);
  float acc[128];
#pragma unroll
  for (int k = 0; k < 128; ++k) acc[k] = 0.0f;
  if (!stereo) {  // stereo edges have wu = wv = 0: H and v are exactly zero
    const SE3f T = rel_se3(d.poses + 7 * i, d.poses + 7 * j);
    const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
    const int HW = d.HW;
    const int p0 = (int)((long)split * HW / d.nsplit), p1 = (int)((long)(split + 1) * HW / d.nsplit);
    const float* tg = d.targets + (long)e * 2 * HW;
    const float* wt = d.weights + (long)e * 2 * HW;
    const float* dp = d.disps + (long)i * HW;
    // the next pixel's five inputs are loaded before this one is linearised, so
    // their HBM latency hides under the ~200 FMAs of the current pixel (164 ->
    // 145 us at C3).  Measured and dropped: summing only S = sum w Jj Jj^T and
    // g = sum w r Jj and mapping them through Ji = -Adj(Tij)^T Jj once per edge
    // (3.3x fewer FMAs, 27 instead of 90 accumulators): M S M^T cancels for
    // long baselines, and even with fp64 sums it moved C3 results across the
    // 1e-4 parity bar, where the reference's per-pixel accumulation stays inside.
    int p = p0 + threadIdx.x;
    float nd = 0.f, ntu = 0.f, ntv = 0.f, nwu = 0.f, nwv = 0.f;
    if (p < p1) { nd = dp[p]; ntu = tg[p]; ntv = tg[HW + p]; nwu = wt[p]; nwv = wt[HW + p]; }
    for (; p < p1; p += 256) {
      const float cd = nd, ctu = ntu, ctv = ntv, cwu = nwu, cwv = nwv;
      const int q = p + 256;
      if (q < p1) { nd = dp[q]; ntu = tg[q]; ntv = tg[HW + q]; nwu = wt[q]; nwv = wt[HW + q]; }
      PixLin L;
      linearize_pixel(T, false, fx, fy, cx, cy, (float)(p % d.W), (float)(p / d.W), cd, ctu, ctv, cwu, cwv, L);
      float Jx[12];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float w = c ? L.wv : L.wu;
        const float r = c ? L.rv : L.ru;
        const float* Jj = c ? L.Jjv : L.Jju;
        ji_from_jj(T, Jj, Jx);
#pragma unroll
        for (int k = 0; k < 6; ++k) Jx[6 + k] = Jj[k];
        int l = 0;
#pragma unroll
        for (int nn = 0; nn < 12; ++nn) {
#pragma unroll
          for (int m = 0; m <= nn; ++m) {
            acc[l] += w * Jx[nn] * Jx[m];
            ++l;
          }
        }
#pragma unroll
        for (int nn = 0; nn < 12; ++nn) acc[78 + nn] += w * r * Jx[nn];
      }
    }
  }
  wave_transpose_reduce128(acc, lane);
  red[wave][2 * lane + 0] = acc[0];
  red[wave][2 * lane + 1] = acc[1];
  __syncthreads();
  if (threadIdx.x < kHessVals) {
    const int k = threadIdx.x;
    const float s = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
    d.hpart[((long)e * d.nsplit + split) * kHessStride + k] = s;
  }
}

// ---------------------------------------------------------------------------
// Kernel B: per depth frame f, per pixel chunk.  For every pixel:
//   C = sum_e wu Jzu^2 + wv Jzv^2 + prior,  w = sum_e ... - prior,  Q = 1/C
//   E rows: [Ei = sum_e wJz*Ji (if pose f optimised), Eij_e = wJz*Jj for each edge]
// and accumulate the Gram G = [E; w] diag(Q) [E; w]^T on f32 MFMA 16x16x4
// (this is S = E Q E^T and the Schur rhs E Q w in one product).
// grid = (nchunk, K), 256 threads, dynamic LDS = 4 * NB*16 * kLdsRow floats.
// ---------------------------------------------------------------------------
template <int NB>
__global__ void __launch_bounds__(256) ba_frame_schur_kernel(BaDev d) {
  constexpr int NT = NB * (NB + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ float Tsh[24 * 8];  // per-edge relative poses (<= 21 edges)
  const int f = blockIdx.y, chunk = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = d.HW;
  const int kf = d.kx[f];
  const int e0 = d.feptr[f], e1 = d.feptr[f + 1];
  const int r0 = d.frptr[f], r1 = d.frptr[f + 1];
  const int nrows = r1 - r0;
  const bool has_ei = nrows > 0 && d.redge[r0] < 0;
  const int ei_off = has_ei ? 1 : 0;
  const int nb = d.fnb[f];
  if (nb > NB) return;  // a wide-path frame (ba_frame_prep + ba_frame_gram_wide)
  const int nv = 6 * nrows + 1;
  const int wcol = 6 * nrows;
  float* m = lds + wave * (NB * 16 * kLdsRow);

  if ((int)threadIdx.x < e1 - e0) {
    const int e = d.fedges[e0 + threadIdx.x];
    const int jx = d.jj[e];
    SE3f T = (jx == kf) ? stereo_se3() : rel_se3(d.poses + 7 * kf, d.poses + 7 * jx);
    float* o = Tsh + 8 * threadIdx.x;
    o[0] = T.t[0]; o[1] = T.t[1]; o[2] = T.t[2];
    o[3] = T.q[0]; o[4] = T.q[1]; o[5] = T.q[2]; o[6] = T.q[3];
    o[7] = (jx == kf) ? 1.0f : 0.0f;
  }
  for (int v = nv; v < NB * 16; ++v) m[v * kLdsRow + lane] = 0.0f;
  __syncthreads();

  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};

  const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
  const int er = (d.eta_rows == 1) ? 0 : f;
  for (int g = 0; g < d.gpw; ++g) {
    const int px = (chunk * d.gpw + g) * 256 + wave * 64 + lane;
    if (px < HW) {
      const float u = (float)(px % d.W), v = (float)(px / d.W);
      const float disp = d.disps[(long)kf * HW + px];
      float C = 0.f, w = 0.f;
      float Ei[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int k = e0; k < e1; ++k) {
        const int e = d.fedges[k];
        const float* to = Tsh + 8 * (k - e0);
        SE3f T;
        T.t[0] = to[0]; T.t[1] = to[1]; T.t[2] = to[2];
        T.q[0] = to[3]; T.q[1] = to[4]; T.q[2] = to[5]; T.q[3] = to[6];
        const bool stereo = to[7] != 0.0f;
        const float* tg = d.targets + (long)e * 2 * HW;
        const float* wt = d.weights + (long)e * 2 * HW;
        PixLin L;
        linearize_pixel(T, stereo, fx, fy, cx, cy, u, v, disp, tg[px], tg[HW + px], wt[px],
                        wt[HW + px], L);
        C += L.C;
        w += L.bz;
        const float au = L.wu * L.Jzu, av = L.wv * L.Jzv;
        float Ji[6];
        float* mr = m + (6 * (ei_off + k - e0)) * kLdsRow + lane;
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) mr[nn * kLdsRow] = au * L.Jju[nn] + av * L.Jjv[nn];
        if (has_ei) {
          ji_from_jj(T, L.Jju, Ji);
#pragma unroll
          for (int nn = 0; nn < 6; ++nn) Ei[nn] += au * Ji[nn];
          ji_from_jj(T, L.Jjv, Ji);
#pragma unroll
          for (int nn = 0; nn < 6; ++nn) Ei[nn] += av * Ji[nn];
        }
      }
      // depth prior / damping (droid_kernels.cu:1396-1400)
      const float ds = d.disps_sens[(long)kf * HW + px];
      const bool msk = ds > 0.0f;
      const float alpha = 0.05f;
      C = msk ? (C + alpha) : (C + d.eta[(long)er * HW + px]);
      if (msk) w = w - alpha * (disp - ds);
      const float Q = 1.0f / C;
      d.qw[(long)f * HW + px] = Q;
      d.qw[(long)d.K * HW + (long)f * HW + px] = w;
      const float sq = sqrtf(Q);
      if (has_ei) {
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) m[nn * kLdsRow + lane] = Ei[nn];
      }
      for (int vv = 0; vv < wcol; ++vv) m[vv * kLdsRow + lane] *= sq;
      m[wcol * kLdsRow + lane] = sq * w;
    } else {
      for (int vv = 0; vv < nv; ++vv) m[vv * kLdsRow + lane] = 0.0f;
    }
    __syncthreads();
    const int ar = lane & 15, ak = lane >> 4;
#pragma unroll
    for (int I = 0; I < NB; ++I) {
#pragma unroll
      for (int J = I; J < NB; ++J) {
        constexpr int dummy = 0;
        (void)dummy;
        const int t = I * NB - I * (I - 1) / 2 + (J - I);
        if (I < nb && J < nb) {
          const float* ma = m + (16 * I + ar) * kLdsRow + ak;
          const float* mb = m + (16 * J + ar) * kLdsRow + ak;
#pragma unroll
          for (int s = 0; s < 16; ++s)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ma[4 * s], mb[4 * s], acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // cross-wave reduction and store: lane l, reg k -> row 4*(l>>4)+k, col l&15
  float* red = lds;
  const int Tf = nb * (nb + 1) / 2;
#pragma unroll
  for (int I = 0; I < NB; ++I) {
#pragma unroll
    for (int J = I; J < NB; ++J) {
      const int t = I * NB - I * (I - 1) / 2 + (J - I);
      if (I < nb && J < nb) {
#pragma unroll
        for (int k = 0; k < 4; ++k) red[wave * 256 + (4 * (lane >> 4) + k) * 16 + (lane & 15)] = acc[t][k];
        __syncthreads();
        const int tf = I * nb - I * (I - 1) / 2 + (J - I);
        const int idx = threadIdx.x;
        const float s = (red[idx] + red[256 + idx]) + (red[512 + idx] + red[768 + idx]);
        d.gram[(long)d.fgoff[f] + ((long)chunk * Tf + tf) * 256 + idx] = s;
        __syncthreads();
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Wide path, for frames whose Gram [E w]^T Q [E w] is larger than kNbMax
// 16-row tiles a side (more than 20 outgoing edges; the reference has no
// degree limit).  Kernel B1: per pixel of each wide frame, C / w / Q over all
// of its edges (any count: the relative poses are staged 256 edges at a time)
// and the Ei row; grid = (ceil(HW/256), nwide).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stash_rel_pose(const BaDev& d, int kf, int e, float* o) {
  const int jx = d.jj[e];
  const SE3f T = (jx == kf) ? stereo_se3() : rel_se3(d.poses + 7 * kf, d.poses + 7 * jx);
  o[0] = T.t[0]; o[1] = T.t[1]; o[2] = T.t[2];
  o[3] = T.q[0]; o[4] = T.q[1]; o[5] = T.q[2]; o[6] = T.q[3];
  o[7] = (jx == kf) ? 1.0f : 0.0f;
}
__device__ __forceinline__ SE3f unstash_rel_pose(const float* to, bool& stereo) {
  SE3f T;
  T.t[0] = to[0]; T.t[1] = to[1]; T.t[2] = to[2];
  T.q[0] = to[3]; T.q[1] = to[4]; T.q[2] = to[5]; T.q[3] = to[6];
  stereo = to[7] != 0.0f;
  return T;
}

__global__ void __launch_bounds__(256) ba_frame_prep_kernel(BaDev d) {
  __shared__ float Tsh[256 * 8];
  const int wf = blockIdx.y;
  const int f = d.widef[wf];
  const int HW = d.HW;
  const int kf = d.kx[f];
  const int e0 = d.feptr[f], e1 = d.feptr[f + 1];
  const bool has_ei = d.redge[d.frptr[f]] < 0;
  const int px = blockIdx.x * 256 + threadIdx.x;
  const bool live = px < HW;
  const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
  const float u = (float)(px % d.W), v = (float)(px / d.W);
  const float disp = live ? d.disps[(long)kf * HW + px] : 0.0f;
  float C = 0.f, w = 0.f;
  float Ei[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int base = e0; base < e1; base += 256) {
    const int cnt = min(256, e1 - base);
    __syncthreads();
    if ((int)threadIdx.x < cnt) stash_rel_pose(d, kf, d.fedges[base + threadIdx.x], Tsh + 8 * threadIdx.x);
    __syncthreads();
    if (!live) continue;
    for (int q = 0; q < cnt; ++q) {
      const int e = d.fedges[base + q];
      bool stereo;
      const SE3f T = unstash_rel_pose(Tsh + 8 * q, stereo);
      const float* tg = d.targets + (long)e * 2 * HW;
      const float* wt = d.weights + (long)e * 2 * HW;
      PixLin L;
      linearize_pixel(T, stereo, fx, fy, cx, cy, u, v, disp, tg[px], tg[HW + px], wt[px], wt[HW + px], L);
      C += L.C;
      w += L.bz;
      if (has_ei) {
        const float au = L.wu * L.Jzu, av = L.wv * L.Jzv;
        float Ji[6];
        ji_from_jj(T, L.Jju, Ji);
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) Ei[nn] += au * Ji[nn];
        ji_from_jj(T, L.Jjv, Ji);
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) Ei[nn] += av * Ji[nn];
      }
    }
  }
  if (!live) return;
  const int er = (d.eta_rows == 1) ? 0 : f;
  const float ds = d.disps_sens[(long)kf * HW + px];
  const bool msk = ds > 0.0f;
  const float alpha = 0.05f;
  C = msk ? (C + alpha) : (C + d.eta[(long)er * HW + px]);
  if (msk) w = w - alpha * (disp - ds);
  d.qw[(long)f * HW + px] = 1.0f / C;
  d.qw[(long)d.K * HW + (long)f * HW + px] = w;
  if (has_ei) {
    float* eo = d.ei + d.wideeoff[wf];
#pragma unroll
    for (int nn = 0; nn < 6; ++nn) eo[(long)nn * HW + px] = Ei[nn];
  }
}

// ---------------------------------------------------------------------------
// Kernel B2: one 64x64-variable block pair (IB <= JB) of a wide frame's Gram,
// per pixel chunk.  Each wave images the scaled variables of both blocks for
// 64 pixels in LDS (an edge row is re-linearised only by the blocks that hold
// its variables; the Ei row comes from B1's image) and multiplies them on f32
// MFMA 16x16x4; the result goes to the same per-frame tile layout as Kernel B,
// so the assembly is unchanged.  grid = (nchunk, #block pairs),
// dynamic LDS = 4 waves x 128 rows x kLdsRow floats.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ba_frame_gram_wide_kernel(BaDev d) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ float Tsh[32 * 8];
  __shared__ int rsh[32];
  const int task = blockIdx.y, chunk = blockIdx.x;
  const int wf = d.widetasks[3 * task], IB = d.widetasks[3 * task + 1], JB = d.widetasks[3 * task + 2];
  const int f = d.widef[wf];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = d.HW;
  const int kf = d.kx[f];
  const int e0 = d.feptr[f];
  const int r0 = d.frptr[f], r1 = d.frptr[f + 1];
  const int nrows = r1 - r0;
  const bool has_ei = d.redge[r0] < 0;
  const int ei_off = has_ei ? 1 : 0;
  const int nb = d.fnb[f];
  const int wcol = 6 * nrows, nv = wcol + 1;
  const bool same = IB == JB;
  // rows (0..nrows; row nrows = the w column) holding the variables of each block
  const int va0 = 64 * IB, vb0 = 64 * JB;
  const int ra0 = va0 / 6, ra1 = min((va0 + 63) / 6, nrows);
  const int rb0 = vb0 / 6, rb1 = min((vb0 + 63) / 6, nrows);
  const int na = ra1 - ra0 + 1, nbr_ = same ? 0 : rb1 - rb0 + 1;
  if ((int)threadIdx.x < na + nbr_) {
    const int q = threadIdx.x;
    const int rho = q < na ? ra0 + q : rb0 + (q - na);
    rsh[q] = rho;
    if (rho >= ei_off && rho < nrows) stash_rel_pose(d, kf, d.fedges[e0 + rho - ei_off], Tsh + 8 * q);
  }
  float* m = lds + wave * (128 * kLdsRow);
  float* mb = same ? m : m + 64 * kLdsRow;
  __syncthreads();

  floatx4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
  const float* eo = d.ei + d.wideeoff[wf];
  for (int g = 0; g < d.gpw; ++g) {
    const int px = (chunk * d.gpw + g) * 256 + wave * 64 + lane;
    const bool live = px < HW;
    const float sq = live ? sqrtf(d.qw[(long)f * HW + px]) : 0.0f;
    const float u = (float)(px % d.W), v = (float)(px / d.W);
    const float disp = live ? d.disps[(long)kf * HW + px] : 0.0f;
    for (int q = 0; q < na + nbr_; ++q) {
      const int rho = rsh[q];
      float val[6];
      int nval = 6;
      if (rho == nrows) {  // the w column
        val[0] = live ? sq * d.qw[(long)d.K * HW + (long)f * HW + px] : 0.0f;
        nval = 1;
      } else if (rho < ei_off) {  // the Ei row
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) val[nn] = live ? sq * eo[(long)nn * HW + px] : 0.0f;
      } else {
        const int e = d.fedges[e0 + rho - ei_off];
        bool stereo;
        const SE3f T = unstash_rel_pose(Tsh + 8 * q, stereo);
        PixLin L;
        if (live) {
          const float* tg = d.targets + (long)e * 2 * HW;
          const float* wt = d.weights + (long)e * 2 * HW;
          linearize_pixel(T, stereo, fx, fy, cx, cy, u, v, disp, tg[px], tg[HW + px], wt[px], wt[HW + px], L);
        }
        const float au = live ? L.wu * L.Jzu : 0.0f, av = live ? L.wv * L.Jzv : 0.0f;
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) val[nn] = live ? sq * (au * L.Jju[nn] + av * L.Jjv[nn]) : 0.0f;
      }
      const int vbase = (rho == nrows) ? wcol : 6 * rho;
      float* dst = q < na ? m : mb;
      const int b0 = q < na ? va0 : vb0;
      for (int c = 0; c < nval; ++c) {
        const int l = vbase + c - b0;
        if (l >= 0 && l < 64) dst[l * kLdsRow + lane] = val[c];
      }
    }
    // variables past the frame's last one are zero rows
    for (int l = max(0, nv - va0); l < 64; ++l) m[l * kLdsRow + lane] = 0.0f;
    if (!same)
      for (int l = max(0, nv - vb0); l < 64; ++l) mb[l * kLdsRow + lane] = 0.0f;
    __syncthreads();
    const int ar = lane & 15, ak = lane >> 4;
#pragma unroll
    for (int I = 0; I < 4; ++I) {
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        if (same && J < I) continue;
        const float* pa = m + (16 * I + ar) * kLdsRow + ak;
        const float* pb = mb + (16 * J + ar) * kLdsRow + ak;
#pragma unroll
        for (int s = 0; s < 16; ++s)
          acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * s], pb[4 * s], acc[I][J], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // cross-wave reduction and store (lane l, reg k -> row 4*(l>>4)+k, col l&15)
  float* red = lds;
  const int Tf = nb * (nb + 1) / 2;
#pragma unroll
  for (int I = 0; I < 4; ++I) {
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      const int GI = 4 * IB + I, GJ = 4 * JB + J;
      if ((same && J < I) || GI >= nb || GJ >= nb) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) red[wave * 256 + (4 * (lane >> 4) + k) * 16 + (lane & 15)] = acc[I][J][k];
      __syncthreads();
      const int tf = GI * nb - GI * (GI - 1) / 2 + (GJ - GI);
      const int idx = threadIdx.x;
      const float s = (red[idx] + red[256 + idx]) + (red[512 + idx] + red[768 + idx]);
      d.gram[(long)d.fgoff[f] + ((long)chunk * Tf + tf) * 256 + idx] = s;
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// Kernel C: deterministic assembly of the lower triangle of A - S (fp64) and
// of the rhs b - E Q w into row n, in the permuted pose order, into the 64x64
// tiles of the factor.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float hess_val(const float* H, int r, int c) {
  if (r < c) { int t = r; r = c; c = t; }
  return H[r * (r + 1) / 2 + c];
}

// chunks c0, c0 + cstep, ... of the per-chunk Gram partials of element (i, j)
__device__ __forceinline__ double gram_sum(const BaDev& d, int f, int i, int j, int c0, int cstep) {
  if (i > j) { int t = i; i = j; j = t; }
  const int nb = d.fnb[f];
  const int I = i >> 4, J = j >> 4;
  const int tf = I * nb - I * (I - 1) / 2 + (J - I);
  const int Tf = nb * (nb + 1) / 2;
  const float* g = d.gram + d.fgoff[f] + (long)tf * 256 + (i & 15) * 16 + (j & 15);
  double s = 0.0;
  for (int c = c0; c < d.nchunk; c += cstep) s += (double)g[(long)c * Tf * 256];
  return s;
}

// element (v, u), v >= u, of the permuted system
__device__ __forceinline__ double& sys_at(const BaDev& d, int v, int u) {
  const int sl = d.slot[(v >> 6) * d.nbc + (u >> 6)];
  return d.M[(size_t)sl * kTile + (v & 63) * 64 + (u & 63)];
}

// One workgroup per 6x6 pose block (36 elements) or rhs block (6): the
// element's partial sums (edge Hessian splits, Gram chunks) are spread over
// 256 / elements thread groups with a fixed stride and the group sums added in
// group order - deterministic, and a small graph's few blocks (C2: one tile)
// no longer sum hundreds of partials per thread.
__global__ void __launch_bounds__(256) ba_assemble_kernel(BaDev d) {
  __shared__ double part[256];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const bool blk = b < d.nblk;
  const int EL = blk ? 36 : 6, G = 256 / EL;
  const int e = t % EL, g = t / EL;
  double s = 0.0;
  if (g < G) {
    if (blk) {
      const int r = e / 6, c = e % 6;
      for (int k = d.blkcptr[b]; k < d.blkcptr[b + 1]; ++k) {
        const int4 q = d.contrib[k];
        if (q.x == kEdgeBlock) {
          for (int sp = g; sp < d.nsplit; sp += G)
            s += (double)hess_val(d.hpart + ((long)q.y * d.nsplit + sp) * kHessStride, q.z + r, q.w + c);
        } else {
          s -= gram_sum(d, q.y, 6 * q.z + r, 6 * q.w + c, g, G);
        }
      }
    } else {
      const int a = b - d.nblk;
      for (int k = d.rhscptr[a]; k < d.rhscptr[a + 1]; ++k) {
        const int4 q = d.rhscontrib[k];
        if (q.x == kEdgeRhs) {
          for (int sp = g; sp < d.nsplit; sp += G)
            s += (double)d.hpart[((long)q.y * d.nsplit + sp) * kHessStride + 78 + q.z + e];
        } else {
          const int wcol = 6 * (d.frptr[q.y + 1] - d.frptr[q.y]);
          s -= gram_sum(d, q.y, 6 * q.z + e, wcol, g, G);
        }
      }
    }
  }
  part[t] = s;
  __syncthreads();
  if (t >= EL) return;
  double tot = 0.0;
  for (int gg = 0; gg < G; ++gg) tot += part[gg * EL + t];
  if (blk) {
    // block (a, b) of the original order (a >= b) sits at permuted positions
    // (pa, pb); its (r, c) element is M'(v, u), stored as M'(u, v) when above
    // the diagonal (a diagonal block's upper half is its lower half mirrored)
    const int r = t / 6, c = t % 6;
    const int pa = d.blka[b], pb = d.blkb[b];
    const int v = 6 * pa + r, u = 6 * pb + c;
    if (v >= u) sys_at(d, v, u) = tot;
    else if (pa != pb) sys_at(d, u, v) = tot;
  } else {
    sys_at(d, d.n, 6 * d.rhspos[b - d.nblk] + t) = tot;
  }
}

// diag += ep + lm * diag  (SparseBlock::solve :1197) and start a new status
// word: flag[0] is this solve's (the kernels after it test its timeout bit),
// flag[1] the sticky OR of every earlier solve's since the caller last cleared
// it (first_solve: droid_ba_run's first GN iteration) - a timeout in GN
// iteration 1 is still reported after iteration 2.
__global__ void ba_damp_kernel(double* M, const int* slot, int nbc, int n, float lm, float ep, int* flag,
                               int first_solve) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    flag[1] = first_solve ? 0 : (flag[1] | flag[0]);
    flag[0] = 0;
  }
  if (i < n) {
    double& dg = M[(size_t)slot[(i >> 6) * nbc + (i >> 6)] * kTile + (i & 63) * 65];
    dg = dg + ((double)ep + (double)lm * dg);
  }
}

// dense lower triangle of A (n x n, lda) and b -> the tiles of a chol plan
__global__ void chol_scatter_kernel(double* M, const int* slot, int nbc, int n, const double* A, int lda,
                                    const double* b) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)(n + 1) * n;
  if (idx >= total) return;
  const int v = (int)(idx / n), u = (int)(idx % n);
  if (u > v) return;
  const double val = v < n ? A[(long)v * lda + u] : b[u];
  M[(size_t)slot[(v >> 6) * nbc + (u >> 6)] * kTile + (v & 63) * 64 + (u & 63)] = val;
}

// ---------------------------------------------------------------------------
// Dataflow Cholesky + solve: ONE persistent launch.
//
// The augmented system (n pivots, rhs as row n) is stored as the structurally
// nonzero 64x64 tiles of its factor (slot map from the plan).  Workgroups (one
// per CU) take tasks by ticket in the host's critical-path order
// (ba_plan.cpp build_chol_structure) and wait for their inputs on per-tile
// version counters: ver(tile) = number of updates applied, fin(tile) = that
// count + 1 once the tile is final.  A task is handed out only after all its
// predecessors were, so it never waits on a workgroup that has not started and
// progress does not depend on residency.  A chained potrf(k+1) runs in the
// workgroup of potrf(k), right after it (its own ticket is a placeholder that
// keeps the order topological: whatever it waits for was handed out earlier).
//
// Cross-workgroup hand-off follows cdna_hip_programming.md Guideline 16 R1:
// every handed-off byte (tiles, y) is stored AND loaded with sc1 buffer
// operations (write-through / L1 bypass), every storing wave drains vmcnt
// before the workgroup barrier (or, where one wave stores alone, before its
// own count), then one lane stores the counter with an agent-scope atomic;
// consumers poll relaxed.  The back solve's x values travel as 16-B {x, tag}
// granules (one sc1 store each, polled directly: no separate counter).  Spins
// are bounded (an abort word stops every workgroup and flag bit 1 is raised;
// the host then reports the timeout and leaves poses and disparities
// untouched).  Tiles are products of f64 MFMA (v_mfma_f64_16x16x4f64); the
// diagonal factor is panel-blocked (16 wide, register rows, readlane pivots)
// and the off-diagonal solves are blocked forward substitutions with the
// diagonal-block inverses D_p (tall_solve).  Round 6 restructured the chain;
// DESIGN.md §3 has the timeline.
// ---------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr int LT = 66;          // LDS tile row stride (doubles): conflict-free f64 MFMA operand reads
constexpr int kSc1 = 16;        // buffer-op aux bit: sc1
constexpr unsigned kOobOff = 0x80000000u;
constexpr unsigned kSpinLimit = 1u << 24;
constexpr unsigned long long kSpinTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
constexpr int kCholLds = (3 * 64 * LT + 256 + 4 * 272) * 8 + 32;

struct CholDev {
  double* M;          // factor tiles: slot s at M + kTile * s, row-major 64 x 64
  int n, nbc, nbr;
  const int* tasks;   // kTaskInts per task
  int ntasks;
  const int* slot;    // [nbr * nbc] tile -> slot, -1 = structural zero
  const int* fin;     // [nslots] final version per slot
  const int* outmap;  // [n] permuted variable -> dx index
  int nslots;
  int* sync;    // [0] ticket [1] abort [4..] ver[nslots] | yver[nbc] | lkk[nbc]  (ba.hpp chol_sync_bytes)
  unsigned* gran;  // x hand-off granules {double x, tag, 0}, 64 per block column (inside the sync area)
  int* flag;    // bit 0: factorisation failed (dx = 0), bit 1: spin timeout
  double* ybuf; // [nbc*64]
  float* dx;    // [n]
  int inject;   // test hook (droid_chol_set_fault_inject): raise the abort at once, as a timeout would
  int epoch;    // this launch's number (never 0): a sync area that holds another launch's number is stale
  long long* prof;  // profiling builds: s_memrealtime per (task, stamp < 16), or null
};

#ifndef DROID_CONV_PROFILE
#define DROID_CONV_PROFILE 0
#endif
#if DROID_CONV_PROFILE
#define CH_STAMPT(t, ph)                                                                      \
  do {                                                                                        \
    if (d.prof && tid == 0) d.prof[(long)(t) * 24 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define CH_STAMPW(t, ph)   /* lane 0 of the calling wave */                                 \
  do {                                                                                        \
    if (d.prof && lane == 0) d.prof[(long)(t) * 24 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CH_STAMPT(t, ph) do { } while (0)
#define CH_STAMPW(t, ph) do { } while (0)
#endif
#define CH_STAMP(ph) CH_STAMPT(tk, ph)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mkrs(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ dbl2 ld2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kSc1));
}
__device__ __forceinline__ void st2(__amdgpu_buffer_rsrc_t r, unsigned off, dbl2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, kSc1);
}
__device__ __forceinline__ double ld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, kSc1));
}
__device__ __forceinline__ void st1(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, kSc1);
}

// rows [0,nr) x cols [0,nc) of stored tile `s` -> LDS T[64][LT]; zeros
// elsewhere (out-of-range offsets read 0).  nc even.
__device__ __forceinline__ unsigned tile_off(int s, int rr, int cc, int nr, int nc) {
  return (rr < nr && cc < nc) ? (unsigned)(((size_t)s * kTile + rr * 64 + cc) * 8) : kOobOff;
}
__device__ __forceinline__ void tile_issue(__amdgpu_buffer_rsrc_t r, int s, int nr, int nc, dbl2 (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    v[q] = ld2(r, tile_off(s, rr, cc, nr, nc));
  }
}
__device__ __forceinline__ void tile_commit(const dbl2 (&v)[8], double* T) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    *reinterpret_cast<dbl2*>(&T[rr * LT + cc]) = v[q];
  }
}
__device__ __forceinline__ void tile_load(__amdgpu_buffer_rsrc_t r, int s, int nr, int nc, double* T) {
  dbl2 v[8];
  tile_issue(r, s, nr, nc, v);
  tile_commit(v, T);
}
__device__ __forceinline__ void tile_store(__amdgpu_buffer_rsrc_t r, int s, int nr, int nc, const double* T) {
  if (nr == 64 && nc == 64) {   // a full tile: all eight LDS reads, then the eight stores (no per-store mask)
    dbl2 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
      v[q] = *reinterpret_cast<const dbl2*>(&T[rr * LT + cc]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
      st2(r, (unsigned)(((size_t)s * kTile + rr * 64 + cc) * 8), v[q]);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    if (rr < nr && cc < nc)
      st2(r, (unsigned)(((size_t)s * kTile + rr * 64 + cc) * 8), *reinterpret_cast<const dbl2*>(&T[rr * LT + cc]));
  }
}

// MFMA f64 16x16x4: A operand lane l = A[l&15][l>>4], B operand lane l =
// B[l>>4][l&15], D: acc[q] = D[4*q + (l>>4)][l&15]  (NOT the f32/f16 16x16
// layout; measured on gfx950 by scripts/probe/mfma_f64_layout.hip).
__device__ __forceinline__ dbl4 mfma64(double a, double b, dbl4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// the wave's 32x32 quadrant (wr, wc) of a 64x64 tile: acc += sgn * A B^T, K = 64
__device__ __forceinline__ void gemm_nt64(const double* A, const double* B, dbl4 (&acc)[2][2], int wr, int wc,
                                          int lane, double sgn) {
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < 64; k0 += 4) {
    const double a0 = sgn * A[(wr + fr) * LT + k0 + fk], a1 = sgn * A[(wr + 16 + fr) * LT + k0 + fk];
    const double b0 = B[(wc + fr) * LT + k0 + fk], b1 = B[(wc + 16 + fr) * LT + k0 + fk];
    acc[0][0] = mfma64(a0, b0, acc[0][0]);
    acc[0][1] = mfma64(a0, b1, acc[0][1]);
    acc[1][0] = mfma64(a1, b0, acc[1][0]);
    acc[1][1] = mfma64(a1, b1, acc[1][1]);
  }
}
__device__ __forceinline__ void acc_load(const double* T, dbl4 (&acc)[2][2], int wr, int wc, int lane) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[a][b][q] = T[(wr + 16 * a + 4 * q + (lane >> 4)) * LT + wc + 16 * b + (lane & 15)];
}
__device__ __forceinline__ void acc_store(double* T, const dbl4 (&acc)[2][2], int wr, int wc, int lane) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        T[(wr + 16 * a + 4 * q + (lane >> 4)) * LT + wc + 16 * b + (lane & 15)] = acc[a][b][q];
}

// every storing wave drains, then one lane publishes (Guideline 16 R1)
__device__ __forceinline__ void publish(int* w, int v, int* w2 = nullptr, int v2 = 0, int* w3 = nullptr, int v3 = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w2) __hip_atomic_store(w2, v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w3) __hip_atomic_store(w3, v3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ bool poll_ge(int* w, int target, int* abort_w, int* flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  for (unsigned s = 0;; ++s) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (s > kSpinLimit || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
      __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicOr(flag, 2);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// A broken invariant of the dataflow state (a sync counter not zeroed before
// the launch, a task record outside the plan): status bits 1 (the solve is
// skipped, as after a timeout) and 2 (kFlagState, reported as such by the
// host), and the abort word so every worker drains.
constexpr int kFlagState = 4;
__device__ __forceinline__ void state_fault(int* abort_w, int* flag) {
  __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicOr(flag, 2 | kFlagState);
}

// wave-uniform lane -> every lane (two v_readlane_b32, no LDS round trip)
__device__ __forceinline__ double bcast_lane(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// 1/sqrt(x) in fp64 with ONE Newton step after v_rsq_f64 (~2^-23 relative ->
// ~2^-46; no division or sqrt expansion on the pivot chain; far inside the 1e-4
// parity bar)
__device__ __forceinline__ double rsqrt_f64_1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return y * fma(-0.5 * x * y, y, 1.5);
}

// 16-wide panel of the diagonal factor (wave 0; lane r owns row r's 16 panel
// values in registers; pivot columns past the block's Bp real columns take a
// unit pivot, so every panel is a full, branch-free 16 columns; lanes above the
// diagonal update their never-read upper-triangle entries too).  Every
// cross-lane value on the column-to-column chain comes by v_readlane: lane r
// keeps its own running diagonal dg = A(r,r) - sum_m L(r,m)^2 (its own x values
// only), so the next pivot is readlane(dg) right after this column's scale, and
// the next column's entry L(c+1,c) comes by one readlane pair too.  Only the
// columns two or more ahead get this column through the LDS broadcast (colbuf),
// which then has a full column step to land.  Chain per column: scale ->
// fma(dg) -> readlane -> rsq + one Newton step -> scale.  dinv[c] = 1/L[c][c];
// flag bit 0 on a non-SPD pivot.  (Round 6; measured at the round-5 column
// panel's 2.0 us per 16 columns: the panel is issue-bound, not chain-bound -
// scripts/probe/f64_latency.hip prices a readlane hop at ~40 clk, an LDS round
// trip at ~130, a dependent f64 op at ~6-7.)
__device__ __forceinline__ void panel_factor(double* T, double* dinv, int c0, int Bp, int lane, int* flag,
                                              double* colbuf) {
  double v[16], invs[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = T[lane * LT + c0 + q];
  double dg = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) dg = (lane == c0 + q) ? v[q] : dg;
  bool bad = false;
  double piv = c0 < Bp ? bcast_lane(dg, c0) : 1.0;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    bad |= !(piv > 0.0 && piv < 1e300);
    const double inv = rsqrt_f64_1(piv);
    invs[jj] = inv;
    const double x = v[jj] * inv;  // L(r, c0+jj); the diagonal lane gets sqrt(piv)
    v[jj] = x;
    if (jj < 15) {
      dg = fma(-x, x, dg);
      piv = c0 + jj + 1 < Bp ? bcast_lane(dg, c0 + jj + 1) : 1.0;   // wave-uniform condition
      const double l1 = bcast_lane(x, c0 + jj + 1);
      v[jj + 1] = fma(-x, l1, v[jj + 1]);
      if (jj < 14) {
        colbuf[lane] = x;
        double lq[16];
#pragma unroll
        for (int q = jj + 2; q < 16; ++q) lq[q] = colbuf[c0 + q];
#pragma unroll
        for (int q = jj + 2; q < 16; ++q) v[q] = fma(-x, lq[q], v[q]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) T[lane * LT + c0 + q] = v[q];
  double mine = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) mine = (lane == q) ? invs[q] : mine;
  if (lane < 16) dinv[c0 + lane] = mine;
  if (bad && lane == 0) atomicOr(flag, 1);
}

// X <- X L^-T for a 64-row tile X in T (trsm against a factored pivot block) by
// blocked forward substitution, X_p = (A_p - sum_{j<p} X_j L_pj^T) D_p^-T per
// 16-column block p: L's strictly-lower 16x16 blocks are read from Lt, the
// diagonal-block inverses D_p = L_pp^-1 from the diagonal blocks of Dt.  Each
// wave owns 16 rows, so the four block steps need no barrier (caller syncs
// before and after).  f64 MFMA: 40 per wave, vs 64 for the product with L^-1.
__device__ __forceinline__ void tall_solve(double* T, const double* Lt, const double* Dt, double* scr, int wave,
                                           int fr, int fk) {
  const int r0 = 16 * wave;
  double* sw = scr + wave * 272;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    dbl4 S;
#pragma unroll
    for (int q = 0; q < 4; ++q) S[q] = T[(r0 + 4 * q + fk) * LT + 16 * p + fr];
#pragma unroll
    for (int j = 0; j < p; ++j)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        S = mfma64(-T[(r0 + fr) * LT + 16 * j + 4 * kk + fk], Lt[(16 * p + fr) * LT + 16 * j + 4 * kk + fk], S);
#pragma unroll
    for (int q = 0; q < 4; ++q) sw[(4 * q + fk) * 17 + fr] = S[q];
    asm volatile("" ::: "memory");
    dbl4 X = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      X = mfma64(sw[fr * 17 + 4 * kk + fk], Dt[(16 * p + fr) * LT + 16 * p + 4 * kk + fk], X);
#pragma unroll
    for (int q = 0; q < 4; ++q) T[(r0 + 4 * q + fk) * LT + 16 * p + fr] = X[q];
    asm volatile("" ::: "memory");
  }
}

// 16x16 block C(cr.., cc..) -= A(ar.., a0 + [0, 4 NK)) B(br.., b0 + [0, 4 NK))^T
// on f64 MFMA, all operands in LDS tiles of row stride LT (one wave).
template <int NK>
__device__ __forceinline__ void blk_sub(double* C, int cr, int cc, const double* A, int ar, int a0,
                                        const double* B, int br, int b0, int lane) {
  const int fr = lane & 15, fk = lane >> 4;
  dbl4 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = C[(cr + 4 * q + fk) * LT + cc + fr];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk)
    acc = mfma64(-A[(ar + fr) * LT + a0 + 4 * kk + fk], B[(br + fr) * LT + b0 + 4 * kk + fk], acc);
#pragma unroll
  for (int q = 0; q < 4; ++q) C[(cr + 4 * q + fk) * LT + cc + fr] = acc[q];
  asm volatile("" ::: "memory");
}

// one wave: rows [r0, r0 + nrows) (nrows a multiple of 16, <= 48) of stored
// tile `s` (nr rows, nc columns real; zeros elsewhere) -> LDS tile B
__device__ __forceinline__ void rows_load(__amdgpu_buffer_rsrc_t r, int s, int nr, int nc, double* B, int r0,
                                          int nrows, int lane) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // two halves of at most 12 16-B pieces per lane in flight
    dbl2 v[12];
#pragma unroll
    for (int q = 0; q < 12; ++q)
      if (2 * (12 * h + q) < nrows) {
        const int rr = r0 + 2 * (12 * h + q) + (lane >> 5), cc = (lane & 31) * 2;
        v[q] = ld2(r, tile_off(s, rr, cc, nr, nc));
      }
#pragma unroll
    for (int q = 0; q < 12; ++q)
      if (2 * (12 * h + q) < nrows) {
        const int rr = r0 + 2 * (12 * h + q) + (lane >> 5), cc = (lane & 31) * 2;
        *reinterpret_cast<dbl2*>(&B[rr * LT + cc]) = v[q];
      }
  }
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int wave_ld(int* w) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// poll_ge by a whole wave (every lane reads the same word; the wave decides on lane 0's value)
__device__ bool wave_poll_ge(int* w, int target, int* abort_w, int* flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned s = 0;; ++s) {
    if (wave_ld(w) >= target) return true;
    if (wave_ld(abort_w)) return false;
    if (s > kSpinLimit || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
      if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicOr(flag, 2);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// x hand-off of the back solve: 16-B granules {x (2 dwords), tag, 0}, each
// written whole by one sc1 store and polled with sc1 loads (the tag is the
// flag: no separate counter, no second round trip).  Lanes < 16 of the wave
// wait for granules g0 .. g0 + 15 and leave their x in dst[lane].
__device__ bool gran_wait(__amdgpu_buffer_rsrc_t rg, unsigned g0, double* dst, int lane, int* abort_w, int* flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned s = 0;; ++s) {
    u32x4 g = {0u, 0u, 1u, 0u};
    if (lane < 16) g = __builtin_amdgcn_raw_buffer_load_b128(rg, (int)((g0 + lane) * 16), 0, kSc1);
    if (__builtin_amdgcn_ballot_w64(g[2] == 0u) == 0) {
      if (lane < 16) dst[lane] = __builtin_bit_cast(double, ((unsigned long long)g[1] << 32) | g[0]);
      return true;
    }
    if (wave_ld(abort_w)) return false;
    if (s > kSpinLimit || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
      if (lane == 0) {
        __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicOr(flag, 2);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");   // re-read the granules every pass
  }
}

// out[j] = sum_t M[t][j] v[t] over the 64 rows of LDS tile M, j = lane: wave w
// sums rows 16w..16w+15 into part[w][j] (the caller adds the four partials in
// wave order after a barrier: a fixed reduction order)
__device__ __forceinline__ void gemv_t_part(const double* M, const double* v, double* part, int wave, int lane) {
  // the wave's 16 v values by eight 16-B broadcast reads from one base, M's
  // rows from one base + immediate offsets (no per-element address registers)
  const dbl2* vv = reinterpret_cast<const dbl2*>(v + 16 * wave);
  const double* m = M + 16 * wave * LT + lane;
  double x[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const dbl2 t = vv[q];
    x[2 * q] = t[0];
    x[2 * q + 1] = t[1];
  }
  double s = 0.0;
#pragma unroll
  for (int t = 0; t < 16; ++t) s = fma(m[t * LT], x[t], s);
  part[64 * wave + lane] = s;
}

// One wave: the four 16x16 diagonal-block inverses D_p = L_pp^-1 of a factored
// 64x64 pivot block (lower triangle of L, row stride LT; rows past the real
// block zero and dinv = 1 there, so D_p is unit-padded) into D's diagonal
// blocks; lane = 16 * block + column.  Right-looking forward substitution down
// the column: once x_t is final it leaves column t of L out of the rows below,
// so the dependent chain per row is one fma and one multiply (the left-looking
// form summed each row's t terms in sequence: a 120-fma chain).
__device__ __forceinline__ void diag_inv_blocks(const double* L, double* D, const double* dinv, int lane) {
  const int base = 16 * (lane >> 4), cc = lane & 15;
  double acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = (t == cc) ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const double x = acc[t] * dinv[base + t];
    acc[t] = x;
#pragma unroll
    for (int m = t + 1; m < 16; ++m) acc[m] = fma(-L[(base + m) * LT + base + t], x, acc[m]);
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) D[(base + t) * LT + base + cc] = acc[t];
}

// every tile a task record names lies in the plan's slot map (wave-uniform)
__device__ __forceinline__ bool task_record_ok(const CholDev& d, int type, int i, int j, int k, int b) {
  if (type < kPotrf || type > kBcol) return false;
  if (i < 0 || i >= d.nbr || j < 0 || j >= d.nbc || k < 0 || k >= d.nbc) return false;
  auto live = [&](int r, int cc) {
    return r < d.nbr && __builtin_amdgcn_readfirstlane(d.slot[r * d.nbc + cc]) >= 0;
  };
  switch (type) {
    case kPotrf: return live(k, k) && (!b || live(k + 1, k));
    case kTrsm: return live(i, k) && live(k, k);
    case kUpdate: return live(i, j) && live(i, k) && live(j, k);
    default: return i < d.nbc && live(i, i);   // kBcol
  }
}

__global__ void __launch_bounds__(256) chol_dataflow_kernel(CholDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* T0 = sm;
  double* T1 = sm + 64 * LT;
  double* T2 = sm + 2 * 64 * LT;
  double* vec = sm + 3 * 64 * LT;        // 256
  double* scr = vec + 256;               // [4][16][17]
  int* shi = reinterpret_cast<int*>(scr + 4 * 272);   // [8]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: wave-conditional code branches, never masks
  const int fr = lane & 15, fk = lane >> 4;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int n = d.n, nbc = d.nbc, nbr = d.nbr;
  const __amdgpu_buffer_rsrc_t rM = mkrs(d.M, (size_t)d.nslots * kTile * 8);
  const __amdgpu_buffer_rsrc_t rY = mkrs(d.ybuf, (size_t)nbc * 64 * 8);
  const __amdgpu_buffer_rsrc_t rG = mkrs(d.gran, (size_t)nbc * 64 * 16);
  int* ticket = d.sync;
  int* abort_w = d.sync + 1;
  int* ver = d.sync + 4;
  int* yver = ver + d.nslots;
  int* lkk = yver + nbc;    // L_kk stored: 3 once potrf(k)'s three storing waves have counted
  auto SL = [&](int i, int j) { return d.slot[i * nbc + j]; };
  if (d.inject && blockIdx.x == 0 && tid == 0) {
    __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicOr(d.flag, 2);
  }
  // every wave's verdict on its own blocking waits -> shi[4 + wave]; all agree after a barrier
  auto all_ok = [&](bool ok) {
    if (lane == 0) shi[4 + wave] = ok ? 1 : 0;
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(shi[4] & shi[5] & shi[6] & shi[7]) != 0;
  };

  // Entry invariant (kFlagState), exact: the sync area was zeroed before this
  // launch.  Every workgroup claims it for this launch (word 2: 0 -> epoch)
  // before it takes a ticket, so an area any earlier launch touched - run to
  // completion or aborted anywhere - holds that launch's number, not 0.
  if (tid == 0) {
    const int e = atomicCAS(d.sync + 2, 0, d.epoch);
    shi[1] = (e == 0 || e == d.epoch) ? 1 : 0;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(shi[1]) == 0) {
    if (tid == 0) state_fault(abort_w, d.flag);
    return;
  }
  for (bool first = true;; first = false) {
    if (tid == 0) shi[0] = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int tk = __builtin_amdgcn_readfirstlane(shi[0]);
    // Second line of the entry check, for replays of a captured graph (whose
    // kernel arguments, the epoch included, are frozen): a launch hands out
    // exactly ntasks + gridDim.x tickets when no worker aborts, so a
    // workgroup's first ticket lies below that unless the counter kept a
    // completed launch's value.
    if (tk < 0 || (first && tk >= d.ntasks + (int)gridDim.x)) {
      if (tid == 0) state_fault(abort_w, d.flag);
      break;
    }
    if (tk >= d.ntasks) break;
    const int* tsk = d.tasks + kTaskInts * tk;
    const int type = __builtin_amdgcn_readfirstlane(tsk[0]), i = __builtin_amdgcn_readfirstlane(tsk[1]);
    const int j = __builtin_amdgcn_readfirstlane(tsk[2]), k = __builtin_amdgcn_readfirstlane(tsk[3]);
    const int ta = __builtin_amdgcn_readfirstlane(tsk[4]), tb = __builtin_amdgcn_readfirstlane(tsk[5]);
    // a chained potrf(k) (record word 7) is run by the workgroup that factored
    // column k-1, straight after it, with L(k,k-1) still in LDS: its ticket is a
    // placeholder that keeps the ticket order topological
    if (type == kPotrf && __builtin_amdgcn_readfirstlane(tsk[7]) != 0) continue;
    CH_STAMP(0);
    // Task-record invariant: every index the task addresses is inside the plan
    // (a corrupted record would otherwise turn into an out-of-range tile access).
    if (!task_record_ok(d, type, i, j, k, tb)) {
      if (tid == 0) state_fault(abort_w, d.flag);
      break;
    }
    if (tid == 0) {
      bool ok = true;
      switch (type) {
        case kPotrf:    // awaited inside the branch (a chained successor awaits the same way)
          break;
        case kTrsm: {
          const int s = SL(i, k);
          ok = poll_ge(&ver[s], d.fin[s] - 1, abort_w, d.flag) && poll_ge(&lkk[k], 3, abort_w, d.flag);
          break;
        }
        case kUpdate: {
          const int s = SL(i, j), si = SL(i, k), sj = SL(j, k);
          ok = poll_ge(&ver[s], ta, abort_w, d.flag) && poll_ge(&ver[si], d.fin[si], abort_w, d.flag) &&
               poll_ge(&ver[sj], d.fin[sj], abort_w, d.flag);
          // the updates of a tile are applied in sequence by this chain alone, so
          // its counter reads exactly `ta` here; more means a stale counter
          if (ok && __hip_atomic_load(&ver[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ta) {
            state_fault(abort_w, d.flag);
            ok = false;
          }
          break;
        }
        default: {  // kBcol: L_cc with its diagonal-block inverses, and the forward value of y_c
          ok = poll_ge(&lkk[i], 3, abort_w, d.flag) && poll_ge(&yver[i], 1, abort_w, d.flag);
          break;
        }
      }
      shi[1] = ok ? 1 : 0;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(shi[1])) break;
    CH_STAMP(1);

    if (type == kPotrf) {
      // Round 6: the diagonal factor's 16-column panels (wave 0) run beside the
      // rest of the tile's last update and the in-tile trailing updates (waves
      // 1-3), and waves 1-3 load tile (k+1,k) as soon as it has its other
      // updates; between two panels only the next block column's update (3
      // blocks, 4 MFMAs each) sits on the chain.  After the panels wave 1 forms
      // the diagonal-block inverses D_p while waves 0, 2, 3 store L_kk and flag
      // it (the trsm tasks below and the back solve read L_kk and form their
      // own D_p); the workgroup solves tile (k+1,k) (tall_solve), publishes it,
      // and - when the plan chains potrf(k+1) to this task - goes straight on
      // to potrf(k+1) with L(k+1,k) still in LDS (no hand-off, no reload; the
      // publish then waits for that task's first barrier, after the stores
      // have landed).
      double* tL = T1;   // L(k,klast) for the last update, then the D_p (diagonal blocks)
      double* tB = T2;   // tile (k+1,k)
      double* dinv = vec + 128;
      int kc = k, ka = ta, kb = tb, tcur = tk;
      const int* rec = tsk;
      bool haveL = false;   // L(k,klast) already in tL (chained from potrf(k-1))
      bool alive = true;
      // inside a pivot chain the publish of tile (k+1,k) and y_k waits for the
      // next potrf's first barrier (its stores have landed by then): the chain
      // does not stall on the store drain
      int pend_s = -1, pend_fin = 0, pend_y = -1;
      for (;;) {
        const int R0 = 64 * kc, Bp = min(64, n - R0), Br = min(64, n + 1 - R0);
        const int np = (Bp + 15) >> 4;
        const int skk = SL(kc, kc);
        const bool fz = kb != 0;
        const int s1 = fz ? SL(kc + 1, kc) : 0, nr1 = fz ? min(64, n + 1 - R0 - 64) : 0;
        if (tid == 0)   // all updates of (k,k) but the last one, which is applied here
          shi[1] = poll_ge(&ver[skk], ka >= 0 ? d.fin[skk] - 2 : 0, abort_w, d.flag) ? 1 : 0;
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(shi[1])) { alive = false; break; }
        CH_STAMPT(tcur, 1);
        // wave w >= 1 loads rows [rlo, rhi) of tile (k+1,k) into tB (16, 16, 32 rows)
        const int rlo = wave == 1 ? 0 : wave == 2 ? 16 : 32, rhi = wave == 1 ? 16 : wave == 2 ? 32 : 64;
        bool ld = false;
        auto load_below = [&](bool block) -> bool {   // this wave's rows of (k+1,k), once final but for the trsm
          if (ld || !fz || wave == 0) return true;
          const int tgt = d.fin[s1] - 1;
          if (block) {
            if (!wave_poll_ge(&ver[s1], tgt, abort_w, d.flag)) return false;
          } else if (wave_ld(&ver[s1]) < tgt) {
            return true;
          }
          rows_load(rM, s1, nr1, Bp, tB, rlo, rhi - rlo, lane);
          ld = true;
          return true;
        };

        dbl2 pre[8];
        tile_issue(rM, skk, Br, Bp, pre);  // A(k,k) is final but for (k,k,klast): load while L(k,klast) is awaited
        if (ka >= 0 && !haveL) {
          const int sl = SL(kc, ka);
          if (tid == 0) shi[3] = poll_ge(&ver[sl], d.fin[sl], abort_w, d.flag) ? 1 : 0;
          __syncthreads();
          if (!__builtin_amdgcn_readfirstlane(shi[3])) { alive = false; break; }
          tile_load(rM, sl, Br, 64, tL);
        }
        tile_commit(pre, T0);
        __syncthreads();
        if (ka >= 0) {  // the last update's block column 0 (one 16x16 block per wave): panel 0 needs only it
          blk_sub<16>(T0, 16 * wave, 0, tL, 16 * wave, 0, tL, 0, 0, lane);
          __syncthreads();
        }
        if (pend_s >= 0) {   // the previous potrf's deferred publish
          publish(&ver[pend_s], pend_fin, pend_y >= 0 ? &yver[pend_y] : nullptr, 1);
          pend_s = -1;
        }
        CH_STAMPT(tcur, 2);
        for (int p = 0; p < np; ++p) {
          if (wave == 0) {
              CH_STAMPT(tcur, 8 + 2 * p);
              panel_factor(T0, dinv, 16 * p, Bp, lane, d.flag, scr);
              CH_STAMPT(tcur, 9 + 2 * p);
          } else {
            int job = 0;
            if (p == 0) {  // the rest of the last update (block columns >= 1)
              if (ka >= 0)
                for (int C = 1; C < np; ++C)
                  for (int R = C; R < 4; ++R, ++job)
                    if (job % 3 == wave - 1) blk_sub<16>(T0, 16 * R, 16 * C, tL, 16 * R, 0, tL, 16 * C, 0, lane);
            } else {       // panel p-1's update of the block columns after the next
              for (int C = p + 1; C < np; ++C)
                for (int R = C; R < 4; ++R, ++job)
                  if (job % 3 == wave - 1)
                    blk_sub<4>(T0, 16 * R, 16 * C, T0, 16 * R, 16 * (p - 1), T0, 16 * C, 16 * (p - 1), lane);
            }
            load_below(false);
          }
          __syncthreads();
          if (p + 1 < np) {  // the next block column gets panel p's update (rows p+1..3, one block per wave)
            const int R = p + wave;
            if (wave >= 1 && R < 4)
              blk_sub<4>(T0, 16 * R, 16 * (p + 1), T0, 16 * R, 16 * p, T0, 16 * (p + 1), 16 * p, lane);
            __syncthreads();
          }
        }
        CH_STAMPT(tcur, 3);
        const bool rhs0 = Br > Bp;                    // the rhs row inside the pivot tile
        const bool rhs1 = fz && kc + 1 == nbr - 1;    // ... or in tile (k+1,k)
        if (wave != 1) {
          // L_kk (rows and columns < Bp) goes out now, a third of it from each
          // of waves 0, 2, 3 (wave 1 forms the D_p meanwhile); each counts its
          // own stores on lkk once they have landed (its own vmcnt(0),
          // Guideline 16 R1): the trsm tasks below and the back solve wait for 3.
          // Split three ways the drain stays under the D_p, off the barrier.
          const int sw = wave == 0 ? 0 : wave - 1;
          if (Bp == 64) {   // row pairs sw, sw + 3, ...: all the LDS reads, then the stores
            // (the 32nd pair is stored by two waves - the same bytes)
            dbl2 sv[11];
#pragma unroll
            for (int j = 0; j < 11; ++j) {
              const int rr = min(sw + 3 * j, 31) * 2 + (lane >> 5), cc2 = (lane & 31) * 2;
              sv[j] = *reinterpret_cast<const dbl2*>(&T0[rr * LT + cc2]);
            }
#pragma unroll
            for (int j = 0; j < 11; ++j) {
              const int rr = min(sw + 3 * j, 31) * 2 + (lane >> 5), cc2 = (lane & 31) * 2;
              st2(rM, (unsigned)(((size_t)skk * kTile + rr * 64 + cc2) * 8), sv[j]);
            }
          } else {
#pragma unroll
            for (int q = 0; q < 32; ++q) {
              const int rr = q * 2 + (lane >> 5), cc2 = (lane & 31) * 2;
              if (q % 3 == sw && rr < Bp && cc2 < Bp)
                st2(rM, (unsigned)(((size_t)skk * kTile + rr * 64 + cc2) * 8), *reinterpret_cast<const dbl2*>(&T0[rr * LT + cc2]));
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_fetch_add(&lkk[kc], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (wave == 1) {
          // y_k (the solved rhs row), the rows past Bp cleared (L_kk^-1 is
          // unit-padded there), then the diagonal-block inverses D_p = L_pp^-1
          // into tL's diagonal blocks; lane = 16 * block + column
          if (rhs0 && lane < 32)
            st2(rY, (unsigned)((R0 + 2 * lane) * 8), *reinterpret_cast<const dbl2*>(&T0[Bp * LT + 2 * lane]));
          for (int r = Bp; r < 64; ++r) T0[r * LT + lane] = 0.0;
          if (lane >= Bp) dinv[lane] = 1.0;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          CH_STAMPW(tcur, 16);
          diag_inv_blocks(T0, tL, dinv, lane);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          CH_STAMPW(tcur, 17);
        }
        if (!all_ok(load_below(true))) { alive = false; break; }
        CH_STAMPT(tcur, 6);
        if (fz) tall_solve(tB, T0, tL, scr, wave, fr, fk);   // trsm(k+1,k) with the D_p, each wave 16 rows
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        CH_STAMPT(tcur, 18);
        if (fz) {
          __syncthreads();
          tile_store(rM, s1, nr1, Bp, tB);
          if (rhs1 && tid < 32)
            st2(rY, (unsigned)((R0 + 2 * tid) * 8), *reinterpret_cast<const dbl2*>(&tB[(n - R0 - 64) * LT + 2 * tid]));
        }
        CH_STAMPT(tcur, 19);
        // chained successor: potrf(k+1), whose last update is L(k+1,k) L(k+1,k)^T
        const int nxt = __builtin_amdgcn_readfirstlane(rec[6]);
        if (nxt > 0 && fz) {   // (the diagonal tile's own version is read by no task)
          __syncthreads();     // the tile stores have read tB
          pend_s = s1;
          pend_fin = d.fin[s1];
          pend_y = (rhs0 || rhs1) ? kc : -1;
        } else {
          publish(&ver[skk], d.fin[skk], fz ? &ver[s1] : nullptr, fz ? d.fin[s1] : 0,
                  (rhs0 || rhs1) ? &yver[kc] : nullptr, 1);
        }
        CH_STAMPT(tcur, 5);
        if (nxt <= 0) break;
        CH_STAMPT(tcur, 7);
        tcur = nxt - 1;
        rec = d.tasks + kTaskInts * tcur;
        const int ntype = __builtin_amdgcn_readfirstlane(rec[0]), nk = __builtin_amdgcn_readfirstlane(rec[3]);
        const int na = __builtin_amdgcn_readfirstlane(rec[4]), nb = __builtin_amdgcn_readfirstlane(rec[5]);
        if (tcur >= d.ntasks || ntype != kPotrf || nk != kc + 1 || na != kc || !fz ||
            !task_record_ok(d, kPotrf, nk, nk, nk, nb)) {
          if (tid == 0) state_fault(abort_w, d.flag);
          alive = false;
          break;
        }
        CH_STAMPT(tcur, 0);
        kc = nk; ka = na; kb = nb;
        double* t = tL; tL = tB; tB = t;   // L(k+1,k) is the next task's last-update operand
        haveL = true;
      }
      if (!alive) break;
      CH_STAMPT(tcur, 7);
      continue;
    } else if (type == kTrsm) {
      // X = A L_kk^-T by blocked forward substitution (tall_solve: 40 f64 MFMAs
      // per wave) against L_kk and its diagonal-block inverses, which potrf(k)
      // stores right after its panels (round 6: the product with the whole
      // L_kk^-1 waited for the end of potrf(k)).  b = 1: then also the update
      // (i,k+1,k) - always that tile's last - with X still in LDS and L(k+1,k)
      // from potrf(k); it is version a+1 of (i,k+1).
      const int R0 = 64 * i, C0 = 64 * k, nr = min(64, n + 1 - R0), nc = min(64, n - C0);
      const int s = SL(i, k);
      dbl2 pa[8];
      tile_issue(rM, s, nr, nc, pa);
      tile_load(rM, SL(k, k), nc, nc, T1);
      tile_commit(pa, T0);
      __syncthreads();
      if (wave == 0) {   // the D_p, from L_kk itself
        vec[lane] = lane < nc ? 1.0 / T1[lane * LT + lane] : 1.0;   // 1 / L[t][t]
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        diag_inv_blocks(T1, T2, vec, lane);
      }
      __syncthreads();
      CH_STAMP(2);
      tall_solve(T0, T1, T2, scr, wave, fr, fk);
      __syncthreads();
      CH_STAMP(3);
      tile_store(rM, s, nr, nc, T0);
      const bool rhs = (i == nbr - 1);
      if (rhs && tid < 32) st2(rY, (unsigned)((C0 + 2 * tid) * 8), *reinterpret_cast<const dbl2*>(&T0[(n - R0) * LT + 2 * tid]));
      publish(&ver[s], d.fin[s], rhs ? &yver[k] : nullptr, 1);
      if (tb) {
        const int su = SL(i, k + 1), sk = SL(k + 1, k);
        const int nc1 = min(64, n - C0 - 64);
        if (tid == 0)
          shi[3] = (poll_ge(&ver[su], ta, abort_w, d.flag) && poll_ge(&ver[sk], d.fin[sk], abort_w, d.flag)) ? 1 : 0;
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(shi[3])) break;
        if (tid == 0 && __hip_atomic_load(&ver[su], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ta) {
          state_fault(abort_w, d.flag);   // this chain applies the tile's updates alone: more is a stale counter
          shi[3] = 0;
        }
        tile_load(rM, sk, nc1, 64, T1);
        tile_load(rM, su, nr, nc1, T2);
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(shi[3])) break;
        CH_STAMP(4);
        dbl4 acc[2][2];
        acc_load(T2, acc, wr, wc, lane);
        gemm_nt64(T0, T1, acc, wr, wc, lane, -1.0);
        acc_store(T2, acc, wr, wc, lane);
        __syncthreads();
        tile_store(rM, su, nr, nc1, T2);
        publish(&ver[su], ta + 1);
      }
    } else if (type == kUpdate) {
      const int Ri = 64 * i, Rj = 64 * j, Ck = 64 * k;
      const int nri = min(64, n + 1 - Ri), ncj = min(64, n - Rj), nck = min(64, n - Ck);
      const int s = SL(i, j);
      tile_load(rM, SL(i, k), nri, nck, T0);
      tile_load(rM, SL(j, k), ncj, nck, T1);
      tile_load(rM, s, nri, ncj, T2);
      __syncthreads();
      CH_STAMP(2);
      dbl4 acc[2][2];
      acc_load(T2, acc, wr, wc, lane);
      gemm_nt64(T0, T1, acc, wr, wc, lane, -1.0);
      acc_store(T2, acc, wr, wc, lane);
      __syncthreads();
      CH_STAMP(3);
      tile_store(rM, s, nri, ncj, T2);
      publish(&ver[s], ta + 1);
    } else {
      // kBcol (round 6): the whole back solve of block column c in one task.
      // x_c = L_cc^-T (y_c - sum_{r>c} L_rc^T x_r).  The rows r > c are the
      // ancestors of c in the elimination tree, so the parent p (the smallest
      // r) publishes last: its term is folded into H = L_pc L_cc^-1, computed
      // while the chain is still above, and x_c = z_c - H^T x_p with z_c =
      // L_cc^-T (y_c - sum_{r>p} L_rc^T x_r).  The chain step is then one
      // granule wait, one 64x64 GEMV and one granule store.
      const int c = i, C0 = 64 * c, Bc = min(64, n - C0);
      const int om = (wave == 0 && lane < Bc) ? d.outmap[C0 + lane] : 0;   // dx index of this lane's variable
      int par = c + 1;
      while (par < nbc && SL(par, c) < 0) ++par;
      const bool haspar = par < nbc;
      dbl2 pc[8], pp[8];
      tile_issue(rM, SL(c, c), Bc, Bc, pc);          // L_cc
      if (haspar) tile_issue(rM, SL(par, c), min(64, n - 64 * par), Bc, pp);
      if (tid < 32) {
        const dbl2 yv = ld2(rY, 2 * tid < Bc ? (unsigned)((C0 + 2 * tid) * 8) : kOobOff);
        vec[2 * tid] = yv[0];
        vec[2 * tid + 1] = yv[1];
      }
      for (int idx = tid; idx < 64 * 64; idx += 256) T2[(idx >> 6) * LT + (idx & 63)] = 0.0;
      tile_commit(pc, T1);
      __syncthreads();
      if (wave == 0) {   // the D_p on T2's diagonal
        vec[128 + lane] = lane < Bc ? 1.0 / T1[lane * LT + lane] : 1.0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        diag_inv_blocks(T1, T2, vec + 128, lane);
      }
      __syncthreads();
      // L_cc^-1 in T2: Linv[I][J] = -D_I sum_{K=J}^{I-1} L[I][K] Linv[K][J]
      for (int I = 1; I < 4; ++I) {
        if (wave < I) {
          const int J = wave;
          dbl4 S = {0.0, 0.0, 0.0, 0.0};
          for (int K = J; K < I; ++K)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
              S = mfma64(T1[(16 * I + fr) * LT + 16 * K + 4 * kk + fk], T2[(16 * K + 4 * kk + fk) * LT + 16 * J + fr], S);
          double* sw = scr + wave * 272;
#pragma unroll
          for (int q = 0; q < 4; ++q) sw[(4 * q + fk) * 17 + fr] = S[q];
          asm volatile("" ::: "memory");
          dbl4 R = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            R = mfma64(-T2[(16 * I + fr) * LT + 16 * I + 4 * kk + fk], sw[(4 * kk + fk) * 17 + fr], R);
#pragma unroll
          for (int q = 0; q < 4; ++q) T2[(16 * I + 4 * q + fk) * LT + 16 * J + fr] = R[q];
        }
        __syncthreads();
      }
      if (haspar) {  // H = L_pc Linv_c -> T1 (each wave a 32x32 quadrant)
        tile_commit(pp, T0);
        __syncthreads();
        dbl4 acc[2][2] = {};
#pragma unroll 4
        for (int k0 = 0; k0 < 64; k0 += 4) {
          const double a0v = T0[(wr + fr) * LT + k0 + fk], a1v = T0[(wr + 16 + fr) * LT + k0 + fk];
          const double b0v = T2[(k0 + fk) * LT + wc + fr], b1v = T2[(k0 + fk) * LT + wc + 16 + fr];
          acc[0][0] = mfma64(a0v, b0v, acc[0][0]);
          acc[0][1] = mfma64(a0v, b1v, acc[0][1]);
          acc[1][0] = mfma64(a1v, b0v, acc[1][0]);
          acc[1][1] = mfma64(a1v, b1v, acc[1][1]);
        }
        acc_store(T1, acc, wr, wc, lane);
      }
      // the other rows, descending, one tile in flight ahead
      int r = nbc - 1;
      while (r > par && SL(r, c) < 0) --r;
      dbl2 pt[8];
      if (r > par) tile_issue(rM, SL(r, c), min(64, n - 64 * r), Bc, pt);
      __syncthreads();
      double* part = scr;   // [4][64]
      bool alive = true;
      while (r > par) {
        int rn = r - 1;
        while (rn > par && SL(rn, c) < 0) --rn;
        tile_commit(pt, T0);
        if (rn > par) tile_issue(rM, SL(rn, c), min(64, n - 64 * rn), Bc, pt);
        if (!all_ok(gran_wait(rG, 64 * r + 16 * wave, vec + 64 + 16 * wave, lane, abort_w, d.flag))) {
          alive = false;
          break;
        }
        gemv_t_part(T0, vec + 64, part, wave, lane);
        __syncthreads();
        if (wave == 0) vec[lane] -= ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
        __syncthreads();
        r = rn;
      }
      if (!alive) break;
      CH_STAMP(2);
      gemv_t_part(T2, vec, part, wave, lane);   // z_c = Linv_c^T y_c
      __syncthreads();
      double xc = ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
      if (haspar) {
        __syncthreads();   // the partials are read
        if (!all_ok(gran_wait(rG, 64 * par + 16 * wave, vec + 64 + 16 * wave, lane, abort_w, d.flag))) break;
        CH_STAMP(3);
        gemv_t_part(T1, vec + 64, part, wave, lane);
        __syncthreads();
        xc -= ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
      }
      if (wave == 0) {
        const double xv = lane < Bc ? xc : 0.0;
        const unsigned long long u = __builtin_bit_cast(unsigned long long, xv);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)u, (unsigned)(u >> 32), 1u, 0u}, rG,
                                               (int)((64 * c + lane) * 16), 0, kSc1);
        if (lane < Bc) d.dx[om] = (float)xv;   // a failed factorisation zeroes dx after the launch
      }
      __syncthreads();   // vec / scr / T0-T2 are reused by the next task
    }
    CH_STAMP(7);
  }
}

// the dense chol API (droid_chol_solve): dx = 0 when the factorisation failed
__global__ void chol_fail_zero_kernel(float* dx, int n, const int* flag) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n && (*flag & 1)) dx[v] = 0.0f;
}

// ---------------------------------------------------------------------------
// Kernel D: back substitution dz = Q (w - sum_rows E_row . dx[pose]) with the
// EvT6x1 skip of rows whose pose index is <= 0 (:1105), then disps += dz.
// A timed-out factorisation (flag bit 1) leaves disparities untouched.
// grid = (ceil(HW/256), K); the frame's edges are staged 256 at a time.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ba_backsub_kernel(BaDev d) {
  __shared__ float Tsh[256 * 8];
  __shared__ float dxs[256 * 8];
  if (*d.flag & 2) return;
  const bool failed = (*d.flag & 1) != 0;   // not SPD: dx = 0 (the solve leaves x undefined there)
  const int f = blockIdx.y;
  const int HW = d.HW;
  const int px = blockIdx.x * 256 + threadIdx.x;
  const bool live = px < HW;
  const int kf = d.kx[f];
  const int e0 = d.feptr[f], e1 = d.feptr[f + 1];
  const int t = threadIdx.x;
  const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
  const float u = (float)(px % d.W), v = (float)(px / d.W);
  const float disp = live ? d.disps[(long)kf * HW + px] : 0.0f;
  const int pi = kf - d.t0;
  const bool use_ei = pi > 0 && pi < d.P;
  float Ei[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float acc = 0.f;
  for (int base = e0; base < e1; base += 256) {
    const int cnt = min(256, e1 - base);
    __syncthreads();
    if (t < cnt) {
      const int e = d.fedges[base + t];
      stash_rel_pose(d, kf, e, Tsh + 8 * t);
      const int pr = d.jj[e] - d.t0;
      for (int k = 0; k < 6; ++k) dxs[8 * t + k] = (pr > 0 && pr < d.P && !failed) ? d.dx[6 * pr + k] : 0.0f;
      dxs[8 * t + 6] = (pr > 0 && pr < d.P && !failed) ? 1.0f : 0.0f;
    }
    __syncthreads();
    if (!live) continue;
    for (int q = 0; q < cnt; ++q) {
      const int e = d.fedges[base + q];
      bool stereo;
      const SE3f T = unstash_rel_pose(Tsh + 8 * q, stereo);
      const float* tg = d.targets + (long)e * 2 * HW;
      const float* wt = d.weights + (long)e * 2 * HW;
      PixLin L;
      linearize_pixel(T, stereo, fx, fy, cx, cy, u, v, disp, tg[px], tg[HW + px], wt[px], wt[HW + px], L);
      const float au = L.wu * L.Jzu, av = L.wv * L.Jzv;
      const float* dxe = dxs + 8 * q;
      if (dxe[6] != 0.0f) {
        float dw = 0.f;
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) dw += (au * L.Jju[nn] + av * L.Jjv[nn]) * dxe[nn];
        acc += dw;
      }
      if (use_ei) {
        float Ji[6];
        ji_from_jj(T, L.Jju, Ji);
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) Ei[nn] += au * Ji[nn];
        ji_from_jj(T, L.Jjv, Ji);
#pragma unroll
        for (int nn = 0; nn < 6; ++nn) Ei[nn] += av * Ji[nn];
      }
    }
  }
  if (!live) return;
  if (use_ei && !failed) {
    float dw = 0.f;
#pragma unroll
    for (int nn = 0; nn < 6; ++nn) dw += Ei[nn] * d.dx[6 * pi + nn];
    acc += dw;
  }
  const float Q = d.qw[(long)f * HW + px];
  const float w = d.qw[(long)d.K * HW + (long)f * HW + px];
  const float dzv = Q * (w - acc);
  d.dz[(long)f * HW + px] = dzv;
  d.disps[(long)kf * HW + px] = disp + dzv;
}

// poses <- Exp(dx) poses; a timed-out factorisation (flag bit 1) changes
// nothing; a failed one (bit 0, not SPD) gives dx = 0, as the reference
// (droid_kernels.cu:1197): the output dx is zeroed here, after the back
// substitution read it as zero
__global__ void ba_retract_kernel(float* poses, float* dx, int t0, int P, const int* flag) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P || (*flag & 2)) return;
  if (*flag & 1) {
    for (int n = 0; n < 6; ++n) dx[6 * k + n] = 0.0f;
    return;
  }
  float xi[6];
  for (int n = 0; n < 6; ++n) xi[n] = dx[6 * k + n];
  retr_se3(xi, poses + 7 * (t0 + k));
}

// ---------------------------------------------------------------------------
template <int NB>
static void launch_schur(const BaDev& d, hipStream_t s) {
  const size_t lds = (size_t)4 * NB * 16 * kLdsRow * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ba_frame_schur_kernel<NB>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 grid(d.nchunk, d.K);
  ba_frame_schur_kernel<NB><<<grid, 256, lds, s>>>(d);
}

static int schur_dispatch(int nb, const BaDev& d, hipStream_t s) {
  switch (nb) {
    case 1: launch_schur<1>(d, s); break;
    case 2: launch_schur<2>(d, s); break;
    case 3: launch_schur<3>(d, s); break;
    case 4: launch_schur<4>(d, s); break;
    case 5: launch_schur<5>(d, s); break;
    case 6: launch_schur<6>(d, s); break;
    case 7: launch_schur<7>(d, s); break;
    case 8: launch_schur<8>(d, s); break;
    default: return fail(kUnsupported, "ba: Schur tile count out of range");
  }
  return kOk;
}

static int launch_wide(const BaPlan& p, const BaDev& d, hipStream_t s) {
  if (p.wide_f.empty()) return kOk;
  ba_frame_prep_kernel<<<dim3(ceil_div(p.HW, 256), (int)p.wide_f.size()), 256, 0, s>>>(d);
  DROID_LAUNCH_CHECK();
  const int lds = 4 * 128 * kLdsRow * (int)sizeof(float);
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&ba_frame_gram_wide_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = true;
  }
  ba_frame_gram_wide_kernel<<<dim3(p.nchunk, (int)p.wide_tasks.size() / 3), 256, lds, s>>>(d);
  DROID_LAUNCH_CHECK();
  return kOk;
}

static BaDev make_dev(BaPlan& p, char* ws) {
  BaDev d{};
  const int* I = reinterpret_cast<const int*>(ws + p.off_ints);
  d.ii = I + p.o_ii; d.jj = I + p.o_jj; d.kx = I + p.o_kx;
  d.feptr = I + p.o_feptr; d.fedges = I + p.o_fedges;
  d.frptr = I + p.o_frptr; d.rpose = I + p.o_rpose; d.redge = I + p.o_redge;
  d.fnb = I + p.o_fnb; d.fgoff = I + p.o_fgoff;
  d.blka = I + p.o_blka; d.blkb = I + p.o_blkb; d.blkcptr = I + p.o_blkcptr;
  d.rhscptr = I + p.o_rhscptr; d.rhspos = I + p.o_rhspos;
  d.contrib = reinterpret_cast<const int4*>(I + p.o_contrib);
  d.rhscontrib = reinterpret_cast<const int4*>(I + p.o_rhscontrib);
  d.widef = I + p.o_widef; d.wideeoff = I + p.o_wideeoff; d.widetasks = I + p.o_widetasks;
  d.slot = I + p.o_slot;
  d.hpart = reinterpret_cast<float*>(ws + p.off_hpart);
  d.gram = reinterpret_cast<float*>(ws + p.off_gram);
  d.qw = reinterpret_cast<float*>(ws + p.off_qw);
  d.ei = reinterpret_cast<float*>(ws + p.off_ei);
  d.M = reinterpret_cast<double*>(ws + p.off_M);
  d.x = reinterpret_cast<double*>(ws + p.off_x);
  d.flag = reinterpret_cast<int*>(ws + p.off_flag);
  d.E = p.E; d.N = p.N; d.H = p.H; d.W = p.W; d.HW = p.HW;
  d.t0 = p.t0; d.t1 = p.t1; d.P = p.P; d.K = p.K; d.n = p.n; d.nbc = p.cs.nbc;
  d.eta_rows = p.eta_rows; d.nsplit = p.nsplit; d.nchunk = p.nchunk; d.gpw = p.group_per_wave;
  d.nblk = (int)p.blk_a.size();
  d.nwide = (int)p.wide_f.size();
  return d;
}

static int num_cus() { return device_cu_count(); }
static long long* g_chol_prof = nullptr;
enum { kInjectOff = 0, kInjectAll = 1, kInjectOnce = 2, kInjectStale = 3 };
static int g_chol_inject = kInjectOff;

static int launch_chol_dataflow(const BaPlan& p, char* ws, float* dx, hipStream_t stream) {
  const int* I = reinterpret_cast<const int*>(ws + p.off_ints);
  CholDev c{};
  c.M = reinterpret_cast<double*>(ws + p.off_M);
  c.n = p.n; c.nbc = p.cs.nbc; c.nbr = p.cs.nbr;
  c.tasks = I + p.o_tasks;
  c.ntasks = p.cs.ntasks;
  c.slot = I + p.o_slot; c.fin = I + p.o_fin; c.outmap = I + p.o_outmap;
  c.nslots = p.cs.nslots;
  c.sync = reinterpret_cast<int*>(ws + p.off_sync);
  c.gran = reinterpret_cast<unsigned*>(ws + p.off_sync + chol_gran_off(p.cs.nslots, p.cs.nbc));
  c.flag = reinterpret_cast<int*>(ws + p.off_flag);
  c.ybuf = reinterpret_cast<double*>(ws + p.off_ybuf);
  c.dx = dx;
  // test hook (droid_chol_set_fault_inject): a timeout in every solve, in the
  // next solve only, or the next solve launched on a stale sync area
  const int inj = g_chol_inject;
  if (inj == kInjectOnce || inj == kInjectStale) g_chol_inject = kInjectOff;
  c.inject = (inj == kInjectAll || inj == kInjectOnce) ? 1 : 0;
  c.prof = g_chol_prof;
  static int epoch = 0;
  epoch = epoch == 0x7fffffff ? 1 : epoch + 1;
  c.epoch = epoch;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&chol_dataflow_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kCholLds));
    attr = true;
  }
  if (inj != kInjectStale)
    if (int st = ba_zero(c.sync, p.sync_bytes, stream)) return st;
  // workers: one per CU on the small task graphs (C3, 2.3k tasks: BA(itrs=2)
  // 1.88 vs 1.95 ms with one per two CUs, the chain's tasks start sooner) and
  // three per four CUs on the large ones (C5, 23.9k tasks: 10.9 vs 11.3 ms; one
  // per CU 11.7 - the extra workers' polling of the hand-off counters costs
  // more than they add), round 6, profiles/r06/r06zd_chol_grid.txt
  const int ncu = num_cus();
  int grid = std::min(p.cs.ntasks, std::max(1, p.cs.ntasks <= 8192 ? ncu : 3 * ncu / 4));
  if (const int g = ab_knob("DROID_CHOL_GRID", 0)) grid = std::max(1, std::min(p.cs.ntasks, g));  // A/B runs
  chol_dataflow_kernel<<<grid, 256, kCholLds, stream>>>(c);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // namespace droid

using namespace droid;

extern "C" {

#if DROID_TESTING
// Test hook for the dataflow solve's failure handling: 0 off, 1 every solve
// aborts as on a dependency-wait timeout (status bit 1), 2 only the next solve
// does, 3 the next solve is launched without zeroing its sync area (the
// kernel's entry check must report it: status bits 1 and 2).  Process-wide.
int droid_chol_set_fault_inject(int mode) {
  if (mode < kInjectOff || mode > kInjectStale) return fail(kInvalidArgument, "chol_set_fault_inject: mode 0..3");
  g_chol_inject = mode;
  return kOk;
}
#endif  // DROID_TESTING

#if DROID_TESTING
// Profiling builds (make prof): per Cholesky task, 24 int64 s_memrealtime
// stamps (100 MHz), scripts/chol_timeline.py names them.
int droid_chol_set_profile(void* buf) {
#if DROID_CONV_PROFILE
  g_chol_prof = static_cast<long long*>(buf);
  return kOk;
#else
  (void)buf;
  return fail(kUnsupported, "chol_set_profile: build with make prof (DROID_CONV_PROFILE=1)");
#endif
}
#endif  // DROID_TESTING

int droid_ba_plan_upload(void* plan, void* workspace, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  if (!p || !workspace) return fail(kInvalidArgument, "ba_plan_upload: null argument");
  DROID_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(workspace) + p->off_ints, p->ints.data(),
                                 p->ints.size() * sizeof(int), hipMemcpyHostToDevice, stream));
  // the status word reads "no failure" until a solve runs
  if (int st = ba_zero(static_cast<char*>(workspace) + p->off_flag, 64, stream)) return st;
  p->uploaded = true;
  p->uploaded_to = workspace;
  return kOk;
}

static int check_ready(const BaPlan* p, void* ws) {
  if (!p || !ws) return fail(kInvalidArgument, "ba: null plan or workspace");
  if (!p->uploaded || p->uploaded_to != ws)
    return fail(kInvalidArgument, "ba: plan not uploaded to this workspace");
  return kOk;
}

// One Gauss-Newton linearisation: fills the augmented reduced system in the
// workspace (droid_kernels.cu:1359-1406 up to the solve).
int droid_ba_build_system(void* plan, void* workspace, float* poses, float* disps,
                          const float* intrinsics, const float* disps_sens, const float* targets,
                          const float* weights, const float* eta, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  BaDev d = make_dev(*p, static_cast<char*>(workspace));
  d.poses = poses; d.disps = disps; d.intr = intrinsics; d.disps_sens = disps_sens;
  d.targets = targets; d.weights = weights; d.eta = eta;
  if (p->E > 0) {
    ba_edge_hessian_kernel<<<dim3(p->nsplit, p->E), 256, 0, stream>>>(d);
    DROID_LAUNCH_CHECK();
  }
  if (!p->motion_only && p->K > 0) {
    if (p->wide_f.size() < (size_t)p->K) {
      st = schur_dispatch(p->nb_max, d, stream);
      if (st) return st;
      DROID_LAUNCH_CHECK();
    }
    st = launch_wide(*p, d, stream);
    if (st) return st;
  }
  if (int st = ba_zero(d.M, (size_t)p->cs.nslots * kTile * sizeof(double), stream)) return st;
  if (d.nblk + p->P > 0) {
    ba_assemble_kernel<<<d.nblk + p->P, 256, 0, stream>>>(d);
    DROID_LAUNCH_CHECK();
  }
  return kOk;
}

// damping + Cholesky + forward/back solve of the reduced system -> dx
static int solve_system(BaPlan* p, void* workspace, float lm, float ep, float* dx, int first_solve,
                        hipStream_t stream) {
  BaDev d = make_dev(*p, static_cast<char*>(workspace));
  const int n = p->n;
  ba_damp_kernel<<<ceil_div(std::max(n, 1), 256), 256, 0, stream>>>(d.M, d.slot, d.nbc, n, lm, ep, d.flag,
                                                                     first_solve);
  DROID_LAUNCH_CHECK();
  if (n > 0) return launch_chol_dataflow(*p, static_cast<char*>(workspace), dx, stream);
  return kOk;
}

// back-substitution of dz + retraction (both skip on flag bit 1)
static int apply_update(BaPlan* p, void* workspace, float* poses, float* disps, const float* intrinsics,
                        const float* disps_sens, const float* targets, const float* weights, const float* eta,
                        float* dx, float* dz, hipStream_t stream) {
  BaDev d = make_dev(*p, static_cast<char*>(workspace));
  d.poses = poses; d.disps = disps; d.intr = intrinsics; d.disps_sens = disps_sens;
  d.targets = targets; d.weights = weights; d.eta = eta; d.dx = dx; d.dz = dz;
  if (!p->motion_only && p->K > 0) {
    if (!dz) return fail(kInvalidArgument, "ba: dz output required unless motion_only");
    ba_backsub_kernel<<<dim3(ceil_div(p->HW, 256), p->K), 256, 0, stream>>>(d);
    DROID_LAUNCH_CHECK();
  }
  if (p->P > 0) {
    ba_retract_kernel<<<ceil_div(p->P, 64), 64, 0, stream>>>(poses, dx, p->t0, p->P, d.flag);
    DROID_LAUNCH_CHECK();
  }
  return kOk;
}

static int solve_update(void* plan, void* workspace, float* poses, float* disps, const float* intrinsics,
                        const float* disps_sens, const float* targets, const float* weights, const float* eta,
                        float lm, float ep, float* dx, float* dz, int first_solve, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  if (!p->motion_only && p->K > 0 && !dz) return fail(kInvalidArgument, "ba: dz output required unless motion_only");
  st = solve_system(p, workspace, lm, ep, dx, first_solve, stream);
  if (st) return st;
  return apply_update(p, workspace, poses, disps, intrinsics, disps_sens, targets, weights, eta, dx, dz, stream);
}

// The two halves of droid_ba_solve_update, for a multi-GPU caller that agrees
// on the status between them (all-reduce MAX of the status words): every rank
// then skips the back-substitution and retraction together when any rank's
// dataflow solve timed out, instead of only the rank that timed out.
int droid_ba_solve_system(void* plan, void* workspace, float lm, float ep, float* dx, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  return solve_system(p, workspace, lm, ep, dx, 0, stream);
}

int droid_ba_apply_update(void* plan, void* workspace, float* poses, float* disps, const float* intrinsics,
                          const float* disps_sens, const float* targets, const float* weights, const float* eta,
                          float* dx, float* dz, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  return apply_update(p, workspace, poses, disps, intrinsics, disps_sens, targets, weights, eta, dx, dz, stream);
}

// Damped Cholesky solve of the (possibly all-reduced) system, back
// substitution and retraction (:1406-1428).  dz may be null for motion_only.
// Earlier solves' status bits accumulate in the sticky word until
// droid_ba_plan_clear_status.
int droid_ba_solve_update(void* plan, void* workspace, float* poses, float* disps,
                          const float* intrinsics, const float* disps_sens, const float* targets,
                          const float* weights, const float* eta, float lm, float ep,
                          float* dx, float* dz, hipStream_t stream) {
  return solve_update(plan, workspace, poses, disps, intrinsics, disps_sens, targets, weights, eta, lm, ep, dx, dz,
                      0, stream);
}

// Zero both status words (stream-ordered): the start of a staged BA call.
int droid_ba_plan_clear_status(void* plan, void* workspace, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  if (int st = ba_zero(static_cast<char*>(workspace) + p->off_flag, 16, stream)) return st;   // the two status words (+ 8 unused bytes of the 64-B flag region)
  return kOk;
}

// Byte offset of the status words in a plan's workspace (two int32): word 0 is
// the last solve's, word 1 the OR of the earlier solves' since the status was
// last cleared; bit 0 = a factorisation was not positive definite (dx = 0, as
// the reference), bit 1 = the dataflow solve timed out (that solve left poses /
// disparities unchanged).
int droid_ba_plan_flag_offset(const void* plan, size_t* offset) {
  auto* p = static_cast<const BaPlan*>(plan);
  if (!p || !offset) return fail(kInvalidArgument, "ba_plan_flag_offset: null argument");
  *offset = p->off_flag;
  return kOk;
}

// Dense lower triangle of A (n x n, row stride lda doubles) and b (n) into the
// tiles of a chol plan (droid_chol_plan_create), both fp64 device pointers.
int droid_chol_set_system(void* plan, void* workspace, const double* A, int lda, const double* b,
                          hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  if (lda < p->n) return fail(kInvalidArgument, "chol_set_system: lda < n");
  char* ws = static_cast<char*>(workspace);
  double* M = reinterpret_cast<double*>(ws + p->off_M);
  if (int st = ba_zero(M, (size_t)std::max(p->cs.nslots, 1) * kTile * sizeof(double), stream)) return st;
  if (p->n == 0) return kOk;
  const long total = (long)(p->n + 1) * p->n;
  chol_scatter_kernel<<<(int)((total + 255) / 256), 256, 0, stream>>>(
      M, reinterpret_cast<const int*>(ws + p->off_ints) + p->o_slot, p->cs.nbc, p->n, A, lda, b);
  DROID_LAUNCH_CHECK();
  return kOk;
}

// Dense damped SPD solve on a chol plan: diag += ep + lm*diag, factor,
// dx = solution (0 and flag bit 0 set if not SPD).
int droid_chol_solve(void* plan, void* workspace, float lm, float ep, float* dx, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  char* ws = static_cast<char*>(workspace);
  double* M = reinterpret_cast<double*>(ws + p->off_M);
  const int* slot = reinterpret_cast<const int*>(ws + p->off_ints) + p->o_slot;
  int* flag = reinterpret_cast<int*>(ws + p->off_flag);
  ba_damp_kernel<<<ceil_div(std::max(p->n, 1), 256), 256, 0, stream>>>(M, slot, p->cs.nbc, p->n, lm, ep, flag, 1);
  DROID_LAUNCH_CHECK();
  if (p->n == 0) return kOk;
  if (int st = launch_chol_dataflow(*p, ws, dx, stream)) return st;
  chol_fail_zero_kernel<<<ceil_div(p->n, 256), 256, 0, stream>>>(dx, p->n, flag);
  DROID_LAUNCH_CHECK();
  return kOk;
}

// Full ba(): `iterations` GN steps on one device (droid_backends.ba).
int droid_ba_run(void* plan, void* workspace, float* poses, float* disps, const float* intrinsics,
                 const float* disps_sens, const float* targets, const float* weights,
                 const float* eta, int iterations, float lm, float ep, float* dx, float* dz,
                 hipStream_t stream) {
  for (int it = 0; it < iterations; ++it) {
    int st = droid_ba_build_system(plan, workspace, poses, disps, intrinsics, disps_sens, targets,
                                   weights, eta, stream);
    if (st) return st;
    st = solve_update(plan, workspace, poses, disps, intrinsics, disps_sens, targets, weights, eta, lm, ep, dx, dz,
                      it == 0, stream);
    if (st) return st;
  }
  return kOk;
}

}  // extern "C"
