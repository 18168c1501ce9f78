// Dense bundle adjustment kernels for gfx950 (see ba.hpp for the pipeline).
// Numerics follow ba_cuda (droid_kernels.cu:176-424, 854-1434): fp32
// linearisation and Schur products, fp64 reduced system and Cholesky.
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
  const int *blka, *blkb, *blkcptr, *rhscptr;
  const int4 *contrib, *rhscontrib;
  float* hpart;
  float* gram;
  float* qw;
  double* M;
  double* x;
  int* flag;
  int E, N, H, W, HW, t0, t1, P, K, n, ld, eta_rows, nsplit, nchunk, gpw, nblk;
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
    for (int p = p0 + threadIdx.x; p < p1; p += 256) {
      PixLin L;
      linearize_pixel(T, false, fx, fy, cx, cy, (float)(p % d.W), (float)(p / d.W), dp[p],
                      tg[p], tg[HW + p], wt[p], wt[HW + p], L);
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
// Kernel C: deterministic assembly of the lower triangle of A - S (fp64) and
// of the rhs b - E Q w into row n of the augmented matrix.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float hess_val(const float* H, int r, int c) {
  if (r < c) { int t = r; r = c; c = t; }
  return H[r * (r + 1) / 2 + c];
}

__device__ __forceinline__ double gram_sum(const BaDev& d, int f, int i, int j) {
  if (i > j) { int t = i; i = j; j = t; }
  const int nb = d.fnb[f];
  const int I = i >> 4, J = j >> 4;
  const int tf = I * nb - I * (I - 1) / 2 + (J - I);
  const int Tf = nb * (nb + 1) / 2;
  const float* g = d.gram + d.fgoff[f] + (long)tf * 256 + (i & 15) * 16 + (j & 15);
  double s = 0.0;
  for (int c = 0; c < d.nchunk; ++c) s += (double)g[(long)c * Tf * 256];
  return s;
}

__global__ void __launch_bounds__(64) ba_assemble_kernel(BaDev d) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b < d.nblk) {
    if (t >= 36) return;
    const int r = t / 6, c = t % 6;
    double s = 0.0;
    for (int k = d.blkcptr[b]; k < d.blkcptr[b + 1]; ++k) {
      const int4 q = d.contrib[k];
      if (q.x == kEdgeBlock) {
        for (int sp = 0; sp < d.nsplit; ++sp)
          s += (double)hess_val(d.hpart + ((long)q.y * d.nsplit + sp) * kHessStride, q.z + r, q.w + c);
      } else {
        s -= gram_sum(d, q.y, 6 * q.z + r, 6 * q.w + c);
      }
    }
    d.M[(long)(6 * d.blka[b] + r) * d.ld + 6 * d.blkb[b] + c] = s;
  } else {
    const int a = b - d.nblk;
    if (t >= 6) return;
    double s = 0.0;
    for (int k = d.rhscptr[a]; k < d.rhscptr[a + 1]; ++k) {
      const int4 q = d.rhscontrib[k];
      if (q.x == kEdgeRhs) {
        for (int sp = 0; sp < d.nsplit; ++sp)
          s += (double)d.hpart[((long)q.y * d.nsplit + sp) * kHessStride + 78 + q.z + t];
      } else {
        const int wcol = 6 * (d.frptr[q.y + 1] - d.frptr[q.y]);
        s -= gram_sum(d, q.y, 6 * q.z + t, wcol);
      }
    }
    d.M[(long)d.n * d.ld + 6 * a + t] = s;
  }
}

// diag += ep + lm * diag  (SparseBlock::solve :1197) and reset the failure flag
__global__ void ba_damp_kernel(double* M, int n, int ld, float lm, float ep, int* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *flag = 0;
  if (i < n) {
    const double dg = M[(long)i * ld + i];
    M[(long)i * ld + i] = dg + ((double)ep + (double)lm * dg);
  }
}

// ---------------------------------------------------------------------------
// Blocked right-looking Cholesky, lower, in place, on the augmented matrix of
// n_aug = n+1 rows (rhs as row n) and n pivot columns: after factorisation,
// row n holds y = L^-1 b.
// ---------------------------------------------------------------------------
constexpr int CB = kCholBlock;

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)(u & 0xffffffffu), lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// Diagonal block: one wave, lane i owns row i of the 64x64 block in
// registers; column j is broadcast with v_readlane (no LDS, no barriers).
__global__ void __launch_bounds__(64) chol_diag_kernel(double* M, int n, int ld, int k0, int* flag) {
  const int i = threadIdx.x;
  const int Br = min(CB, n + 1 - k0);
  const int Bp = min(CB, n - k0);
  double r[CB];
  const double* src = M + (long)(k0 + i) * ld + k0;
#pragma unroll
  for (int c = 0; c < CB; ++c) r[c] = (i < Br && c <= i && c < Bp) ? src[c] : 0.0;
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    if (j < Bp) {
      const double piv = readlane_f64(r[j], j);
      if (i == 0 && !(piv > 0.0 && piv < 1e300)) atomicOr(flag, 1);
      const double sd = sqrt(piv);
      if (i == j) r[j] = sd;
      else if (i > j) r[j] = r[j] / sd;
      const double lij = r[j];
#pragma unroll
      for (int c = j + 1; c < CB; ++c) {
        const double lcj = readlane_f64(lij, c);
        r[c] = (c <= i) ? fma(-lij, lcj, r[c]) : r[c];
      }
    }
  }
  if (i < Br) {
    double* dst = M + (long)(k0 + i) * ld + k0;
#pragma unroll
    for (int c = 0; c < CB; ++c)
      if (c <= i && c < Bp) dst[c] = r[c];
  }
}

// rows below the diagonal block: X = A_ik L_kk^-T.  L_kk and the rows of X
// live in LDS; column-oriented elimination keeps every inner-loop update of a
// lane independent (pipelined LDS traffic, broadcast reads of L).
__global__ void __launch_bounds__(64) chol_trsm_kernel(double* M, int n, int ld, int k0) {
  __shared__ double L[CB][CB + 1];
  __shared__ double X[CB][CB + 1];
  const int i = threadIdx.x;
  const int Bp = min(CB, n - k0);
  const int row = k0 + CB * (blockIdx.x + 1) + i;
  for (int r = 0; r < CB; ++r) L[r][i] = (r < Bp && i <= r) ? M[(long)(k0 + r) * ld + k0 + i] : (r == i ? 1.0 : 0.0);
  const bool live = row <= n;
  const double* src = M + (long)row * ld + k0;
  for (int c = 0; c < CB; ++c) X[i][c] = (live && c < Bp) ? src[c] : 0.0;
  __syncthreads();
  for (int c = 0; c < CB; ++c) {
    const double xc = X[i][c] / L[c][c];
    X[i][c] = xc;
#pragma unroll 8
    for (int t = c + 1; t < CB; ++t) X[i][t] = fma(-xc, L[t][c], X[i][t]);
  }
  if (!live) return;
  double* dst = M + (long)row * ld + k0;
  for (int c = 0; c < Bp; ++c) dst[c] = X[i][c];
}

// trailing update: M[rb][cb] -= L[rb][k] L[cb][k]^T for k0 < cb <= rb
__global__ void __launch_bounds__(256) chol_update_kernel(double* M, int n, int ld, int k0) {
  __shared__ double Lr[CB][CB + 1];
  __shared__ double Lc[CB][CB + 1];
  const int kb = k0 / CB;
  const int rb = kb + 1 + blockIdx.y;
  const int cb = kb + 1 + blockIdx.x;
  const int nrowblk = ceil_div(n + 1, CB);
  const int ncolblk = ceil_div(n, CB);
  if (cb > rb || rb >= nrowblk || cb >= ncolblk) return;
  const int Bp = min(CB, n - k0);
  const int R0 = CB * rb, C0 = CB * cb;
  const int Br = min(CB, n + 1 - R0), Bc = min(CB, n - C0);
  for (int idx = threadIdx.x; idx < CB * CB; idx += 256) {
    const int r = idx / CB, t = idx % CB;
    Lr[r][t] = (r < Br && t < Bp) ? M[(long)(R0 + r) * ld + k0 + t] : 0.0;
    Lc[r][t] = (r < Bc && t < Bp) ? M[(long)(C0 + r) * ld + k0 + t] : 0.0;
  }
  __syncthreads();
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  for (int t = 0; t < Bp; ++t) {
    double ra[4], cbv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) ra[a] = Lr[4 * ty + a][t];
#pragma unroll
    for (int b = 0; b < 4; ++b) cbv[b] = Lc[tx + 16 * b][t];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] += ra[a] * cbv[b];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int r = 4 * ty + a;
    if (r >= Br) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = tx + 16 * b;
      if (c >= Bc) continue;
      if (rb == cb && c > r) continue;
      M[(long)(R0 + r) * ld + C0 + c] -= acc[a][b];
    }
  }
}

// back substitution L^T x = y (y = row n), one workgroup; writes dx (fp32),
// zeroed when the factorisation failed (SparseBlock::solve :1207-1210).
// Per 64-column block: stage L_bb in LDS, wave 0 solves it with register
// broadcasts, then all 1024 threads update the rhs of the earlier blocks with
// coalesced reads of the block's 64 rows.
__global__ void __launch_bounds__(1024) chol_backsolve_kernel(const double* M, int n, int ld,
                                                              const int* flag, double* xout,
                                                              float* dx) {
  extern __shared__ __attribute__((aligned(16))) double y[];
  __shared__ double Lb[CB][CB + 1];
  for (int k = threadIdx.x; k < n; k += blockDim.x) y[k] = M[(long)n * ld + k];
  const int ncolblk = ceil_div(n, CB);
  for (int cb = ncolblk - 1; cb >= 0; --cb) {
    const int c0 = CB * cb;
    const int Bc = min(CB, n - c0);
    for (int idx = threadIdx.x; idx < CB * CB; idx += blockDim.x) {
      const int r = idx / CB, c = idx % CB;
      Lb[r][c] = (r < Bc && c <= r) ? M[(long)(c0 + r) * ld + c0 + c] : (r == c ? 1.0 : 0.0);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int i = threadIdx.x;
      double yi = (i < Bc) ? y[c0 + i] : 0.0;
#pragma unroll
      for (int c = CB - 1; c >= 0; --c) {
        const double xc = readlane_f64(yi, c) / Lb[c][c];
        if (i == c) yi = xc;
        else if (i < c) yi = fma(-Lb[c][i], xc, yi);
      }
      if (i < Bc) y[c0 + i] = yi;
    }
    __syncthreads();
    for (int jx = threadIdx.x; jx < c0; jx += blockDim.x) {
      double s = 0.0;
      for (int c = 0; c < Bc; ++c) s = fma(M[(long)(c0 + c) * ld + jx], y[c0 + c], s);
      y[jx] -= s;
    }
    __syncthreads();
  }
  const bool failed = *flag != 0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    xout[k] = y[k];
    dx[k] = failed ? 0.0f : (float)y[k];
  }
}

// ---------------------------------------------------------------------------
// Kernel D: back substitution dz = Q (w - sum_rows E_row . dx[pose]) with the
// EvT6x1 skip of rows whose pose index is <= 0 (:1105), then disps += dz.
// grid = (ceil(HW/256), K).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ba_backsub_kernel(BaDev d) {
  __shared__ float Tsh[24 * 8];
  __shared__ float dxs[24 * 8];
  const int f = blockIdx.y;
  const int HW = d.HW;
  const int px = blockIdx.x * 256 + threadIdx.x;
  const int kf = d.kx[f];
  const int e0 = d.feptr[f], e1 = d.feptr[f + 1];
  const int t = threadIdx.x;
  if (t < e1 - e0) {
    const int e = d.fedges[e0 + t];
    const int jx = d.jj[e];
    SE3f T = (jx == kf) ? stereo_se3() : rel_se3(d.poses + 7 * kf, d.poses + 7 * jx);
    float* o = Tsh + 8 * t;
    o[0] = T.t[0]; o[1] = T.t[1]; o[2] = T.t[2];
    o[3] = T.q[0]; o[4] = T.q[1]; o[5] = T.q[2]; o[6] = T.q[3];
    o[7] = (jx == kf) ? 1.0f : 0.0f;
    const int pr = jx - d.t0;
    for (int k = 0; k < 6; ++k) dxs[8 * t + k] = (pr > 0 && pr < d.P) ? d.dx[6 * pr + k] : 0.0f;
    dxs[8 * t + 6] = (pr > 0 && pr < d.P) ? 1.0f : 0.0f;
  }
  __syncthreads();
  if (px >= HW) return;
  const float fx = d.intr[0], fy = d.intr[1], cx = d.intr[2], cy = d.intr[3];
  const float u = (float)(px % d.W), v = (float)(px / d.W);
  const float disp = d.disps[(long)kf * HW + px];
  const int pi = kf - d.t0;
  const bool use_ei = pi > 0 && pi < d.P;
  float Ei[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float acc = 0.f;
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
    linearize_pixel(T, stereo, fx, fy, cx, cy, u, v, disp, tg[px], tg[HW + px], wt[px], wt[HW + px], L);
    const float au = L.wu * L.Jzu, av = L.wv * L.Jzv;
    const float* dxe = dxs + 8 * (k - e0);
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
  if (use_ei) {
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

__global__ void ba_retract_kernel(float* poses, const float* dx, int t0, int P) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P) return;
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

static BaDev make_dev(BaPlan& p, char* ws) {
  BaDev d{};
  const int* I = reinterpret_cast<const int*>(ws + p.off_ints);
  d.ii = I + p.o_ii; d.jj = I + p.o_jj; d.kx = I + p.o_kx;
  d.feptr = I + p.o_feptr; d.fedges = I + p.o_fedges;
  d.frptr = I + p.o_frptr; d.rpose = I + p.o_rpose; d.redge = I + p.o_redge;
  d.fnb = I + p.o_fnb; d.fgoff = I + p.o_fgoff;
  d.blka = I + p.o_blka; d.blkb = I + p.o_blkb; d.blkcptr = I + p.o_blkcptr;
  d.rhscptr = I + p.o_rhscptr;
  d.contrib = reinterpret_cast<const int4*>(I + p.o_contrib);
  d.rhscontrib = reinterpret_cast<const int4*>(I + p.o_rhscontrib);
  d.hpart = reinterpret_cast<float*>(ws + p.off_hpart);
  d.gram = reinterpret_cast<float*>(ws + p.off_gram);
  d.qw = reinterpret_cast<float*>(ws + p.off_qw);
  d.M = reinterpret_cast<double*>(ws + p.off_M);
  d.x = reinterpret_cast<double*>(ws + p.off_x);
  d.flag = reinterpret_cast<int*>(ws + p.off_flag);
  d.E = p.E; d.N = p.N; d.H = p.H; d.W = p.W; d.HW = p.HW;
  d.t0 = p.t0; d.t1 = p.t1; d.P = p.P; d.K = p.K; d.n = p.n; d.ld = p.n + 1;
  d.eta_rows = p.eta_rows; d.nsplit = p.nsplit; d.nchunk = p.nchunk; d.gpw = p.group_per_wave;
  d.nblk = (int)p.blk_a.size();
  return d;
}

}  // namespace droid

using namespace droid;

extern "C" {

int droid_ba_plan_upload(void* plan, void* workspace, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  if (!p || !workspace) return fail(kInvalidArgument, "ba_plan_upload: null argument");
  DROID_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(workspace) + p->off_ints, p->ints.data(),
                                 p->ints.size() * sizeof(int), hipMemcpyHostToDevice, stream));
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
    st = schur_dispatch(p->nb_max, d, stream);
    if (st) return st;
    DROID_LAUNCH_CHECK();
  }
  DROID_HIP_CHECK(hipMemsetAsync(d.M, 0, (size_t)(p->n + 1) * (p->n + 1) * sizeof(double), stream));
  ba_assemble_kernel<<<d.nblk + p->P, 64, 0, stream>>>(d);
  DROID_LAUNCH_CHECK();
  return kOk;
}

// Damped Cholesky solve of the (possibly all-reduced) system, back
// substitution and retraction (:1406-1428).  dz may be null for motion_only.
int droid_ba_solve_update(void* plan, void* workspace, float* poses, float* disps,
                          const float* intrinsics, const float* disps_sens, const float* targets,
                          const float* weights, const float* eta, float lm, float ep,
                          float* dx, float* dz, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  BaDev d = make_dev(*p, static_cast<char*>(workspace));
  d.poses = poses; d.disps = disps; d.intr = intrinsics; d.disps_sens = disps_sens;
  d.targets = targets; d.weights = weights; d.eta = eta; d.dx = dx; d.dz = dz;
  d.lm = lm; d.ep = ep;
  const int n = p->n, ld = p->n + 1;
  ba_damp_kernel<<<ceil_div(n, 256), 256, 0, stream>>>(d.M, n, ld, lm, ep, d.flag);
  DROID_LAUNCH_CHECK();
  const int ncolblk = ceil_div(n, CB), nrowblk = ceil_div(n + 1, CB);
  for (int kb = 0; kb < ncolblk; ++kb) {
    const int k0 = CB * kb;
    chol_diag_kernel<<<1, 64, 0, stream>>>(d.M, n, ld, k0, d.flag);
    const int below = nrowblk - kb - 1;
    if (below > 0) {
      chol_trsm_kernel<<<below, 64, 0, stream>>>(d.M, n, ld, k0);
      chol_update_kernel<<<dim3(below, below), 256, 0, stream>>>(d.M, n, ld, k0);
    }
  }
  DROID_LAUNCH_CHECK();
  static int backsolve_lds = 0;
  const int need = n * (int)sizeof(double);
  if (need > backsolve_lds) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&chol_backsolve_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, need));
    backsolve_lds = need;
  }
  if (need > 160 * 1024) return fail(kUnsupported, "ba: reduced system too large for the single-WG back solve");
  chol_backsolve_kernel<<<1, 1024, (size_t)n * sizeof(double), stream>>>(d.M, n, ld, d.flag, d.x, dx);
  DROID_LAUNCH_CHECK();
  if (!p->motion_only && p->K > 0) {
    if (!dz) return fail(kInvalidArgument, "ba: dz output required unless motion_only");
    ba_backsub_kernel<<<dim3(ceil_div(p->HW, 256), p->K), 256, 0, stream>>>(d);
    DROID_LAUNCH_CHECK();
  }
  ba_retract_kernel<<<ceil_div(p->P, 64), 64, 0, stream>>>(poses, dx, p->t0, p->P);
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
    st = droid_ba_solve_update(plan, workspace, poses, disps, intrinsics, disps_sens, targets,
                               weights, eta, lm, ep, dx, dz, stream);
    if (st) return st;
  }
  return kOk;
}

}  // extern "C"
