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
// Dataflow Cholesky + solve: ONE persistent launch.
//
// The augmented system (n pivots, rhs as row n, rows of ld doubles) is cut
// into 64x64 tiles.  Workgroups (one per CU) take tasks by ticket in the
// host's critical-path order (ba_plan.cpp build_chol_tasks) and wait for
// their inputs on per-tile version counters: ver(i,j) = number of updates
// applied, +1 when the tile is final.  A task that is handed out only after
// all its predecessors were handed out never waits on a workgroup that has
// not started, so progress does not depend on residency.
//
// Cross-workgroup hand-off follows cdna_hip_programming.md Guideline 16 R1:
// every handed-off byte (tiles, Linv, y, x) is stored AND loaded with sc1
// buffer operations (write-through / L1 bypass), every storing wave drains
// vmcnt before the workgroup barrier, then one lane stores the counter with
// an agent-scope atomic; consumers poll relaxed.  Spins are bounded (an
// abort word stops every workgroup).  Tiles are products of f64 MFMA
// (v_mfma_f64_16x16x4f64); the diagonal factor is panel-blocked (16 wide)
// with register rows and LDS column broadcasts, and also returns L_kk^-1 so
// the off-diagonal solves are GEMMs.
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
constexpr int kCholLds = (3 * 64 * LT + 256 + 4 * 272) * 8 + 16;
#ifdef DROID_CHOL_TRACE
#define CHOL_TRACE(...) do { if (threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
#else
#define CHOL_TRACE(...) do { } while (0)
#endif
// debug-only progress marks (DROID_CHOL_MARKS=<device address of an int[grid*4]>):
// per workgroup {ticket, phase, wave-0 phase, heartbeat}, system-scope stores a
// host copy engine can read while the kernel runs
#define CHOL_MARK(slot, v)                                                                          \
  do {                                                                                              \
    if (d.marks && (threadIdx.x & 63) == 0)                                                         \
      __hip_atomic_store(d.marks + 16 * blockIdx.x + 4 * (threadIdx.x >> 6) + (slot), (v),          \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                              \
  } while (0)

struct CholDev {
  double* M;
  int n, ld, nbc, nbr;
  const int4* tasks;
  int ntasks;
  int* sync;    // [0] ticket [1] abort [4..] ver[nbr*nbc] | yver[nbc] | xdone[nbc]
  int* flag;    // bit 0: factorisation failed (dx = 0), bit 1: spin timeout
  double* linv; // [nbc][64][64]
  double* ybuf; // [nbc*64]
  double* x;    // [n]
  float* dx;    // [n]
  int debug;    // unused (tracing is compile-time: DROID_CHOL_TRACE)
  int* marks;   // debug progress marks or null
  long long* tprof;  // debug per-ticket timeline {wg|type<<12|i<<16|j<<32|k<<48, got, deps ok, published} (s_memrealtime) or null
};

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

// rows [R0,R0+nr) x cols [C0,C0+nc) of a row-major matrix with `ld` doubles per
// row -> LDS T[64][LT]; zeros elsewhere (out-of-range offsets read 0).  nc even.
__device__ __forceinline__ void tile_load(__amdgpu_buffer_rsrc_t r, int ld, int R0, int C0, int nr, int nc,
                                          double* T) {
  dbl2 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    const unsigned off = (rr < nr && cc < nc) ? (unsigned)(((size_t)(R0 + rr) * ld + C0 + cc) * 8) : kOobOff;
    v[q] = ld2(r, off);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    *reinterpret_cast<dbl2*>(&T[rr * LT + cc]) = v[q];
  }
}
// the same load split in two, so the global latency overlaps other work
__device__ __forceinline__ void tile_issue(__amdgpu_buffer_rsrc_t r, int ld, int R0, int C0, int nr, int nc,
                                           dbl2 (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    const unsigned off = (rr < nr && cc < nc) ? (unsigned)(((size_t)(R0 + rr) * ld + C0 + cc) * 8) : kOobOff;
    v[q] = ld2(r, off);
  }
}
__device__ __forceinline__ void tile_commit(const dbl2 (&v)[8], double* T) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    *reinterpret_cast<dbl2*>(&T[rr * LT + cc]) = v[q];
  }
}
__device__ __forceinline__ void tile_store(__amdgpu_buffer_rsrc_t r, int ld, int R0, int C0, int nr, int nc,
                                           const double* T) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + 256 * q, rr = p >> 5, cc = (p & 31) * 2;
    if (rr < nr && cc < nc)
      st2(r, (unsigned)(((size_t)(R0 + rr) * ld + C0 + cc) * 8), *reinterpret_cast<const dbl2*>(&T[rr * LT + cc]));
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

// wave-uniform lane -> every lane (two v_readlane_b32, no LDS round trip)
__device__ __forceinline__ double bcast_lane(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// 1/sqrt(x) in fp64: v_rsq_f64 + two Newton steps (no division, no sqrt
// expansion on the critical path; ~1 ulp, far inside the 1e-4 parity bar)
__device__ __forceinline__ double rsqrt_f64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  y = y * fma(-hx * y, y, 1.5);
  return y;
}

// 16-wide panel of the diagonal factor: wave 0, lane r owns row r's panel
// values in registers; pivots and scaled column entries are broadcast with
// v_readlane (wave-synchronous: no LDS, no waits, no branches).  Lanes above
// the diagonal update their (never read) upper-triangle entries too, and
// pivot columns past the block's Bp real columns use a unit pivot, so every
// panel is a full, branch-free 16 columns.
// dinv[c] = 1 / L[c][c].
__device__ __forceinline__ void panel_factor(double* T, double* dinv, int c0, int Bp, int lane, int* flag) {
  double v[16], invs[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = T[lane * LT + c0 + q];
  bool bad = false;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    const bool real = c0 + jj < Bp;  // wave-uniform
    const double piv = real ? bcast_lane(v[jj], c0 + jj) : 1.0;
    bad |= !(piv > 0.0 && piv < 1e300);
    const double inv = rsqrt_f64(piv);
    invs[jj] = inv;
    v[jj] *= inv;  // the diagonal lane gets piv / sqrt(piv)
#pragma unroll
    for (int q = jj + 1; q < 16; ++q) v[q] = fma(-v[jj], bcast_lane(v[jj], c0 + q), v[q]);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) T[lane * LT + c0 + q] = v[q];
  double mine = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) mine = (lane == q) ? invs[q] : mine;
  if (lane < 16) dinv[c0 + lane] = mine;
  if (bad && lane == 0) atomicOr(flag, 1);
}

__global__ void __launch_bounds__(256) chol_dataflow_kernel(CholDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* T0 = sm;
  double* T1 = sm + 64 * LT;
  double* T2 = sm + 2 * 64 * LT;
  double* vec = sm + 3 * 64 * LT;        // 256
  double* scr = vec + 256;               // [4][16][17]
  int* shi = reinterpret_cast<int*>(scr + 4 * 272);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: wave-conditional code branches, never masks
  const int fr = lane & 15, fk = lane >> 4;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int n = d.n, ld = d.ld, nbc = d.nbc, nbr = d.nbr;
  const __amdgpu_buffer_rsrc_t rM = mkrs(d.M, (size_t)(n + 1) * ld * 8);
  const __amdgpu_buffer_rsrc_t rL = mkrs(d.linv, (size_t)nbc * 4096 * 8);
  const __amdgpu_buffer_rsrc_t rY = mkrs(d.ybuf, (size_t)nbc * 64 * 8);
  const __amdgpu_buffer_rsrc_t rX = mkrs(d.x, (size_t)n * 8);
  int* ticket = d.sync;
  int* abort_w = d.sync + 1;
  int* ver = d.sync + 4;
  int* yver = ver + nbr * nbc;
  int* xdone = yver + nbc;

  int nbar = 0;
#define BAR() do { ++nbar; CHOL_MARK(3, nbar); __syncthreads(); } while (0)
  for (;;) {
    if (tid == 0) shi[0] = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    BAR();
    const int tk = __builtin_amdgcn_readfirstlane(shi[0]);
    const unsigned long long t_got = d.tprof ? __builtin_amdgcn_s_memrealtime() : 0ull;
    CHOL_MARK(0, tk);
    CHOL_MARK(1, 1);
    CHOL_TRACE("[chol] wg %d got ticket %d\n", (int)blockIdx.x, tk);
    if (tk >= d.ntasks) break;
    const int4 tsk = d.tasks[tk];
    const int type = __builtin_amdgcn_readfirstlane(tsk.x), i = __builtin_amdgcn_readfirstlane(tsk.y);
    const int j = __builtin_amdgcn_readfirstlane(tsk.z), k = __builtin_amdgcn_readfirstlane(tsk.w);
    CHOL_TRACE("[chol] wg %d ticket %d task %d (%d,%d,%d)\n", (int)blockIdx.x, tk, type, i, j, k);
    if (tid == 0) {
      bool ok = true;
      switch (type) {
        case kPotrf:  // all updates of the tile but the last (done here); L(k, k-1) is awaited below
          ok = poll_ge(&ver[k * nbc + k], k > 0 ? k - 1 : 0, abort_w, d.flag);
          break;
        case kTrsm:
          ok = poll_ge(&ver[i * nbc + k], k, abort_w, d.flag) && poll_ge(&ver[k * nbc + k], k + 1, abort_w, d.flag);
          break;
        case kUpdate:
          ok = poll_ge(&ver[i * nbc + j], k, abort_w, d.flag) && poll_ge(&ver[i * nbc + k], k + 1, abort_w, d.flag) &&
               poll_ge(&ver[j * nbc + k], k + 1, abort_w, d.flag);
          break;
        case kBsolve:
          ok = poll_ge(&ver[i * nbc + i], i + 1, abort_w, d.flag) &&
               poll_ge(&yver[i], 1 + (nbc - 1 - i), abort_w, d.flag);
          break;
        default:  // kBupd (r = i, c = j)
          ok = poll_ge(&xdone[i], 1, abort_w, d.flag) && poll_ge(&ver[i * nbc + j], j + 1, abort_w, d.flag) &&
               poll_ge(&yver[j], 1 + (nbc - 1 - i), abort_w, d.flag);
          break;
      }
      shi[1] = ok ? 1 : 0;
    }
    BAR();
    CHOL_TRACE("[chol] wg %d ticket %d deps %s\n", (int)blockIdx.x, tk, shi[1] ? "ok" : "ABORT");
    if (!__builtin_amdgcn_readfirstlane(shi[1])) break;
    CHOL_MARK(1, 2);
    if (d.tprof && tid == 0) {
      d.tprof[4 * tk + 0] = (long long)blockIdx.x | ((long long)type << 12) | ((long long)i << 16) | ((long long)j << 32) |
                           ((long long)k << 48);
      d.tprof[4 * tk + 1] = (long long)t_got;
      d.tprof[4 * tk + 2] = (long long)__builtin_amdgcn_s_memrealtime();
    }

    if (type == kPotrf) {
      int ps = 0;
#define PSTAMP() do { if (d.tprof && tid == 0) d.tprof[65536 + 16 * k + (ps < 15 ? ps : 15)] = (long long)__builtin_amdgcn_s_memrealtime(); ++ps; } while (0)
      const int R0 = 64 * k, Bp = min(64, n - R0), Br = min(64, n + 1 - R0);
      dbl2 pre[8];
      tile_issue(rM, ld, R0, R0, Br, Bp, pre);  // A(k,k) is final but for (k,k,k-1): load while L(k,k-1) is awaited
      if (k > 0) {  // the tile's last update (k, k, k-1): T0 -= L(k,k-1) L(k,k-1)^T
        if (tid == 0) shi[1] = poll_ge(&ver[k * nbc + k - 1], k, abort_w, d.flag) ? 1 : 0;
        BAR();
        if (!__builtin_amdgcn_readfirstlane(shi[1])) break;
        tile_load(rM, ld, R0, R0 - 64, Br, 64, T1);
        tile_commit(pre, T0);
        BAR();
        dbl4 acc[2][2];
        acc_load(T0, acc, wr, wc, lane);
        gemm_nt64(T1, T1, acc, wr, wc, lane, -1.0);
        acc_store(T0, acc, wr, wc, lane);
      } else {
        tile_commit(pre, T0);
      }
      BAR(); PSTAMP();
      CHOL_TRACE("[chol] potrf %d loaded Bp %d Br %d\n", k, Bp, Br);
      for (int c0 = 0; c0 < Bp; c0 += 16) {  // whole 16-wide panels (unit-padded)
        CHOL_MARK(1, 100 + c0);
        if (wave == 0) panel_factor(T0, vec + 128, c0, Bp, lane, d.flag);
        if (wave == 0) CHOL_MARK(2, 100 + c0);
        BAR(); PSTAMP();
        CHOL_MARK(1, 200 + c0);
        CHOL_TRACE("[chol] potrf %d panel %d done\n", k, c0);
        const int s0 = c0 + 16;
        const int nt = (64 - s0) / 16;
        for (int ti = wave; ti < nt * nt; ti += 4) {
          const int R = s0 + 16 * (ti / nt), C = s0 + 16 * (ti % nt);
          if (C > R) continue;
          dbl4 acc;
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = T0[(R + 4 * q + fk) * LT + C + fr];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            acc = mfma64(-T0[(R + fr) * LT + c0 + 4 * kk + fk], T0[(C + fr) * LT + c0 + 4 * kk + fk], acc);
#pragma unroll
          for (int q = 0; q < 4; ++q) T0[(R + 4 * q + fk) * LT + C + fr] = acc[q];
        }
        BAR(); PSTAMP();
      }
      CHOL_TRACE("[chol] potrf %d factored\n", k);
      CHOL_MARK(1, 300);
      const bool below = k + 1 < nbr;  // trsm(k+1, k) runs in this task
      const int R1 = R0 + 64, nr1 = below ? min(64, n + 1 - R1) : 0;
      if (below && tid == 0) shi[2] = poll_ge(&ver[(k + 1) * nbc + k], k, abort_w, d.flag) ? 1 : 0;
      // Linv of the Bp x Bp pivot block (unit-diagonal padding past Bp)
      for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int r = idx >> 6, c = idx & 63;
        T2[r * LT + c] = (r < Bp) ? (c <= r ? T0[r * LT + c] : 0.0) : (r == c ? 1.0 : 0.0);
        T1[r * LT + c] = 0.0;
      }
      if (tid >= Bp && tid < 64) vec[128 + tid] = 1.0;  // unit padding of the pivot block
      BAR(); PSTAMP();
      if (below) {
        if (!__builtin_amdgcn_readfirstlane(shi[2])) break;
        tile_issue(rM, ld, R1, R0, nr1, Bp, pre);  // lands during the Linv work
      }
      if (wave == 0) {  // the four 16x16 diagonal blocks; lane = 16 * block + column
        const int base = 16 * (lane >> 4), cc = lane & 15;
        double xv[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          double sacc = (t == cc) ? 1.0 : 0.0;
#pragma unroll
          for (int u = 0; u < t; ++u) sacc = fma(-T2[(base + t) * LT + base + u], xv[u], sacc);
          xv[t] = sacc * vec[128 + base + t];  // 1 / L[t][t] from the panel
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) T1[(base + t) * LT + base + cc] = xv[t];
      }
      BAR(); PSTAMP();
      for (int I = 1; I < 4; ++I) {  // Linv[I][J] = -Dinv_I sum_{K=J}^{I-1} L[I][K] Linv[K][J]
        if (wave < I) {
          const int J = wave;
          dbl4 S = {0.0, 0.0, 0.0, 0.0};
          for (int K = J; K < I; ++K)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
              S = mfma64(T2[(16 * I + fr) * LT + 16 * K + 4 * kk + fk], T1[(16 * K + 4 * kk + fk) * LT + 16 * J + fr], S);
          double* sw = scr + wave * 272;
#pragma unroll
          for (int q = 0; q < 4; ++q) sw[(4 * q + fk) * 17 + fr] = S[q];
          asm volatile("" ::: "memory");
          dbl4 R = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            R = mfma64(-T1[(16 * I + fr) * LT + 16 * I + 4 * kk + fk], sw[(4 * kk + fk) * 17 + fr], R);
#pragma unroll
          for (int q = 0; q < 4; ++q) T1[(16 * I + 4 * q + fk) * LT + 16 * J + fr] = R[q];
        }
        BAR(); PSTAMP();
        CHOL_TRACE("[chol] potrf %d linv row %d\n", k, I);
      }
      CHOL_MARK(1, 400);
      tile_store(rM, ld, R0, R0, Br, Bp, T0);
      tile_store(rL, 64, R0, 0, 64, 64, T1);
      const bool rhs = Br > Bp;
      if (rhs && tid < 32) st2(rY, (unsigned)((R0 + 2 * tid) * 8), *reinterpret_cast<const dbl2*>(&T0[Bp * LT + 2 * tid]));
      CHOL_TRACE("[chol] potrf %d stored\n", k);
      if (below) {  // trsm(k+1, k): L(k+1,k) = A(k+1,k) L_kk^-T with L_kk^-1 still in T1
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        BAR();  // T0's store reads are done
        tile_commit(pre, T0);
        BAR();
        dbl4 acc[2][2] = {};
        gemm_nt64(T0, T1, acc, wr, wc, lane, 1.0);
        BAR();
        acc_store(T0, acc, wr, wc, lane);
        BAR();
        tile_store(rM, ld, R1, R0, nr1, Bp, T0);
        const bool rhs1 = (k + 1 == nbr - 1);
        if (rhs1 && tid < 32) st2(rY, (unsigned)((R0 + 2 * tid) * 8), *reinterpret_cast<const dbl2*>(&T0[(n - R1) * LT + 2 * tid]));
        publish(&ver[k * nbc + k], k + 1, &ver[(k + 1) * nbc + k], k + 1, rhs1 ? &yver[k] : nullptr, 1);
      } else {
        publish(&ver[k * nbc + k], k + 1, rhs ? &yver[k] : nullptr, 1);
      }
      CHOL_TRACE("[chol] potrf %d published\n", k);
      PSTAMP();
#undef PSTAMP
    } else if (type == kTrsm) {
      const int R0 = 64 * i, C0 = 64 * k, nr = min(64, n + 1 - R0), nc = min(64, n - C0);
      tile_load(rM, ld, R0, C0, nr, nc, T0);
      tile_load(rL, 64, C0, 0, 64, 64, T1);
      BAR();
      CHOL_TRACE("[chol] trsm %d,%d loaded\n", i, k);
      dbl4 acc[2][2] = {};
      gemm_nt64(T0, T1, acc, wr, wc, lane, 1.0);
      BAR();
      CHOL_TRACE("[chol] trsm %d,%d gemm\n", i, k);
      acc_store(T0, acc, wr, wc, lane);
      BAR();
      tile_store(rM, ld, R0, C0, nr, nc, T0);
      const bool rhs = (i == nbr - 1);
      if (rhs && tid < 32) st2(rY, (unsigned)((C0 + 2 * tid) * 8), *reinterpret_cast<const dbl2*>(&T0[(n - R0) * LT + 2 * tid]));
      CHOL_TRACE("[chol] trsm %d,%d stored\n", i, k);
      publish(&ver[i * nbc + k], k + 1, rhs ? &yver[k] : nullptr, 1);
      CHOL_TRACE("[chol] trsm %d,%d published\n", i, k);
    } else if (type == kUpdate) {
      const int Ri = 64 * i, Rj = 64 * j, Ck = 64 * k;
      const int nri = min(64, n + 1 - Ri), ncj = min(64, n - Rj), nck = min(64, n - Ck);
      tile_load(rM, ld, Ri, Ck, nri, nck, T0);
      tile_load(rM, ld, Rj, Ck, ncj, nck, T1);
      tile_load(rM, ld, Ri, Rj, nri, ncj, T2);
      BAR();
      dbl4 acc[2][2];
      acc_load(T2, acc, wr, wc, lane);
      gemm_nt64(T0, T1, acc, wr, wc, lane, -1.0);
      acc_store(T2, acc, wr, wc, lane);
      BAR();
      tile_store(rM, ld, Ri, Rj, nri, ncj, T2);
      publish(&ver[i * nbc + j], k + 1);
    } else if (type == kBsolve) {  // x_i = L_ii^-T y_i, then bupd(i, i-1): y_{i-1} -= L(i,i-1)^T x_i
      const int C0 = 64 * i, Bp = min(64, n - C0);
      tile_load(rL, 64, C0, 0, 64, 64, T1);
      if (i > 0) tile_load(rM, ld, C0, C0 - 64, Bp, 64, T0);
      CHOL_TRACE("[chol] bsolve %d tile issued\n", i);
      if (tid < 32) {
        const dbl2 yv = ld2(rY, 2 * tid < Bp ? (unsigned)((C0 + 2 * tid) * 8) : kOobOff);
        vec[2 * tid] = yv[0];
        vec[2 * tid + 1] = yv[1];
      }
      BAR();
      if (wave == 0) {
        double sacc = 0.0;
#pragma unroll 8
        for (int t = 0; t < 64; ++t) sacc = fma(T1[t * LT + lane], vec[t], sacc);
        const bool failed = (__hip_atomic_load(d.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1) != 0;
        if (lane < Bp) {
          st1(rX, (unsigned)((C0 + lane) * 8), sacc);
          d.dx[C0 + lane] = failed ? 0.0f : (float)sacc;
        }
        vec[64 + lane] = lane < Bp ? sacc : 0.0;
      }
      CHOL_TRACE("[chol] bsolve %d computed\n", i);
      publish(&xdone[i], 1);
      CHOL_TRACE("[chol] bsolve %d published\n", i);
      if (i > 0) {
        if (tid == 0) shi[1] = poll_ge(&yver[i - 1], 1 + (nbc - 1 - i), abort_w, d.flag) ? 1 : 0;
        BAR();
        if (!__builtin_amdgcn_readfirstlane(shi[1])) break;
        if (tid < 64) vec[128 + tid] = ld1(rY, (unsigned)((C0 - 64 + tid) * 8));
        BAR();
        if (wave == 0) {
          double sacc = vec[128 + lane];
#pragma unroll 8
          for (int t = 0; t < 64; ++t) sacc = fma(-T0[t * LT + lane], vec[64 + t], sacc);
          st1(rY, (unsigned)((C0 - 64 + lane) * 8), sacc);
        }
        publish(&yver[i - 1], 1 + (nbc - i));
      }
    } else {  // kBupd: y_c -= L_rc^T x_r
      const int R0 = 64 * i, C0 = 64 * j, nr = min(64, n - R0), nc = min(64, n - C0);
      tile_load(rM, ld, R0, C0, nr, nc, T0);
      if (tid < 64) vec[tid] = ld1(rX, tid < nr ? (unsigned)((R0 + tid) * 8) : kOobOff);
      else if (tid < 128) vec[tid] = ld1(rY, tid - 64 < nc ? (unsigned)((C0 + tid - 64) * 8) : kOobOff);
      BAR();
      if (wave == 0) {
        double sacc = vec[64 + lane];
#pragma unroll 8
        for (int t = 0; t < 64; ++t) sacc = fma(-T0[t * LT + lane], vec[t], sacc);
        if (lane < nc) st1(rY, (unsigned)((C0 + lane) * 8), sacc);
      }
      publish(&yver[j], 1 + (nbc - i));
    }
    if (d.tprof && tid == 0) d.tprof[4 * tk + 3] = (long long)__builtin_amdgcn_s_memrealtime();
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
  d.t0 = p.t0; d.t1 = p.t1; d.P = p.P; d.K = p.K; d.n = p.n; d.ld = p.ld;
  d.eta_rows = p.eta_rows; d.nsplit = p.nsplit; d.nchunk = p.nchunk; d.gpw = p.group_per_wave;
  d.nblk = (int)p.blk_a.size();
  return d;
}

// the previous launch-per-step blocked factorisation (A/B reference: DROID_CHOL=blocked)
static int chol_blocked(const BaDev& d, int n, int ld, float* dx, hipStream_t stream) {
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
  return kOk;
}

static bool use_dataflow_chol() {
  static const bool on = [] {
    const char* e = getenv("DROID_CHOL");
    return !(e && std::string(e) == "blocked");
  }();
  return on;
}

static int num_cus() { return device_cu_count(); }

static int launch_chol_dataflow(const BaPlan& p, char* ws, const BaDev& bd, float* dx, hipStream_t stream) {
  if ((size_t)(p.n + 1) * p.ld * 8 >= 0x80000000ull)
    return fail(kUnsupported, "ba: reduced system exceeds the 2 GB dense-solver limit");
  CholDev c{};
  c.M = bd.M; c.n = p.n; c.ld = p.ld; c.nbc = p.nbc; c.nbr = p.nbr;
  c.tasks = reinterpret_cast<const int4*>(reinterpret_cast<const int*>(ws + p.off_ints) + p.o_tasks);
  c.ntasks = p.ntasks;
  c.sync = reinterpret_cast<int*>(ws + p.off_sync);
  c.flag = bd.flag;
  c.linv = reinterpret_cast<double*>(ws + p.off_linv);
  c.ybuf = reinterpret_cast<double*>(ws + p.off_ybuf);
  c.x = bd.x;
  c.dx = dx;
  static int* const marks = getenv("DROID_CHOL_MARKS") ? reinterpret_cast<int*>(strtoull(getenv("DROID_CHOL_MARKS"), nullptr, 0)) : nullptr;
  c.marks = marks;
  static long long* const tprof =
      getenv("DROID_CHOL_TPROF") ? reinterpret_cast<long long*>(strtoull(getenv("DROID_CHOL_TPROF"), nullptr, 0)) : nullptr;
  c.tprof = tprof;
  static bool attr = false;
  if (!attr) {
    DROID_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&chol_dataflow_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kCholLds));
    attr = true;
  }
  DROID_HIP_CHECK(hipMemsetAsync(c.sync, 0, p.sync_bytes, stream));
  const int grid = std::min(p.ntasks, num_cus());
  chol_dataflow_kernel<<<grid, 256, kCholLds, stream>>>(c);
  DROID_LAUNCH_CHECK();
  return kOk;
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
  DROID_HIP_CHECK(hipMemsetAsync(d.M, 0, (size_t)(p->n + 1) * p->ld * sizeof(double), stream));
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
  const int n = p->n, ld = p->ld;
  ba_damp_kernel<<<ceil_div(std::max(n, 1), 256), 256, 0, stream>>>(d.M, n, ld, lm, ep, d.flag);
  DROID_LAUNCH_CHECK();
  if (n > 0 && use_dataflow_chol()) {
    st = launch_chol_dataflow(*p, static_cast<char*>(workspace), d, dx, stream);
    if (st) return st;
  } else if (n > 0) {
    st = chol_blocked(d, n, ld, dx, stream);
    if (st) return st;
  }
  if (!p->motion_only && p->K > 0) {
    if (!dz) return fail(kInvalidArgument, "ba: dz output required unless motion_only");
    ba_backsub_kernel<<<dim3(ceil_div(p->HW, 256), p->K), 256, 0, stream>>>(d);
    DROID_LAUNCH_CHECK();
  }
  ba_retract_kernel<<<ceil_div(std::max(p->P, 1), 64), 64, 0, stream>>>(poses, dx, p->t0, p->P);
  DROID_LAUNCH_CHECK();
  return kOk;
}


// Dense damped SPD solve on a chol plan (droid_chol_plan_create): diag += ep +
// lm*diag, factor, dx = solution (0 and flag bit 0 set if not SPD).
int droid_chol_solve(void* plan, void* workspace, float lm, float ep, float* dx, hipStream_t stream) {
  auto* p = static_cast<BaPlan*>(plan);
  int st = check_ready(p, workspace);
  if (st) return st;
  char* ws = static_cast<char*>(workspace);
  BaDev d{};
  d.M = reinterpret_cast<double*>(ws + p->off_M);
  d.x = reinterpret_cast<double*>(ws + p->off_x);
  d.flag = reinterpret_cast<int*>(ws + p->off_flag);
  d.n = p->n;
  d.ld = p->ld;
  ba_damp_kernel<<<ceil_div(std::max(p->n, 1), 256), 256, 0, stream>>>(d.M, p->n, p->ld, lm, ep, d.flag);
  DROID_LAUNCH_CHECK();
  if (p->n == 0) return kOk;
  return use_dataflow_chol() ? launch_chol_dataflow(*p, ws, d, dx, stream) : chol_blocked(d, p->n, p->ld, dx, stream);
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
