// Geometry kernels for gfx950.
//
//  projective_transform  DepthVideo.reproject -> pops.projective_transform
//                        (projective_ops.py:96-125) fused with the update()
//                        motion features (factor_graph.py:202-204)
//  frame_distance        droid_kernels.cu:518-657
//  projmap               droid_kernels.cu:427-516
//  iproj                 droid_kernels.cu:779-850
//  depth_filter          droid_kernels.cu:661-775 (per-pixel loop over the 6
//                        neighbours instead of atomics: deterministic)
#include "common.hpp"

namespace droid {

__device__ __forceinline__ SE3f load_pose_mul_inv(const float* poses, int i, int j) {
  // lietorch: Gij = poses[j] * poses[i].inv()  -> (q_j q_i^*, t_j - R(q_j) R(q_i)^-1 t_i)
  SE3f Ti = load_pose(poses, i), Tj = load_pose(poses, j);
  const float qi_inv[4] = {-Ti.q[0], -Ti.q[1], -Ti.q[2], Ti.q[3]};
  float ti_inv[3], tmp[3];
  act_so3(qi_inv, Ti.t, tmp);
  ti_inv[0] = -tmp[0]; ti_inv[1] = -tmp[1]; ti_inv[2] = -tmp[2];
  SE3f G;
  // Hamilton product qj (x) qi_inv
  const float* a = Tj.q; const float* b = qi_inv;
  G.q[0] = a[3] * b[0] + b[3] * a[0] + a[1] * b[2] - a[2] * b[1];
  G.q[1] = a[3] * b[1] + b[3] * a[1] + a[2] * b[0] - a[0] * b[2];
  G.q[2] = a[3] * b[2] + b[3] * a[2] + a[0] * b[1] - a[1] * b[0];
  G.q[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  float rt[3];
  act_so3(Tj.q, ti_inv, rt);
  G.t[0] = Tj.t[0] + rt[0]; G.t[1] = Tj.t[1] + rt[1]; G.t[2] = Tj.t[2] + rt[2];
  return G;
}

// coords (E,H,W,2); valid (E,H,W) optional; motn (E,4,H,W) optional (needs target (E,H,W,2)).
__global__ void __launch_bounds__(256)
projective_transform_kernel(const float* __restrict__ poses, const float* __restrict__ disps,
                            const float* __restrict__ intr, const int64_t* __restrict__ ii,
                            const int64_t* __restrict__ jj, int H, int W,
                            float* __restrict__ coords, float* __restrict__ valid,
                            const float* __restrict__ target, float* __restrict__ motn) {
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = blockIdx.y;
  if (p >= HW) return;
  const int i = (int)ii[e], j = (int)jj[e];
  SE3f G;
  if (i == j) G = stereo_se3();
  else G = load_pose_mul_inv(poses, i, j);
  const float* ki = intr + 4 * i;
  const float* kj = intr + 4 * j;
  const float u = (float)(p % W), v = (float)(p / W);
  const float X0[4] = {(u - ki[2]) / ki[0], (v - ki[3]) / ki[1], 1.0f, disps[(long)i * HW + p]};
  float X1[4];
  act_se3(G, X0, X1);
  const float Z = (X1[2] < 0.1f) ? 1.0f : X1[2];
  const float d = 1.0f / Z;
  const float x = kj[0] * (X1[0] * d) + kj[2];
  const float y = kj[1] * (X1[1] * d) + kj[3];
  const long o = (long)e * HW + p;
  coords[2 * o + 0] = x;
  coords[2 * o + 1] = y;
  if (valid) valid[o] = (X1[2] > 0.2f && X0[2] > 0.2f) ? 1.0f : 0.0f;
  if (motn) {
    const float tx = target[2 * o + 0], ty = target[2 * o + 1];
    float* m = motn + (long)e * 4 * HW + p;
    m[0] = fminf(fmaxf(x - u, -64.f), 64.f);
    m[HW] = fminf(fmaxf(y - v, -64.f), 64.f);
    m[2 * HW] = fminf(fmaxf(tx - x, -64.f), 64.f);
    m[3 * HW] = fminf(fmaxf(ty - y, -64.f), 64.f);
  }
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
  return s;
}

__global__ void __launch_bounds__(256)
frame_distance_kernel(const float* __restrict__ poses, const float* __restrict__ disps,
                      const float* __restrict__ intr, const int64_t* __restrict__ ii,
                      const int64_t* __restrict__ jj, int H, int W, float beta,
                      float* __restrict__ dist) {
  __shared__ float red[4];
  const int e = blockIdx.x;
  const int ix = (int)ii[e], jx = (int)jj[e];
  const int HW = H * W;
  const float fx = intr[0], fy = intr[1], cx = intr[2], cy = intr[3];
  const SE3f T = rel_se3(poses + 7 * ix, poses + 7 * jx);
  float accum = 0.f, valid = 0.f, total = 0.f;
  for (int k = threadIdx.x; k < HW; k += blockDim.x) {
    const float u = (float)(k % W), v = (float)(k / W);
    const float Xi[4] = {(u - cx) / fx, (v - cy) / fy, 1.0f, disps[(long)ix * HW + k]};
    float Xj[4];
    act_se3(T, Xi, Xj);
    float du = fx * (Xj[0] / Xj[2]) + cx - u;
    float dv = fy * (Xj[1] / Xj[2]) + cy - v;
    float d = sqrtf(du * du + dv * dv);
    total += beta;
    if (Xj[2] > kMinDepth) { accum += beta * d; valid += beta; }
    Xj[0] = Xi[0] + Xi[3] * T.t[0];
    Xj[1] = Xi[1] + Xi[3] * T.t[1];
    Xj[2] = Xi[2] + Xi[3] * T.t[2];
    du = fx * (Xj[0] / Xj[2]) + cx - u;
    dv = fy * (Xj[1] / Xj[2]) + cy - v;
    d = sqrtf(du * du + dv * dv);
    total += (1 - beta);
    if (Xj[2] > kMinDepth) { accum += (1 - beta) * d; valid += (1 - beta); }
  }
  accum = block_sum256(accum, red);
  total = block_sum256(total, red);
  valid = block_sum256(valid, red);
  if (threadIdx.x == 0) dist[e] = (valid / (total + 1e-8f) < 0.75f) ? 1000.0f : accum / valid;
}

__global__ void __launch_bounds__(256)
projmap_kernel(const float* __restrict__ poses, const float* __restrict__ disps,
               const float* __restrict__ intr, const int64_t* __restrict__ ii,
               const int64_t* __restrict__ jj, int H, int W,
               float* __restrict__ coords, float* __restrict__ valid) {
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = blockIdx.y;
  if (p >= HW) return;
  const int ix = (int)ii[e], jx = (int)jj[e];
  const float fx = intr[0], fy = intr[1], cx = intr[2], cy = intr[3];
  const SE3f T = rel_se3(poses + 7 * ix, poses + 7 * jx);
  const float u = (float)(p % W), v = (float)(p / W);
  const float Xi[4] = {(u - cx) / fx, (v - cy) / fy, 1.0f, disps[(long)ix * HW + p]};
  float Xj[4];
  act_se3(T, Xi, Xj);
  const long o = (long)e * HW + p;
  float x = u, y = v;
  if (Xj[2] > 0.01f) {
    x = fx * (Xj[0] / Xj[2]) + cx;
    y = fy * (Xj[1] / Xj[2]) + cy;
  }
  coords[3 * o + 0] = x;
  coords[3 * o + 1] = y;
  coords[3 * o + 2] = 0.f;
  valid[o] = (Xj[2] > kMinDepth) ? 1.0f : 0.0f;
}

__global__ void __launch_bounds__(256)
iproj_kernel(const float* __restrict__ poses, const float* __restrict__ disps,
             const float* __restrict__ intr, int H, int W, float* __restrict__ points) {
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  if (p >= HW) return;
  const float fx = intr[0], fy = intr[1], cx = intr[2], cy = intr[3];
  const SE3f T = load_pose(poses, n);
  const float u = (float)(p % W), v = (float)(p / W);
  const float Xi[4] = {(u - cx) / fx, (v - cy) / fy, 1.0f, disps[(long)n * HW + p]};
  float Xj[4];
  act_se3(T, Xi, Xj);
  const long o = (long)n * HW + p;
  points[3 * o + 0] = Xj[0] / Xj[3];
  points[3 * o + 1] = Xj[1] / Xj[3];
  points[3 * o + 2] = Xj[2] / Xj[3];
}

__global__ void __launch_bounds__(256)
depth_filter_kernel(const float* __restrict__ poses, const float* __restrict__ disps,
                    const float* __restrict__ intr, const int64_t* __restrict__ inds,
                    const float* __restrict__ thresh, int num, int H, int W,
                    float* __restrict__ counter) {
  const int HW = H * W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HW) return;
  const float fx = intr[0], fy = intr[1], cx = intr[2], cy = intr[3];
  const int ix = (int)inds[b];
  const float t = thresh[b];
  const int i = p / W, j = p % W;
  const float Xi[4] = {((float)j - cx) / fx, ((float)i - cy) / fy, 1.0f, disps[(long)ix * HW + p]};
  float count = 0.f;
  for (int neigh = 0; neigh < 6; ++neigh) {
    const int jx = (neigh < 3) ? ix - neigh - 1 : ix + neigh;
    if (jx < 0 || jx >= num) continue;
    const SE3f T = rel_se3(poses + 7 * ix, poses + 7 * jx);
    float Xj[4];
    act_se3(T, Xi, Xj);
    const float uj = fx * (Xj[0] / Xj[2]) + cx;
    const float vj = fy * (Xj[1] / Xj[2]) + cy;
    const float dj = Xj[3] / Xj[2];
    const int u0 = (int)floorf(uj), v0 = (int)floorf(vj);
    if (u0 >= 0 && v0 >= 0 && u0 < W - 1 && v0 < H - 1) {
      const float* D = disps + (long)jx * HW;
      const float d00 = D[(v0 + 0) * W + u0 + 0];
      const float d01 = D[(v0 + 0) * W + u0 + 1];
      const float d10 = D[(v0 + 1) * W + u0 + 0];
      const float d11 = D[(v0 + 1) * W + u0 + 1];
      // the reference's test is in double (droid_kernels.cu:768-772: 1.0 / dj
      // with a double literal), so a count at the threshold flips the same way
      const double idj = 1.0 / (double)dj, td = (double)t;
      if (fabs(idj - 1.0 / (double)d00) < td || fabs(idj - 1.0 / (double)d01) < td ||
          fabs(idj - 1.0 / (double)d10) < td || fabs(idj - 1.0 / (double)d11) < td)
        count += 1.0f;
    }
  }
  counter[(long)b * HW + p] = count;
}

}  // namespace droid

using namespace droid;

extern "C" {

int droid_projective_transform(const float* poses, const float* disps, const float* intrinsics,
                               const int64_t* ii, const int64_t* jj, int E, int H, int W,
                               float* coords, float* valid, const float* target, float* motn,
                               hipStream_t stream) {
  if (E < 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "projective_transform: bad shape");
  if (motn && !target) return fail(kInvalidArgument, "projective_transform: motn needs target");
  if (E == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), E);
  projective_transform_kernel<<<grid, 256, 0, stream>>>(poses, disps, intrinsics, ii, jj, H, W,
                                                       coords, valid, target, motn);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_frame_distance(const float* poses, const float* disps, const float* intrinsics,
                         const int64_t* ii, const int64_t* jj, int E, int H, int W, float beta,
                         float* dist, hipStream_t stream) {
  if (E < 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "frame_distance: bad shape");
  if (E == 0) return kOk;
  frame_distance_kernel<<<E, 256, 0, stream>>>(poses, disps, intrinsics, ii, jj, H, W, beta, dist);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_projmap(const float* poses, const float* disps, const float* intrinsics,
                  const int64_t* ii, const int64_t* jj, int E, int H, int W,
                  float* coords, float* valid, hipStream_t stream) {
  if (E < 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "projmap: bad shape");
  if (E == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), E);
  projmap_kernel<<<grid, 256, 0, stream>>>(poses, disps, intrinsics, ii, jj, H, W, coords, valid);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_iproj(const float* poses, const float* disps, const float* intrinsics, int N, int H, int W,
                float* points, hipStream_t stream) {
  if (N < 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "iproj: bad shape");
  if (N == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), N);
  iproj_kernel<<<grid, 256, 0, stream>>>(poses, disps, intrinsics, H, W, points);
  DROID_LAUNCH_CHECK();
  return kOk;
}

int droid_depth_filter(const float* poses, const float* disps, const float* intrinsics,
                       const int64_t* ix, const float* thresh, int n, int num, int H, int W,
                       float* counter, hipStream_t stream) {
  if (n < 0 || num <= 0 || H <= 0 || W <= 0) return fail(kInvalidArgument, "depth_filter: bad shape");
  if (n == 0) return kOk;
  dim3 grid(ceil_div(H * W, 256), n);
  depth_filter_kernel<<<grid, 256, 0, stream>>>(poses, disps, intrinsics, ix, thresh, num, H, W, counter);
  DROID_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
