// Latency probe for the Cholesky panel's column chain (one wave, s_memtime
// cycles): dependent v_fma_f64, v_rsq_f64 + one Newton step, the v_readlane
// pair -> SGPR -> VALU hop, and the LDS store -> broadcast load round trip.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double rl(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__global__ void probe(double seed, long long* out, double* sink) {
  __shared__ double buf[64];
  const int lane = threadIdx.x;
  double a = seed + lane * 1e-3, b = 1.0000001, c = 1e-9;
  constexpr int N = 256;
  long long t0, t1;
  // 1. dependent fma chain
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; ++i) a = fma(a, b, c);
  asm volatile("" :: "v"(a));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (t1 - t0);
  // 2. dependent rsq chain (+ one Newton step)
  double x = 1.5 + a * 1e-12;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < N; ++i) {
    const double y = __builtin_amdgcn_rsq(x);
    x = y * fma(-0.5 * x * y, y, 1.5) + 1.0;
  }
  asm volatile("" :: "v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (t1 - t0);
  // 3. bare rsq chain
  double z = 1.5 + x * 1e-12;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < N; ++i) z = __builtin_amdgcn_rsq(z) + 0.5;
  asm volatile("" :: "v"(z));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (t1 - t0);
  // 4. readlane pair -> VALU (fma with the SGPR pair) -> readlane
  double w = z;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < N; ++i) w = fma(rl(w, i & 63), b, c);
  asm volatile("" :: "v"(w));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (t1 - t0);
  // 5. LDS round trip: store, broadcast load of another lane's slot, fma
  double u = w;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int i = 0; i < N; ++i) {
    buf[lane] = u;
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    u = fma(buf[(i + 5) & 63], b, c);
  }
  asm volatile("" :: "v"(u));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (t1 - t0);
  // 6. independent fma throughput (8 chains)
  double q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q[k] = u + k;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = fma(q[k], b, c);
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += q[k];
  asm volatile("" :: "v"(s));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = (t1 - t0);
  sink[lane] = s;
}

int main() {
  long long* d_out;
  double* d_sink;
  hipMalloc(&d_out, 8 * sizeof(long long));
  hipMalloc(&d_sink, 64 * sizeof(double));
  for (int rep = 0; rep < 3; ++rep) {
    probe<<<1, 64>>>(1.25, d_out, d_sink);
    hipDeviceSynchronize();
  }
  long long h[8];
  hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[6] = {"dependent v_fma_f64", "v_rsq_f64 + Newton (5 dep ops)", "v_rsq_f64 + add",
                       "readlane pair -> fma", "LDS store -> load -> fma", "8 independent fma (per 8)"};
  for (int i = 0; i < 6; ++i) printf("%-34s %7.1f clk per step\n", nm[i], (double)h[i] / 256.0);
  hipFree(d_out);
  hipFree(d_sink);
  return 0;
}
