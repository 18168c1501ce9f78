// Achievable dense f16 MFMA rate on the whole chip: 8 waves/CU, register-only
// v_mfma_f32_16x16x32_f16 chains (16 independent accumulators per wave), plus
// the shader clock measured as s_memtime ticks per s_memrealtime tick.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(512) peak(float* out, int iters, long long* clk) {
  half8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(i * 0.5f); }
  floatx4 acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}
int main() {
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu, iters = 20000;
  float* out; long long* clk;
  hipMalloc(&out, grid * 512 * 4); hipMalloc(&clk, 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  peak<<<grid, 512>>>(out, 100, clk);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    peak<<<grid, 512>>>(out, iters, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double flops = (double)grid * 8 * iters * 16 * 16384.0;
    printf("CUs %d: %.3f ms  %.1f TFLOP/s  shader clock %.2f GHz (memtime %lld / realtime %lld ticks @100MHz)\n",
           ncu, ms, flops / ms / 1e9, (double)c[0] / c[1] * 0.1, c[0], c[1]);
  }
  return 0;
}
