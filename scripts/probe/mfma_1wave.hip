// One wave per SIMD (4 waves / CU): can a single wave keep its SIMD's matrix
// core busy?  Register-only v_mfma_f32_16x16x32_f16 over NACC independent
// accumulators (builtin, or inline asm with the accumulators pinned in AGPRs),
// and the same with one ds_read_b128 per RD MFMAs feeding the A operand.
// Compare with 8 waves / CU (mfma_peak.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int NACC, bool ASM, int RD>
__global__ void __launch_bounds__(256) one_wave(float* out, int iters, long long* clk) {
  __shared__ half8 lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 256)
    for (int k = 0; k < 8; ++k) lds[i][k] = (_Float16)(0.001f * (i + k));
  __syncthreads();
  half8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(i * 0.5f); }
  floatx4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  int off = threadIdx.x & 63;
  for (int it = 0; it < iters; ++it) {
    half8 ar[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) ar[q] = a;
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      // the read for the group two ahead (its latency hidden under 2 x RD MFMAs)
      if (RD && j % RD == 0) ar[(j / RD + 2) & 3] = lds[(off + 64 * (j / RD)) & 2047];
      const half8 av = RD ? ar[(j / RD) & 3] : a;
      if constexpr (ASM) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(av), "v"(b));
      else acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b, acc[j], 0, 0, 0);
    }
    off += 7;
  }
  if constexpr (ASM) asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int NACC, bool ASM, int RD>
static void run(const char* name, int ncu, float* out, long long* clk) {
  const int iters = 320000 / NACC;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  one_wave<NACC, ASM, RD><<<ncu, 256>>>(out, 10, clk);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  one_wave<NACC, ASM, RD><<<ncu, 256>>>(out, iters, clk);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
  const double mfmas = (double)iters * NACC;            // per wave
  const double flops = (double)ncu * 4 * mfmas * 16384.0;
  printf("%-34s %.3f ms  %7.1f TFLOP/s  clock %.2f GHz  %.1f clk/MFMA/wave\n", name, ms, flops / ms / 1e9,
         (double)c[0] / c[1] * 0.1, (double)c[0] / mfmas);
}

int main() {
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out; long long* clk;
  hipMalloc(&out, ncu * 256 * 4); hipMalloc(&clk, 16);
  run<16, false, 0>("builtin, 16 acc", ncu, out, clk);
  run<64, false, 0>("builtin, 64 acc", ncu, out, clk);
  run<16, true, 0>("asm +a, 16 acc", ncu, out, clk);
  run<64, true, 0>("asm +a, 64 acc", ncu, out, clk);
  run<64, true, 4>("asm +a, 64 acc, ds_read / 4 MFMA", ncu, out, clk);
  run<64, true, 8>("asm +a, 64 acc, ds_read / 8 MFMA", ncu, out, clk);
  run<64, true, 2>("asm +a, 64 acc, ds_read / 2 MFMA", ncu, out, clk);
  return 0;
}
