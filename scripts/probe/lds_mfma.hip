// Microbenchmark of the band conv's inner loop without DMA, barriers or
// epilogue: 8 waves / CU (2 per SIMD), each a 64x128 accumulator tile, per
// "stage" 64 v_mfma_f32_16x16x32_f16 whose fragments come from LDS (24
// ds_read_b128, the kernel's ratio) - or from registers only (mode 0), or with
// v_mfma_f32_32x32x16_f16 (mode 2: 32 MFMAs, same 24 reads).  Tells how much
// of the MFMA rate the LDS fragment reads cost by themselves.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ void __launch_bounds__(512) loop(float* out, int stages) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 65536 / 16; i += 512)
    reinterpret_cast<uint4*>(lds)[i] = make_uint4(0x3c003c00u ^ i, 0x3c00u, 0x3c003c00u, i);
  __syncthreads();
  // per-lane fragment addresses: 16-B pieces, XOR-swizzled rows as in the kernel
  const int fr = lane & 15, kq = lane >> 4;
  const int abase = ((wave * 64 + fr) * 128 + ((kq ^ (fr & 7)) << 4)) & 32767;
  const int bbase = 32768 + (((wave & 1) * 128 + fr) * 128 + ((kq ^ (fr & 7)) << 4)) % 32768;
  if constexpr (MODE == 2) {
    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    for (int s = 0; s < stages; ++s) {
      const int so = (s & 7) * 1024;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        half8 a[2], b[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const half8*>(lds + ((abase + so + i * 4096 + ks * 64) & 32767));
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const half8*>(lds + 32768 + ((bbase + so + j * 4096 + ks * 64) & 32767));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) t += acc[i][j][q];
    out[blockIdx.x * 512 + tid] = t;
  } else {
    floatx4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 ra[2][4], rb[2][8];
    if constexpr (MODE == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[h][i] = *reinterpret_cast<const half8*>(lds + ((abase + i * 8192 + h * 64) & 32767));
#pragma unroll
        for (int j = 0; j < 8; ++j) rb[h][j] = *reinterpret_cast<const half8*>(lds + 32768 + ((bbase + j * 2048 + h * 64) & 32767));
      }
    }
    for (int s = 0; s < stages; ++s) {
      const int so = (s & 7) * 1024;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        half8 a[4], b[8];
        if constexpr (MODE == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = ra[h][i];
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = rb[h][j];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const half8*>(lds + ((abase + so + i * 8192 + h * 64) & 32767));
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const half8*>(lds + 32768 + ((bbase + so + j * 2048 + h * 64) & 32767));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 512 + tid] = t;
  }
}

template <int MODE>
static void run(const char* name, float* out, int ncu) {
  const int stages = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  loop<MODE><<<ncu, 512>>>(out, 10);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    loop<MODE><<<ncu, 512>>>(out, stages);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  // per stage per wave: 64 x (16x16x32) = 32 x (32x32x16) = 64 x 16384 FLOP
  const double flops = (double)ncu * 8 * stages * 64 * 16384.0;
  printf("%-44s %.3f ms  %.1f TFLOP/s\n", name, best, flops / best / 1e9);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, ncu * 512 * 4);
  run<0>("16x16x32, fragments in registers", out, ncu);
  run<1>("16x16x32, 24 ds_read_b128 per 64 MFMA", out, ncu);
  run<2>("32x32x16, 24 ds_read_b128 per 32 MFMA", out, ncu);
  return 0;
}
