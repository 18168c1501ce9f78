// Probe: issue cost of LDS-DMA (buffer_load_dwordx4 ... lds) per wave vs a plain
// buffer_load_dwordx4 into VGPRs.  One workgroup per CU, NW waves; every wave
// issues K loads of 1 KB (16 B / lane) from an L2-resident 8 MB buffer and
// stamps s_memtime before the first issue, after the last issue and after
// vmcnt(0).  Output per (mode, NW, K): median issue clocks and drain clocks of
// wave 0.  Build: hipcc --offload-arch=gfx950 -O3 -I../../droid-slam_amd/csrc
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"

#include <algorithm>
#include <cstdio>
#include <vector>

#include "lds_dma.hpp"

using namespace droid;

template <int MODE, int K>
__global__ void __launch_bounds__(512) probe(const char* src, unsigned bytes, long long* out, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const rsrc_t rs = make_rsrc(src, bytes);
  const unsigned base = lds_addr(lds) + wave * K * 1024;
  const unsigned off0 = ((blockIdx.x * 37 + wave * 11) % 4096) * 1024 + lane * 16;
  uint4 acc = {0, 0, 0, 0};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) dma16(rs, base + k * 1024, off0 + k * 1024);
  } else {
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      v[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                 __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), (short)0, (int)bytes, kBufFlags),
                 (int)(off0 + k * 1024), 0, 0));
    asm volatile("" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < K; ++k) acc.x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    const long long t2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      out[(blockIdx.x * 8 + wave) * 2 + 0] = t1 - t0;
      out[(blockIdx.x * 8 + wave) * 2 + 1] = t2 - t0;
    }
    if (acc.x == 0x12345678u) sink[0] = 1;
    return;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t2 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[(blockIdx.x * 8 + wave) * 2 + 0] = t1 - t0;
    out[(blockIdx.x * 8 + wave) * 2 + 1] = t2 - t0;
  }
}

template <int MODE, int K>
static void run(const char* src, unsigned bytes, long long* dout, int* sink, int nw, int cus) {
  std::vector<long long> h((size_t)cus * 16, 0);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(dout, 0, h.size() * 8);
    probe<MODE, K><<<cus, nw * 64, 8 * K * 1024>>>(src, bytes, dout, sink);
    hipDeviceSynchronize();
  }
  hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<long long> is, dr;
  for (int b = 0; b < cus; ++b)
    for (int w = 0; w < nw; ++w) {
      is.push_back(h[(b * 8 + w) * 2]);
      dr.push_back(h[(b * 8 + w) * 2 + 1]);
    }
  std::sort(is.begin(), is.end());
  std::sort(dr.begin(), dr.end());
  printf("%-10s waves %d K %2d: issue median %6lld clk (%5.1f / instr), issue+drain median %6lld clk\n",
         MODE == 0 ? "lds-dma" : "vgpr-load", nw, K, is[is.size() / 2], (double)is[is.size() / 2] / K,
         dr[dr.size() / 2]);
}

int main() {
  const unsigned bytes = 8u << 20;
  char* src;
  long long* dout;
  int* sink;
  hipMalloc(&src, bytes);
  hipMemset(src, 1, bytes);
  hipMalloc(&dout, 256 * 16 * 8);
  hipMalloc(&sink, 4);
  hipFuncSetAttribute((const void*)&probe<0, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 16 * 1024);
  hipFuncSetAttribute((const void*)&probe<1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 16 * 1024);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int nw : {1, 8}) {
    run<0, 1>(src, bytes, dout, sink, nw, cus);
    run<0, 4>(src, bytes, dout, sink, nw, cus);
    run<0, 16>(src, bytes, dout, sink, nw, cus);
    run<1, 4>(src, bytes, dout, sink, nw, cus);
    run<1, 16>(src, bytes, dout, sink, nw, cus);
  }
  return 0;
}
