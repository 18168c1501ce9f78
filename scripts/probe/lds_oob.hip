// Probe: what a ds_read_b128 beyond the workgroup's LDS allocation returns on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out, unsigned off) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  for (int i = threadIdx.x; i < 163840 / 16; i += blockDim.x) ((uint4*)smem)[i] = make_uint4(0xdeadbeef, 1, 2, 3);
  __syncthreads();
  const unsigned addr = off + threadIdx.x * 16;
  uint4 v = *(const uint4*)(smem + addr);
  out[threadIdx.x] = v.x | v.y | v.z | v.w;
}
int main() {
  unsigned* d; hipMalloc(&d, 256 * 4);
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  unsigned offs[] = {0u, 163840u - 1024u, 163840u, 163840u + 4096u, 0x100000u, 0x40000000u};
  for (unsigned off : offs) {
    k<<<1, 64, 163840>>>(d, off);
    unsigned h[64]; hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
    unsigned any = 0; for (int i = 0; i < 64; ++i) any |= h[i];
    printf("offset 0x%08x: %s (or=0x%08x)\n", off, any ? "nonzero" : "ZERO", any);
  }
  // smaller allocation: 64 KB, read at 96 KB
  k<<<1, 64, 65536>>>(d, 98304);
  unsigned h[64]; hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
  unsigned any = 0; for (int i = 0; i < 64; ++i) any |= h[i];
  printf("alloc 64K, offset 96K: %s\n", any ? "nonzero" : "ZERO");
  return 0;
}
