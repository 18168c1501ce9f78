// Probe (round 6): __builtin_bit_cast of an ext_vector
// element.  Build the device assembly:
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only scripts/probe/bitcast_vec.hip -o /tmp/bitcast_vec.s
// scripts/probe/bitcast_vec.txt holds the relevant lines of that output
// (ROCm 7.2 hipcc, this image).  Finding: with `w` of a clang ext_vector type
// (u32x2_t below), __builtin_bit_cast(h2_t, w[1]) and (h2_t, w.y) read
// ELEMENT 0 - the kernel loads one dword (ds_read_b32 at the vector's base)
// and stores the same halves for both casts.  With HIP's uint2 (a struct
// whose .x/.y are members) and with a named scalar the second dword is read.
// The bit-cast of an ext_vector element lvalue takes the vector's base
// address instead of the element's; a value (a named scalar, a member of a
// struct, a plain array element) is cast correctly.
#include <hip/hip_runtime.h>

typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));

#define FILL_LDS()                                                 \
  __shared__ __attribute__((aligned(16))) char lds[4096];          \
  const int i = threadIdx.x;                                       \
  reinterpret_cast<unsigned*>(lds)[i] = in[i];                     \
  reinterpret_cast<unsigned*>(lds)[i + 256] = in[i + 256];         \
  __syncthreads();

// miscompiled: ext_vector element by subscript
extern "C" __global__ void ext_subscript(const unsigned* __restrict__ in, h2_t* __restrict__ out) {
  FILL_LDS();
  const u32x2_t w = *reinterpret_cast<const u32x2_t*>(lds + (i & 63) * 16 + 8);
  out[2 * i] = __builtin_bit_cast(h2_t, w[0]);
  out[2 * i + 1] = __builtin_bit_cast(h2_t, w[1]);
}

// miscompiled: ext_vector element by swizzle
extern "C" __global__ void ext_swizzle(const unsigned* __restrict__ in, h2_t* __restrict__ out) {
  FILL_LDS();
  const u32x2_t w = *reinterpret_cast<const u32x2_t*>(lds + (i & 63) * 16 + 8);
  out[2 * i] = __builtin_bit_cast(h2_t, w.x);
  out[2 * i + 1] = __builtin_bit_cast(h2_t, w.y);
}

// correct: the element through a named scalar first (the rule the kernels follow)
extern "C" __global__ void ext_named(const unsigned* __restrict__ in, h2_t* __restrict__ out) {
  FILL_LDS();
  const u32x2_t w = *reinterpret_cast<const u32x2_t*>(lds + (i & 63) * 16 + 8);
  const unsigned w0 = w[0], w1 = w[1];
  out[2 * i] = __builtin_bit_cast(h2_t, w0);
  out[2 * i + 1] = __builtin_bit_cast(h2_t, w1);
}

// correct: HIP's uint2 (struct members)
extern "C" __global__ void hip_uint2(const unsigned* __restrict__ in, h2_t* __restrict__ out) {
  FILL_LDS();
  const uint2 w = *reinterpret_cast<const uint2*>(lds + (i & 63) * 16 + 8);
  out[2 * i] = __builtin_bit_cast(h2_t, w.x);
  out[2 * i + 1] = __builtin_bit_cast(h2_t, w.y);
}
