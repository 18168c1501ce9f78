// MFMA operand types and LDS-DMA helpers shared by the gfx950 kernels.
#pragma once

#include "common.hpp"

namespace droid {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));

constexpr unsigned kOob = 0x80000000u;  // buffer offset past any descriptor: loads return 0
constexpr int kBufFlags = 0x00020000;   // raw buffer descriptor word 3 (gfx950)

// LDS-DMA of 16 B per lane (buffer_load_dwordx4 ... lds): lane l's bytes land at
// LDS byte address `lds` + 16 l.  Issued as inline asm so that hipcc does not
// treat every later ds_read as dependent on the DMA (it inserts vmcnt(0) before
// them otherwise); the kernel orders the DMA with explicit counted vmcnt waits +
// s_barrier.  `rs` is a raw buffer descriptor in SGPRs; out-of-range offsets
// (kOob) land as zeros.
typedef int rsrc_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char* lds_cptr_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, unsigned bytes) {
  // wave-uniform by construction; readfirstlane keeps the descriptor in SGPRs
  const unsigned long long pa = (unsigned long long)base;
  return rsrc_t{__builtin_amdgcn_readfirstlane((int)(unsigned)pa),
                __builtin_amdgcn_readfirstlane((int)((unsigned)(pa >> 32) & 0xffffu)),
                __builtin_amdgcn_readfirstlane((int)bytes), kBufFlags};
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(lds_cptr_t)(p);
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(rsrc_t rs, unsigned lds, unsigned voff) {
  const rsrc_t r = {__builtin_amdgcn_readfirstlane(rs.x), __builtin_amdgcn_readfirstlane(rs.y),
                    __builtin_amdgcn_readfirstlane(rs.z), __builtin_amdgcn_readfirstlane(rs.w)};
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
               : "memory", "m0");
}
// the same with the non-temporal policy (nt): for streams that one workgroup
// reads once, past L2 and the Infinity Cache
__device__ __forceinline__ void dma16_nt(rsrc_t rs, unsigned lds, unsigned voff) {
  const rsrc_t r = {__builtin_amdgcn_readfirstlane(rs.x), __builtin_amdgcn_readfirstlane(rs.y),
                    __builtin_amdgcn_readfirstlane(rs.z), __builtin_amdgcn_readfirstlane(rs.w)};
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
               : "memory", "m0");
}
#pragma clang diagnostic pop

}  // namespace droid
