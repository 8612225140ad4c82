// mx_dma.h — LDS-DMA and vmcnt helpers shared by the ring kernels (gfx950).
#pragma once
#include "mx_common.h"

namespace mx {

#define LDS_AS __attribute__((address_space(3)))
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt encoding: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// LDS-DMA (buffer_load_dwordx4 ... lds, 16 B per lane) issued from inline asm. Through the builtin
// the compiler tracks the load as an LDS write it cannot place, so SIInsertWaitcnts puts an
// s_waitcnt vmcnt(0) in front of the first later ds_read that may alias it: in the ring kernels that
// is the current tile's fragment read, right after the next tiles' DMA was issued -- every K-tile
// then waited for its successors' loads and the STAGES-deep ring never had more than one tile in
// flight during the MFMAs. Hidden from the compiler, the loads are ordered only by the kernels'
// own counted wait_vmcnt<> + barrier (the ring's protocol): ds_reads of tile t never alias the
// slots being filled. `lds` (M0) and the descriptor are wave-uniform SGPRs; M0 -> LDS-DMA needs one
// wait state.
__device__ __forceinline__ i32x4 dma_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(LDS_AS const void*)p);
}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // M0 is reserved: the kernels using this set it only here
__device__ __forceinline__ void lds_dma16(i32x4 rsrc, uint32_t lds, uint32_t voff, uint32_t soff) {
  const int l = __builtin_amdgcn_readfirstlane((int)lds), so = __builtin_amdgcn_readfirstlane((int)soff);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(l), "v"(voff), "s"(rsrc), "s"(so) : "memory", "m0");
}
#pragma clang diagnostic pop

// 4 B per lane (buffer_load_dword ... lds): lane l's dword lands at M0 + 4 l
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma4(i32x4 rsrc, uint32_t lds, uint32_t voff, uint32_t soff) {
  const int l = __builtin_amdgcn_readfirstlane((int)lds), so = __builtin_amdgcn_readfirstlane((int)soff);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               :: "s"(l), "v"(voff), "s"(rsrc), "s"(so) : "memory", "m0");
}
#pragma clang diagnostic pop

}  // namespace mx
