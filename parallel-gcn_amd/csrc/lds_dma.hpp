// parallel-gcn_amd/csrc/lds_dma.hpp -- device helpers shared by the LDS-staged kernels
// (k_graphsum_lds.hip, k_graphsum_ring.hip, k_xstream_lds.hip): LDS-DMA pieces issued from inline asm,
// LDS hand-off words, float4 accumulation.
#pragma once
#include "common.hpp"

namespace pgcn {

__device__ __forceinline__ void f4_acc(float4 &a, const float4 &x) {
  a.x += x.x;
  a.y += x.y;
  a.z += x.z;
  a.w += x.w;
}

// One LDS-DMA piece: 16 B per active lane to LDS byte address lds_dst + 16 * lane.  Inline
// asm keeps the DMA out of hipcc's waitcnt bookkeeping (it would otherwise drain it with
// vmcnt(0) before unrelated LDS reads); completion is counted by hand (s_waitcnt vmcnt).
__device__ __forceinline__ void glds16(const void *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// The same piece with the nontemporal hint (a stream read once: X in the X-stream kernels)
__device__ __forceinline__ void glds16_nt(const void *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// Four consecutive 1-KB pieces: gsrc .. gsrc + 3 KB -> lds_dst .. lds_dst + 3 KB.  The
// instruction offset steps the global AND the LDS address (LDS = M0 + offset + 16 * lane),
// so one M0 write and one address VGPR serve all four.
__device__ __forceinline__ void glds16x4(const void *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024\n\t"
      "global_load_lds_dwordx4 %1, off offset:2048\n\t"
      "global_load_lds_dwordx4 %1, off offset:3072\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

__device__ __forceinline__ unsigned lds_wait_ge(const unsigned *p, unsigned target) {
  unsigned spins = 0;
  while (true) {
    const unsigned v = __builtin_amdgcn_readfirstlane(__atomic_load_n(p, __ATOMIC_RELAXED));
    if (v >= target) break;
    __builtin_amdgcn_s_sleep(1);
    spins++;
  }
  asm volatile("" ::: "memory");
  return spins;
}

}  // namespace pgcn
