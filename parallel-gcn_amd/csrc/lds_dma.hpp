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

typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));

// LDS reads issued from inline asm (LDS byte addresses): hipcc does not count them, so its
// automatic waits do not drain them; every use goes behind an lgkm_wait<N> naming the
// registers it waits for (the asm operands order the uses after it).
// Invariants the compiler does not guarantee (checked on the built code object by
// tests/test_cpu_host.py test_ring_kernel_lds_reads_wait_before_use):
//  * the destination registers stay where the read lands them until the tied lgkm_wait: hipcc
//    takes the asm outputs as ready at once, so a v_mov of one of them placed before the wait
//    would copy stale data -- no instruction may name them before the next lgkmcnt(0);
//  * an LDS atomic issued under a forced exec mask (k_graphsum_ring's hand-off count) sits in
//    wave-uniform control flow with lane 0 active, and restores exec inside the same asm
//    statement, so the hazard recognizer never sees a live exec write across statements.
__device__ __forceinline__ f4v ds_rd128(unsigned addr) {
  f4v r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ u2v ds_rd64(unsigned addr) {
  u2v r;
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
// the same read into registers that hold the previous value (read first by earlier code)
__device__ __forceinline__ void ds_rd64_into(u2v &r, unsigned addr) {
  asm volatile("ds_read_b64 %0, %1" : "+v"(r) : "v"(addr));
}
// s_waitcnt lgkmcnt(N): at most N LDS operations of this wave still in flight
template <int N>
__device__ __forceinline__ void lgkm_wait(u2v &e) {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%c1)" : "+v"(e) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(f4v &x0, f4v &x1, f4v &x2, f4v &x3, u2v &e) {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%c5)"
               : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(e)
               : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(f4v &x0, f4v &x1, f4v &x2, f4v &x3, u2v &e0, u2v &e1) {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%c6)"
               : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(e0), "+v"(e1)
               : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(f4v &x0, f4v &x1, f4v &x2, f4v &x3) {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%c4)" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "n"(N));
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
