// parallel-gcn_amd/csrc/peer_sync.hpp -- device side of the peer-mapped exchange's hand-off
// (k_peer.hip, and k_gs_lds_combine's push mode in k_graphsum_ring.hip).
//
// Flags and arrival counters live in uncached device memory (MTYPE UC): no cache on this GPU
// or a peer holds their lines.  The receive slots are plain device memory that the pushers
// write through with system-scope (sc0 sc1) 16-B stores: no cache keeps a dirty copy, so once
// every store is acknowledged the flag may follow, with no L2 write-back; the receiver reads
// them in a later kernel (a kernel boundary invalidates its L1; its L2's lines of local memory
// are kept coherent by the memory probes).  (r05: uncached slots moved 0.3 TB/s, 48.6 vs
// 13 us per combine.)
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace pgcn {

// every store this wave issued acknowledged (gfx9 counts stores in vmcnt)
__device__ __forceinline__ void stores_acked() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void flag_store(unsigned *p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned flag_load(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// v -> float4 element i of the slot at `base` (bytes: the slot's size from base on), written
// through to memory at system scope (buffer_store_dwordx4 ... sc0 sc1); `base` wave-uniform
__device__ __forceinline__ void peer_store16(float *base, long long bytes, long long i, float4 v) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
  const u4 d = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 16), 0, 17 /* sc0 sc1 */);
}
__device__ __forceinline__ void peer_store4(float *base, long long bytes, long long i, float v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(i * 4), 0, 17 /* sc0 sc1 */);
}

// The end of a pushing workgroup (every thread calls it): its stores acknowledged, one arrival
// on the launch's counter; the launch's last workgroup resets the counter and (k.signal: the
// last pass of a multi-pass push) stores the generation into every receiver's flag of this rank
__device__ __forceinline__ void peer_arrive(const PeerSink &k) {
  stores_acked();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = gridDim.x * gridDim.y;
    const unsigned old =
        __hip_atomic_fetch_add(k.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old == n - 1) {
      __hip_atomic_store(k.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (k.signal)
        for (int q = 0; q < k.world; q++) flag_store(k.flag[q], k.gen);
      stores_acked();
    }
  }
}

}  // namespace pgcn
