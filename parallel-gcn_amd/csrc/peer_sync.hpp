// parallel-gcn_amd/csrc/peer_sync.hpp -- device side of the peer-mapped exchange's hand-off
// (k_peer.hip, and k_gs_lds_combine's push mode in k_graphsum_ring.hip).
//
// Receive slots, flags and arrival counters live in uncached device memory (MTYPE UC): no
// cache on this GPU or a peer holds their lines, so an acknowledged store is visible to every
// later load, here or over xGMI, and no cache write-back or invalidate is needed.
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
