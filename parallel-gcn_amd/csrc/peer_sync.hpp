// parallel-gcn_amd/csrc/peer_sync.hpp -- device side of the peer-mapped exchange's hand-off
// (k_peer.hip, and k_gs_lds_combine's push mode in k_graphsum_ring.hip).
//
// Flags and arrival counters live in uncached device memory (MTYPE UC): no cache on this GPU
// or a peer holds their lines.  The receive slots are plain device memory, written with plain
// 16-B stores; every pushing workgroup then makes them visible at system scope with ONE
// release (an L2 write-back of its XCD's dirty lines, `buffer_wbl2 sc0 sc1`, waited for)
// before its arrival, so when the last arrival stores the flags every slot byte has left this
// GPU's caches.  The receiver reads them in a later kernel whose every workgroup starts with
// a system-scope acquire (acquire_system_workgroup: `buffer_inv sc0 sc1`, waited for, then the
// workgroup's barrier) -- the consumer half of the gfx942/gfx950 memory model's system-scope
// hand-off.  That drops this CU's L1 and the XCD L2's non-coherent (NC) lines; the slots are
// local VRAM, which the kernel driver maps MTYPE RW with the snoop bit on these parts (as it
// maps fine-grained VRAM: the same MTYPE), so a peer's write-back over xGMI invalidates any L2
// copy by the memory probes ("MTYPE RW and CC memory will never be stale due to the memory
// probes", the LLVM AMDGPU memory model for GFX942 system-scope acquire).  A knob allocates
// the slots uncached instead (`peer_uncached`, MTYPE UC: no L2 copy at all) for a machine
// where that assumption fails; bench.py checks every N > 1 run's logits against a one-GPU
// engine and falls back to RCCL when they differ.
// r05, measured on one GPU (the solo form, every slot local): write-through pushes (sc0 sc1
// stores, or uncached slots) moved 0.3 TB/s -- 49 us per GraphSum combine at W = 8 against
// 12.7 us for the combine that writes its own rows (profiles/r05/g/rank8_breakdown.txt).
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

// Everything this thread's workgroup stored so far visible at system scope: the stores
// acknowledged, then (one lane) a system-scope release -- the L2 write-back -- and its
// completion (inline-asm wait: the compiler may drop the one after the write-back when it
// believes nothing is outstanding).  Call with every thread; lane 0 of wave 0 fences.
__device__ __forceinline__ void release_workgroup_stores() {
  stores_acked();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    stores_acked();
  }
}

// The receiving side of a hand-off at system scope (every thread calls it, before any early
// exit): lane 0 of wave 0 issues the system-scope acquire and waits for it, then the
// workgroup's barrier orders every wave's slot loads after it
__device__ __forceinline__ void acquire_system_workgroup() {
#ifdef PGCN_ABL_NO_ACQUIRE  // timing-only diagnostic build (the cost of the acquire): unsafe
  return;
#endif
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: buffer_inv sc0 sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// grad[k][j] of a deferred reduction (TnDeferred, kernels.hpp): k_gemm_tn_reduce's loads in
// batches of 16 and its ordered adds, the same bits (the Adam launch and the weight
// gradients' peer push run it)
__device__ __forceinline__ float tn_deferred_sum(const TnDeferred &d, long long i) {
  const int k = (int)(i / d.N), j = (int)(i - (long long)k * d.N);
  const long long e = (long long)k * d.ldp + j, stride = (long long)d.K * d.ldp;
  float s = 0.0f;
  for (int b0 = 0; b0 < d.n_groups; b0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = b0 + u < d.n_groups ? d.src[(b0 + u) * stride + e] : 0.0f;
#pragma unroll
    for (int u = 0; u < 16; u++)
      if (b0 + u < d.n_groups) s += v[u];
  }
  return s;
}

// v -> float4 element i of the slot at `base` (bytes: the slot's size from base on: a store
// past it is dropped by the buffer resource's range check); `base` wave-uniform
__device__ __forceinline__ void peer_store16(float *base, long long bytes, long long i, float4 v) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
  const u4 d = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 16), 0, 0);
}
__device__ __forceinline__ void peer_store4(float *base, long long bytes, long long i, float v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(i * 4), 0, 0);
}

// The end of a pushing workgroup (every thread calls it): its stores released at system scope,
// one arrival on the launch's counter; the launch's last workgroup resets the counter and
// (k.signal: the last pass of a multi-pass push) stores the generation into every receiver's
// flag of this rank
__device__ __forceinline__ void peer_arrive(const PeerSink &k) {
  release_workgroup_stores();
  if (threadIdx.x == 0) {
    const unsigned n = gridDim.x * gridDim.y;
    const unsigned old =
        __hip_atomic_fetch_add(k.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old == n - 1) {
      __hip_atomic_store(k.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (k.signal) {
        for (int q = 0; q < k.world; q++) flag_store(k.flag[q], k.gen);
        stores_acked();
        // the receiver's wait, fused (separate processes): the launch ends once every sender
        // of this rank has signalled, so the next kernel may read the slots
        if (k.nwait && !flag_load(k.err)) {
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          for (int q = 0; q < k.nwait; q++) {
            while ((int)(flag_load(k.wait_flags + q) - k.gen) < 0) {
              __builtin_amdgcn_s_sleep(2);
              if (__builtin_amdgcn_s_memrealtime() - t0 > kPeerTimeoutTicks) {
                __hip_atomic_store(k.err, 0x10000u | (unsigned)q, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                return;
              }
            }
          }
        }
      } else {
        stores_acked();
      }
    }
  }
}

// A small all-reduce inside ONE workgroup (every thread calls it; separate processes only:
// their kernels never share a hardware queue, so this rank's spin cannot sit ahead of a peer's
// push): buf [n] pushed to every receiver's slot of this rank, released, the flags; one wave
// polls this rank's flags (p.waited[q], q < p.nwait), one system-scope acquire (the slots were
// written by other agents within this kernel's lifetime: no kernel boundary in between), the
// rank-order sum back into buf.  Returns false (buf untouched) when a peer never signalled.
// buf must be visible to the whole workgroup (written before a barrier).
__device__ __forceinline__ bool peer_allreduce_block(float *buf, int n, const PeerSmall &p) {
  const PeerSink &k = p.k;
  const bool v4 = (n & 3) == 0;
  for (int q = 0; q < k.world; q++) {
    if (v4)
      for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
        peer_store16(k.dst[q], k.slot_bytes, i, reinterpret_cast<const float4 *>(buf)[i]);
    else
      for (int i = threadIdx.x; i < n; i += blockDim.x) peer_store4(k.dst[q], k.slot_bytes, i, buf[i]);
  }
  release_workgroup_stores();
  if (threadIdx.x == 0) {
    for (int q = 0; q < k.world; q++) flag_store(k.flag[q], k.gen);
    stores_acked();
  }
  __shared__ int failed;
  if (threadIdx.x < 64) {
    const int q = threadIdx.x;
    bool bad = flag_load(p.err) != 0;
    if (!bad && q < p.nwait) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while ((int)(flag_load(p.waited + q) - k.gen) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kPeerTimeoutTicks) {
          __hip_atomic_store(p.err, 0x10000u | (unsigned)q, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          bad = true;
          break;
        }
      }
    }
    const unsigned long long any_bad = __ballot(bad);
    if (threadIdx.x == 0) {
      failed = any_bad != 0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: L1 (and NC lines) dropped
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (failed) return false;
  const PeerRecv &r = p.r;
  if (v4) {
    for (int i = threadIdx.x; i < n / 4; i += blockDim.x) {
      float4 a = reinterpret_cast<const float4 *>(r.slot[0])[i];
      for (int q = 1; q < r.world; q++) {
        const float4 b = reinterpret_cast<const float4 *>(r.slot[q])[i];
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
      }
      reinterpret_cast<float4 *>(buf)[i] = a;
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      float a = r.slot[0][i];
      for (int q = 1; q < r.world; q++) a += r.slot[q][i];
      buf[i] = a;
    }
  }
  return true;
}

}  // namespace pgcn
