// parallel-gcn_amd/csrc/k_peer.hip -- the edge-cut engine's peer-mapped exchange (PeerComm,
// host/comm.cpp): every rank's receive region is mapped into every other rank's address space
// (hipIpcOpenMemHandle across processes; plain pointers between the in-process loopback
// ranks), so a collective is one-sided stores over xGMI plus a flag per (receiver, sender).
//
// Replaces, for the reference's GraphSum at partition boundaries (src/module.cu:188-210) and
// the weight-gradient all-reduce, RCCL's reduce-scatter / all-reduce: rank r's partial sums of
// the rows owned by rank q are written straight into q's slot r (in the kernel that forms
// them: k_gs_lds_combine's push mode), and q sums its W slots in rank order (deterministic,
// the same order on every rank).
//
// Ordering, with flags and arrival counters in uncached device memory (MTYPE UC: no cache
// holds a line of them, on this GPU or a peer) and the receive slots in plain device memory:
//   producer  -- every store of a workgroup acknowledged (s_waitcnt vmcnt(0)), the workgroup's
//                barrier, one system-scope release (L2 write-back, waited for), one arrival on
//                the launch's counter; the last workgroup to arrive stores gen into flag[rank]
//                of every peer, and resets the counter (peer_sync.hpp);
//   consumer  -- one wave polls its own flags until every peer's reads gen (bounded: an error
//                word and an early exit after kPeerTimeoutTicks), then the sum kernel reads
//                the slots (stream order after the wait), each of its workgroups after a
//                system-scope acquire (acquire_system_workgroup).
// Slots are double-buffered by generation parity: a rank's push of generation g + 2 into
// peer q's slot follows (in its stream) its wait for g + 1, which needs q's push of g + 1,
// which follows (in q's stream) q's reads of generation g.
#include "common.hpp"
#include "kernels.hpp"
#include "lds_dma.hpp"
#include "peer_sync.hpp"

namespace pgcn {

// send [world][count] (stride 0: the same count floats for every receiver) -> receiver q's
// slot (sink.dst[q]); blockIdx.x = q (consecutive workgroups push to different peers: every
// link busy at once), blockIdx.y = the workgroup's piece of the count
// (T = float4 when count % 4 == 0, else float)
template <typename T>
__global__ __launch_bounds__(256) void k_peer_push(const T *__restrict__ send, long long n,
                                                   long long stride, PeerSink k) {
  const int q = blockIdx.x;
  const T *src = send + (long long)q * stride;
  for (long long i = (long long)blockIdx.y * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.y * blockDim.x) {
    if constexpr (sizeof(T) == 16)
      peer_store16(k.dst[q], k.slot_bytes, i, src[i]);
    else
      peer_store4(k.dst[q], k.slot_bytes, i, src[i]);
  }
  peer_arrive(k);
}

// one wave: lane q < world polls flags[q] (this rank's own flag words) until it reads gen;
// after kPeerTimeoutTicks of the 100 MHz clock an error word names the peer and every later
// wait returns at once (the host turns it into PGCN_E_COMM)
__global__ __launch_bounds__(64) void k_peer_wait(const unsigned *flags, int world, unsigned gen,
                                                  unsigned *err) {
  const int q = threadIdx.x;
  if (flag_load(err)) return;
  if (q >= world) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(flag_load(flags + q) - gen) < 0) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kPeerTimeoutTicks) {
      __hip_atomic_store(err, 0x10000u | (unsigned)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}

__device__ __forceinline__ void peer_acc(float &a, float b) { a += b; }
__device__ __forceinline__ void peer_acc(float4 &a, const float4 &b) { f4_acc(a, b); }

// A small all-reduce in ONE workgroup (peer_allreduce_block): replaces push + wait + sum
// launches (3 x ~5 us per collective at W = 8) for the loss scalars between processes.
__global__ __launch_bounds__(256) void k_peer_allreduce_small(float *__restrict__ buf, int n,
                                                              PeerSmall p) {
  (void)peer_allreduce_block(buf, n, p);
}

void launch_peer_allreduce_small(float *buf, int n, const PeerSink &k, const PeerRecv &r,
                                 const unsigned *waited, int nwait, unsigned *err,
                                 hipStream_t s) {
  PGCN_CHECK(k.world >= 1 && k.world <= kPeerMaxRanks && r.world == k.world && n >= 0 &&
                 n <= kPeerSmallAllreduce,
             PGCN_E_INVALID, "peer_allreduce_small: shape");
  PeerSmall p;
  p.k = k;
  p.r = r;
  p.waited = waited;
  p.nwait = nwait;
  p.err = err;
  PGCN_LAUNCH(k_peer_allreduce_small, dim3(1), dim3(256), 0, s, buf, n, p);
  PGCN_HIP(hipGetLastError());
}

// dst[i] = sum over q (rank order) of slot[q][i]
template <typename T>
__global__ __launch_bounds__(256) void k_peer_sum(PeerRecv r, T *__restrict__ dst, long long n) {
  acquire_system_workgroup();  // the peers' pushes (peer_sync.hpp)
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T p[kPeerMaxRanks];
#pragma unroll
  for (int q = 0; q < kPeerMaxRanks; q++)
    if (q < r.world) p[q] = reinterpret_cast<const T *>(r.slot[q])[i];
  T a = p[0];
#pragma unroll
  for (int q = 1; q < kPeerMaxRanks; q++)
    if (q < r.world) peer_acc(a, p[q]);
  dst[i] = a;
}

__global__ __launch_bounds__(256) void k_peer_push_grads(const float *__restrict__ arena, long long n,
                                                          GradRegions r, PeerSink k) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float v = arena[i];
    for (int t = 0; t < r.n; t++) {
      const long long rel = i - r.off[t];
      if (rel >= 0 && rel < (long long)r.d[t].K * r.d[t].N) v = tn_deferred_sum(r.d[t], rel);
    }
    for (int q = 0; q < k.world; q++) peer_store4(k.dst[q], k.slot_bytes, i, v);
  }
  peer_arrive(k);
}

void launch_peer_push_grads(const float *arena, long long n, const GradRegions &r,
                            const PeerSink &k, hipStream_t s) {
  PGCN_CHECK(k.world >= 1 && k.world <= kPeerMaxRanks && r.n >= 0 && r.n <= 4 && n > 0,
             PGCN_E_INVALID, "peer_push_grads: shape");
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(ceil_div(n, 256), 64));
  PGCN_LAUNCH(k_peer_push_grads, dim3(grid), dim3(256), 0, s, arena, n, r, k);
  PGCN_HIP(hipGetLastError());
}

void launch_peer_push(const float *send, size_t count, const PeerSink &k, hipStream_t s,
                      bool same_for_all) {
  PGCN_CHECK(k.world >= 1 && k.world <= kPeerMaxRanks, PGCN_E_INVALID, "peer_push: world");
  const bool v4 = count % 4 == 0;
  const long long n = (long long)(v4 ? count / 4 : count);
  const dim3 grid((unsigned)k.world,
                  (unsigned)std::max<long long>(1, std::min<long long>(ceil_div(n, 256), 64)));
  const long long stride = same_for_all ? 0 : n;
  if (v4)
    PGCN_LAUNCH(k_peer_push<float4>, grid, dim3(256), 0, s, reinterpret_cast<const float4 *>(send),
                n, stride, k);
  else
    PGCN_LAUNCH(k_peer_push<float>, grid, dim3(256), 0, s, send, n, stride, k);
  PGCN_HIP(hipGetLastError());
}

void launch_peer_wait(const unsigned *flags, int world, unsigned gen, unsigned *err,
                      hipStream_t s) {
  PGCN_LAUNCH(k_peer_wait, dim3(1), dim3(64), 0, s, flags, world, gen, err);
  PGCN_HIP(hipGetLastError());
}

void launch_peer_sum(const PeerRecv &r, float *dst, size_t count, hipStream_t s) {
  PGCN_CHECK(r.world >= 1 && r.world <= kPeerMaxRanks, PGCN_E_INVALID, "peer_sum: world");
  const bool v4 = count % 4 == 0;
  const long long n = (long long)(v4 ? count / 4 : count);
  if (n == 0) return;
  if (v4)
    PGCN_LAUNCH(k_peer_sum<float4>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, r,
                reinterpret_cast<float4 *>(dst), n);
  else
    PGCN_LAUNCH(k_peer_sum<float>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, r, dst, n);
  PGCN_HIP(hipGetLastError());
}

}  // namespace pgcn
