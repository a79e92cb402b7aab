// parallel-gcn_amd/csrc/host/comm.hpp -- edge-cut partition + RCCL communicator.
//
// New relative to the reference (single GPU, no collectives).  The graph is
// cut into `world` contiguous node ranges balanced by adjacency nnz.  Rank r owns the rows
// of its range: its features, activations, labels.  For GraphSum, rank r holds the columns
// of Â that belong to its range (the edges whose SOURCE feature row it owns), computes the
// partial sum for EVERY row from those columns alone (gathers hit only the local table,
// 1/world of the features), and the partials are summed into their owners with one RCCL
// reduce-scatter per GraphSum call.  Weight gradients and loss scalars are all-reduced.
#pragma once
#include <cstddef>
#include <functional>
#include <memory>
#include <vector>

#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "../kernels.hpp"

namespace pgcn {

// "peer_uncached" (read at engine build): the peer exchange's receive slots in uncached device
// memory (hipDeviceMallocUncached, MTYPE UC) instead of plain device memory -- no cache holds
// a slot line on the receiver; the pushes are then write-through (0.3 TB/s on one GPU, r05)
extern int g_peer_uncached;

struct Partition {
  int world = 1, rank = 0;
  std::vector<int> bounds;  // world + 1 node boundaries
  int maxrows = 0;          // padded rows per rank (equal reduce-scatter counts)
  int chunks = 1;           // reduce-scatter row chunks (maxrows is a multiple of chunks)
  int chunk_rows() const { return maxrows / chunks; }
  int first() const { return bounds[rank]; }
  int last() const { return bounds[rank + 1]; }
  int local_rows() const { return last() - first(); }
  int owner(int node) const;
};

// contiguous nnz-balanced ranges (every rank gets >= 1 node); maxrows rounded up to a
// multiple of `chunks`
Partition make_partition(int n, const int *indptr, int world, int rank, int chunks = 1);

// Chunk k of rank `part.rank`'s column block, rows in chunk-major padded order: row
// q*h + j (h = chunk_rows()) is global node bounds[q] + k*h + j of owner q (no edges past the
// owner's range).  Chunk k's reduce-scatter then hands rank q exactly its rows k*h .. k*h+h-1,
// so the sum of chunk k can travel while chunk k+1 is computed.
void partition_subgraph_chunk(const Partition &part, int n, const int *indptr,
                              const int *indices, int k, std::vector<int> *sub_indptr,
                              std::vector<int> *sub_indices);

// Rank `part.rank`'s column block of Â in padded row layout: rows = world*maxrows (row of
// global node i = owner(i)*maxrows + i - bounds[owner(i)]), columns = local node ids,
// values = the global Â coefficients.
void partition_subgraph(const Partition &part, int n, const int *indptr, const int *indices,
                        std::vector<int> *sub_indptr, std::vector<int> *sub_indices,
                        std::vector<float> *sub_vals);

// The collectives the edge-cut engine needs, stream-ordered like RCCL's: a call enqueues its
// work on `s` and returns; buffers may be reused by later work on `s`.
class Comm {
 public:
  Comm(int rank, int world) : rank_(rank), world_(world) {}
  virtual ~Comm() = default;
  Comm(const Comm &) = delete;
  Comm &operator=(const Comm &) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  virtual void allreduce_sum(float *buf, size_t n, hipStream_t s) = 0;
  // recv[0, recvcount) = sum over ranks of send[rank * recvcount, (rank + 1) * recvcount)
  virtual void reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                                  hipStream_t s) = 0;
  virtual const char *kind() const = 0;
  static void unique_id(void *out128);  // RCCL unique id (rank 0 creates, all share)
  // collectives enqueued and the bytes this rank sends into them (a ring reduce-scatter of a
  // send buffer of B bytes moves B (world - 1) / world per rank; an all-reduce 2x that)
  long long calls = 0;
  double bytes = 0.0;
  // a collective enqueued outside the calls above (PeerComm's fused GraphSum exchange)
  void note(size_t send_bytes, double factor) { count(send_bytes, factor); }
  // Work on another stream that the next collective must follow (eval_tail: the eval pass's
  // last exchange on comm_stream shares the slots' parity and the arrival counter): every
  // collective entry point calls enter(s) first, which makes `s` wait for it once
  void defer(hipEvent_t e) { pending_ = e; }
  void enter(hipStream_t s) {
    if (!pending_) return;
    if (hipStreamWaitEvent(s, pending_, 0) != hipSuccess)
      throw Error(PGCN_E_COMM, "comm: stream wait on the pending tail");
    pending_ = nullptr;
  }
  bool pending() const { return pending_ != nullptr; }
  // every rank has reached this point on the host (before the first device collective after
  // seconds of per-rank host set-up, so no rank's bounded device wait starts far ahead)
  virtual void host_barrier() {}

 protected:
  hipEvent_t pending_ = nullptr;
  void count(size_t send_bytes, double factor) {
    calls++;
    bytes += factor * (double)send_bytes * (world_ - 1) / world_;
  }
  int rank_, world_;
};


// One process per GPU over RCCL (xGMI on one node).
class RcclComm : public Comm {
 public:
  RcclComm(int rank, int world, const void *unique_id_128);
  ~RcclComm() override;
  void allreduce_sum(float *buf, size_t n, hipStream_t s) override;
  void reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                          hipStream_t s) override;
  const char *kind() const override { return "rccl"; }

 private:
  void *comm_ = nullptr;  // ncclComm_t
};

// In-process ranks (SURVEY.md §4 "fake RCCL"): `world` engines in one process on one device,
// each driven by its own host thread; their PeerComms exchange raw device pointers through
// this group's host rendezvous, and then run exactly the multi-process exchange's kernels
// (RCCL itself refuses two ranks on one device).
class LoopbackGroup {
 public:
  explicit LoopbackGroup(int world);
  int world() const { return world_; }
  // rendezvous `phase` of the current collective: publish (ptr, ev) of `rank`, wait for all
  // ranks, return every rank's (ptr, ev).  Throws PGCN_E_COMM after `timeout_s` seconds.
  void exchange(int rank, const void *ptr, hipEvent_t ev, std::vector<const void *> *ptrs,
                std::vector<hipEvent_t> *evs);
  // PeerComm::AllGather between the group's ranks (host threads of one process)
  void allgather(int rank, const void *mine, size_t bytes, void *all);
  void barrier(int rank);  // every rank of the group has called it
  double timeout_s = 60.0;

 private:
  struct Impl;
  std::shared_ptr<Impl> impl_;
  int world_;
};

// One-sided exchange over peer-mapped receive slots (k_peer.hip).  Every rank
// owns two device regions: 2 x world receive slots (generation parity x sender) of slot_floats
// floats, and an uncached header of flag words (one per sender), an arrival counter and an
// error word.
// Every region is mapped into every rank: hipIpcGetMemHandle / hipIpcOpenMemHandle between
// processes (`ipc`, one process per GPU), raw device pointers between the in-process loopback
// ranks on one device.  A collective is: pushes into the receivers' slots (k_peer_push, or the
// GraphSum combine itself: k_gs_lds_combine's push mode), the flags, one wave waiting for them,
// a rank-order sum of the received slots.  Stream-ordered like RCCL; every collective of a
// rank runs on one stream, in the same order on every rank.
class PeerComm : public Comm {
 public:
  // all[q * bytes, (q + 1) * bytes) = rank q's `mine` (every rank calls it, in the same order;
  // throws on failure).  The engine calls it at construction and destruction only.
  using AllGather = std::function<void(const void *mine, size_t bytes, void *all)>;
  // slot_floats: the largest collective's floats per rank
  // host_order (in-process ranks): before a rank enqueues a wait, every rank has enqueued the
  // push it waits for -- ranks of one process may share hardware queues (GPU_MAX_HW_QUEUES),
  // where a wait ahead of a peer's push would block that push (a host rendezvous per wait)
  // solo (timing only, tools/rank_epoch.py): rank `rank` of `world` with no peers -- every
  // peer's region is this rank's own, so the pushes, waits and sums run with this rank's
  // kernels and bytes (every store local), but the results are not the model's
  PeerComm(int rank, int world, size_t slot_floats, AllGather ag, bool ipc,
           std::function<void()> host_order = nullptr, bool solo = false);
  ~PeerComm() override;
  void allreduce_sum(float *buf, size_t n, hipStream_t s) override;
  void reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                          hipStream_t s) override;
  const char *kind() const override { return solo_ ? "solo" : ipc_ ? "peer" : "loopback"; }
  void host_barrier() override;
  bool slots_uncached() const { return uncached_; }
  // The GraphSum exchange fused into the combine: sink() opens the next collective and returns
  // where this rank's rows go (rows_per_rank padded rows per owner, owner-major); after the
  // push, wait() enqueues the wait for every sender and recv() names the received slots
  PeerSink sink(int rows_per_rank, size_t row_floats);
  void wait(hipStream_t s);
  PeerRecv recv() const;
  size_t slot_floats() const { return slot_floats_; }
  bool host_ordered() const { return (bool)host_order_; }  // in-process ranks
  // An all-reduce of n floats that the caller's own one-workgroup kernel completes
  // (peer_allreduce_block): opens the collective and fills *p, or returns false when that
  // form does not apply (in-process ranks, n above kPeerSmallAllreduce, world 1)
  bool small_allreduce(size_t n, PeerSmall *p);
  // The weight gradients' all-reduce between processes (or solo) with the deferred last TN
  // passes folded into its push (launch_peer_push_grads); the sum is left to the consumer:
  // *rv names the received slots, which the Adam launch sums in rank order.  Returns false
  // (nothing enqueued) where that form does not apply: in-process ranks, world 1.
  bool allreduce_grads(float *buf, size_t n, const GradRegions &r, hipStream_t s, PeerRecv *rv);
  // throws PGCN_E_COMM when a wait gave up (a peer never signalled); call after a sync
  void check() const;

 private:
  float *slot(char *slots, int parity, int sender) const;
  void unmap();
  char *slots_ = nullptr, *header_ = nullptr;     // this rank's regions
  std::vector<char *> peer_slots_, peer_header_;  // every rank's regions as mapped here
  size_t slot_floats_ = 0, bytes_ = 0;
  unsigned gen_ = 0;                         // the last collective's generation
  AllGather ag_;
  bool ipc_ = false, solo_ = false, uncached_ = false;
  std::function<void()> host_order_;
};


}  // namespace pgcn
