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
#include <memory>
#include <vector>

#include <hip/hip_runtime.h>

namespace pgcn {

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

 protected:
  void count(size_t send_bytes, double factor) {
    calls++;
    bytes += factor * (double)send_bytes * (world_ - 1) / world_;
  }
  int rank_, world_;
};

// Timing only (tools/rank_epoch.py): rank `rank` of `world` with no peers -- a reduce-scatter
// keeps this rank's own share, an all-reduce leaves the buffer.  The rank's kernels and
// stream order are the edge-cut engine's; its numbers are not (no other rank contributes).
class SoloComm : public Comm {
 public:
  SoloComm(int rank, int world) : Comm(rank, world) {}
  void allreduce_sum(float *buf, size_t n, hipStream_t s) override;
  void reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                          hipStream_t s) override;
  const char *kind() const override { return "solo"; }
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

// In-process "fake RCCL" (SURVEY.md §4): `world` engines in one process on one device, each
// driven by its own host thread.  A collective is a host rendezvous of the ranks (each posts
// its buffer and an event recorded after its producer), then every rank's stream waits for
// all peers' events and sums the peers' buffers in rank order with a device kernel, then a
// second rendezvous on "read done" events before any rank may overwrite its send buffer.
// Same stream semantics as RCCL, so the edge-cut engine runs unchanged at world 2, 4, ... on
// one GPU (RCCL itself refuses two ranks on one device).
class LoopbackGroup {
 public:
  explicit LoopbackGroup(int world);
  int world() const { return world_; }
  // rendezvous `phase` of the current collective: publish (ptr, ev) of `rank`, wait for all
  // ranks, return every rank's (ptr, ev).  Throws PGCN_E_COMM after `timeout_s` seconds.
  void exchange(int rank, const void *ptr, hipEvent_t ev, std::vector<const void *> *ptrs,
                std::vector<hipEvent_t> *evs);
  double timeout_s = 60.0;

 private:
  struct Impl;
  std::shared_ptr<Impl> impl_;
  int world_;
};

class LoopbackComm : public Comm {
 public:
  LoopbackComm(int rank, std::shared_ptr<LoopbackGroup> group);
  ~LoopbackComm() override;
  void allreduce_sum(float *buf, size_t n, hipStream_t s) override;
  void reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                          hipStream_t s) override;
  const char *kind() const override { return "loopback"; }

 private:
  void collective(const float *send, float *dst, size_t count, size_t src_offset, hipStream_t s);
  std::shared_ptr<LoopbackGroup> group_;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
  float *tmp_ = nullptr;  // all-reduce result before it overwrites `buf`
  size_t tmp_n_ = 0;
};

}  // namespace pgcn
