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

class Comm {
 public:
  Comm(int rank, int world, const void *unique_id_128);
  ~Comm();
  Comm(const Comm &) = delete;
  Comm &operator=(const Comm &) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  void allreduce_sum(float *buf, size_t n, hipStream_t s);
  void reduce_scatter_sum(const float *send, float *recv, size_t recvcount, hipStream_t s);
  static void unique_id(void *out128);

 private:
  int rank_, world_;
  void *comm_ = nullptr;  // ncclComm_t
};

}  // namespace pgcn
