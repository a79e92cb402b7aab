// parallel-gcn_amd/csrc/host/graph.hpp -- device adjacency for GraphSum.
//
// The reference keeps the adjacency as DevSparseIndex (include/sparse.cuh:21-29) plus a
// separately uploaded dev_graph_value array (src/parser.cpp:164-181, src/gcn.cu:30-43).  Here
// DevGraph owns the CSR column ids, the Â coefficients and, per row width, the wavefront
// work schedule of k_graphsum (built once; the graph is static across epochs).
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <vector>

#include "../kernels.hpp"
#include "runtime.hpp"

namespace pgcn {

// hpdga module.cpp:88-90 coefficient, bit-exact: (float)(1.0 / (double)sqrtf((float)(di*dj)))
float graph_coef(int deg_src, int deg_dst);

// Coefficients for every slot of a CSR whose degrees are the row lengths (single graph).
std::vector<float> graph_coefs(int n, const int *indptr, const int *indices);

// Runs f(begin, end) over [0, n) on up to `threads` host threads.
void parallel_for(long long n, const std::function<void(long long, long long)> &f,
                  int threads = 0);

class DevGraph {
 public:
  // CSR with n_rows rows; `vals` aligned with `indices` (coefficients).
  DevGraph(int n_rows, const int *indptr, const int *indices, const float *vals);
  int rows() const { return n_rows_; }
  long long nnz() const { return nnz_; }
  const int *indices() const { return indices_.get(); }
  const float *vals() const { return vals_.get(); }
  const std::vector<int> &host_indptr() const { return h_indptr_; }
  // out[i,:dim] = sum_j val_ij * in[col_j,:dim]
  void graphsum(const float *in, int ld_in, float *out, int ld_out, int dim, hipStream_t s);
  // bytes the kernel must move at minimum (SURVEY.md §8d formula, per call)
  double algorithmic_bytes(int dim, long long n_in_rows) const;

 private:
  struct Sched {
    GraphSchedule s;
    DeviceBuffer<int4> items, comb;
    DeviceBuffer<float> partial;
  };
  Sched &schedule(int vec);
  int n_rows_;
  long long nnz_;
  std::vector<int> h_indptr_;
  DeviceBuffer<int> indices_;
  DeviceBuffer<float> vals_;
  std::map<int, std::unique_ptr<Sched>> scheds_;
};

}  // namespace pgcn
