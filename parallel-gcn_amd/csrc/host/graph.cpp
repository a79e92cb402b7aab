// parallel-gcn_amd/csrc/host/graph.cpp
#include "graph.hpp"

#include <cmath>
#include <functional>
#include <thread>

namespace pgcn {

float graph_coef(int deg_src, int deg_dst) {
  // hpdga-spring23/src/module.cpp:88-90: int product -> float for sqrtf, double division,
  // stored to float.  (src/parser.cpp:164-181 precomputes the same expression.)
  return (float)(1.0 / (double)sqrtf((float)(deg_src * deg_dst)));
}

void parallel_for(long long n, const std::function<void(long long, long long)> &f, int threads) {
  if (threads <= 0) {
    threads = (int)std::thread::hardware_concurrency();
    if (threads > 16) threads = 16;  // the GPU box grants 16 CPUs per GPU
    if (threads < 1) threads = 1;
  }
  if (n < 100000 || threads == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const long long step = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    const long long b = t * step, e = std::min(n, b + step);
    if (b >= e) break;
    ts.emplace_back([=, &f] { f(b, e); });
  }
  for (auto &t : ts) t.join();
}

std::vector<float> graph_coefs(int n, const int *indptr, const int *indices) {
  std::vector<float> v((size_t)indptr[n]);
  parallel_for(n, [&](long long b, long long e) {
    for (long long src = b; src < e; src++) {
      const int ds = indptr[src + 1] - indptr[src];
      for (int i = indptr[src]; i < indptr[src + 1]; i++) {
        const int dst = indices[i];
        v[i] = graph_coef(ds, indptr[dst + 1] - indptr[dst]);
      }
    }
  });
  return v;
}

DevGraph::DevGraph(int n_rows, const int *indptr, const int *indices, const float *vals)
    : n_rows_(n_rows), nnz_(indptr[n_rows]), h_indptr_(indptr, indptr + n_rows + 1) {
  indices_.allocate((size_t)nnz_ + 64);  // slack: unrolled loads never step past the end
  vals_.allocate((size_t)nnz_ + 64);
  indices_.upload(indices, (size_t)nnz_);
  vals_.upload(vals, (size_t)nnz_);
  PGCN_HIP(hipMemset(indices_.get() + nnz_, 0, 64 * sizeof(int)));
  PGCN_HIP(hipMemset(vals_.get() + nnz_, 0, 64 * sizeof(float)));
}

DevGraph::Sched &DevGraph::schedule(int vec) {
  auto it = scheds_.find(vec);
  if (it != scheds_.end()) return *it->second;
  PGCN_CHECK(graphsum_vec_supported(vec), PGCN_E_INVALID,
             "graphsum: row width not supported: " + std::to_string(4 * vec));
  auto sp = std::make_unique<Sched>();
  const int nb = 64 / vec;
  const int chunk = nb * 32;  // 32 wave iterations per work item
  std::vector<int4> items, comb;
  items.reserve((size_t)n_rows_ + (size_t)(nnz_ / chunk) + 1);
  long long slots = 0;
  for (int r = 0; r < n_rows_; r++) {
    const int b = h_indptr_[r], e = h_indptr_[r + 1];
    if (e - b <= chunk) {
      items.push_back(make_int4(r, b, e, -1));
    } else {
      const int first = (int)slots;
      int cnt = 0;
      for (int p = b; p < e; p += chunk) {
        items.push_back(make_int4(r, p, std::min(e, p + chunk), (int)slots++));
        cnt++;
      }
      comb.push_back(make_int4(r, first, cnt, 0));
    }
  }
  sp->s.vec = vec;
  sp->s.chunk = chunk;
  sp->s.n_items = (int)items.size();
  sp->s.n_comb = (int)comb.size();
  sp->s.n_slots = slots;
  sp->items.allocate(items.size());
  sp->items.upload(items);
  if (!comb.empty()) {
    sp->comb.allocate(comb.size());
    sp->comb.upload(comb);
  }
  if (slots) sp->partial.allocate((size_t)slots * vec * 4);
  sp->s.items = sp->items.get();
  sp->s.comb = sp->comb.get();
  auto &ref = *sp;
  scheds_[vec] = std::move(sp);
  return ref;
}

void DevGraph::graphsum(const float *in, int ld_in, float *out, int ld_out, int dim,
                        hipStream_t s) {
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0 && ld_in >= dim && ld_out >= dim,
             PGCN_E_INVALID, "graphsum: leading dims must be multiples of 4 and >= dim");
  const int vec = (dim + 3) / 4;
  Sched &sc = schedule(vec);
  launch_graphsum(sc.s, indices_.get(), vals_.get(), in, ld_in, out, ld_out, sc.partial.get(), s);
}

double DevGraph::algorithmic_bytes(int dim, long long n_in_rows) const {
  // 4(N+1) indptr + 8 nnz (index + value) + 4 N_in d (read) + 4 N d (write)
  return 4.0 * (n_rows_ + 1) + 8.0 * (double)nnz_ + 4.0 * (double)n_in_rows * dim +
         4.0 * (double)n_rows_ * dim;
}

}  // namespace pgcn
