// parallel-gcn_amd/csrc/capi.cpp -- the extern "C" boundary declared in include/pgcn.h.
#include <atomic>
#include <cstring>
#include <memory>

#include "../../include/pgcn.h"
#include "common.hpp"
#include "host/comm.hpp"
#include "host/data.hpp"
#include "host/gcn.hpp"
#include "host/graph.hpp"
#include "kernels.hpp"
#include "rng.hpp"

#include <cmath>

using namespace pgcn;

namespace pgcn {
// engine knobs (pgcn_debug_set): defaults and meaning at their definitions
extern int g_train_ahead;           // host/gcn.cpp
extern int g_split_rows;            // host/gcn.cpp
extern int g_split_cols;            // host/gcn.cpp
extern int g_fuse_epilogue;         // host/gcn.cpp
extern int g_fuse_output;           // host/gcn.cpp
extern int g_mm_side;               // host/gcn.cpp
extern int g_eval_tail;             // host/gcn.cpp
extern int g_peer_uncached;         // host/comm.cpp
extern int g_tn_fold;               // host/gcn.cpp
extern int g_fuse_finish;           // host/gcn.cpp
extern int g_mask_per;              // host/gcn.cpp
extern int g_mask_adam;             // host/gcn.cpp
extern int g_mask_xstream;          // host/gcn.cpp
extern int g_reassoc_small;         // host/gcn.cpp
extern int g_defer_small_wgrad;     // host/module.cpp
extern int g_eval_ax;               // host/gcn.cpp
extern int g_epoch_graph;           // host/gcn.cpp
extern long long g_lds_min_bytes;   // host/graph.cpp
extern int g_lds_blocks;            // host/graph.cpp
extern int g_xstream_ring;          // k_xstream_lds.hip
extern int g_gs_split;              // host/graph.cpp
extern int g_co_draw;               // host/gcn.cpp
extern int g_sparse_dual;           // host/gcn.cpp
extern int g_gs_item_iters;         // host/graph.cpp
extern int g_gs_orig_cols;          // host/graph.cpp
extern int g_gs16_gather;           // host/graph.cpp
extern int g_parse_threads;         // host/data.cpp: pieces of the parallel text parse

namespace {
std::atomic<long long> g_path_hits[KP_COUNT];
thread_local long long t_path_hits[KP_COUNT];  // the launching host thread's (loopback ranks)
const char *const kPathNames[KP_COUNT] = {"xs_nn_ring", "xs_tn_ring", "xs_nn",   "xs_tn",
                                          "gs_ring",    "gs_gather",  "out_xent", "gemm_nn",
                                          "gemm_tn",    "gemm_nn_w",  "gemm_tn_w", "launches"};
}  // namespace
void note_path(KernelPath p) {
  g_path_hits[p].fetch_add(1, std::memory_order_relaxed);
  t_path_hits[p]++;
}
}  // namespace pgcn

struct pgcn_graph {
  std::unique_ptr<DevGraph> g;
};
struct pgcn_gcn {
  std::unique_ptr<GCN> g;
};
struct pgcn_dataset {
  GCNData d;
};
struct pgcn_loopback {
  std::shared_ptr<LoopbackGroup> g;
};

namespace {
void check_device() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    throw Error(PGCN_E_NODEVICE, "no HIP device visible: the engine has no CPU fallback");
}

GCNParams to_params(const pgcn_params *p, const pgcn_data *d) {
  GCNParams q;
  q.num_nodes = d->num_nodes;
  q.input_dim = p->input_dim;
  q.output_dim = p->output_dim;
  q.n_layers = p->n_layers;
  q.hidden_dims.assign(p->hidden_dims, p->hidden_dims + std::max(0, p->n_layers - 1));
  q.dropouts.assign(p->dropouts, p->dropouts + std::max(0, p->n_layers));
  q.epochs = p->epochs;
  q.early_stopping = p->early_stopping;
  q.reassociate_last = p->reassociate_last != 0;
  q.seed = p->seed;
  return q;
}
AdamParams to_adam(const pgcn_params *p) {
  AdamParams a;
  a.learning_rate = p->learning_rate;
  a.weight_decay = p->weight_decay;
  a.beta1 = p->beta1;
  a.beta2 = p->beta2;
  a.eps = p->eps;
  return a;
}
// GCNData view -> owned GCNData (the engine uploads from it once)
GCNData to_data(const pgcn_data *d, const pgcn_params *p) {
  GCNData g;
  const int n = d->num_nodes;
  g.num_nodes = n;
  g.input_dim = p->input_dim;
  g.output_dim = p->output_dim;
  g.graph.indptr.assign(d->graph_indptr, d->graph_indptr + n + 1);
  g.graph.indices.assign(d->graph_indices, d->graph_indices + d->graph_indptr[n]);
  g.feature_index.indptr.assign(d->feat_indptr, d->feat_indptr + n + 1);
  g.feature_index.indices.assign(d->feat_indices, d->feat_indices + d->feat_indptr[n]);
  g.feature_value.assign(d->feat_values, d->feat_values + d->feat_indptr[n]);
  g.label.assign(d->label, d->label + n);
  g.split.assign(d->split, d->split + n);
  return g;
}
}  // namespace

extern "C" {

const char *pgcn_status_string(int s) {
  switch (s) {
    case PGCN_OK: return "ok";
    case PGCN_E_INVALID: return "invalid argument";
    case PGCN_E_NOMEM: return "out of device memory";
    case PGCN_E_IO: return "cannot read input";
    case PGCN_E_COMM: return "RCCL error";
    case PGCN_E_NODEVICE: return "no HIP device";
    default: return s > 0 ? hipGetErrorString((hipError_t)s) : "unknown";
  }
}

int pgcn_version(void) { return 100; }

// ---------------------------------------------------------------- graph + kernels
int pgcn_graph_create(int n, const int *indptr, const int *indices, pgcn_graph **out) {
  return guarded([&] {
    PGCN_CHECK(n > 0 && indptr && indices && out, PGCN_E_INVALID, "graph_create args");
    check_device();
    std::vector<float> v = graph_coefs(n, indptr, indices);
    auto h = std::make_unique<pgcn_graph>();
    h->g = std::make_unique<DevGraph>(n, n, indptr, indices, v.data());
    std::vector<float> sc = degree_scales(n, indptr);
    h->g->set_scales(sc, sc);
    *out = h.release();
  });
}
int pgcn_graph_create_values(int n, const int *indptr, const int *indices, const float *values,
                             pgcn_graph **out) {
  return guarded([&] {
    PGCN_CHECK(n > 0 && indptr && indices && values && out, PGCN_E_INVALID,
               "graph_create_values args");
    PGCN_CHECK(indptr[0] == 0 && indptr[n] >= 0, PGCN_E_INVALID, "graph_create_values: indptr");
    for (int i = 0; i < n; i++)
      PGCN_CHECK(indptr[i + 1] >= indptr[i], PGCN_E_INVALID, "graph_create_values: indptr order");
    for (long long k = 0; k < indptr[n]; k++)
      PGCN_CHECK(indices[k] >= 0 && indices[k] < n, PGCN_E_INVALID,
                 "graph_create_values: column id out of range");
    check_device();
    auto h = std::make_unique<pgcn_graph>();
    h->g = std::make_unique<DevGraph>(n, n, indptr, indices, values);
    // the parser's coefficients exactly: the factorised LDS path applies
    const std::vector<float> coef = graph_coefs(n, indptr, indices);
    if (std::memcmp(coef.data(), values, coef.size() * sizeof(float)) == 0) {
      std::vector<float> sc = degree_scales(n, indptr);
      h->g->set_scales(sc, sc);
    }
    *out = h.release();
  });
}

int pgcn_debug_rank_graph(int n, const int *indptr, const int *indices, int world, int rank,
                          int chunks, int chunk, pgcn_graph **out, int *rows, int *cols) {
  return guarded([&] {
    PGCN_CHECK(n > 0 && indptr && indices && out && world >= 1 && rank >= 0 && rank < world &&
                   chunks >= 1 && chunk >= 0 && chunk < chunks,
               PGCN_E_INVALID, "rank_graph args");
    check_device();
    const Partition part = make_partition(n, indptr, world, rank, chunks);
    const std::vector<float> sg = degree_scales(n, indptr);
    const int h = part.chunk_rows();
    std::vector<int> sp, si;
    partition_subgraph_chunk(part, n, indptr, indices, chunk, &sp, &si);
    // the same values and scales as GCN::build's chunk graphs
    std::vector<float> rs((size_t)part.world * h, 0.0f), cs((size_t)part.local_rows()), sv(si.size());
    for (int c = 0; c < part.local_rows(); c++) cs[(size_t)c] = sg[(size_t)part.first() + c];
    for (int q = 0; q < part.world; q++)
      for (int j = 0; j < h; j++) {
        const int i = part.bounds[(size_t)q] + chunk * h + j;
        if (i >= part.bounds[(size_t)q + 1]) continue;
        const size_t r = (size_t)q * h + j;
        rs[r] = sg[(size_t)i];
        for (int t = sp[r]; t < sp[r + 1]; t++) {
          const int gj = part.first() + si[(size_t)t];
          sv[(size_t)t] = graph_coef(indptr[i + 1] - indptr[i], indptr[gj + 1] - indptr[gj]);
        }
      }
    auto g = std::make_unique<pgcn_graph>();
    g->g = std::make_unique<DevGraph>(part.world * h, part.local_rows(), sp.data(), si.data(),
                                      sv.data());
    g->g->set_scales(std::move(rs), cs);
    if (rows) *rows = part.world * h;
    if (cols) *cols = part.local_rows();
    *out = g.release();
  });
}

int pgcn_graph_destroy(pgcn_graph *g) {
  delete g;
  return PGCN_OK;
}
long long pgcn_graph_nnz(const pgcn_graph *g) { return g ? g->g->nnz() : -1; }

int pgcn_graphsum(const pgcn_graph *g, const float *in, int ld_in, float *out, int ld_out,
                  int dim, void *stream) {
  return guarded([&] {
    PGCN_CHECK(g && in && out && dim > 0, PGCN_E_INVALID, "graphsum args");
    g->g->graphsum(in, ld_in, out, ld_out, dim, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm(int M, int N, int K, const float *A, int lda, const float *B, int ldb, int trans_b,
              float *C, int ldc, const uint64_t *a_mask, long long mask_base, long long mask_ld,
              float a_scale, void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && B && C && M >= 0 && K > 0 && ldc >= N, PGCN_E_INVALID, "gemm args");
    launch_gemm_nn(M, N, K, A, lda, B, ldb, trans_b, C, ldc, a_mask, mask_base, mask_ld, a_scale,
                   as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

size_t pgcn_gemm_tn_workspace(int M, int N, int K) { return gemm_tn_workspace(M, N, K); }

int pgcn_gemm_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg, float *C,
                 int ldc, const uint64_t *a_mask, long long mask_base, long long mask_ld,
                 float a_scale, void *workspace, void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && G && C && workspace && K > 0 && ldc >= N, PGCN_E_INVALID, "gemm_tn args");
    launch_gemm_tn(M, N, K, A, lda, G, ldg, C, ldc, a_mask, mask_base, mask_ld, a_scale,
                   workspace, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_mask_nibbles(const uint64_t *mask, long long mask_base, long long mask_ld, int M, int K,
                      uint64_t *out, void *stream) {
  return guarded([&] {
    PGCN_CHECK(mask && out && M >= 0 && K > 0, PGCN_E_INVALID, "mask_nibbles args");
    launch_mask_nibbles(mask, mask_base, mask_ld, M, K, out, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm_xstream(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                      int trans_b, float *C, int ldc, const uint64_t *mask_nib, float a_scale,
                      void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && B && C && M >= 0 && ldc >= N, PGCN_E_INVALID, "gemm_xstream args");
    launch_xstream_nn(M, N, K, A, lda, B, ldb, trans_b, C, ldc, mask_nib, a_scale,
                      as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm_xstream_dual(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                           int trans_b, float *C, float *C2, int ldc, const uint64_t *mask_nib,
                           float a_scale, void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && B && C && C2 && mask_nib && M >= 0 && ldc >= N, PGCN_E_INVALID,
               "gemm_xstream_dual args");
    launch_xstream_nn(M, N, K, A, lda, B, ldb, trans_b, C, ldc, mask_nib, a_scale,
                      as_stream(stream), C2);
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm_tn_xstream(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *mask_nib, float a_scale,
                         void *workspace, void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && G && C && workspace && M >= 0 && ldc >= N, PGCN_E_INVALID,
               "gemm_tn_xstream args");
    launch_xstream_tn(M, N, K, A, lda, G, ldg, C, ldc, mask_nib, a_scale, workspace,
                      as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm_xstream_flat(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                           int trans_b, float *C, float *C2, int ldc, const uint64_t *mask,
                           long long mask_base, long long mask_words, float a_scale,
                           void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && B && C && mask && mask_words > 0 && mask_base >= 0 && M >= 0 && ldc >= N &&
                   xstream_ring_ok(K, lda),
               PGCN_E_INVALID, "gemm_xstream_flat args");
    const XsMask fm{mask, mask_base, K, mask_words};
    launch_xstream_nn(M, N, K, A, lda, B, ldb, trans_b, C, ldc, nullptr, a_scale,
                      as_stream(stream), C2, nullptr, &fm);
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_gemm_tn_xstream_flat(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                              float *C, int ldc, const uint64_t *mask, long long mask_base,
                              long long mask_words, float a_scale, void *workspace, void *stream) {
  return guarded([&] {
    PGCN_CHECK(A && G && C && workspace && mask && mask_words > 0 && mask_base >= 0 && M >= 0 &&
                   ldc >= N && xstream_ring_ok(K, lda),
               PGCN_E_INVALID, "gemm_tn_xstream_flat args");
    const XsMask fm{mask, mask_base, K, mask_words};
    launch_xstream_tn(M, N, K, A, lda, G, ldg, C, ldc, nullptr, a_scale, workspace,
                      as_stream(stream), &fm);
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_spmm_csr(int m, int p, const int *indptr, const int *indices, const float *a,
                  const uint64_t *a_mask, float a_scale, const float *b, float *c, void *stream) {
  return guarded([&] {
    launch_spmm_csr(m, p, p, indptr, indices, a, a_mask, 0, a_scale, b, c, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_spmm_csc_bwd(int nf, int p, const int *csc_ptr, const int *csc_row, const int *csc_pos,
                      const float *a, const uint64_t *a_mask, float a_scale, const float *cgrad,
                      float *bgrad, void *stream) {
  return guarded([&] {
    launch_spmm_csc_bwd(nf, p, p, csc_ptr, csc_row, csc_pos, a, a_mask, 0, a_scale, cgrad, bgrad,
                        as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_csr_transpose(int m, int n_cols, const int *indptr, const int *indices, int *csc_ptr,
                       int *csc_row, int *csc_pos) {
  return guarded([&] {
    std::memset(csc_ptr, 0, sizeof(int) * (size_t)(n_cols + 1));
    for (int k = 0; k < indptr[m]; k++) {
      PGCN_CHECK(indices[k] >= 0 && indices[k] < n_cols, PGCN_E_INVALID, "column id");
      csc_ptr[indices[k] + 1]++;
    }
    for (int f = 0; f < n_cols; f++) csc_ptr[f + 1] += csc_ptr[f];
    std::vector<int> fill(csc_ptr, csc_ptr + n_cols);
    for (int i = 0; i < m; i++)
      for (int k = indptr[i]; k < indptr[i + 1]; k++) {
        const int o = fill[(size_t)indices[k]]++;
        csc_row[o] = i;
        csc_pos[o] = k;
      }
  });
}

int pgcn_dropout_mask(uint64_t *chunk_states, long long n_chunks, long long n_elems,
                      long long elem0, float p, uint64_t *mask, const void *dev_jump_table,
                      void *stream) {
  return guarded([&] {
    launch_dropout_mask(chunk_states, n_chunks, elem0, n_elems, p, mask, dev_jump_table,
                        as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_dropout_apply(float *x, long long n, const uint64_t *mask, float scale, void *stream) {
  return guarded([&] {
    launch_dropout_apply_based(x, n, mask, 0, scale, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_relu_fwd(float *x, long long n, uint8_t *mask, int training, void *stream) {
  return guarded([&] { launch_relu_fwd(x, n, mask, training, as_stream(stream)); });
}
int pgcn_relu_bwd(float *g, long long n, const uint8_t *mask, void *stream) {
  return guarded([&] { launch_relu_bwd(g, n, mask, as_stream(stream)); });
}

int pgcn_xent_blocks(int n) { return xent_blocks(n); }

int pgcn_xent_fwd(float *logits, int ld, float *grad, const int *truth, int n, int c, int count,
                  int training, float *partials, void *stream) {
  return guarded([&] {
    launch_xent_fwd(logits, ld, grad, truth, n, c, count, training, partials, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_finalize(const float *partials, int n_blocks, int count, const float *w_l2,
                  long long n_l2, float weight_decay, float *out4, void *stream) {
  return guarded([&] {
    // out4[0..1] = {loss, acc}; out4[2..3] hold the raw sums (loss_sum, wrong); one launch
    launch_reduce_scalars(partials, n_blocks, w_l2, n_l2, out4 + 2, as_stream(stream), count,
                          weight_decay, out4);
  });
}

int pgcn_adam(float *w, const float *g, float *m, float *v, long long n, float step_size,
              float beta1, float beta2, float eps, float weight_decay, int decay, void *stream) {
  return guarded([&] {
    launch_adam(w, g, m, v, n, step_size, beta1, beta2, eps, weight_decay, decay,
                as_stream(stream));
  });
}

float pgcn_adam_step_size(float lr, float beta1, float beta2, int t) {
  return lr * sqrtf(1.0f - powf(beta2, (float)t)) / (1.0f - powf(beta1, (float)t));
}

// ---------------------------------------------------------------- engine
void pgcn_params_default(pgcn_params *p) {
  std::memset(p, 0, sizeof *p);
  p->n_layers = 2;
  p->hidden_dims[0] = 16;
  p->dropouts[0] = 0.5f;
  p->dropouts[1] = 0.5f;
  p->epochs = 100;
  p->early_stopping = 0;
  p->learning_rate = 0.01f;
  p->weight_decay = 5e-4f;
  p->beta1 = 0.9f;
  p->beta2 = 0.999f;
  p->eps = 1e-8f;
  p->reassociate_last = 1;
  p->seed = 0;
}

int pgcn_gcn_create(const pgcn_params *p, const pgcn_data *d, int device, pgcn_gcn **out) {
  return guarded([&] {
    PGCN_CHECK(p && d && out, PGCN_E_INVALID, "gcn_create args");
    check_device();
    GCNData data = to_data(d, p);
    auto h = std::make_unique<pgcn_gcn>();
    h->g = std::make_unique<GCN>(to_params(p, d), to_adam(p), data, device, nullptr);
    *out = h.release();
  });
}

int pgcn_comm_unique_id(void *uid) {
  return guarded([&] { Comm::unique_id(uid); });
}

int pgcn_gcn_create_dist(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                         int world, const void *uid, pgcn_gcn **out) {
  return guarded([&] {
    PGCN_CHECK(p && d && out && uid, PGCN_E_INVALID, "gcn_create_dist args");
    check_device();
    GCNData data = to_data(d, p);
    DistSpec ds;
    ds.rank = rank;
    ds.world = world;
    ds.unique_id = uid;
    auto h = std::make_unique<pgcn_gcn>();
    h->g = std::make_unique<GCN>(to_params(p, d), to_adam(p), data, device, &ds);
    *out = h.release();
  });
}

int pgcn_gcn_create_peer(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                         int world, pgcn_allgather_fn allgather, void *user, pgcn_gcn **out) {
  return guarded([&] {
    PGCN_CHECK(p && d && out && allgather && world >= 1 && world <= kPeerMaxRanks && rank >= 0 &&
                   rank < world,
               PGCN_E_INVALID, "gcn_create_peer args");
    check_device();
    GCNData data = to_data(d, p);
    DistSpec ds;
    ds.rank = rank;
    ds.world = world;
    ds.allgather = [allgather, user](const void *mine, size_t bytes, void *all) {
      if (allgather(mine, bytes, all, user) != 0)
        throw Error(PGCN_E_COMM, "peer comm: the caller's all-gather failed");
    };
    auto h = std::make_unique<pgcn_gcn>();
    h->g = std::make_unique<GCN>(to_params(p, d), to_adam(p), data, device, &ds);
    *out = h.release();
  });
}

int pgcn_debug_gcn_create_solo(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                               int world, pgcn_gcn **out) {
  return guarded([&] {
    PGCN_CHECK(p && d && out && world >= 1 && rank >= 0 && rank < world, PGCN_E_INVALID,
               "gcn_create_solo args");
    check_device();
    GCNData data = to_data(d, p);
    DistSpec ds;
    ds.rank = rank;
    ds.world = world;
    ds.solo = true;
    auto h = std::make_unique<pgcn_gcn>();
    h->g = std::make_unique<GCN>(to_params(p, d), to_adam(p), data, device, &ds);
    *out = h.release();
  });
}

int pgcn_loopback_create(int world, pgcn_loopback **out) {
  return guarded([&] {
    PGCN_CHECK(out, PGCN_E_INVALID, "loopback_create args");
    auto h = std::make_unique<pgcn_loopback>();
    h->g = std::make_shared<LoopbackGroup>(world);
    *out = h.release();
  });
}

int pgcn_loopback_destroy(pgcn_loopback *g) {
  delete g;  // engines keep the group alive until they are destroyed
  return PGCN_OK;
}

int pgcn_gcn_create_loopback(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                             pgcn_loopback *group, pgcn_gcn **out) {
  return guarded([&] {
    PGCN_CHECK(p && d && out && group && group->g, PGCN_E_INVALID, "gcn_create_loopback args");
    check_device();
    GCNData data = to_data(d, p);
    DistSpec ds;
    ds.rank = rank;
    ds.world = group->g->world();
    ds.loopback = group->g;
    auto h = std::make_unique<pgcn_gcn>();
    h->g = std::make_unique<GCN>(to_params(p, d), to_adam(p), data, device, &ds);
    *out = h.release();
  });
}

long long pgcn_gcn_query(pgcn_gcn *g, const char *key) {
  if (!g || !key) return PGCN_E_INVALID;
  const GCN &e = *g->g;
  const Comm *c = e.communicator();
  if (!std::strcmp(key, "world")) return c ? c->world() : 1;
  if (!std::strcmp(key, "rank")) return c ? c->rank() : 0;
  if (!std::strcmp(key, "comm"))
    return c ? (!std::strcmp(c->kind(), "rccl")       ? 1
                : !std::strcmp(c->kind(), "loopback") ? 2
                : !std::strcmp(c->kind(), "solo")     ? 3
                                                      : 4)
             : 0;
  if (!std::strcmp(key, "comm_calls")) return c ? c->calls : 0;
  if (!std::strcmp(key, "peer_uncached")) {  // the peer exchange's slots are uncached memory
    const auto *pc = dynamic_cast<const pgcn::PeerComm *>(c);
    return pc && pc->slots_uncached() ? 1 : 0;
  }
  if (!std::strcmp(key, "comm_bytes")) return c ? (long long)c->bytes : 0;
  if (!std::strcmp(key, "reassociated")) return e.reassociated() ? 1 : 0;
  if (!std::strcmp(key, "fused_tails")) return e.fused_tails();
  if (!std::strcmp(key, "graph_symmetric")) return e.symmetric() ? 1 : 0;
  if (!std::strcmp(key, "graphsum_lds")) return e.graphsum_lds() ? 1 : 0;
  if (!std::strcmp(key, "epochs")) return e.epochs_run();
  if (!std::strcmp(key, "eval_ax_us")) return (long long)(e.eval_ax_build_ms() * 1000.0f);
  return PGCN_E_INVALID;
}

int pgcn_gcn_destroy(pgcn_gcn *g) {
  delete g;
  return PGCN_OK;
}

int pgcn_gcn_train_epoch(pgcn_gcn *g, float out2[2]) {
  return guarded([&] {
    auto r = g->g->train_epoch();
    out2[0] = r.first;
    out2[1] = r.second;
  });
}

int pgcn_gcn_eval(pgcn_gcn *g, int split, float out2[2]) {
  return guarded([&] {
    auto r = g->g->eval(split);
    out2[0] = r.first;
    out2[1] = r.second;
  });
}

int pgcn_gcn_epoch_async(pgcn_gcn *g) {
  return guarded([&] { g->g->epoch_async(); });
}
int pgcn_gcn_sync(pgcn_gcn *g) {
  return guarded([&] { g->g->sync(); });
}
int pgcn_gcn_results(pgcn_gcn *g, int n, float *host_out) {
  int rows = 0;
  const int st = guarded([&] {
    PGCN_CHECK(n >= 0 && (n == 0 || host_out), PGCN_E_INVALID, "gcn_results args");
    auto r = g->g->results(n);
    std::memcpy(host_out, r.data(), r.size() * sizeof(float));
    rows = (int)(r.size() / 4);
  });
  return st == PGCN_OK ? rows : st;
}
int pgcn_gcn_run(pgcn_gcn *g, int verbose) {
  return guarded([&] { g->g->run(verbose != 0); });
}
long long pgcn_gcn_get_var(pgcn_gcn *g, int idx, int which, float *dst) {
  long long n = -1;
  const int st = guarded([&] {
    auto v = g->g->get_var(idx, which);
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(float));
    n = (long long)v.size();
  });
  return st == PGCN_OK ? n : st;
}
int pgcn_gcn_num_vars(pgcn_gcn *g) { return g->g->num_vars(); }
int pgcn_gcn_profile(pgcn_gcn *g, int enable) {
  return guarded([&] { g->g->set_profile(enable != 0); });
}
int pgcn_gcn_profile_read(pgcn_gcn *g, double *ms, long long *calls, double *bytes) {
  return guarded([&] { g->g->profile_read(ms, calls, bytes); });
}
int pgcn_gcn_profile_read_mm(pgcn_gcn *g, double *ms, long long *calls, double *flops) {
  return guarded([&] { g->g->profile_read_mm(ms, calls, flops); });
}
int pgcn_gcn_node_range(pgcn_gcn *g, int *first, int *last) {
  *first = g->g->partition().first();
  *last = g->g->partition().last();
  return PGCN_OK;
}

// ---------------------------------------------------------------- data
int pgcn_dataset_load(const char *root, const char *name, pgcn_dataset **out) {
  return guarded([&] {
    auto h = std::make_unique<pgcn_dataset>();
    Parser parser(&h->d, name, root ? root : ".");
    if (!parser.parse()) throw Error(PGCN_E_IO, std::string("Cannot read input: ") + name);
    *out = h.release();
  });
}

int pgcn_dataset_load_cached(const char *root, const char *name, pgcn_dataset **out,
                             int *from_cache) {
  return guarded([&] {
    auto h = std::make_unique<pgcn_dataset>();
    bool hit = false;
    if (!load_dataset_cached(&h->d, root ? root : ".", name, &hit))
      throw Error(PGCN_E_IO, std::string("Cannot read input: ") + name);
    if (from_cache) *from_cache = hit ? 1 : 0;
    *out = h.release();
  });
}

int pgcn_dataset_save(const pgcn_dataset *ds, const char *path) {
  return guarded([&] {
    PGCN_CHECK(ds && path, PGCN_E_INVALID, "dataset_save: null argument");
    if (!save_binary(ds->d, path, nullptr))
      throw Error(PGCN_E_IO, std::string("cannot write ") + path);
  });
}

int pgcn_dataset_binarize(pgcn_dataset *ds) {
  if (!ds) return PGCN_E_INVALID;
  std::fill(ds->d.feature_value.begin(), ds->d.feature_value.end(), 1.0f);
  return PGCN_OK;
}

int pgcn_dataset_load_binary(const char *path, pgcn_dataset **out) {
  return guarded([&] {
    PGCN_CHECK(path && out, PGCN_E_INVALID, "dataset_load_binary: null argument");
    auto h = std::make_unique<pgcn_dataset>();
    if (!load_binary(&h->d, path, nullptr))
      throw Error(PGCN_E_IO, std::string("not a valid dataset cache: ") + path);
    *out = h.release();
  });
}

int pgcn_dataset_synthetic(int n, int f, int c, long long undirected_edges, uint64_t seed,
                           pgcn_dataset **out) {
  return guarded([&] {
    PGCN_CHECK(n > 1 && f > 0 && c > 0 && undirected_edges >= 0, PGCN_E_INVALID, "synthetic args");
    auto h = std::make_unique<pgcn_dataset>();
    make_synthetic(&h->d, n, f, c, undirected_edges, seed);
    *out = h.release();
  });
}

int pgcn_dataset_view(const pgcn_dataset *ds, pgcn_data *v, int *input_dim, int *output_dim) {
  if (!ds || !v) return PGCN_E_INVALID;
  v->num_nodes = ds->d.num_nodes;
  v->graph_indptr = ds->d.graph.indptr.data();
  v->graph_indices = ds->d.graph.indices.data();
  v->feat_indptr = ds->d.feature_index.indptr.data();
  v->feat_indices = ds->d.feature_index.indices.data();
  v->feat_values = ds->d.feature_value.data();
  v->label = ds->d.label.data();
  v->split = ds->d.split.data();
  if (input_dim) *input_dim = ds->d.input_dim;
  if (output_dim) *output_dim = ds->d.output_dim;
  return PGCN_OK;
}

int pgcn_dataset_free(pgcn_dataset *ds) {
  delete ds;
  return PGCN_OK;
}

// ---------------------------------------------------------------- diagnostics
int pgcn_debug_set(const char *key, int value) {
  if (!key) return PGCN_E_INVALID;
  // every key's value range is checked: an out-of-range value is refused, never reinterpreted
  auto in = [&](int lo, int hi) { return value >= lo && value <= hi; };
  if (!std::strcmp(key, "train_ahead")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_train_ahead = value;
  } else if (!std::strcmp(key, "split_rows")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_split_rows = value;
  } else if (!std::strcmp(key, "split_cols")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_split_cols = value;
  } else if (!std::strcmp(key, "eval_ax")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_eval_ax = value;
  } else if (!std::strcmp(key, "epoch_graph")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_epoch_graph = value;
  } else if (!std::strcmp(key, "fuse_epilogue")) {
    if (!in(0, 15)) return PGCN_E_INVALID;
    pgcn::g_fuse_epilogue = value;
  } else if (!std::strcmp(key, "fuse_output")) {
    if (!in(0, 3)) return PGCN_E_INVALID;
    pgcn::g_fuse_output = value;
  } else if (!std::strcmp(key, "mm_side")) {
    if (!in(0, 2)) return PGCN_E_INVALID;
    pgcn::g_mm_side = value;
  } else if (!std::strcmp(key, "eval_tail")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_eval_tail = value;
  } else if (!std::strcmp(key, "mask_xstream")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_mask_xstream = value;
  } else if (!std::strcmp(key, "mask_adam")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_mask_adam = value;
  } else if (!std::strcmp(key, "defer_wgrad")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_defer_small_wgrad = value;
  } else if (!std::strcmp(key, "reassoc_small")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_reassoc_small = value;
  } else if (!std::strcmp(key, "csc_tree")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_csc_tree = value;
  } else if (!std::strcmp(key, "mask_per")) {
    if (!in(0, 2)) return PGCN_E_INVALID;
    pgcn::g_mask_per = value;
  } else if (!std::strcmp(key, "fuse_finish")) {
    if (!in(0, 2)) return PGCN_E_INVALID;
    pgcn::g_fuse_finish = value;
  } else if (!std::strcmp(key, "tn_fold")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_tn_fold = value;
  } else if (!std::strcmp(key, "ring_window")) {
    if (value != 0 && value != 2 && value != 3) return PGCN_E_INVALID;
    pgcn::g_ring_window = value;
  } else if (!std::strcmp(key, "ring_pair")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_ring_pair = value;
  } else if (!std::strcmp(key, "peer_uncached")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_peer_uncached = value;
  } else if (!std::strcmp(key, "xstream_ring")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_xstream_ring = value;
  } else if (!std::strcmp(key, "lds_min_kb")) {  // < 0: the default
    pgcn::g_lds_min_bytes = value < 0 ? DevGraph::kLdsMinBytes : 1024LL * value;
  } else if (!std::strcmp(key, "lds_blocks")) {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16 &&
        value != 32)
      return PGCN_E_INVALID;
    pgcn::g_lds_blocks = value;
  } else if (!std::strcmp(key, "gs_orig_cols")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_gs_orig_cols = value;
  } else if (!std::strcmp(key, "gs16_gather")) {
    if (!in(0, 2)) return PGCN_E_INVALID;
    pgcn::g_gs16_gather = value;
  } else if (!std::strcmp(key, "sparse_dual")) {
    if (!in(0, 1)) return PGCN_E_INVALID;
    pgcn::g_sparse_dual = value;
  } else if (!std::strcmp(key, "co_draw")) {
    if (!in(0, 2)) return PGCN_E_INVALID;
    pgcn::g_co_draw = value;
  } else if (!std::strcmp(key, "gs_split")) {
    if (!in(0, 3)) return PGCN_E_INVALID;
    pgcn::g_gs_split = value;
  } else if (!std::strcmp(key, "gs_item_iters")) {
    if (value != 0 && value != 2 && value != 4 && value != 8 && value != 16 && value != 32)
      return PGCN_E_INVALID;
    pgcn::g_gs_item_iters = value;
  } else if (!std::strcmp(key, "parse_threads")) {
    if (!in(0, 4096)) return PGCN_E_INVALID;
    pgcn::g_parse_threads = value;
  } else {
    return PGCN_E_INVALID;
  }
  return PGCN_OK;
}

// CPU check of the d = 16 ring schedule of a CSR pattern: builds it, walks it as the kernel
// does over a seeded input and reports the max relative error of the sums against a direct CSR
// sum, and the number of entry blocks.  No device needed.  (window: kRingWindow, the only
// schedule.)  Diagnostics: the schedule's step counts [wg][t_max][LDS_CW][LDS_SLOTS] (uint16)
// and its shape {n_batches, t_max, LDS_CW, LDS_SLOTS, window} (balance analysis on the host).
long long pgcn_debug_lds_counts(int n_rows, int n_cols, const int *indptr, const int *indices,
                                int window, unsigned short *dst, long long cap, int *shape5) {
  long long n = -1;
  const int st = guarded([&] {
    PGCN_CHECK(n_rows > 0 && n_cols > 0 && indptr && indices && window == kRingWindow,
               PGCN_E_INVALID, "lds_counts args");
    std::vector<int> ip(indptr, indptr + n_rows + 1), ix(indices, indices + indptr[n_rows]);
    const std::vector<int> cut = ring_cuts(n_cols, ix, lds_blocks(n_rows, n_cols));
    const LdsHost h = build_ring_host(
        n_rows, n_cols, ip, ix, cut, lds_slots(n_rows, n_cols), -1,
        ring_window_for(n_rows, n_cols, (long long)ix.size(), (int)cut.size() - 1));
    n = (long long)h.counts.size();
    if (dst) std::copy(h.counts.begin(), h.counts.begin() + std::min(n, cap), dst);
    if (shape5) {
      shape5[0] = h.n_batches;
      shape5[1] = h.t_max;
      shape5[2] = LDS_CW;
      shape5[3] = h.ns;
      shape5[4] = kRingWindow;
    }
  });
  return st == PGCN_OK ? n : -1;
}

int pgcn_debug_lds_check(int n_rows, int n_cols, const int *indptr, const int *indices,
                         int window, double *max_rel_err, long long *n_blocks) {
  return guarded([&] {
    PGCN_CHECK(n_rows > 0 && n_cols > 0 && indptr && indices && window == kRingWindow,
               PGCN_E_INVALID, "lds_check args");
    std::vector<int> ip(indptr, indptr + n_rows + 1), ix(indices, indices + indptr[n_rows]);
    const std::vector<int> cut = ring_cuts(n_cols, ix, lds_blocks(n_rows, n_cols));
    const LdsHost h = build_ring_host(
        n_rows, n_cols, ip, ix, cut, lds_slots(n_rows, n_cols), -1,
        ring_window_for(n_rows, n_cols, (long long)ix.size(), (int)cut.size() - 1));
    std::vector<float> in((size_t)n_cols);
    uint64_t st[2] = {12345, 67890};
    for (auto &x : in) x = (float)((double)(xs_next(st) & 0xffffff) / (double)0x1000000 - 0.5);
    std::vector<double> out((size_t)n_rows, 0.0);
    ring_emulate(h, n_rows, in.data(), out.data());
    double err = 0;
    for (int r = 0; r < n_rows; r++) {
      double ref = 0, mag = 0;
      for (int k = ip[(size_t)r]; k < ip[(size_t)r + 1]; k++) {
        ref += in[(size_t)ix[(size_t)k]];
        mag += std::fabs(in[(size_t)ix[(size_t)k]]);
      }
      err = std::max(err, std::fabs(out[(size_t)r] - ref) / (mag + 1e-30));
    }
    if (max_rel_err) *max_rel_err = err;
    if (n_blocks) *n_blocks = h.wave_off.back();
  });
}

int pgcn_debug_empty_launches(int n, void *stream) {
  return guarded([&] {
    PGCN_CHECK(n >= 0, PGCN_E_INVALID, "empty_launches: n >= 0");
    launch_empty(n, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_debug_exp_check(const float *x, long long n, float *mine, float *lib, void *stream) {
  return guarded([&] {
    PGCN_CHECK(n >= 0 && (n == 0 || (x && mine && lib)), PGCN_E_INVALID, "exp_check args");
    launch_exp_check(x, n, mine, lib, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

int pgcn_debug_div_check(const float *a, const float *b, long long n, float *q, void *stream) {
  return guarded([&] {
    PGCN_CHECK(n >= 0 && (n == 0 || (a && b && q)), PGCN_E_INVALID, "div_check args");
    launch_div_check(a, b, n, q, as_stream(stream));
    PGCN_HIP(hipGetLastError());
  });
}

long long pgcn_debug_path_count(const char *name, int reset) {
  const bool thread = (reset & 2) != 0, zero = (reset & 1) != 0;
  if (reset & ~3) return PGCN_E_INVALID;
  if (!name) {
    if (!zero) return PGCN_E_INVALID;
    for (int p = 0; p < KP_COUNT; p++) {
      if (thread) pgcn::t_path_hits[p] = 0;
      else pgcn::g_path_hits[p].store(0);
    }
    return 0;
  }
  for (int p = 0; p < KP_COUNT; p++)
    if (!std::strcmp(name, pgcn::kPathNames[p])) {
      if (thread) {
        const long long n = pgcn::t_path_hits[p];
        if (zero) pgcn::t_path_hits[p] = 0;
        return n;
      }
      return zero ? pgcn::g_path_hits[p].exchange(0) : pgcn::g_path_hits[p].load();
    }
  return PGCN_E_INVALID;
}

// ---------------------------------------------------------------- partition (host only)
int pgcn_partition_bounds(int n, const int *indptr, int world, int *bounds_out, int *maxrows) {
  return guarded([&] {
    Partition p = make_partition(n, indptr, world, 0);
    std::memcpy(bounds_out, p.bounds.data(), sizeof(int) * (size_t)(world + 1));
    if (maxrows) *maxrows = p.maxrows;
  });
}

// Rank `rank`'s column block in the padded row layout (sizes: call with null arrays first
// to get nnz; indptr needs world*maxrows+1 entries).
long long pgcn_partition_subgraph(int n, const int *indptr, const int *indices, int world,
                                  int rank, int *sub_indptr, int *sub_indices, float *sub_vals) {
  long long nnz = -1;
  const int st = guarded([&] {
    Partition p = make_partition(n, indptr, world, rank);
    std::vector<int> sp, si;
    std::vector<float> sv;
    partition_subgraph(p, n, indptr, indices, &sp, &si, &sv);
    nnz = (long long)si.size();
    if (sub_indptr) std::memcpy(sub_indptr, sp.data(), sp.size() * sizeof(int));
    if (sub_indices) std::memcpy(sub_indices, si.data(), si.size() * sizeof(int));
    if (sub_vals) std::memcpy(sub_vals, sv.data(), sv.size() * sizeof(float));
  });
  return st == PGCN_OK ? nnz : st;
}

}  // extern "C"
