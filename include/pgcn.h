/* include/pgcn.h -- the drop-in C ABI of the MI355X GCN engine (libpgcn.so).
 *
 * Two layers, both plain C: caller-owned device pointers, sizes, a hipStream_t passed as
 * `void *`, int status returns (0 = OK, >0 = hipError_t, <0 = PGCN_E_*). Kernel entry
 * points never allocate (workspace is passed in or owned by a handle created beforehand),
 * are asynchronous on the given stream and are safe to capture into a hipGraph.
 *
 *  (1) Kernel ABI -- one entry per reference kernel family it replaces
 *      (reference: src/module.cu, src/optim.cu, src/gcn.cu of parallel-GCN).
 *  (2) Engine ABI -- the GCN object of include/gcn.cuh (ctor + train_epoch/eval/run),
 *      plus the edge-cut multi-GPU variant (new: the reference is single-GPU).
 *
 * The reference's C++ classes (Module and its subclasses, Variable, Adam, GCN, Parser) with
 * their constructor shapes are published in include/pgcn.hpp (namespace pgcn::api, the same
 * library); INTEGRATION.md shows the bindings a reference maintainer would add.
 */
#ifndef PGCN_H
#define PGCN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGCN_OK 0
#define PGCN_E_INVALID (-1)   /* bad argument / shape */
#define PGCN_E_NOMEM (-2)     /* device allocation failed */
#define PGCN_E_IO (-3)        /* dataset could not be read (Parser::parse() == false) */
#define PGCN_E_COMM (-4)      /* RCCL error */
#define PGCN_E_NODEVICE (-5)  /* no HIP device: the product has no CPU fallback */

const char *pgcn_status_string(int status);
int pgcn_version(void);

/* ===================================================================================== */
/* (1) Kernel ABI                                                                          */
/* ===================================================================================== */

/* --- xorshift128+ (hpdga-spring23/src/rand.cpp:17-28), host helpers ------------------- */
/* Default seed state of hpdga init_rand_state() (rand.cpp:6-14). */
void pgcn_rng_seed(uint64_t state[2]);
/* the same two draws after srand(seed), on a private glibc random_r state */
void pgcn_rng_seed_glibc(unsigned int seed, uint64_t state[2]);
/* state <- state advanced by `k` draws (GF(2) jump-ahead; exact). */
void pgcn_rng_jump(uint64_t state[2], uint64_t k);

/* --- Graph (DevSparseIndex + precomputed Â values; include/sparse.cuh:21-29,
 *     src/parser.cpp:164-181) ------------------------------------------------------------ */
typedef struct pgcn_graph pgcn_graph;
/* Uploads a CSR adjacency (implicit self loops already present, as the hpdga Parser builds
 * it), computes coef = 1/sqrtf(deg_src*deg_dst) bit-exactly as hpdga module.cpp:88-90 and
 * builds the wavefront work schedule. Host pointers. */
int pgcn_graph_create(int n_nodes, const int *indptr, const int *indices, pgcn_graph **out);
/* The reference's full GraphSum contract (include/module.cuh:82, the dev_graph_value array of
 * src/gcn.cu:30-43): any per-slot values, aligned with `indices` (host pointers).  Values equal
 * to the parser's coefficients (as pgcn_graph_create computes them) take the LDS ring path;
 * any other values take the per-edge gather kernels.  The pattern need not be symmetric (the
 * call is out = A in for the given A; the engine's backward identity needs A = A^T). */
int pgcn_graph_create_values(int n_nodes, const int *indptr, const int *indices,
                             const float *values, pgcn_graph **out);
int pgcn_graph_destroy(pgcn_graph *g);
long long pgcn_graph_nnz(const pgcn_graph *g);
/* out[i, 0:dim] = sum_j coef_ij * in[j, 0:dim]  (GraphSum::forward/backward,
 * src/module.cu:172-210; the backward is the same gather on grads because Â is symmetric).
 * Row-major, leading dims ld_in/ld_out (multiples of 4, >= dim). Device pointers. */
int pgcn_graphsum(const pgcn_graph *g, const float *in, int ld_in, float *out, int ld_out,
                  int dim, void *stream);

/* --- dense GEMMs on fp32 MFMA (Matmul, src/module.cu:274-472; dense X * W1) ------------- */
/* C[M,N] = A[M,K] * op(B)   (op(B) = B[K,N] if trans_b == 0 else B^T with B stored [N,K]).
 * Optional dropout on A: element (m,k) is kept iff bit (mask_base + m*mask_ld + k) of
 * `a_mask` is set, kept values scaled by `a_scale` (a_mask NULL: no dropout). */
int pgcn_gemm(int M, int N, int K, const float *A, int lda, const float *B, int ldb, int trans_b,
              float *C, int ldc, const uint64_t *a_mask, long long mask_base, long long mask_ld,
              float a_scale, void *stream);
/* C[K,N] = A[M,K]^T * G[M,N], reduced over M deterministically (split-M slabs + ordered
 * reduction; replaces the atomicAdd kernels matmul_kernel_backward_2 and
 * sparse_matmul_kernel_backward). `workspace` >= pgcn_gemm_tn_workspace(M,N,K) bytes. */
size_t pgcn_gemm_tn_workspace(int M, int N, int K);
int pgcn_gemm_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                 float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                 long long mask_ld, float a_scale, void *workspace, void *stream);

/* X-stream forms of the two contractions over the dense feature matrix (N <= 16, K <= 640;
 * SparseMatmul::forward/backward on dense X, src/module.cu:104-163), with the dropout keep
 * bits in the "nibble" layout: mask_nib[m][j] (16 words per row) holds in nibble c the bits of
 * A[m][64c + 4j .. 64c + 4j + 3].  pgcn_mask_nibbles builds it from the flat bitmap of
 * pgcn_gemm (bit mask_base + m*mask_ld + k).  mask_nib NULL: no dropout.  The TN form needs
 * pgcn_gemm_tn_workspace(M, N, K) bytes of workspace.  Same results as pgcn_gemm /
 * pgcn_gemm_tn up to fp32 summation order. */
int pgcn_mask_nibbles(const uint64_t *mask, long long mask_base, long long mask_ld, int M, int K,
                      uint64_t *mask_nib, void *stream);
int pgcn_gemm_xstream(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                      int trans_b, float *C, int ldc, const uint64_t *mask_nib, float a_scale,
                      void *stream);
/* Both first-layer products from one pass over A: C = A B (no dropout) and C2 = drop(A) B,
 * C2 bit-identical to pgcn_gemm_xstream with the same mask.  The engine uses it for eval's
 * forward together with the next training forward (same weights: no optimizer step between),
 * replacing the reference's two separate SparseMatmul::forward passes (src/module.cu:104-126,
 * called by src/gcn.cu:293-343). */
int pgcn_gemm_xstream_dual(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                           int trans_b, float *C, float *C2, int ldc, const uint64_t *mask_nib,
                           float a_scale, void *stream);
int pgcn_gemm_tn_xstream(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *mask_nib, float a_scale,
                         void *workspace, void *stream);
/* The same products with the flat bitmap itself (keep bit of A[m][k] at mask_base + m*K + k;
 * mask_words uint64 words at mask, an even count), which the engine passes on the shapes the
 * loader-wave kernels take (K in 577..640, lda = K rounded up to 4; others: PGCN_E_INVALID):
 * their loader waves stage each 16-row group's bits beside its rows, no pgcn_mask_nibbles
 * pass.  C2 NULL: the single product.  Bit-identical to the nibble forms with the nibbles of
 * the same bitmap. */
int pgcn_gemm_xstream_flat(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                           int trans_b, float *C, float *C2, int ldc, const uint64_t *mask,
                           long long mask_base, long long mask_words, float a_scale, void *stream);
int pgcn_gemm_tn_xstream_flat(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                              float *C, int ldc, const uint64_t *mask, long long mask_base,
                              long long mask_words, float a_scale, void *workspace, void *stream);

/* --- sparse X (SparseMatmul, src/module.cu:104-163) ----------------------------------- */
/* c[i,:] = sum_jj drop(a[jj]) * b[indices[jj], :], CSR order (bit-exact vs hpdga). */
int pgcn_spmm_csr(int m, int p, const int *indptr, const int *indices, const float *a,
                  const uint64_t *a_mask, float a_scale, const float *b, float *c, void *stream);
/* bgrad[f,:] = sum over (i,jj) with indices[jj]==f, in CSR order: drop(a[jj]) * cgrad[i,:],
 * using the transposed index (csc_ptr/csc_row/csc_pos) built by pgcn_csr_transpose. */
int pgcn_spmm_csc_bwd(int n_features, int p, const int *csc_ptr, const int *csc_row,
                      const int *csc_pos, const float *a, const uint64_t *a_mask, float a_scale,
                      const float *cgrad, float *bgrad, void *stream);
/* host helper: CSR (m rows, nnz, column ids < n_cols) -> CSC with original positions */
int pgcn_csr_transpose(int m, int n_cols, const int *indptr, const int *indices, int *csc_ptr,
                       int *csc_row, int *csc_pos);

/* --- dropout (Dropout, src/module.cu:16-99; hpdga module.cpp:208-228) ------------------ */
/* Bit-exact hpdga masks: chunk c holds the xorshift128+ state at the draw that element
 * 64*c of the variable consumes.  One call generates words [c0, c0+n_chunks) and advances
 * every chunk state by `period` draws via the byte tables built by pgcn_rng_jump_table. */
int pgcn_rng_jump_table(uint64_t period, void *host_table /* 16*256*16 bytes */);
int pgcn_dropout_mask(uint64_t *chunk_states, long long n_chunks, long long n_elems,
                      long long elem0, float p, uint64_t *mask, const void *dev_jump_table,
                      void *stream);
/* x[i] *= bit(i) ? scale : 0 for i in [0,n) (also the backward on grads). */
int pgcn_dropout_apply(float *x, long long n, const uint64_t *mask, float scale, void *stream);

/* --- ReLU (src/module.cu:215-265) ------------------------------------------------------- */
int pgcn_relu_fwd(float *x, long long n, uint8_t *mask, int training, void *stream);
int pgcn_relu_bwd(float *g, long long n, const uint8_t *mask, void *stream);

/* --- cross entropy + accuracy (src/module.cu:484-541, src/gcn.cu:264-289) -------------- */
/* Rows with truth >= 0: logits max-shifted in place; if training grad = (softmax - 1[t])
 * / count, zero elsewhere.  Writes per-block partial sums (loss, wrong) to `partials`
 * (>= 2*pgcn_xent_blocks(n) floats); pgcn_finalize reduces them. */
int pgcn_xent_blocks(int n);
int pgcn_xent_fwd(float *logits, int ld, float *grad, const int *truth, int n, int c,
                  int count, int training, float *partials, void *stream);
/* out4[0] = loss/count + wd*sum(w^2)/2, out4[1] = (count-wrong)/count   (device) */
int pgcn_finalize(const float *partials, int n_blocks, int count, const float *w_l2,
                  long long n_l2, float weight_decay, float *out4, void *stream);

/* --- Adam (src/optim.cu:42-95; hpdga optim.cpp:23-35) ---------------------------------- */
int pgcn_adam(float *w, const float *g, float *m, float *v, long long n, float step_size,
              float beta1, float beta2, float eps, float weight_decay, int decay, void *stream);
/* host: lr*sqrtf(1-powf(b2,t))/(1-powf(b1,t)) exactly as hpdga optim.cpp:24 */
float pgcn_adam_step_size(float lr, float beta1, float beta2, int t);

/* ===================================================================================== */
/* (2) Engine ABI                                                                          */
/* ===================================================================================== */

#define PGCN_MAX_LAYERS 16

/* GCNParams + AdamParams (include/gcn.cuh:40-47, include/optim.cuh:16-19) */
typedef struct {
  int num_nodes, input_dim, output_dim; /* filled by the loader */
  int n_layers;                          /* >= 2 */
  int hidden_dims[PGCN_MAX_LAYERS];      /* n_layers - 1 */
  float dropouts[PGCN_MAX_LAYERS];       /* n_layers */
  int epochs, early_stopping;
  float learning_rate, weight_decay, beta1, beta2, eps;
  /* 1: compute the output layer as (Â H) W instead of Â (H W) when hidden < classes, so its
   * GraphSum gathers hidden-width rows.  Exact algebra when Â is symmetric (checked at engine
   * build: a non-symmetric pattern keeps the reference's order); only the fp32 rounding order
   * differs from the reference.  0: the reference's module order. */
  int reassociate_last;
  /* PART2 `seed` (src/parser.cpp:234): 0 = hpdga's unseeded glibc rand() (init_rand_state,
   * hpdga rand.cpp:6-14); else the xorshift state is the first two rand() values after
   * srand(seed).  Glorot init and every dropout mask follow from it. */
  unsigned int seed;
} pgcn_params;

/* hpdga defaults: 2 layers, hidden 16, dropout .5/.5, 100 epochs, Adam lr .01, wd 5e-4,
 * reassociate_last = 1 */
void pgcn_params_default(pgcn_params *p);

/* GCNData in host memory (include/gcn.cuh:51-58): CSRs as the hpdga Parser builds them. */
typedef struct {
  int num_nodes;
  const int *graph_indptr, *graph_indices;            /* n+1, nnz */
  const int *feat_indptr, *feat_indices;              /* n+1, nnz_x */
  const float *feat_values;                           /* nnz_x */
  const int *label, *split;                           /* n, n */
} pgcn_data;

typedef struct pgcn_gcn pgcn_gcn;

/* GCN::GCN (include/gcn.cuh:79) on HIP device `device`. */
int pgcn_gcn_create(const pgcn_params *p, const pgcn_data *d, int device, pgcn_gcn **out);
/* Edge-cut variant: this process is rank `rank` of `world` (one process per GPU); the
 * graph is partitioned into contiguous nnz-balanced node ranges; GraphSum partials are
 * combined with RCCL reduce-scatter, weight grads and scalars with all-reduce.
 * `unique_id` = 128 bytes from pgcn_comm_unique_id on rank 0, shared by the caller. */
int pgcn_comm_unique_id(void *unique_id_128);
int pgcn_gcn_create_dist(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                         int world, const void *unique_id_128, pgcn_gcn **out);
/* Edge-cut variant over peer-mapped memory instead of RCCL (one process per GPU, DESIGN.md
 * §6): every rank's receive slots are mapped into every other rank with hipIpc handles, and a
 * GraphSum's partial sums travel as one-sided stores over xGMI straight from the kernel that
 * forms them into their owner's slot, summed there in rank order (deterministic).  `allgather`
 * is the caller's host channel (MPI_Allgather, torch.distributed, ...): the engine calls it
 * with every rank in the same order -- at creation (the handles; all ranks fail together with
 * PGCN_E_COMM if any cannot map its peers) and at destruction (a barrier before the regions are
 * unmapped and freed) -- and it must fill all[q * bytes, (q + 1) * bytes) with rank q's `mine`
 * and return 0.  A peer that never signals fails the next sync with PGCN_E_COMM after 20 s. */
typedef int (*pgcn_allgather_fn)(const void *mine, size_t bytes, void *all, void *user);
int pgcn_gcn_create_peer(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                         int world, pgcn_allgather_fn allgather, void *user, pgcn_gcn **out);
/* In-process ranks ("fake RCCL"): `world` edge-cut engines in ONE process on
 * one device, each created and driven by its own host thread (creation and destruction
 * rendezvous with the peers' same call).  Their collectives are pgcn_gcn_create_peer's
 * kernels over raw device pointers (the same pushes, flags and rank-order sums), so the
 * multi-rank engine (partition, peer exchange, global dropout offsets, weight all-reduce)
 * runs unchanged without RCCL.  The group may be destroyed after the engines are created
 * (they keep it alive). */
typedef struct pgcn_loopback pgcn_loopback;
int pgcn_loopback_create(int world, pgcn_loopback **out);
int pgcn_loopback_destroy(pgcn_loopback *group);
int pgcn_gcn_create_loopback(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                             pgcn_loopback *group, pgcn_gcn **out);
/* Diagnostics (timing only, tools/rank_epoch.py): rank `rank` of a `world`-rank edge-cut
 * engine with no peers -- its kernels and stream order, collectives reduced to this rank's
 * share ("comm" 3).  Its results are not the model's. */
int pgcn_debug_gcn_create_solo(const pgcn_params *p, const pgcn_data *d, int device, int rank,
                               int world, pgcn_gcn **out);
int pgcn_gcn_destroy(pgcn_gcn *g);
/* Engine facts: "world", "rank", "comm" (0 none, 1 RCCL, 2 loopback, 3 solo, 4 peer), "comm_calls" /
 * "comm_bytes" (collectives enqueued since creation and the bytes this rank sends in them,
 * ring algorithm: a reduce-scatter (W-1)/W of its send buffer, an all-reduce twice that), "reassociated",
 * "graph_symmetric", "graphsum_lds" (width-16 GraphSums take the LDS kernel), "epochs",
 * "eval_ax_us" (device time of the Â X precompute at engine build, µs; 0 when not used).
 * Returns the value (>= 0) or PGCN_E_INVALID for an unknown key. */
long long pgcn_gcn_query(pgcn_gcn *g, const char *key);
/* GCN::train_epoch / GCN::eval (src/gcn.cu:293-343): out2 = {loss, accuracy} */
int pgcn_gcn_train_epoch(pgcn_gcn *g, float out2[2]);
int pgcn_gcn_eval(pgcn_gcn *g, int split, float out2[2]);
/* One "epoch" as the reference times it (train_epoch + eval(2)) without a host sync;
 * results land in an on-device ring read by pgcn_gcn_results. */
int pgcn_gcn_epoch_async(pgcn_gcn *g);
int pgcn_gcn_sync(pgcn_gcn *g);
/* copies the last min(n, epochs run, 1024) epoch results {train_loss, train_acc, val_loss,
 * val_acc}, oldest first; returns the number of rows copied (>= 0) or a status (< 0) */
int pgcn_gcn_results(pgcn_gcn *g, int n, float *host_out);
/* GCN::run (src/gcn.cu:347-436): prints the reference's epoch lines when verbose */
int pgcn_gcn_run(pgcn_gcn *g, int verbose);
/* Variables in reference order (input, then per layer var1, weight, var2; see
 * include/gcn.cuh:85). which: 0 data, 1 grad. Returns element count (>= 0) or status. For
 * the edge-cut engine node-sized variables cover this rank's rows only.  PGCN_E_INVALID for
 * the output layer's node variables after a forward with the diagnostic row restriction
 * ("split_rows" on): their rows outside the split are stale. */
long long pgcn_gcn_get_var(pgcn_gcn *g, int idx, int which, float *host_dst);
int pgcn_gcn_num_vars(pgcn_gcn *g);
/* per-call device timing of the GraphSum kernels (enable before the timed region) */
int pgcn_gcn_profile(pgcn_gcn *g, int enable);
int pgcn_gcn_profile_read(pgcn_gcn *g, double *graphsum_ms_total, long long *graphsum_calls,
                          double *graphsum_bytes_total);
/* The same for the XW contractions on the MFMA kernels (dense X W1 / its weight gradient,
 * H W / its two gradients): summed event time, launches, 2*M*N*K flops. */
int pgcn_gcn_profile_read_mm(pgcn_gcn *g, double *ms_total, long long *calls,
                             double *flops_total);
/* this rank's node range [first, last) (edge-cut engine; whole graph otherwise) */
int pgcn_gcn_node_range(pgcn_gcn *g, int *first, int *last);

/* --- data (kept hpdga loader + synthetic inputs) ---------------------------------------- */
typedef struct pgcn_dataset pgcn_dataset;
/* Parser(GCNParams*, GCNData*, name).parse(): reads data/<name>.{graph,split,svmlight}
 * under `root` with hpdga-spring23/src/parser.cpp:6-140 semantics. */
int pgcn_dataset_load(const char *root, const char *name, pgcn_dataset **out);
/* The same load through the binary cache <root>/data/<name>.pgcnbin:
 * read when its recorded size + mtime of the three text files match, else the text is parsed
 * (identical arrays) and the cache rewritten, best effort.  *from_cache (may be NULL) = 1 on a
 * cache hit.  Errors as pgcn_dataset_load. */
int pgcn_dataset_load_cached(const char *root, const char *name, pgcn_dataset **out,
                             int *from_cache);
/* Write / read the parsed arrays as one binary file (any dataset, synthetic ones included).
 * PGCN_E_IO on a write failure or an invalid / truncated / corrupted file. */
int pgcn_dataset_save(const pgcn_dataset *ds, const char *path);
/* PART2 NO_FEATURE (src/parser.cpp:100-104): every feature value of `ds` becomes 1.0 (the
 * feature ids stay, so input_dim is unchanged). */
int pgcn_dataset_binarize(pgcn_dataset *ds);
int pgcn_dataset_load_binary(const char *path, pgcn_dataset **out);
/* Seeded reddit-shaped synthetic: n nodes, f dense features, c classes,
 * Chung-Lu power-law undirected graph with `undirected_edges` edges (2x directed slots). */
int pgcn_dataset_synthetic(int n, int f, int c, long long undirected_edges, uint64_t seed,
                           pgcn_dataset **out);
int pgcn_dataset_view(const pgcn_dataset *ds, pgcn_data *view, int *input_dim, int *output_dim);
int pgcn_dataset_free(pgcn_dataset *ds);

/* --- edge-cut partition plan (host only; no device needed) ------------------------------ */
/* contiguous nnz-balanced node ranges: bounds_out[world+1], padded rows per rank */
int pgcn_partition_bounds(int n, const int *indptr, int world, int *bounds_out, int *maxrows);
/* rank's column block of Â in padded row layout (world*maxrows rows, local column ids,
 * global coefficients). Returns nnz (call with null arrays to size them) or a status < 0. */
long long pgcn_partition_subgraph(int n, const int *indptr, const int *indices, int world,
                                  int rank, int *sub_indptr, int *sub_indices, float *sub_vals);

/* --- diagnostics (profiling ablations; not for production use) ------------------------ */
/* The edge-cut engine's GraphSum graph of rank `rank`, reduce-scatter chunk `chunk` of
 * `chunks` at `world` ranks (rows world*maxrows/chunks, columns = the rank's nodes, global
 * coefficients and scales), as GCN builds it: times the per-rank GraphSum of an N-GPU run on
 * one GPU.  *rows / *cols give its shape. */
int pgcn_debug_rank_graph(int n, const int *indptr, const int *indices, int world, int rank,
                          int chunks, int chunk, pgcn_graph **out, int *rows, int *cols);
/* Engine options (process-wide; most are read when an engine is built).  Each selects between
 * bit-identical or oracle-tested forms of the same reference epoch (19 keys, r05):
 *   "train_ahead" 0/1, "eval_ax" 0/1, "split_cols" 0/1, "epoch_graph" 0/1, "mm_side" 0/1/2,
 *   "eval_tail" 0/1 (edge-cut between processes: the eval pass's last exchange and output
 *   layer beside the next epoch's first kernels, default 0),
 *   "fuse_epilogue" bits 1 tails | 2 prestaged tables | 4 X-stream epilogue | 8 Dropout /
 *   ReLU backward in a Matmul's input-grad product (default 15),
 *   "fuse_output" 0..3 (default 2), "xstream_ring" 0/1, "lds_min_kb" (< 0: default),
 *   "lds_blocks" 0 (by shape) or 1..32, "parse_threads" (0: up to 16),
 *   "co_draw" 0/1 (sparse X: the hidden dropout's mask drawn in the input dropout's launch,
 *   default 1), "sparse_dual" 0/1 (sparse X: eval's first-layer product also computes the next
 *   training forward's, default 1), "gs_split" 0..3 (the plain GraphSum's rows longer than one
 *   work item on graphs of <= 2^20 slots: 0 a combine launch, 1 the row's last item sums the
 *   slots, 2 long rows as one item, 3 (default) rows of up to 8 workgroup iterations summed
 *   by one workgroup, longer ones as 1), "gs_item_iters" 0/2/4/8/16/32 (group iterations per
 *   work item there; 0 (default): by shape, the shortest leaving <= 1,536 workgroup items),
 *   "gs_orig_cols" 0/1 (a column subset's plain GraphSum gathers through the original column
 *   ids instead of compacting its input, default 1), "gs16_gather" 0..2 (the blocked d = 16
 *   gather kernel: 0 (default) by mean segment length, 1 k_graphsum16, 2 interleaved slots);
 *   r06 (30 keys): "co_draw" also 2 (dense X too, the default), "tn_fold" 0/1 (one GPU and
 *   edge-cut ranks between processes: the weight gradients' last reduction pass inside the
 *   Adam launch / the all-reduce push, default 1), "fuse_finish" 0..2 (one GPU, <= 512 loss
 *   blocks: the loss kernel's last block finishes the pass's scalars, default 1; 2: above 512
 *   blocks too, two levels of arrivals), "mask_per"
 *   0..2 (64-draw mask words per stored RNG state; default 0: 2 for masks of >= 2^20 words,
 *   else 1), "csc_tree" 0/1 (sparse X's
 *   W1.grad as a fixed tree over each feature's entries; default 0: the reference's sequential
 *   order, bit-exact; the tree measured slower), "mask_adam" 0/1 (one GPU: the next epoch's
 *   input mask drawn by the Adam launch, default 1, bit-identical), "mask_xstream" 0/1 (dense X, eval_ax: that mask drawn by
 *   two extra waves of eval's first-layer X-stream pass instead, bit-identical, default 0:
 *   measured slower), "reassoc_small" 0/1 (graphs
 *   under 65,536 nodes: the output layer as (A H) W with its Matmul in the loss kernel even when
 *   the classes are no more than the last hidden width <= 16, default 1; fp32 order only),
 *   "defer_wgrad" 0/1 (one GPU, <= 128 loss blocks: the output layer's W.grad block partials
 *   summed by the Adam launch, default 1; another grouping of the same sums), "peer_uncached" 0/1 (the peer
 *   exchange's receive slots in uncached memory, default 0), and the ring GraphSum's schedule
 *   shapes "ring_pair" 0/1 and "ring_window" 0/2/3 (0: the default window 3), both measured
 *   slower and off;
 * and one diagnostic, not reference-equivalent: "split_rows" 0/1 (the output layer's forward
 *   over the current split's rows only: stale logits elsewhere, which get_var refuses).
 * Returns PGCN_E_INVALID on an unknown key or on a value outside the key's range (nothing is
 * changed then). */
int pgcn_debug_set(const char *key, int value);
/* Host-only check of the d = 16 LDS ring schedule (window must be 5) of a CSR pattern: builds
 * it, walks it as k_graphsum_ring consumes it over a seeded input and returns the max relative
 * error of the row sums against a direct CSR sum, and the number of 4-step entry blocks. */
int pgcn_debug_lds_check(int n_rows, int n_cols, const int *indptr, const int *indices,
                         int window, double *max_rel_err, long long *n_blocks);
/* Host-only: the same schedule's per-(workgroup, slice, wave, slot) step counts (uint16, up to
 * cap) and its shape {n_batches, t_max, waves, slots, window}; returns the count or -1. */
long long pgcn_debug_lds_counts(int n_rows, int n_cols, const int *indptr, const int *indices,
                                int window, unsigned short *dst, long long cap, int *shape5);
/* Launch counts of the engine's kernel families since the last reset (process-wide), so a test
 * can assert which kernels a configuration took: "xs_nn_ring" / "xs_tn_ring" (loader + MFMA-wave
 * X-stream kernels), "xs_nn" / "xs_tn" (register-streamed X-stream kernels), "gs_ring" (LDS ring
 * GraphSum), "gs_gather" (gather GraphSum), "out_xent" (output layer fused into the loss),
 * "gemm_nn" / "gemm_tn" (general MFMA GEMMs), "launches" (every kernel launch of the library).
 * A non-null name returns its count (then zeroes it
 * when reset bit 0 is set); a null name with reset bit 0 zeroes every counter.  Bit 1 of reset
 * selects the counters of the calling host thread instead of the process-wide ones (each rank
 * of an in-process loopback group runs on a thread of its own).  Status < 0 on an unknown
 * name. */
long long pgcn_debug_path_count(const char *name, int reset);
/* n empty kernels back to back on `stream` (the per-launch floor the small graphs' epochs are
 * compared with: launches per epoch x the time of one empty launch). */
int pgcn_debug_empty_launches(int n, void *stream);
/* mine[i] = the loss kernel's exp of x[i] (x <= 0: the device expf sequence without its
 * overflow select), lib[i] = the device library's expf(x[i]); device pointers */
int pgcn_debug_exp_check(const float *x, long long n, float *mine, float *lib, void *stream);
/* q[i] = the loss kernel's quotient a[i] / b[i] (div_rn: from the reciprocal of b[i], the IEEE
 * division below 2^-125); device pointers */
int pgcn_debug_div_check(const float *a, const float *b, long long n, float *q, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PGCN_H */
