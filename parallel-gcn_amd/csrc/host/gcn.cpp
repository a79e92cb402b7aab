// parallel-gcn_amd/csrc/host/gcn.cpp
#include "gcn.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "../kernels.hpp"
#include "../rng.hpp"

namespace pgcn {

// "train_ahead" (pgcn_debug_set, read at engine build): eval's first-layer forward also
// computes the next training forward's product (SparseMatmul, one pass over dense X)
int g_train_ahead = 1;
// "eval_ax" (read at engine build): eval's first layer as (Â X) W1 from Â X computed once
// (Â and X are constants: exact algebra, fp32 rounding order differs)
int g_eval_ax = 1;
// "epoch_graph" (read per epoch_async): replay a captured per-epoch hipGraph when eligible;
int g_epoch_graph = 0;  // measured no faster than eager launches (r01: GPU-bound epochs)
// "split_rows" (read at each split switch): the output layer's GraphSum forward computes only
// the current split's labelled rows.  Off by default: the reference's forward produces the
// logits of every row, and so does the default engine (r02); on, rows outside the split keep
// stale logits (get_var refuses them)
int g_split_rows = 0;
// "split_cols" (read at each split switch): the output layer's GraphSum backward keeps only the
// edges from the training split's columns.  The loss gradient is exactly zero on every other
// row, so the skipped terms are exact zeros: in.grad is the full gradient of every row
int g_split_cols = 1;
// "fuse_epilogue" (read at engine build), bits, all bit-identical to separate launches:
//   1 (kFuseTails)    the ReLU / Dropout modules next to a GraphSum run in its final-write
//                     epilogue (gs_epilogue.hpp);
//   2 (kFusePrestage) ... and that epilogue also writes the next GraphSum's prescaled input
//                     table, which then skips its prescale launch;
//   4 (kFuseXstream)  the first layer's X-stream product applies the eval ReLU / writes the
//                     first GraphSum's table;
//   8 (kFuseMatmulTails) the Dropout / ReLU backward before a Matmul run in its input-grad
//                     product's final write (k_xstream_nn: outputs of <= 16 columns; the
//                     small graphs' second layer -- two launches fewer per epoch).
int g_fuse_epilogue = kFuseTails | kFusePrestage | kFuseXstream | kFuseMatmulTails;
// "fuse_output" (read at engine build): 0 = separate Matmul + loss; 1 = the output layer's
// Matmul forward and input grad run inside the loss (launch_out_xent) when the Matmul produces
// the logits (the reassociated order: GraphSum, then Matmul) from at most 16 columns
// (bit-identical); 2 (default) = ... and its weight grad's block partials on graphs of >=
// 65,536 rows or on an edge-cut rank (the same sums in another grouping); 3 = ... on any graph
int g_fuse_output = 2;
// "co_draw" (read at engine build): the hidden dropout's mask drawn in the input dropout's
// launch (1: sparse X; 2: dense X too; bit-identical)
int g_co_draw = 2;
// "fuse_finish" (read per pass): one GPU, the loss kernel's last block sums the pass's
// scalars and writes its results ring slot (XentFinal; one launch fewer per pass): 1 (default)
// up to kFinishMaxBlocks loss blocks, 2 also above them with two levels of arrivals (reddit:
// measured even, 615.2-616.0 vs 615.4 epochs/s -- the loss kernels' tails grew by what the
// reduce launches cost, profiles/r06/x)
int g_fuse_finish = 1;
// "mask_adam" (read per epoch): one GPU, the next input mask drawn by the Adam launch
int g_mask_adam = 1;
// "mask_xstream" (read per epoch): dense X with eval_ax, one GPU -- the next input mask drawn
// by eval's first-layer X-stream pass instead (GCN::mask_in_eval).  Off: bit-identical but
// slower -- two drawing waves per CU (all the VGPR budget leaves beside the consumers) take
// 202 us for what k_dropout_mask's 32 waves per CU draw in 63, so the pass doubles (reddit
// 604-605 vs 617-619 epochs/s, profiles/r06/z2)
int g_mask_xstream = 0;
constexpr int kFinishMaxBlocks = 512, kFinishGroup = 64;
// "tn_fold" (read per epoch): one GPU, the weight gradients' last reduction pass runs inside
// the Adam launch (GCN::backward_pass; bit-identical)
int g_tn_fold = 1;
// "sparse_dual" (read per eval forward): sparse X with train_ahead: eval's first-layer product
// also computes the next training forward's (k_spmm_csr<true>, one pass; bit-identical)
int g_sparse_dual = 1;
// "mm_side" (read at engine build): Matmul weight gradients on the side stream (ModuleContext)
// on graphs of at least kMmSideRows rows; 2 = on every graph.  Off: r02 A/B on reddit-114M,
// three runs each, 486.5 (on) vs 487.4 (off) epochs/s -- the LDS GraphSum holds every CU with
// one workgroup, so the side kernels find no room to overlap; cora 5,957 vs 7,136 (the
// stream hand-offs cost more than the ~7 us of kernels they hide)
int g_mm_side = 0;
constexpr int kMmSideRows = 65536;
// "reassoc_small" (read at engine build): on graphs of fewer than kMmSideRows nodes the output
// layer runs in the reassociated order (Â H) W even when the classes are no more than the last
// hidden width (<= 16), so its Matmul runs inside the loss kernel: a small graph's epoch is
// bound by its launches, not by the GraphSum's width (the fp32 order differs, like reddit's)
int g_reassoc_small = 1;
// "eval_tail" (read at engine build): the edge-cut eval pass's last exchange and output layer
// on the (high-priority) comm stream beside the next epoch's mask draw and first-layer product
// (ModuleContext::tail_stream; peer exchange between processes only; bit-identical).  Off: on
// the solo timing form, where the push has no link time to hide, the overlapped kernels slow
// each other -- W = 8 rank epoch 0.511-0.514 vs 0.489-0.495 ms (0.502-0.506 on the low-priority
// side stream; profiles/r05/s).  An 8-GPU run with slow links may still gain (the eval push's
// link time beside ~48 us of compute): `bench.py --knob eval_tail=1`
int g_eval_tail = 0;

// ------------------------------------------------------------------------------------------
// Adam (src/optim.cu:7-95; hpdga optim.cpp:16-35)
// ------------------------------------------------------------------------------------------
Adam::Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
           const AdamParams &p)
    : params(p) {
  PGCN_CHECK(weights.size() == decays.size(), PGCN_E_INVALID,
             "Adam: weights and decays must have the same size");
  for (size_t i = 0; i < weights.size(); i++) {
    Var v;
    v.w = weights[i];
    v.m.allocate((size_t)v.w->size);
    v.v.allocate((size_t)v.w->size);
    v.m.zero();
    v.v.zero();
    v.decay = decays[i];
    vars.push_back(std::move(v));
  }
}

float Adam::step_size(int t) const {
  // hpdga optim.cpp:24, host float arithmetic with glibc powf/sqrtf
  return params.learning_rate * sqrtf(1.0f - powf(params.beta2, (float)t)) /
         (1.0f - powf(params.beta1, (float)t));
}

void Adam::step(const Stream &s, TnDeferList *defer, const PeerRecv *peer, const float *arena,
                const MaskDraw *draws, int n_draws, const void *table) {
  step_count++;
  launch(s, step_size(step_count), nullptr, nullptr, 1, defer, peer, arena, draws, n_draws, table);
}

void Adam::step_each(const std::vector<hipStream_t> &streams,
                     const std::vector<hipEvent_t> &events) {
  PGCN_CHECK(streams.size() == vars.size() && events.size() == vars.size(), PGCN_E_INVALID,
             "Adam: one stream and one event per weight");
  step_count++;
  const float st = step_size(step_count);
  for (size_t i = 0; i < vars.size(); i++) {
    const Var &v = vars[i];
    launch_adam(v.w->dev_data.get(), v.w->dev_grad.get(), v.m.get(), v.v.get(), v.w->size, st,
                params.beta1, params.beta2, params.eps, params.weight_decay, v.decay ? 1 : 0,
                streams[i]);
    if (events[i]) PGCN_HIP(hipEventRecord(events[i], streams[i]));
  }
}

void Adam::step_graph(const Stream &s, const float *table, const int *ctr, int cap,
                      TnDeferList *defer, const PeerRecv *peer, const float *arena) const {
  launch(s, 0.0f, table, ctr, cap, defer, peer, arena);
}

// every weight in one launch when they fit one AdamBatch (the 2-layer model: W1 and W2); a
// deferred reduction pass that writes a tensor's whole gradient runs inside it (tn_defer)
void Adam::launch(const Stream &s, float st, const float *table, const int *ctr, int cap,
                  TnDeferList *defer, const PeerRecv *peer, const float *arena,
                  const MaskDraw *draws, int n_draws, const void *jump_table) const {
  PGCN_CHECK(!peer || (arena && vars.size() <= (size_t)kAdamBatch), PGCN_E_INVALID,
             "Adam: the all-reduce's received slots need the gradient arena and one batch");
  PGCN_CHECK(n_draws == 0 || (vars.size() <= (size_t)kAdamBatch && !peer && !table),
             PGCN_E_INVALID, "Adam: masks only in an eager one-batch step");
  if (vars.size() <= (size_t)kAdamBatch) {
    AdamBatch b{};
    if (peer) b.peer = *peer;
    for (const auto &v : vars) {
      b.w[b.count] = v.w->dev_data.get();
      b.g[b.count] = v.w->dev_grad.get();
      b.m[b.count] = v.m.get();
      b.v[b.count] = v.v.get();
      b.n[b.count] = v.w->size;
      b.decay[b.count] = v.decay ? 1 : 0;
      if (peer) b.arena_off[b.count] = v.w->dev_grad.get() - arena;
      for (int i = 0; defer && i < defer->n; i++) {
        TnDeferred &d = defer->d[i];
        if (d.src && d.C == v.w->dev_grad.get() && (long long)d.K * d.N == v.w->size) {
          b.red[b.count] = d;
          d.src = nullptr;  // taken
        }
      }
      b.count++;
    }
    if (defer) tn_defer_flush(*defer, s.get());  // passes no tensor took: before the update
    launch_adam_multi(b, st, params.beta1, params.beta2, params.eps, params.weight_decay, s.get(),
                      table, ctr, cap, draws, n_draws, jump_table);
    return;
  }
  if (defer) tn_defer_flush(*defer, s.get());
  for (auto &v : vars)
    launch_adam(v.w->dev_data.get(), v.w->dev_grad.get(), v.m.get(), v.v.get(), v.w->size, st,
                params.beta1, params.beta2, params.eps, params.weight_decay, v.decay ? 1 : 0,
                s.get(), table, ctr, cap);
}

// ------------------------------------------------------------------------------------------
// GCN
// ------------------------------------------------------------------------------------------
namespace {
// hpdga variable.cpp:15-19 (glorot), drawing from the shared xorshift state
void glorot_host(std::vector<float> &w, int in_size, int out_size, uint64_t s[2]) {
  const float range = sqrtf(6.0f / (float)(in_size + out_size));
  for (auto &x : w) {
    const float r = (float)xs_next(s) / (float)0x7fffffff;
    x = (float)((((double)r - 0.5) * (double)range) * 2.0);
  }
}
}  // namespace

// hpdga variable.cpp:15-19 (glorot) from the shared xorshift state (GCN and the C++ API)
void glorot_fill(std::vector<float> &w, int in_size, int out_size, uint64_t s[2]) {
  glorot_host(w, in_size, out_size, s);
}

// X on the device for rows [first, first + rows) of a CSR feature matrix (GCN::upload_features;
// also the public C++ API's SparseMatmul).  dense: [rows][round_up4(F)] fp32 + the X-stream
// nibble-mask buffer when hidden0 fits the X-stream kernels; sparse: CSR + transposed index.
void build_dev_features(DevFeatures &feats, const int *fptr, const int *indices,
                        const float *values, int first, int rows, int F, bool dense, int hidden0) {
  feats.rows = rows;
  feats.cols = F;
  feats.dense = dense;
  const long long p0 = fptr[(size_t)first], p1 = fptr[(size_t)first + rows];
  feats.nnz = p1 - p0;
  if (feats.dense) {
    feats.ldx = round_up4(F);
    std::vector<float> x((size_t)rows * feats.ldx, 0.0f);
    parallel_for(rows, [&](long long b, long long e) {
      for (long long i = b; i < e; i++)
        std::memcpy(&x[(size_t)i * feats.ldx], &values[(size_t)(first + i) * F],
                    sizeof(float) * (size_t)F);
    });
    feats.x.allocate(x.size() + 4);
    feats.x.upload(x);
    if (xstream_ok(hidden0, F)) {
      feats.maskT.allocate((size_t)std::max(rows, 1) * 16);
      feats.maskT.zero();
    } else if (gemm_wide_ok(std::min(hidden0, 128)) && F <= 1024) {
      feats.maskW.allocate((size_t)std::max(rows, 1) * 16);
      feats.maskW.zero();
    }
  } else {
    std::vector<int> ip((size_t)rows + 1);
    for (int i = 0; i <= rows; i++) ip[(size_t)i] = (int)(fptr[(size_t)first + i] - p0);
    const int *idx = indices + p0;
    feats.host_values.assign(values + p0, values + p1);
    // transposed index for the weight gradient: stable counting sort by feature id
    std::vector<int> cptr((size_t)F + 1, 0), crow((size_t)feats.nnz), cpos((size_t)feats.nnz);
    for (long long k = 0; k < feats.nnz; k++) {
      PGCN_CHECK(idx[k] >= 0 && idx[k] < F, PGCN_E_INVALID, "feature id out of range");
      cptr[(size_t)idx[k] + 1]++;
    }
    for (int f = 0; f < F; f++) cptr[(size_t)f + 1] += cptr[(size_t)f];
    std::vector<int> fill(cptr.begin(), cptr.end() - 1);
    for (int i = 0; i < rows; i++)
      for (int k = ip[(size_t)i]; k < ip[(size_t)i + 1]; k++) {
        const int o = fill[(size_t)idx[k]]++;
        crow[(size_t)o] = i;
        cpos[(size_t)o] = k;
      }
    feats.indptr.allocate(ip.size());
    feats.indptr.upload(ip);
    feats.indices.allocate((size_t)feats.nnz + 1);
    feats.indices.upload(idx, (size_t)feats.nnz);
    feats.values.allocate((size_t)feats.nnz + 1);
    feats.values.upload(feats.host_values);
    feats.csc_ptr.allocate(cptr.size());
    feats.csc_ptr.upload(cptr);
    feats.csc_row.allocate(crow.size() + 1);
    feats.csc_row.upload(crow);
    feats.csc_pos.allocate(cpos.size() + 1);
    feats.csc_pos.upload(cpos);
    // the weight-gradient pass's workgroups in descending column length: a column is one
    // serial chain, so the longest ones start first and the short ones fill in around them
    std::vector<int> order((size_t)F);
    for (int f = 0; f < F; f++) order[(size_t)f] = f;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      return cptr[(size_t)a + 1] - cptr[(size_t)a] > cptr[(size_t)b + 1] - cptr[(size_t)b];
    });
    feats.csc_order.allocate(order.size() + 1);
    feats.csc_order.upload(order);
  }
}

// Chunk states of a dropout over global elements [elem_begin, elem_end) whose first training
// forward draws stream positions offset + element (hpdga: one xorshift128+ draw per element,
// module.cpp:208-219), each 64-element chunk's state jumped to from the seed state.
// "mask_per" (read at engine build): 64-draw mask words per stored RNG state (1 or 2); 0 = by
// size: 2 from kMaskPer2Chunks words on (reddit's input mask: half the period jumps, 68.3 ->
// 65.2 us for both masks), else 1 (a W = 8 rank's input mask, 274 k words: twice the threads,
// each chain half as long -- 17.3 -> 14.5 us, profiles/r06/o)
int g_mask_per = 0;
constexpr long long kMaskPer2Chunks = 1LL << 20;

void init_dropout_rng_range(DropoutRng &r, const uint64_t seed[2], unsigned long long offset,
                            long long elem_begin, long long elem_end) {
  r.elem_begin = elem_begin;
  r.elem_end = elem_end;
  r.chunk_lo = r.elem_begin / kDropChunk;
  const long long chunk_hi = ceil_div(r.elem_end, kDropChunk);
  r.n_chunks = std::max(0LL, chunk_hi - r.chunk_lo);
  r.per = g_mask_per ? g_mask_per : (r.n_chunks >= kMaskPer2Chunks ? 2 : 1);
  r.mask_base = r.elem_begin - kDropChunk * r.chunk_lo;
  // one state per r.per mask words: the stream's state at the first draw of words per * k
  const long long n_states = ceil_div(r.n_chunks, (long long)r.per);
  const int span = kDropChunk * r.per;
  std::vector<uint64_t> st((size_t)std::max(1LL, n_states) * 2, 0);
  const unsigned long long base = offset + (unsigned long long)kDropChunk * r.chunk_lo;
  parallel_for(n_states, [&](long long b, long long e) {
    uint64_t s[2] = {seed[0], seed[1]};
    xs_jump(s, base + (unsigned long long)span * b);
    for (long long c = b; c < e; c++) {
      st[(size_t)c * 2] = s[0];
      st[(size_t)c * 2 + 1] = s[1];
      for (int k = 0; k < span; k++) xs_advance(s);
    }
  });
  r.states.allocate(st.size());
  r.states.upload(st);
  // (+1, rounded up to an even count: the X-stream ring kernels stage the bitmap in 16-B pieces)
  r.mask.allocate(((size_t)std::max(1LL, r.n_chunks) + 2) & ~(size_t)1);
  r.mask.zero();
}

GCN::GCN(const GCNParams &params_, const AdamParams &adam, const GCNData &data, int device_,
         const DistSpec *dist)
    : params(params_), adam_params(adam), device(device_) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    throw Error(PGCN_E_NODEVICE, "no HIP device visible: the engine has no CPU fallback");
  PGCN_CHECK(device >= 0 && device < ndev, PGCN_E_INVALID, "bad device index");
  PGCN_HIP(hipSetDevice(device));
  L = params.n_layers;
  PGCN_CHECK(L >= 2 && L <= PGCN_MAX_LAYERS, PGCN_E_INVALID, "n_layers must be in [2,16]");
  PGCN_CHECK((int)params.hidden_dims.size() == L - 1, PGCN_E_INVALID,
             "Number of hidden dimensions must be 1 - n_layers");
  PGCN_CHECK((int)params.dropouts.size() == L, PGCN_E_INVALID,
             "Number of dropouts must match number of layers");
  for (int h : params.hidden_dims)
    PGCN_CHECK(h > 0 && h % 4 == 0 && h <= 4096, PGCN_E_INVALID,
               "hidden dims must be multiples of 4 in [4,4096]");
  PGCN_CHECK(params.output_dim >= 1 && params.output_dim <= 128, PGCN_E_INVALID,
             "output_dim must be in [1,128]");
  PGCN_CHECK(data.num_nodes == params.num_nodes, PGCN_E_INVALID, "num_nodes mismatch");
  int lo_prio = 0, hi_prio = 0;
  PGCN_HIP(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
  stream = Stream::create(hi_prio);  // the reference uses High priority streams
  // side stream: weight gradients beside the rest of the backward pass (mm_side)
  side_stream = Stream::create(lo_prio);
  ctx.side_stream = side_stream.get();
  const int world = dist ? dist->world : 1, rank = dist ? dist->rank : 0;
  // one row chunk on one rank: nothing to exchange, nothing to overlap
  part = make_partition(params.num_nodes, data.graph.indptr.data(), world, rank,
                        1);
  if (dist) {  // the edge-cut path (also at world == 1, which exercises it on one GPU)
    if (dist->loopback || dist->allgather || dist->solo) {
      // peer-mapped slots sized for the largest collective: a GraphSum's rows of one owner at
      // the widest row, the weight-gradient all-reduce, Â X's 16-column reduce-scatters
      size_t ld = 16;
      for (int h : params.hidden_dims) ld = std::max(ld, (size_t)round_up4(h));
      ld = std::max(ld, (size_t)round_up4(params.output_dim));
      long long wtotal = 0;
      for (int l = 0; l < L; l++) {
        const int a = l == 0 ? params.input_dim : params.hidden_dims[(size_t)l - 1];
        const int b = l == L - 1 ? params.output_dim : params.hidden_dims[(size_t)l];
        wtotal += (long long)a * b;
      }
      const size_t cap = std::max((size_t)part.maxrows * ld, (size_t)wtotal);
      if (dist->solo) {  // timing only: every peer is this rank (PeerComm's solo form)
        comm = std::make_unique<PeerComm>(rank, world, cap, nullptr, false, nullptr, true);
      } else if (dist->loopback) {
        auto grp = dist->loopback;
        comm = std::make_unique<PeerComm>(
            rank, world, cap,
            [grp, rank](const void *m, size_t b, void *all) { grp->allgather(rank, m, b, all); },
            false, [grp, rank] { grp->barrier(rank); });
      } else {
        comm = std::make_unique<PeerComm>(rank, world, cap, dist->allgather, true);
      }
    } else {
      comm = std::make_unique<RcclComm>(rank, world, dist->unique_id);
    }
    ctx.comm = comm.get();
    comm_stream = Stream::create(hi_prio);
    ctx.comm_stream = comm_stream.get();
  }
  build(data);
}

GCN::~GCN() {
  if (stream.get()) (void)hipStreamSynchronize(stream.get());
  drop_epoch_graph();
  if (side_stream.get()) (void)hipStreamSynchronize(side_stream.get());
  if (comm_stream.get()) (void)hipStreamSynchronize(comm_stream.get());
}

void GCN::upload_features(const GCNData &data) {
  const auto &fptr = data.feature_index.indptr;
  feat_indptr_global = fptr;
  nnz_x_global = fptr[(size_t)params.num_nodes];
  build_dev_features(feats, fptr.data(), data.feature_index.indices.data(),
                     data.feature_value.data(), part.first(), part.local_rows(), params.input_dim,
                     features_dense(data), params.hidden_dims.front());
}

void GCN::init_dropout_rng(const GCNData &data, long long glorot_draws) {
  const int N = params.num_nodes, first = part.first(), last = part.last();
  std::vector<int> dims;
  dims.push_back(params.input_dim);
  for (int h : params.hidden_dims) dims.push_back(h);
  dims.push_back(params.output_dim);
  // draws per training epoch: the input dropout (nnz_X) then each hidden dropout (N*h_l)
  unsigned long long period = (unsigned long long)nnz_x_global;
  for (int l = 1; l < L; l++) period += (unsigned long long)N * dims[(size_t)l];
  std::vector<uint64_t> table(16 * 256 * 2);
  xs_byte_tables(xs_jump_matrix(period), table.data());
  jump_table.allocate(table.size() * sizeof(uint64_t));
  jump_table.upload(reinterpret_cast<const uint8_t *>(table.data()), table.size() * sizeof(uint64_t));
  ctx.jump_table = jump_table.get();
  mask_lut.allocate(32 * 16);
  launch_mask_lut(jump_table.get(), mask_lut.get(), stream.get());

  uint64_t seed[2];
  if (params.seed) pgcn_rng_seed_glibc(params.seed, seed);
  else pgcn_rng_seed(seed);
  unsigned long long offset = (unsigned long long)glorot_draws;
  for (int l = 0; l < L; l++) {
    auto r = std::make_shared<DropoutRng>();
    if (l == 0)
      init_dropout_rng_range(*r, seed, offset, data.feature_index.indptr[(size_t)first],
                             data.feature_index.indptr[(size_t)last]);
    else
      init_dropout_rng_range(*r, seed, offset, (long long)first * dims[(size_t)l],
                             (long long)last * dims[(size_t)l]);
    rngs.push_back(r);
    offset += (l == 0) ? (unsigned long long)nnz_x_global
                       : (unsigned long long)N * dims[(size_t)l];
  }
}

void GCN::build(const GCNData &data) {
  const int N = params.num_nodes;
  graph_symmetric = csr_symmetric(N, data.graph.indptr.data(), data.graph.indices.data());
  // adjacency
  if (comm) {
    // one column block per reduce-scatter chunk (rows in chunk-major padded order,
    // partition_subgraph_chunk); vals = s_row * s_col with s = 1/sqrt(global degree)
    const std::vector<float> sg = degree_scales(N, data.graph.indptr.data());
    const int h = part.chunk_rows();
    std::vector<float> cs((size_t)part.local_rows());
    for (int c = 0; c < part.local_rows(); c++) cs[(size_t)c] = sg[(size_t)part.first() + c];
    for (int k = 0; k < part.chunks; k++) {
      std::vector<int> sp, si;
      partition_subgraph_chunk(part, N, data.graph.indptr.data(), data.graph.indices.data(), k,
                               &sp, &si);
      std::vector<float> rs((size_t)part.world * h, 0.0f), sv(si.size());
      for (int q = 0; q < part.world; q++)
        for (int j = 0; j < h; j++) {
          const int i = part.bounds[(size_t)q] + k * h + j;
          if (i < part.bounds[(size_t)q + 1]) rs[(size_t)q * h + j] = sg[(size_t)i];
        }
      // the plain kernels' per-edge values: hpdga's coefficient (graph_coef), bit-exact
      const int *ip = data.graph.indptr.data();
      for (int q = 0; q < part.world; q++)
        for (int j = 0; j < h; j++) {
          const int i = part.bounds[(size_t)q] + k * h + j;
          if (i >= part.bounds[(size_t)q + 1]) continue;
          const size_t r = (size_t)q * h + j;
          for (int t = sp[r]; t < sp[r + 1]; t++) {
            const int gj = part.first() + si[(size_t)t];
            sv[(size_t)t] = graph_coef(ip[i + 1] - ip[i], ip[gj + 1] - ip[gj]);
          }
        }
      auto gk = std::make_unique<DevGraph>(part.world * h, part.local_rows(), sp.data(), si.data(),
                                           sv.data());
      gk->set_scales(std::move(rs), cs);
      chunk_graphs.push_back(std::move(gk));
    }
    // the chunks' columns are this rank's rows: one prescaled table serves them all
    for (size_t k = 1; k < chunk_graphs.size(); k++) chunk_graphs[k]->share_tables(chunk_graphs[0].get());
    for (auto &gk : chunk_graphs) ctx.chunk_graphs.push_back(gk.get());
    ctx.local_rows = part.local_rows();
  } else {
    std::vector<float> v = graph_coefs(N, data.graph.indptr.data(), data.graph.indices.data());
    graph = std::make_unique<DevGraph>(N, N, data.graph.indptr.data(), data.graph.indices.data(),
                                       v.data());
    const std::vector<float> sg = degree_scales(N, data.graph.indptr.data());
    graph->set_scales(sg, sg);
  }
  upload_features(data);
  // eval_ax (dense X): Â X's buffer now -- the modules built below read it -- and its sums at
  // the end of the build (build_eval_ax)
  if (g_eval_ax && feats.dense && feats.cols >= 16 && (comm || graph)) {
    feats.ax.allocate(feats.x.size());
    feats.ax.zero();
  }
  // truth per split for this rank's rows, padded with -1 (set_truth, src/gcn.cu:204-226)
  const int first = part.first(), rows = part.local_rows(), prow = part.maxrows;
  for (int s = 1; s <= 3; s++) {
    std::vector<int> t((size_t)prow, -1);
    for (int i = 0; i < rows; i++)
      t[(size_t)i] = data.split[(size_t)first + i] == s ? data.label[(size_t)first + i] : -1;
    truth[s].allocate(t.size());
    truth[s].upload(t);
    split_rows_host[s].clear();
    std::vector<int> tc;
    for (int i = 0; i < rows; i++)
      if (t[(size_t)i] >= 0) {
        split_rows_host[s].push_back(i);
        tc.push_back(t[(size_t)i]);
      }
    truth_compact[s].allocate(std::max<size_t>(tc.size(), 1));
    if (!tc.empty()) truth_compact[s].upload(tc);
    int c = 0;
    split_rows_global[s].clear();
    for (int i = 0; i < N; i++)
      if (data.split[(size_t)i] == s && data.label[(size_t)i] >= 0) {
        c++;
        if (comm) split_rows_global[s].push_back(i);  // edge-cut row restriction (set_split)
      }
    counts[s] = c;
  }
  // weights: glorot in layer order from the default seed (hpdga gcn.cpp:64-128)
  std::vector<int> dims;
  dims.push_back(params.input_dim);
  for (int h : params.hidden_dims) dims.push_back(h);
  dims.push_back(params.output_dim);
  long long wtotal = 0;
  for (int l = 0; l < L; l++) wtotal += (long long)dims[(size_t)l] * dims[(size_t)l + 1];
  grad_arena.allocate((size_t)wtotal);
  grad_arena.zero();
  uint64_t rs[2];
  if (params.seed) pgcn_rng_seed_glibc(params.seed, rs);
  else pgcn_rng_seed(rs);
  long long woff = 0;
  std::vector<std::vector<float>> winit;
  for (int l = 0; l < L; l++) {
    auto w = std::make_shared<Variable>(dims[(size_t)l], dims[(size_t)l + 1], false);
    std::vector<float> h((size_t)w->size);
    glorot_host(h, dims[(size_t)l], dims[(size_t)l + 1], rs);
    w->dev_data.upload(h);
    w->dev_grad = grad_arena.slice((size_t)woff, (size_t)w->size);
    woff += w->size;
    weights.push_back(w);
    decays.push_back(l == 0);
  }
  init_dropout_rng(data, wtotal);

  // context buffers
  xent_partials.allocate((size_t)xent_blocks(prow) * 2 + 2);
  sums.allocate(4);
  results_ring.allocate((size_t)ring_cap * 4);
  results_ring.zero();
  if (comm) {
    raw_ring.allocate((size_t)ring_cap * 8);
    raw_ring.zero();
  }
  pinned = PinnedBuffer<float>(8);
  size_t ws = 0;
  for (int l = 0; l < L; l++)
    ws = std::max(ws, gemm_tn_workspace(rows, dims[(size_t)l + 1], dims[(size_t)l]));
  // the fused loss kernel's per-block W.grad partials of the output layer (fuse_output >= 2)
  ws = std::max(ws, tn_reduce_blocks_workspace(xent_blocks(prow), 16, 48));
  gemm_ws.allocate(ws / sizeof(float) + 64);
  if (g_mm_side == 2 || (g_mm_side == 1 && rows >= kMmSideRows)) {
    // the side stream's Matmul weight gradients have a workspace of their own
    gemm_ws_side.allocate(ws / sizeof(float) + 64);
    ctx.mm_side = true;
    ctx.gemm_workspace_side = gemm_ws_side.get();
    ctx.mm_fork = Event::create();
    ctx.side_join = Event::create();
  }
  ctx.train_ahead = g_train_ahead != 0;
  ctx.xent_partials = xent_partials.get();
  ctx.xent_blocks = xent_blocks(prow);
  ctx.gemm_workspace = gemm_ws.get();
  ctx.gemm_workspace_bytes = gemm_ws.size() * sizeof(float);
  ctx.gs_events = &gs_events;
  ctx.gs_bytes = &gs_bytes;
  ctx.mm_events = &mm_events;
  ctx.mm_flops = &mm_flops;

  // layers (src/gcn.cu:146-177)
  variables.push_back(nullptr);  // "input": the features, kept in `feats`
  insert_first_layer();
  for (int l = 1; l < L - 1; l++)
    insert_layer(params.hidden_dims[(size_t)l - 1], params.hidden_dims[(size_t)l],
                 params.dropouts[(size_t)l], l);
  insert_last_layer();
  // (edge-cut: the tails run in k_gs_finish on the rank's rows after the reduce-scatter)
  if (g_fuse_epilogue & kFuseTails) fuse_epilogues();
  if (g_fuse_epilogue & kFuseMatmulTails) fuse_matmul_tails();
  if (g_co_draw && dropouts_.size() >= 2 && (g_co_draw == 2 || !feats.dense) && dropouts_[0] &&
      dropouts_[1])
    const_cast<Dropout *>(dropouts_[0])->co_draw = dropouts_[1];
  if (g_fuse_output) fuse_output_layer();
  optimizer = Adam(weights, decays, adam_params);
  prepare_graphs();
  build_eval_ax();
  // eval_tail: the peer exchange between processes (or the solo timing form) -- in-process
  // ranks may share hardware queues, where a wait on one rank's side stream could sit ahead
  // of the push it waits for
  const auto *pc = dynamic_cast<const PeerComm *>(comm.get());
  if (g_eval_tail && pc && !pc->host_ordered() && comm->world() > 1) {
    for (int i = 0; i < (int)modules.size(); i++)
      if (dynamic_cast<const GraphSum *>(modules[(size_t)i].get())) tail_gs = i;
    ctx.tail_fork = Event::create();
    ctx.tail_done = Event::create();
  }
  PGCN_HIP(hipDeviceSynchronize());
  if (comm) comm->host_barrier();  // every rank built: the first epoch's waits start together
}

// eval_ax's Â X, computed last in build(): the engine's only long GPU work before the first
// epoch then runs right before it (the GPU's clocks ramp up over its first ~30 ms of load after
// an idle spell, profiles/r05/ramp.json)
void GCN::build_eval_ax() {
  // eval_ax: Â X once (16 columns per d = 16 GraphSum; the last chunk overlaps the one
  // before it so it never reads past a row), single GPU, dense X (eval's (Â X) W1 runs on the
  // X-stream kernel for hidden <= 16, the MFMA GEMM for wider first layers)
  // (its device time is kept in ax_build_ms: bench.py amortises it over the reference's
  // 100-epoch run)
  Event ax0 = Event::create(true), ax1 = Event::create(true);
  if (feats.ax && !comm) {
    graph->prepare(16);  // the schedule's host build is set-up, not Â X's device time
    ax0.record(stream.get());
    for (int c0 = 0; c0 < feats.cols; c0 += 16) {
      const int c = std::min(c0, feats.ldx - 16);
      graph->graphsum(feats.x.get() + c, feats.ldx, feats.ax.get() + c, feats.ldx, 16, stream.get());
    }
    ax1.record(stream.get());
    stream.sync();
    PGCN_HIP(hipEventElapsedTime(&ax_build_ms, ax0.get(), ax1.get()));
  }
  // the same for the edge-cut engine: per 16-column chunk of X, every row chunk's partial
  // sums from this rank's columns reduce-scattered exactly as GraphSum::run does (this rank
  // receives its own rows), then placed into Â X's columns
  if (feats.ax && comm) {
    const int h = part.chunk_rows(), nk = (int)chunk_graphs.size();
    DeviceBuffer<float> partial((size_t)part.world * h * 16), own((size_t)nk * h * 16);
    for (auto &gk : chunk_graphs) gk->prepare(16);
    // the engine's first device collective follows seconds of per-rank host set-up: every rank
    // arrives first, so no rank's bounded wait (kPeerTimeoutTicks) starts far ahead of a peer
    comm->host_barrier();
    ax0.record(stream.get());
    for (int c0 = 0; c0 < feats.cols; c0 += 16) {
      const int c = std::min(c0, feats.ldx - 16);
      for (int k = 0; k < nk; k++) {
        chunk_graphs[(size_t)k]->graphsum(feats.x.get() + c, feats.ldx, partial.get(), 16, 16,
                                          stream.get());
        comm->reduce_scatter_sum(partial.get(), own.get() + (size_t)k * h * 16, (size_t)h * 16,
                                 stream.get());
      }
      PGCN_HIP(hipMemcpy2DAsync(feats.ax.get() + c, sizeof(float) * feats.ldx, own.get(),
                                sizeof(float) * 16, sizeof(float) * 16, (size_t)part.local_rows(),
                                hipMemcpyDeviceToDevice, stream.get()));
    }
    ax1.record(stream.get());
    stream.sync();
    PGCN_HIP(hipEventElapsedTime(&ax_build_ms, ax0.get(), ax1.get()));
  }
}

// Every graph an epoch sums over, and its LDS schedule, built now (host set-up) rather than
// at its first use: the training split's column subset used to be built inside the first
// epoch (~1.9 s of host work while the GPU idled)
void GCN::prepare_graphs() {
  for (int split = 1; split <= 2; split++) {
    set_split(split);
    for (const auto &m : modules) {
      const auto *gs = dynamic_cast<const GraphSum *>(m.get());
      if (!gs) continue;
      const int d = gs->width();
      for (DevGraph *g : {gs->forward_graph(), gs->backward_graph()})
        if (g) g->prepare(d);
      for (DevGraph *g : ctx.chunk_graphs) g->prepare(d);
      for (DevGraph *g : ctx.chunk_split_graphs) g->prepare(d);
      for (DevGraph *g : ctx.chunk_col_graphs) g->prepare(d);
    }
  }
  set_split(1);
}

void GCN::fuse_output_layer() {
  const size_t n = modules.size();
  if (n < 2) return;
  auto *ce = dynamic_cast<CrossEntropyLoss *>(modules[n - 1].get());
  auto *mm = dynamic_cast<Matmul *>(modules[n - 2].get());
  if (!ce || !mm || mm->output() != ce->input() || mm->inner() > 16 || mm->inner() < 1) return;
  if (ce->input()->ld > 116 || mm->input()->rows != ce->input()->rows) return;
  ce->fused = mm;
  mm->fused_forward = true;
  // the reassociated output layer: GraphSum -> Matmul -> loss, the GraphSum's backward reads
  // the Matmul's input grad, which the fused kernel writes
  auto *gs = n >= 3 ? dynamic_cast<GraphSum *>(modules[n - 3].get()) : nullptr;
  if (gs && gs->output() == mm->input()) ce->dh_reader = gs;
}

// GraphSum -> ReLU(out) [-> Dropout(out)] in the module list: the ReLU and the Dropout run in
// the GraphSum's epilogue (forward); Dropout(in) <- ReLU(in) <- GraphSum, i.e. the backward
// of a GraphSum followed by those of the Dropout and ReLU on its input: same (backward).
// Only where the element order of the variable is its storage order (ld == cols).
void GCN::fuse_epilogues() {
  const size_t n = modules.size();
  for (size_t i = 0; i < n; i++) {
    auto *gs = dynamic_cast<GraphSum *>(modules[i].get());
    if (!gs) continue;
    const Variable *out = gs->output(), *in = gs->input();
    if (i + 1 < n && out->ld == out->cols) {
      auto *relu = dynamic_cast<ReLU *>(modules[i + 1].get());
      if (relu && relu->variable() == out) {
        gs->fwd_relu = relu;
        auto *drop = i + 2 < n ? dynamic_cast<Dropout *>(modules[i + 2].get()) : nullptr;
        if (drop && drop->variable() == out) gs->fwd_drop = drop;
        fused_tails_++;
        // the next forward module reading `out` is a GraphSum (the reassociated output layer)
        const size_t k = i + (gs->fwd_drop ? 3 : 2);
        auto *next = k < n ? dynamic_cast<GraphSum *>(modules[k].get()) : nullptr;
        if (next && next->input() == out) gs->fwd_next = next;
      }
    }
    if (i >= 1 && in->ld == in->cols) {
      auto *drop = dynamic_cast<Dropout *>(modules[i - 1].get());
      const size_t ri = drop && drop->variable() == in ? i - 2 : i - 1;
      auto *relu = ri < n ? dynamic_cast<ReLU *>(modules[ri].get()) : nullptr;
      if (relu && relu->variable() == in) {
        gs->bwd_relu = relu;
        if (ri + 1 < i) gs->bwd_drop = drop;
        fused_tails_++;
        // the next backward after ReLU(in)'s is a GraphSum's whose output is `in`
        auto *next = ri >= 1 ? dynamic_cast<GraphSum *>(modules[ri - 1].get()) : nullptr;
        if (next && next->output() == in) gs->bwd_next = next;
      }
    }
  }
}

// ReLU(a) [-> Dropout(a)] -> Matmul(a, W): the backward of the Dropout and the ReLU follow the
// Matmul's, which applies them to a.grad as it writes it (Matmul::backward decides per call
// whether its product runs on the kernel that can).  Only where a's element order is its
// storage order, and not for a ReLU a GraphSum backward already applies.
void GCN::fuse_matmul_tails() {
  const size_t n = modules.size();
  for (size_t i = 1; i < n; i++) {
    auto *mm = dynamic_cast<Matmul *>(modules[i].get());
    if (!mm || mm->input()->ld != mm->input()->cols) continue;
    const Variable *a = mm->input(), *c = mm->output();
    if (!xstream_ok(a->cols, c->cols) || xstream_ring_ok(c->cols, c->ld)) continue;
    auto *drop = dynamic_cast<Dropout *>(modules[i - 1].get());
    if (drop && drop->variable() != a) drop = nullptr;
    const size_t ri = drop ? i - 2 : i - 1;
    auto *relu = ri < n ? dynamic_cast<ReLU *>(modules[ri].get()) : nullptr;
    if (!relu || relu->variable() != a) continue;
    bool taken = false;
    for (auto &m : modules) {
      auto *gs = dynamic_cast<GraphSum *>(m.get());
      if (gs && gs->bwd_relu == relu) taken = true;
    }
    if (taken) continue;
    mm->bwd_relu = relu;
    mm->bwd_drop = drop;
    fused_tails_++;
  }
}

// src/gcn.cu:47-81
void GCN::insert_first_layer() {
  const int prow = part.maxrows, h = params.hidden_dims.front();
  auto drop = std::make_unique<Dropout>(nullptr, params.dropouts.front(), rngs[0], &ctx);
  const Dropout *dptr = drop.get();
  dropouts_.push_back(dptr);
  modules.push_back(std::move(drop));
  auto var1 = std::make_shared<Variable>(prow, h, true, round_up4(h));
  variables.push_back(var1);
  variables.push_back(weights[0]);
  auto sm = std::make_unique<SparseMatmul>(&feats, weights[0], var1, dptr, &ctx);
  SparseMatmul *smp = sm.get();
  modules.push_back(std::move(sm));
  auto var2 = std::make_shared<Variable>(prow, h, true, round_up4(h));
  variables.push_back(var2);
  auto gs = std::make_unique<GraphSum>(var1, var2, graph.get(), h, &ctx);
  smp->consumer = gs.get();
  if (feats.ax) {  // eval: (Â X) W1 -> var2 directly, the GraphSum is skipped
    smp->eval_out = var2;
    gs->first_layer = true;
  }
  modules.push_back(std::move(gs));
  modules.push_back(std::make_unique<ReLU>(var2));
}

// src/gcn.cu:85-112
void GCN::insert_layer(int in_dim, int out_dim, float dropout, int layer) {
  const int prow = part.maxrows;
  shared_ptr<Variable> prev = variables.back();
  auto drop = std::make_unique<Dropout>(prev, dropout, rngs[(size_t)layer], &ctx);
  dropouts_.push_back(drop.get());
  modules.push_back(std::move(drop));
  auto var1 = std::make_shared<Variable>(prow, out_dim, true, round_up4(out_dim));
  variables.push_back(var1);
  variables.push_back(weights[(size_t)layer]);
  modules.push_back(std::make_unique<Matmul>(prev, weights[(size_t)layer], var1,
                                             part.local_rows(), in_dim, out_dim, &ctx));
  auto var2 = std::make_shared<Variable>(prow, out_dim, true, round_up4(out_dim));
  variables.push_back(var2);
  modules.push_back(std::make_unique<GraphSum>(var1, var2, graph.get(), out_dim, &ctx));
  modules.push_back(std::make_unique<ReLU>(var2));
}

// src/gcn.cu:116-142
void GCN::insert_last_layer() {
  const int prow = part.maxrows, C = params.output_dim, hl = params.hidden_dims.back();
  shared_ptr<Variable> prev = variables.back();
  auto drop = std::make_unique<Dropout>(prev, params.dropouts.back(), rngs[(size_t)L - 1], &ctx);
  dropouts_.push_back(drop.get());
  modules.push_back(std::move(drop));
  const bool small = g_reassoc_small && hl <= 16 && part.bounds.back() < kMmSideRows;
  if (params.reassociate_last && (hl < C || small) && graph_symmetric) {
    // out = Â (H W) computed as (Â H) W: the same product (Â is symmetric, so the backward
    // Â dOut W^T = Â (dOut W^T) and W.grad = H^T Â dOut = (Â H)^T dOut also match), but the
    // GraphSum gathers rows of width hl instead of C.  Only the fp32 rounding order differs.
    // A non-symmetric pattern (directed edge list) keeps the reference's module order: there
    // (Â H)^T dOut = H^T Â^T dOut is not the reference's H^T Â dOut (hpdga module.cpp:98-111).
    reassociated_ = true;
    auto z = std::make_shared<Variable>(prow, hl, true, round_up4(hl));
    restricted_vars.push_back((int)variables.size());
    variables.push_back(z);
    variables.push_back(weights.back());
    modules.push_back(std::make_unique<GraphSum>(prev, z, graph.get(), hl, &ctx, true));
    auto out = std::make_shared<Variable>(prow, C, true, round_up4(C));
    restricted_vars.push_back((int)variables.size());
    variables.push_back(out);
    auto mm = std::make_unique<Matmul>(z, weights.back(), out, part.local_rows(), hl, C, &ctx);
    mm->last_layer = true;
    modules.push_back(std::move(mm));
    modules.push_back(std::make_unique<CrossEntropyLoss>(out, C, &ctx));
    if (!comm && graph) {  // compact output layer buffers (split rows, see ModuleContext)
      size_t mx = 1;
      for (int sp = 1; sp <= 3; sp++) mx = std::max(mx, split_rows_host[sp].size());
      compact_z = std::make_unique<Variable>((int)mx, hl, true, round_up4(hl));
      compact_out = std::make_unique<Variable>((int)mx, C, true, round_up4(C));
      ctx.compact_z = compact_z.get();
      ctx.compact_out = compact_out.get();
    }
    return;
  }
  auto var1 = std::make_shared<Variable>(prow, C, true, round_up4(C));
  variables.push_back(var1);
  variables.push_back(weights.back());
  modules.push_back(std::make_unique<Matmul>(prev, weights.back(), var1, part.local_rows(), hl,
                                             C, &ctx));
  auto out = std::make_shared<Variable>(prow, C, true, round_up4(C));
  restricted_vars.push_back((int)variables.size());
  variables.push_back(out);
  modules.push_back(std::make_unique<GraphSum>(var1, out, graph.get(), C, &ctx, true));
  modules.push_back(std::make_unique<CrossEntropyLoss>(out, C, &ctx));
}

void GCN::set_split(int split) {
  ctx.truth = truth[split].get();
  ctx.count = counts[split];
  modules.back()->set_num_samples(counts[split]);
  // output-layer row restriction: Â restricted to the split's labelled rows, built at the
  // split's first use (single GPU; the edge-cut engine restricts its chunk graphs below)
  ctx.split_graph = nullptr;
  ctx.split_rows = nullptr;
  ctx.split_colgraph = nullptr;
  if (g_split_rows && !comm && graph) {
    if (!split_graphs[split]) {
      split_graphs[split] = graph->row_subset(split_rows_host[split]);
      split_rows_dev[split].allocate(std::max<size_t>(split_rows_host[split].size(), 1));
      split_rows_dev[split].upload(split_rows_host[split]);
    }
    ctx.split_graph = split_graphs[split].get();
    ctx.split_rows = split_rows_dev[split].get();
  }
  ctx.chunk_split_graphs.clear();
  ctx.chunk_split_rows.clear();
  if (g_split_rows && comm && !chunk_graphs.empty()) {
    // edge-cut: the output layer's forward sums only the split's labelled rows of every RS
    // chunk (padded chunk row q*h + j = global node bounds[q] + k*h + j)
    if (chunk_split_graphs[split].empty()) {
      const int h = part.chunk_rows();
      std::vector<char> in_split((size_t)params.num_nodes, 0);
      for (int i : split_rows_global[split]) in_split[(size_t)i] = 1;
      for (size_t k = 0; k < chunk_graphs.size(); k++) {
        std::vector<int> rows;
        for (int q = 0; q < part.world; q++)
          for (int j = 0; j < h; j++) {
            const long long i = (long long)part.bounds[(size_t)q] + (long long)k * h + j;
            if (i < part.bounds[(size_t)q + 1] && in_split[(size_t)i]) rows.push_back(q * h + j);
          }
        chunk_split_graphs[split].push_back(chunk_graphs[k]->row_subset(rows));
        chunk_split_rows[split].emplace_back();
        chunk_split_rows[split].back().allocate(std::max<size_t>(rows.size(), 1));
        if (!rows.empty()) chunk_split_rows[split].back().upload(rows);
      }
    }
    for (size_t k = 0; k < chunk_graphs.size(); k++) {
      ctx.chunk_split_graphs.push_back(chunk_split_graphs[split][k].get());
      ctx.chunk_split_rows.push_back(chunk_split_rows[split][k].get());
    }
  }
  ctx.chunk_col_graphs.clear();
  if (g_split_cols && comm && !chunk_graphs.empty() && split == 1 &&
      !split_rows_host[1].empty()) {  // backward follows training
    if (chunk_col_graphs.empty()) {
      for (auto &gk : chunk_graphs) chunk_col_graphs.push_back(gk->col_subset(split_rows_host[1]));
      for (size_t k = 1; k < chunk_col_graphs.size(); k++)
        chunk_col_graphs[k]->share_tables(chunk_col_graphs[0].get());
    }
    for (auto &cg : chunk_col_graphs) ctx.chunk_col_graphs.push_back(cg.get());
  }
  if (g_split_cols && !comm && graph && split == 1) {  // backward only follows training
    if (!split_colgraphs[split]) split_colgraphs[split] = graph->col_subset(split_rows_host[split]);
    ctx.split_colgraph = split_colgraphs[split].get();
  }
  out_restricted = ctx.split_graph != nullptr || !ctx.chunk_split_graphs.empty();
  // compact output layer: with the row restriction on the reassociated output layer
  const int n_s = (int)split_rows_host[split].size();
  if (ctx.split_graph && ctx.compact_z && n_s > 0) {
    ctx.compact_n = n_s;
    ctx.compact_truth = truth_compact[split].get();
    ctx.xent_blocks = xent_blocks(n_s);
  } else {
    ctx.compact_n = 0;
    ctx.compact_truth = nullptr;
    ctx.xent_blocks = xent_blocks(part.maxrows);
  }
}

// One GPU ("mask_adam", default on): the next training forward's input mask (and the hidden mask
// co-drawn with it) drawn by the optimizer's launch -- the two are independent, and the masks
// come from the same stream positions whenever they are drawn; the next forward then finds
// them drawn ahead (Dropout::ahead_descs).  One launch fewer per epoch.
int GCN::mask_with_adam(MaskDraw out[2]) {
  // (not with epoch graphs: a capture after an eager epoch would find the mask drawn ahead and
  // record a forward without its draw)
  if (!g_mask_adam || g_epoch_graph || comm || dropouts_.empty() || !dropouts_[0] ||
      dropouts_[0]->variable() || optimizer.size() > (size_t)kAdamBatch || mask_in_eval())
    return 0;
  return dropouts_[0]->ahead_descs(out);
}

// One GPU, dense X with eval_ax ("mask_xstream"): the next training forward's input mask (and
// the co-drawn hidden mask) drawn by two extra waves of eval's (A X) W1 pass -- an unmasked
// X-stream pass, HBM-bound, whose VALU is otherwise idle -- instead of by the Adam launch
// before it.  The same stream positions whenever they are drawn: bit-identical.  A training
// epoch with no eval after it draws its next mask in its own forward, as without the knob.
bool GCN::mask_in_eval() const {
  return g_mask_xstream && !g_epoch_graph && !comm && feats.ax && !dropouts_.empty() &&
         dropouts_[0] && !dropouts_[0]->variable();
}

// One GPU ("fuse_finish", default on): the next pass's loss kernel finishes its scalars itself
// into results_ring slot dst_offset (XentFinal), so finalize() launches nothing
void GCN::arm_finish(int dst_offset, bool graph) {
  ctx.fin = nullptr;
  ctx.fin_taken = false;
  // every block adds to ONE ticket: cheap for the small graphs' 43-310 loss blocks (cora 11.1k
  // -> 11.8k, citeseer 10.6k -> 11.5k epochs/s, same box, profiles/r06/e), but reddit's 3,641
  // serialised device-scope adds took the loss kernels from 21 + 39 to 58 + 69 us: there the
  // separate one-block launch stays
  // r06 late (fuse_finish 2): above that, two levels -- the blocks arrive on one ticket per
  // group of kFinishGroup, the group's last block sums the group and arrives on the top ticket
  // (reddit: 57 groups of 64 instead of 3,641 adds on one address)
  if (!g_fuse_finish || comm) return;
  const bool two = ctx.xent_blocks > kFinishMaxBlocks;
  if (two && g_fuse_finish < 2) return;
  const int groups = two ? (ctx.xent_blocks + kFinishGroup - 1) / kFinishGroup : 0;
  if (!fin_ticket || fin_blocks < ctx.xent_blocks) {
    fin_ticket.allocate(1);
    fin_ticket.zero();
    fin_part4.allocate((size_t)std::max(1, ctx.xent_blocks) * 4);
    fin_blocks = ctx.xent_blocks;
    if (two) {
      fin_gticket.allocate((size_t)groups * 16);
      fin_gticket.zero();
      fin_gpart4.allocate((size_t)groups * 4);
    }
  }
  const auto &w1 = weights.front();
  fin_desc = XentFinal{};
  fin_desc.w = w1->dev_data.get();
  fin_desc.n_w = w1->size;
  fin_desc.wd = adam_params.weight_decay;
  fin_desc.out2 = results_ring.get() + dst_offset;
  fin_desc.ctr = graph ? dev_ctr.get() : nullptr;
  fin_desc.ring_cap = ring_cap;
  fin_desc.sums = sums.get();
  fin_desc.ticket = fin_ticket.get();
  fin_desc.part4 = reinterpret_cast<float4 *>(fin_part4.get());
  if (two) {
    fin_desc.group = kFinishGroup;
    fin_desc.gticket = fin_gticket.get();
    fin_desc.gpart4 = reinterpret_cast<float4 *>(fin_gpart4.get());
  }
  ctx.fin = &fin_desc;
}

// loss/acc of the pass just enqueued -> results_ring slot (finalize, src/gcn.cu:440-455);
// graph: the slot from the device epoch counter
void GCN::finalize(int dst_offset, bool graph, hipStream_t s) {
  const auto &w1 = weights.front();
  if (!s) s = stream.get();
  if (ctx.fin_taken) {  // the loss kernel's last block did it (fuse_finish)
    ctx.fin_taken = false;
    ctx.fin = nullptr;
    return;
  }
  ctx.fin = nullptr;
  if (!comm) {  // one launch: reduce + compose
    launch_reduce_scalars(xent_partials.get(), ctx.xent_blocks, w1->dev_data.get(), w1->size,
                          sums.get(), stream.get(), ctx.count, adam_params.weight_decay,
                          results_ring.get() + dst_offset, graph ? dev_ctr.get() : nullptr,
                          ring_cap);
    return;
  }
  // edge-cut: {loss sum, wrong, sum W1^2, count} into the raw ring slot, the first two summed
  // over the ranks in place; the host composes them when it reads the results (compose_raw:
  // k_compose's arithmetic in the same float operations, the same bits)
  PGCN_CHECK(!graph, PGCN_E_INVALID, "edge-cut epochs are not captured");
  float *raw = raw_ring.get() + (size_t)dst_offset * 2;  // slot * 8 + pass * 4
  PeerSmall ps;
  auto *pc = dynamic_cast<PeerComm *>(comm.get());
  comm->enter(s);  // (eval_tail) after the last eval pass's tail
  const bool fused = pc && pc->small_allreduce(2, &ps);  // between processes: in this launch
  launch_reduce_scalars(xent_partials.get(), ctx.xent_blocks, w1->dev_data.get(), w1->size,
                        nullptr, s, ctx.count, 0.0f, nullptr, nullptr, 1, raw,
                        fused ? &ps : nullptr);
  if (!fused) comm->allreduce_sum(raw, 2, s);
}

// eval's forward pass (src/gcn.cu:293-303).  eval_tail: from its last GraphSum's push on, the
// pass runs on comm_stream (ModuleContext::tail_stream), so the next epoch's mask draw and
// first-layer product proceed on the stream beside the exchange and the output layer; the
// next GraphSum waits for tail_done.
void GCN::eval_forward(int off, bool graph) {
  const bool tail = tail_gs >= 0;
  arm_finish(off, graph);
  ctx.xs_draw.n = 0;
  if (!graph && mask_in_eval()) {
    const int n = dropouts_[0]->ahead_descs(ctx.xs_draw_md);
    for (int i = 0; i < n; i++) ctx.xs_draw.seg[i] = mask_seg_of(ctx.xs_draw_md[i]);
    ctx.xs_draw.lut = mask_lut.get();
    ctx.xs_draw.n = n;
  }
  for (int i = 0; i < (int)modules.size(); i++) {
    if (tail && i == tail_gs) {
      ctx.tail_stream = comm_stream.get();
      ctx.tail_used = false;
    }
    modules[(size_t)i]->forward(false, tail && i > tail_gs ? comm_stream : stream);
    if (tail && i == tail_gs) {
      ctx.tail_stream = nullptr;
      if (!ctx.tail_used) {  // that GraphSum ran whole on the stream: the rest follows it
        ctx.tail_fork.record(stream.get());
        ctx.tail_fork.wait_on(comm_stream.get());
      }
    }
  }
  finalize(off, graph, tail ? comm_stream.get() : nullptr);
  if (tail) {
    ctx.tail_done.record(comm_stream.get());
    ctx.tail_pending = true;
    comm->defer(ctx.tail_done.get());  // the next collective on any stream follows it
  }
}

// k_compose (hpdga gcn.cpp:167-198) on the host: {loss_sum/count + wd*l2/2, (count-wrong)/count}
void GCN::compose_raw(const float *raw4, float *out2) const {
  const int count = (int)raw4[3];
  const float loss = raw4[0] / (float)count;
  const float l2 = adam_params.weight_decay * raw4[2] / 2.0f;
  out2[0] = loss + l2;
  const int wrong = (int)raw4[1];
  out2[1] = (float)(count - wrong) / (float)count;
}

// the weight gradients a Matmul::backward left on the side stream are complete on `stream`
void GCN::join_side() {
  if (!ctx.side_pending) return;
  ctx.side_join.record(side_stream.get());
  ctx.side_join.wait_on(stream.get());
  ctx.side_pending = false;
}

// One GPU ("tn_fold"): from the training forward (the fused loss kernel's W2.grad partials) to
// the end of the backward pass the weight gradients' last ordered reduction passes are
// recorded for the Adam launch, which runs them (the same bits, two launches fewer per epoch;
// tn_defer).  An edge-cut rank all-reduces finished gradients instead: no fold.
struct GCN::FoldScope {
  explicit FoldScope(GCN &g, TnDeferList *d) {
    g.adam_peer = PeerRecv{};
    // one GPU, or the peer exchange between processes (the passes then ride the gradients'
    // all-reduce push: GCN::backward_pass); in-process ranks and RCCL all-reduce finished
    // gradients
    const auto *pc = dynamic_cast<const PeerComm *>(g.comm.get());
    if (!g_tn_fold || (g.comm && !(pc && !pc->host_ordered() && g.comm->world() > 1))) return;
    // the deferred passes' inputs: 64 first-pass groups of every weight's [K][16-padded]
    // gradient (reddit: 0.8 MB)
    if (!g.tn_pool) {
      size_t f = 0;
      for (const auto &w : g.weights) f += (size_t)64 * w->rows * ((w->cols + 15) / 16 * 16) + 64;
      // the small graphs' loss-kernel W.grad block partials ([16][48] per block)
      f += (size_t)g.ctx.xent_blocks * 16 * 48 + 64;
      g.tn_pool.allocate(f);
    }
    d->pool = g.tn_pool.get();
    d->pool_floats = g.tn_pool.size();
    tn_defer(d);
  }
  ~FoldScope() { tn_defer(nullptr); }
  void end() { tn_defer(nullptr); }
};

// The backward modules in reverse order (src/gcn.cu:318-330), the side stream joined, the
// gradients all-reduced (edge-cut)
void GCN::backward_pass(FoldScope &fold, TnDeferList *defer) {
  for (int i = (int)modules.size() - 1; i >= 0; i--) modules[(size_t)i]->backward(stream);
  fold.end();
  join_side();
  if (!comm) return;
  auto *pc = dynamic_cast<PeerComm *>(comm.get());
  if (pc && defer->n > 0) {
    // the deferred passes ride the all-reduce's push (their sums pushed straight from the
    // group partials), and the Adam launch sums the received slots (adam_peer): three launches
    // fewer than passes + push + sum
    GradRegions r;
    const float *arena = grad_arena.get();
    for (int i = 0; i < defer->n; i++) {
      TnDeferred &d = defer->d[i];
      const long long off = d.C - arena, len = (long long)d.K * d.N;
      if (!d.src || off < 0 || off + len > (long long)grad_arena.size() || r.n >= 4) continue;
      r.off[r.n] = off;
      r.d[r.n++] = d;
      d.src = nullptr;  // taken
    }
    tn_defer_flush(*defer, stream.get());  // (any pass outside the arena: before the push)
    if (pc->allreduce_grads(grad_arena.get(), grad_arena.size(), r, stream.get(), &adam_peer))
      return;
    // (not applicable: nothing enqueued) the passes as launches, then the plain all-reduce
    defer->n = 0;
    for (int i = 0; i < r.n; i++) defer->d[defer->n++] = r.d[i];
    tn_defer_flush(*defer, stream.get());
  }
  comm->allreduce_sum(grad_arena.get(), grad_arena.size(), stream.get());
}

// train_epoch (src/gcn.cu:307-343) + eval(2) (src/gcn.cu:293-303), host-sync free
void GCN::enqueue_epoch(bool graph) {
  const int slot4 = graph ? 0 : (int)(epoch_count % ring_cap) * 4;
  set_split(1);
  TnDeferList defer;
  FoldScope fold(*this, &defer);
  arm_finish(slot4, graph);
  for (const auto &m : modules) m->forward(true, stream);
  finalize(slot4, graph);
  backward_pass(fold, &defer);
  const PeerRecv *pr = adam_peer.world ? &adam_peer : nullptr;
  if (graph) {
    optimizer.step_graph(stream, step_table.get(), dev_ctr.get(), kStepTable, &defer, pr,
                         grad_arena.get());
  } else {
    MaskDraw md[2];
    const int nd = mask_with_adam(md);
    optimizer.step(stream, &defer, pr, grad_arena.get(), md, nd, ctx.jump_table);
  }
  set_split(2);
  eval_forward(slot4 + 2, graph);
  if (graph) launch_counters(dev_ctr.get(), 0, 0, 0, stream.get());
}

// A replayed epoch must launch exactly what an eager one would: no host-side state may change
// between epochs.  Excluded: the edge-cut engine (RCCL calls), GraphSum profiling (host
// events), and train-ahead over dense X without eval_ax (it swaps buffers on the host between
// eval and the next training forward).
bool GCN::graph_eligible() const {
  if (!g_epoch_graph || !warm || comm || ctx.profile) return false;
  if (ctx.train_ahead && feats.dense && feats.maskT && !feats.ax) return false;
  if (ctx.train_ahead && !feats.dense && g_sparse_dual) return false;  // (the same host swaps)
  return true;
}

void GCN::drop_epoch_graph() {
  if (epoch_exec) (void)hipGraphExecDestroy(epoch_exec);
  if (epoch_graph) (void)hipGraphDestroy(epoch_graph);
  epoch_exec = nullptr;
  epoch_graph = nullptr;
}

void GCN::capture_epoch() {
  if (!dev_ctr) {
    dev_ctr.allocate(2);
    step_table.allocate(kStepTable);
  }
  PGCN_HIP(hipStreamBeginCapture(stream.get(), hipStreamCaptureModeThreadLocal));
  const bool side = ctx.mm_side;
  ctx.mm_side = false;  // the captured epoch keeps every launch on the captured stream
  try {
    enqueue_epoch(true);
    ctx.mm_side = side;
  } catch (...) {
    ctx.mm_side = side;
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(stream.get(), &g);
    if (g) (void)hipGraphDestroy(g);
    throw;
  }
  PGCN_HIP(hipStreamEndCapture(stream.get(), &epoch_graph));
  PGCN_HIP(hipGraphInstantiate(&epoch_exec, epoch_graph, nullptr, nullptr, 0));
}

void GCN::epoch_async() {
  if (!graph_eligible()) {
    enqueue_epoch(false);
    ctr_valid = false;
    warm = true;
  } else {
    if (!epoch_exec) capture_epoch();
    // the step size table covers this epoch's Adam step (index = steps done % cap)
    const long long t = optimizer.steps(), block = t / kStepTable;
    if (block != table_block) {
      stream.sync();  // replays already queued read the old table
      std::vector<float> tab(kStepTable);
      for (int i = 0; i < kStepTable; i++)
        tab[(size_t)i] = optimizer.step_size((int)(block * kStepTable + i + 1));
      step_table.upload(tab);
      table_block = block;
    }
    if (!ctr_valid) {
      launch_counters(dev_ctr.get(), 1, (int)t, (int)epoch_count, stream.get());
      ctr_valid = true;
    }
    PGCN_HIP(hipGraphLaunch(epoch_exec, stream.get()));
    optimizer.advance();
    set_split(2);  // host context as after an eager epoch
  }
  last_forward_training = false;
  epoch_count++;
}

std::pair<float, float> GCN::train_epoch() {
  const long long slot = epoch_count % ring_cap;
  set_split(1);
  TnDeferList defer;
  FoldScope fold(*this, &defer);
  arm_finish((int)(slot * 4), false);
  for (const auto &m : modules) m->forward(true, stream);
  finalize((int)(slot * 4));
  backward_pass(fold, &defer);
  MaskDraw md[2];
  const int nd = mask_with_adam(md);
  optimizer.step(stream, &defer, adam_peer.world ? &adam_peer : nullptr, grad_arena.get(), md, nd,
                 ctx.jump_table);
  ctr_valid = false;
  last_forward_training = true;
  return read_slot((int)(slot * 4));
}

// results_ring[off .. off + 1] (one GPU), or the host's composition of the raw ring's sums of
// that pass (edge-cut)
std::pair<float, float> GCN::read_slot(int off) {
  if (comm) {
    if (ctx.tail_pending) comm_stream.sync();  // an eval pass's scalars (eval_tail)
    PGCN_HIP(hipMemcpyAsync(pinned.get(), raw_ring.get() + (size_t)off * 2, 4 * sizeof(float),
                            hipMemcpyDeviceToHost, stream.get()));
    stream.sync();
    check_comm();
    float r[2];
    compose_raw(pinned.get(), r);
    return {r[0], r[1]};
  }
  PGCN_HIP(hipMemcpyAsync(pinned.get(), results_ring.get() + off, 2 * sizeof(float),
                          hipMemcpyDeviceToHost, stream.get()));
  stream.sync();
  return {pinned.get()[0], pinned.get()[1]};
}

std::pair<float, float> GCN::eval(int split) {
  PGCN_CHECK(split >= 1 && split <= 3, PGCN_E_INVALID, "split must be 1, 2 or 3");
  const long long slot = epoch_count % ring_cap;
  set_split(split);
  eval_forward((int)(slot * 4 + 2), false);
  last_forward_training = false;
  ctr_valid = false;
  const std::pair<float, float> r = read_slot((int)(slot * 4 + 2));
  if (split == 2) epoch_count++;  // a train_epoch + eval(2) pair fills one ring slot
  return r;
}

void GCN::sync() {
  stream.sync();
  side_stream.sync();
  if (comm_stream.get()) comm_stream.sync();  // (eval_tail)
  check_comm();
}

// a peer exchange that gave up waiting (a rank never signalled) fails the call that syncs
void GCN::check_comm() const {
  if (const auto *pc = dynamic_cast<const PeerComm *>(comm.get())) pc->check();
}

std::vector<float> GCN::results(int n) {
  sync();
  std::vector<float> all((size_t)ring_cap * 4);
  if (comm) {
    std::vector<float> raw((size_t)ring_cap * 8);
    raw_ring.download(raw.data(), raw.size());
    for (int k = 0; k < ring_cap * 2; k++) compose_raw(&raw[(size_t)k * 4], &all[(size_t)k * 2]);
  } else {
    results_ring.download(all.data(), all.size());
  }
  n = (int)std::min<long long>(n, std::min<long long>(epoch_count, ring_cap));
  std::vector<float> out((size_t)n * 4);
  for (int k = 0; k < n; k++) {
    const long long e = epoch_count - n + k;
    std::memcpy(&out[(size_t)k * 4], &all[(size_t)(e % ring_cap) * 4], 4 * sizeof(float));
  }
  return out;
}

// src/gcn.cu:347-436 / hpdga gcn.cpp:214-274
void GCN::run(bool verbose) {
  std::vector<float> loss_history;
  double total = 0;
  int epoch = 1;
  for (; epoch <= params.epochs; epoch++) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    auto tr = train_epoch();
    auto va = eval(2);
    const float dt = std::chrono::duration<float>(std::chrono::high_resolution_clock::now() - t0).count();
    total += dt;
    if (verbose)
      printf("epoch=%d train_loss=%.5f train_acc=%.5f val_loss=%.5f val_acc=%.5f time=%.5f\n",
             epoch, tr.first, tr.second, va.first, va.second, dt);
    loss_history.push_back(va.first);
    if (params.early_stopping > 0 && epoch >= params.early_stopping) {
      float recent = 0.0f;
      for (int i = epoch - params.early_stopping; i < epoch; i++) recent += loss_history[(size_t)i];
      if (va.first > recent / (float)params.early_stopping) {
        if (verbose) printf("Early stopping...\n");
        break;
      }
    }
  }
  if (verbose) {
    const int done = std::min(epoch, params.epochs);
    printf("TMR_TRAIN average time: %.3fms\n", total * 1000.0 / done);
    const auto t0 = std::chrono::high_resolution_clock::now();
    auto te = eval(3);
    const float dt = std::chrono::duration<float>(std::chrono::high_resolution_clock::now() - t0).count();
    printf("test_loss=%.5f test_acc=%.5f time=%.5f\n", te.first, te.second, dt);
  }
}

bool GCN::graphsum_lds() const {
  if (graph) return graph->uses_lds(16);
  return !chunk_graphs.empty() && chunk_graphs.front()->uses_lds(16);
}

std::vector<float> GCN::get_var(int idx, int which) {
  sync();
  PGCN_CHECK(idx >= 0 && idx < (int)variables.size(), PGCN_E_INVALID, "variable index");
  if (idx == 0) {  // the input features (dropped, if the last forward was a training one)
    if (which) return {};
    std::vector<float> x;
    if (feats.dense) {
      std::vector<float> raw((size_t)feats.rows * feats.ldx);
      feats.x.download(raw.data(), raw.size());
      x.resize((size_t)feats.rows * feats.cols);
      for (int i = 0; i < feats.rows; i++)
        std::memcpy(&x[(size_t)i * feats.cols], &raw[(size_t)i * feats.ldx],
                    sizeof(float) * (size_t)feats.cols);
    } else {
      x = feats.host_values;
    }
    if (last_forward_training) {
      const DropoutRng &r = *rngs[0];
      std::vector<uint64_t> m((size_t)r.n_chunks);
      r.mask.download(m.data(), m.size());
      const float scale = dropouts_[0]->scale();
      for (size_t k = 0; k < x.size(); k++) {
        const long long b = r.mask_base + (long long)k;
        x[k] *= ((m[(size_t)(b >> 6)] >> (b & 63)) & 1) ? scale : 0.0f;
      }
    }
    return x;
  }
  // the output-layer row restriction (split_rows) leaves these rows stale or unwritten
  PGCN_CHECK(!out_restricted || std::find(restricted_vars.begin(), restricted_vars.end(), idx) ==
                                    restricted_vars.end(),
             PGCN_E_INVALID,
             "get_var: the output layer ran restricted to the split's rows (split_rows on); its "
             "other rows are stale");
  const auto &v = variables[(size_t)idx];
  std::vector<float> out = v->to_host(which);
  const bool node_var = v->rows == part.maxrows &&
                        std::find(weights.begin(), weights.end(), v) == weights.end();
  if (node_var) out.resize((size_t)part.local_rows() * v->cols);
  return out;
}

void GCN::set_profile(bool on) {
  sync();
  ctx.profile = on;
  gs_events.clear();
  gs_bytes.clear();
  mm_events.clear();
  mm_flops.clear();
}

void GCN::profile_read_mm(double *ms, long long *calls, double *flops) {
  sync();
  double t = 0, f = 0;
  for (size_t i = 0; i < mm_events.size(); i++) {
    float e = 0;
    PGCN_HIP(hipEventElapsedTime(&e, mm_events[i].first.get(), mm_events[i].second.get()));
    t += e;
    f += mm_flops[i];
  }
  if (ms) *ms = t;
  if (calls) *calls = (long long)mm_events.size();
  if (flops) *flops = f;
}

void GCN::profile_read(double *ms, long long *calls, double *bytes) {
  sync();
  double t = 0, b = 0;
  for (size_t i = 0; i < gs_events.size(); i++) {
    float e = 0;
    PGCN_HIP(hipEventElapsedTime(&e, gs_events[i].first.get(), gs_events[i].second.get()));
    t += e;
    b += gs_bytes[i];
  }
  if (ms) *ms = t;
  if (calls) *calls = (long long)gs_events.size();
  if (bytes) *bytes = b;
}

}  // namespace pgcn
