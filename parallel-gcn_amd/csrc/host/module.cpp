// parallel-gcn_amd/csrc/host/module.cpp
#include "module.hpp"

#include <utility>

#include "../kernels.hpp"

namespace pgcn {

namespace {
// Profiling scope of one XW contraction (MFMA kernels): HIP events around the launches on
// the module's stream and the contraction's 2*M*N*K flops (ctx->profile only).
struct MmProfile {
  ModuleContext *ctx;
  hipStream_t s;
  double flops;
  Event e0, e1;
  MmProfile(ModuleContext *c, hipStream_t st, double f) : ctx(c), s(st), flops(f) {
    if (!on()) return;
    e0 = Event::create(true);
    e1 = Event::create(true);
    e0.record(s);
  }
  bool on() const { return ctx->profile && ctx->mm_events && flops > 0; }
  ~MmProfile() {
    if (!on()) return;
    e1.record(s);
    ctx->mm_events->emplace_back(e0, e1);
    ctx->mm_flops->push_back(flops);
  }
};
}  // namespace

Variable::Variable(int rows_, int cols_, bool requires_grad, int ld_)
    : rows(rows_), cols(cols_), ld(ld_ < 0 ? cols_ : ld_), size((long long)rows_ * cols_) {
  const size_t n = (size_t)rows * (size_t)ld;
  dev_data.allocate(n);
  dev_data.zero();
  if (requires_grad) {
    dev_grad.allocate(n);
    dev_grad.zero();
  }
}

std::vector<float> Variable::to_host(int which) const {
  const DeviceBuffer<float> &b = which ? dev_grad : dev_data;
  std::vector<float> out;
  if (!b) return out;
  std::vector<float> raw((size_t)rows * ld);
  b.download(raw.data(), raw.size());
  out.resize((size_t)rows * cols);
  for (int r = 0; r < rows; r++)
    for (int c = 0; c < cols; c++) out[(size_t)r * cols + c] = raw[(size_t)r * ld + c];
  return out;
}

// "csc_tree" (read per launch): sparse X's W1.grad summed as a fixed tree over each feature's
// entries (k_spmm_csc_tree) instead of hpdga's sequential scatter order (k_spmm_csc_bwd,
// bit-exact); deterministic, the sums in another order.  Off: measured slower where it counts
// (same box, 400 epochs, profiles/r06/k: citeseer 11.6-11.7k vs 12.1k epochs/s, pubmed_synth
// 6.57-6.59k vs 7.06k, cora 10.7-12.4k vs 12.3k) -- the chain's one-wave tail is not what
// bounds the launch
int g_csc_tree = 0;
// "defer_wgrad" (read per pass): a small graph's fused loss kernel writes the output layer's
// W.grad block partials into the deferred-reduction pool (tn_fold), summed by the Adam launch
int g_defer_small_wgrad = 1;
// up to this many loss blocks (cora 43, citeseer 52): pubmed_synth's 309 partials per weight
// element made the Adam launch's sum as long as the two launches it saved (7.73-7.74k vs
// 7.78-7.80k epochs/s, profiles/r06/s)
constexpr int kDeferWgradMaxBlocks = 128;

// ------------------------------------------------------------------------------------------
// Dropout (src/module.cu:6-99; hpdga module.cpp:196-228)
// ------------------------------------------------------------------------------------------
Dropout::Dropout(shared_ptr<Variable> in_, float p_, shared_ptr<DropoutRng> rng_,
                 ModuleContext *ctx_)
    : in(std::move(in_)), rng(std::move(rng_)), p(p_), ctx(ctx_) {}

void Dropout::draw(hipStream_t s, uint64_t *mask, int max_blocks) const {
  const DropoutRng &r = *rng;
  launch_dropout_mask(r.states.get(), r.n_chunks, 64 * r.chunk_lo, r.elem_end, p, mask,
                      ctx->jump_table, s, max_blocks, r.per);
}

void Dropout::draw_ahead(hipStream_t s, const Event *ready) const {
  PGCN_CHECK(!ahead && !in, PGCN_E_INVALID, "dropout: one mask ahead, input dropout only");
  // into its own buffer: `mask` stays the last training forward's (backward, get_var)
  if (!rng->mask_ahead) {
    rng->mask_ahead.allocate(rng->mask.size());
    rng->mask_ahead.zero();
  }
  if (co_draw && !ready && !co_draw->pre_drawn && !co_draw->ahead) {
    // with the hidden dropout's next mask (co_draw; the eval forward uses neither)
    const DropoutRng &r = *rng, &q = co_draw->state();
    const MaskDraw a{r.states.get(), r.n_chunks, 64 * r.chunk_lo, r.elem_end, p,
                     rng->mask_ahead.get(), r.per};
    const MaskDraw b{q.states.get(), q.n_chunks, 64 * q.chunk_lo, q.elem_end, co_draw->p,
                     q.mask.get(), q.per};
    launch_dropout_mask2(a, b, ctx->jump_table, s);
    co_draw->pre_drawn = true;
  } else {
    // on a side stream: two workgroups per CU, leaving room for the main stream's kernels
    draw(s, rng->mask_ahead.get(), ready ? 2 * kCUs : 0);
  }
  if (ready) ready->record(s);
  ahead_ready = ready;
  ahead = true;
}

int Dropout::ahead_descs(MaskDraw out[2]) const {
  PGCN_CHECK(!in, PGCN_E_INVALID, "dropout: one mask ahead, input dropout only");
  if (ahead) return 0;
  if (!rng->mask_ahead) {
    rng->mask_ahead.allocate(rng->mask.size());
    rng->mask_ahead.zero();
  }
  const DropoutRng &r = *rng;
  out[0] = MaskDraw{r.states.get(), r.n_chunks, 64 * r.chunk_lo, r.elem_end, p,
                    rng->mask_ahead.get(), r.per};
  int n = 1;
  if (co_draw && !co_draw->pre_drawn && !co_draw->ahead) {
    const DropoutRng &q = co_draw->state();
    out[1] = MaskDraw{q.states.get(), q.n_chunks, 64 * q.chunk_lo, q.elem_end, co_draw->p,
                      q.mask.get(), q.per};
    co_draw->pre_drawn = true;
    n = 2;
  }
  ahead_ready = nullptr;
  ahead = true;
  return n;
}

void Dropout::wait_ahead(hipStream_t s) const {
  if (ahead && ahead_ready) {
    ahead_ready->wait_on(s);
    ahead_ready = nullptr;
  }
}

void Dropout::draw_fused(hipStream_t s) const {
  PGCN_CHECK(in && !ahead, PGCN_E_INVALID, "dropout: fused draw of a hidden dropout only");
  if (pre_drawn)
    pre_drawn = false;
  else
    draw(s, rng->mask.get());
  skip_forward = true;
}

void Dropout::forward(bool training, const Stream &s) const {
  if (!training) return;  // hpdga module.cpp:209
  if (skip_forward) {  // drawn and applied by the GraphSum before it (epilogue)
    skip_forward = false;
    return;
  }
  const DropoutRng &r = *rng;
  if (ahead) {  // drawn ahead (during the last weight-gradient pass, or by the eval forward)
    wait_ahead(s.get());
    std::swap(rng->mask, rng->mask_ahead);
    ahead = false;
  } else if (pre_drawn) {  // drawn with the input dropout's mask (co_draw)
    pre_drawn = false;
  } else if (co_draw && !co_draw->pre_drawn && !co_draw->ahead) {
    const DropoutRng &q = co_draw->state();
    const MaskDraw a{r.states.get(), r.n_chunks, 64 * r.chunk_lo, r.elem_end, p, r.mask.get(),
                     r.per};
    const MaskDraw b{q.states.get(), q.n_chunks, 64 * q.chunk_lo, q.elem_end, co_draw->p,
                     q.mask.get(), q.per};
    launch_dropout_mask2(a, b, ctx->jump_table, s.get());
    co_draw->pre_drawn = true;
  } else {
    draw(s.get(), rng->mask.get());
  }
  if (in) {
    // a grad-carrying variable is dropped in place (module.cpp:215); its rows are the
    // first (elem_end - elem_begin) elements of the local variable
    launch_dropout_apply_based(in->dev_data.get(), r.elem_end - r.elem_begin, r.mask.get(),
                               r.mask_base, scale(), s.get());
  }
}

void Dropout::backward(const Stream &s) const {
  if (!in || !in->dev_grad) return;  // module.cpp:222: no mask => nothing to do
  if (skip_backward) {  // applied by the GraphSum backward before it (epilogue)
    skip_backward = false;
    return;
  }
  const DropoutRng &r = *rng;
  launch_dropout_apply_based(in->dev_grad.get(), r.elem_end - r.elem_begin, r.mask.get(),
                             r.mask_base, scale(), s.get());
}

// ------------------------------------------------------------------------------------------
// SparseMatmul (src/module.cu:104-163; hpdga module.cpp:49-72)
// ------------------------------------------------------------------------------------------
SparseMatmul::SparseMatmul(const DevFeatures *x_, shared_ptr<Variable> b_,
                           shared_ptr<Variable> c_, const Dropout *drop_, ModuleContext *ctx_)
    : x(x_), b(std::move(b_)), c(std::move(c_)), drop(drop_), ctx(ctx_) {}

// The X-stream ring kernels (xstream_ring_ok) read the dropout bitmap as it was drawn (XsMask);
// the register-streamed ones read the nibble layout k_mask_nibbles builds from it (x->maskT)
static bool xs_flat(const DevFeatures *x) { return xstream_ring_ok(x->cols, x->ldx); }

void SparseMatmul::forward(bool training, const Stream &s) const {
  last_training = training;
  const uint64_t *mask = training ? drop->state().mask.get() : nullptr;
  const long long base = drop->state().mask_base;
  const float scale = drop->scale();
  if (!training && x->ax && eval_out) {  // eval_ax: (Â X) W1 straight into the GraphSum's output
    if (xstream_ok(b->cols, x->cols)) {
      // eval: out = relu(Â X W1) (GraphSum, then its fused ReLU; the Dropout after it is the
      // identity in eval), which the reassociated output layer's GraphSum reads next
      XsEpilogue e;
      if ((g_fuse_epilogue & kFuseXstream) && consumer && consumer->fwd_relu) {
        e.relu = 1;
        consumer->fwd_relu->skip_forward = true;
        if (consumer->fwd_next)
          e.next_table =
              consumer->fwd_next->claim_forward_table(x->rows, eval_out->ld, &e.next_scale);
        e.next_sr = RING_SR;
      }
      // mask_xstream: the next training forward's masks drawn by extra waves of this product
      // (an unmasked pass on the ring kernel), else by their own launch below
      XsDraw dr;
      if (ctx->xs_draw.n > 0 && xstream_ring_ok(x->cols, x->ldx)) {
        dr = ctx->xs_draw;
        e.draw = &dr;
        ctx->xs_draw.n = 0;
      }
      launch_xstream_nn(x->rows, b->cols, x->cols, x->ax.get(), x->ldx, b->dev_data.get(), b->ld,
                        0, eval_out->dev_data.get(), eval_out->ld, nullptr, 1.0f, s.get(), nullptr,
                        &e);
    } else
      launch_gemm_nn(x->rows, b->cols, x->cols, x->ax.get(), x->ldx, b->dev_data.get(), b->ld, 0,
                     eval_out->dev_data.get(), eval_out->ld, nullptr, 0, 0, 1.0f, s.get());
    if (ctx->xs_draw.n > 0) {  // drawn ahead all the same: the forward expects them
      if (ctx->xs_draw.n == 2)
        launch_dropout_mask2(ctx->xs_draw_md[0], ctx->xs_draw_md[1], ctx->jump_table, s.get());
      else
        launch_dropout_mask(ctx->xs_draw_md[0].states, ctx->xs_draw_md[0].n_chunks,
                            ctx->xs_draw_md[0].elem0, ctx->xs_draw_md[0].elem_end,
                            ctx->xs_draw_md[0].p, ctx->xs_draw_md[0].mask, ctx->jump_table,
                            s.get(), 0, ctx->xs_draw_md[0].per);
      ctx->xs_draw.n = 0;
    }
    return;
  }
  if (training && ahead_valid) {  // computed by the eval forward before this one
    std::swap(c->dev_data, ahead);
    ahead_valid = false;
    return;
  }
  if (!training && ctx->train_ahead && !x->dense && g_sparse_dual && !ahead_valid) {
    // sparse X: eval's X W1 and the next training forward's drop(X) W1 from one pass over X
    // (k_spmm_csr<true>; the next input mask -- and its co-drawn hidden mask -- drawn now)
    if (!ahead) {
      ahead.allocate(c->dev_data.size());
      ahead.zero();
    }
    if (drop->drawn_ahead())
      drop->wait_ahead(s.get());
    else
      drop->draw_ahead(s.get());
    launch_spmm_csr_dual(x->rows, b->cols, c->ld, x->indptr.get(), x->indices.get(),
                         x->values.get(), drop->mask_ahead(), base, scale, b->dev_data.get(),
                         c->dev_data.get(), ahead.get(), s.get());
    ahead_valid = true;
    return;
  }
  if (!training && ctx->train_ahead && x->dense && x->maskT && !ahead_valid) {
    // eval forward + the next training forward's product, one pass over X (the next mask is
    // usually drawn already, on the side stream during the last weight-gradient pass)
    if (!ahead) {
      ahead.allocate(c->dev_data.size());
      ahead.zero();  // rows past x->rows (edge-cut padding) and padding columns stay zero
    }
    if (drop->drawn_ahead())
      drop->wait_ahead(s.get());
    else
      drop->draw_ahead(s.get());
    const uint64_t *m = drop->mask_ahead();
    const bool flat = xs_flat(x);
    const XsMask fm{m, base, x->cols, (long long)drop->state().mask.size()};  // (ahead: same size)
    if (!flat) launch_mask_nibbles(m, base, x->cols, x->rows, x->cols, x->maskT.get(), s.get());
    launch_xstream_nn(x->rows, b->cols, x->cols, x->x.get(), x->ldx, b->dev_data.get(), b->ld, 0,
                      c->dev_data.get(), c->ld, flat ? nullptr : x->maskT.get(), scale, s.get(),
                      ahead.get(), nullptr, flat ? &fm : nullptr);
    ahead_valid = true;
    return;
  }
  MmProfile prof(ctx, s.get(), x->dense ? 2.0 * x->rows * b->cols * x->cols : 0.0);
  if (x->dense && x->maskT) {  // X-stream kernels (N <= 16, K <= 640)
    const bool flat = mask && xs_flat(x);
    const XsMask fm{mask, base, x->cols, (long long)drop->state().mask.size()};
    if (mask && !flat)
      launch_mask_nibbles(mask, base, x->cols, x->rows, x->cols, x->maskT.get(), s.get());
    XsEpilogue e;  // the first GraphSum's prescaled input, written beside c
    if ((g_fuse_epilogue & kFuseXstream) && consumer && (training || !eval_out)) {
      e.next_table = consumer->claim_forward_table(x->rows, c->ld, &e.next_scale);
      e.next_sr = RING_SR;
    }
    launch_xstream_nn(x->rows, b->cols, x->cols, x->x.get(), x->ldx, b->dev_data.get(), b->ld, 0,
                      c->dev_data.get(), c->ld, mask && !flat ? x->maskT.get() : nullptr, scale,
                      s.get(), nullptr, &e, flat ? &fm : nullptr);
  } else if (x->dense) {
    // wide outputs: the mask in the nibble layout too (one pass over the bitmap; the wide
    // kernels then read one word per row and 4 steps, and the backward reuses it)
    const uint64_t *mw = mask && x->maskW ? x->maskW.get() : nullptr;
    if (mw)
      launch_mask_nibbles(mask, base, x->cols, x->rows, x->cols, x->maskW.get(), s.get());
    launch_gemm_nn(x->rows, b->cols, x->cols, x->x.get(), x->ldx, b->dev_data.get(), b->ld, 0,
                   c->dev_data.get(), c->ld, mask, base, x->cols, scale, s.get(), mw);
  } else {
    launch_spmm_csr(x->rows, b->cols, c->ld, x->indptr.get(), x->indices.get(), x->values.get(),
                    mask, base, scale, b->dev_data.get(), c->dev_data.get(), s.get());
  }
}

void SparseMatmul::backward(const Stream &s) const {
  // b.grad = drop(X)^T * c.grad  (the dropped X of the last training forward)
  const uint64_t *mask = last_training ? drop->state().mask.get() : nullptr;
  const long long base = drop->state().mask_base;
  const float scale = drop->scale();
  MmProfile prof(ctx, s.get(), x->dense ? 2.0 * x->rows * b->cols * x->cols : 0.0);
  if (x->dense && x->maskT) {  // the mask of the last training forward (flat or nibbles)
    const bool flat = mask && xs_flat(x);
    const XsMask fm{mask, base, x->cols, (long long)drop->state().mask.size()};
    launch_xstream_tn(x->rows, b->cols, x->cols, x->x.get(), x->ldx, c->dev_grad.get(), c->ld,
                      b->dev_grad.get(), b->ld, mask && !flat ? x->maskT.get() : nullptr, scale,
                      ctx->gemm_workspace, s.get(), flat ? &fm : nullptr);
  } else if (x->dense) {
    launch_gemm_tn(x->rows, b->cols, x->cols, x->x.get(), x->ldx, c->dev_grad.get(), c->ld,
                   b->dev_grad.get(), b->ld, mask, base, x->cols, scale, ctx->gemm_workspace,
                   s.get(), mask && x->maskW ? x->maskW.get() : nullptr);
  } else {
    launch_spmm_csc_bwd(x->cols, b->cols, c->ld, x->csc_ptr.get(), x->csc_row.get(),
                        x->csc_pos.get(), x->values.get(), mask, base, scale, c->dev_grad.get(),
                        b->dev_grad.get(), s.get(), x->nnz, x->csc_order.get(), g_csc_tree != 0);
  }
}

// ------------------------------------------------------------------------------------------
// GraphSum (src/module.cu:168-210; hpdga module.cpp:82-111)
// ------------------------------------------------------------------------------------------
GraphSum::GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevGraph *graph_,
                   int dim_, ModuleContext *ctx_, bool last_layer_)
    : in(std::move(in_)), out(std::move(out_)), graph(graph_), dim(dim_), ctx(ctx_),
      last_layer(last_layer_) {
  if (ctx->comm && ctx->comm->world() > 1) {  // (one rank sums straight into `out`)
    for (DevGraph *gk : ctx->chunk_graphs) {
      partial.emplace_back();
      partial.back().allocate((size_t)gk->rows() * out->ld);
      partial.back().zero();
      computed.push_back(Event::create());
    }
    reduced = Event::create();
  }
}

DevGraph *GraphSum::forward_graph() const {
  if (ctx->comm) return nullptr;
  return last_layer && ctx->split_graph ? ctx->split_graph : graph;
}

DevGraph *GraphSum::backward_graph() const {
  if (ctx->comm) return nullptr;
  return last_layer && ctx->split_colgraph ? ctx->split_colgraph : graph;
}

// the graph whose prescaled input table this module's next forward / backward reads first
// (edge-cut: row chunk 0's, which the other chunks share)
DevGraph *GraphSum::forward_table_graph() const {
  if (!ctx->comm) return forward_graph();
  if (last_layer && !ctx->chunk_split_graphs.empty()) return nullptr;
  return ctx->chunk_graphs.empty() ? nullptr : ctx->chunk_graphs[0];
}

DevGraph *GraphSum::backward_table_graph() const {
  if (!ctx->comm) return backward_graph();
  if (last_layer && !ctx->chunk_col_graphs.empty()) return ctx->chunk_col_graphs[0];
  return ctx->chunk_graphs.empty() ? nullptr : ctx->chunk_graphs[0];
}

float4 *GraphSum::claim_forward_table(int rows, int ld, const float **scale) const {
  DevGraph *g = forward_table_graph();
  if (!g || !(g_fuse_epilogue & kFusePrestage) || dim != 16 || in->ld != 16 || ld != 16 || g->cols() != rows)
    return nullptr;
  float *t = g->ring_table(dim, scale);
  if (!t) return nullptr;
  prestaged_fwd = true;
  return reinterpret_cast<float4 *>(t);
}

bool GraphSum::claim_backward_table(int rows, int ld, XentTable *t) const {
  if (ctx->comm || !(g_fuse_epilogue & kFusePrestage) || dim != 16 || ld != 16 ||
      out->ld != 16 || out->rows != rows)
    return false;
  DevGraph *g = backward_graph();
  const float *sc = nullptr;
  const int *pos = nullptr;
  int pos_rows = 0;
  float *tab = g ? g->ring_table_mapped(dim, &sc, &pos, &pos_rows) : nullptr;
  if (!tab || pos_rows != rows) return false;
  t->table = tab;
  t->scale = sc;
  t->pos = pos;
  t->rows = pos_rows;
  prestaged_bwd = true;
  return true;
}

void GraphSum::stage_next(GsEpilogue &e, GraphSum *next, DevGraph *ng, bool fwd) const {
  if (!next || !ng || !(g_fuse_epilogue & kFusePrestage)) return;
  const float *sc = nullptr;
  float *t = ng->ring_table(next->dim, &sc);
  if (!t) return;
  e.next_table = reinterpret_cast<float4 *>(t);
  e.next_scale = sc;
  e.next_sr = RING_SR;
  (fwd ? next->prestaged_fwd : next->prestaged_bwd) = true;
}

// Where this GraphSum's fused tails can run: in the kernel that forms the final rows (one
// GPU: `g`'s combine), or (edge-cut) in k_gs_finish on this rank's rows once the
// reduce-scatter has summed them
bool GraphSum::tail_ok(const DevGraph *g, int ld_in, int ld_out) const {
  if (ctx->comm) {
    if (dim % 4 != 0 || ld_out % 4 != 0) return false;
    if (ctx->comm->world() > 1) return true;
    // one rank: run() hands the tail to the column block's own GraphSum (its combine)
    const DevGraph *cg = g ? g : (ctx->chunk_graphs.empty() ? nullptr : ctx->chunk_graphs[0]);
    return cg && cg->epilogue_ok(dim, ld_in, ld_out);
  }
  return g && g->epilogue_ok(dim, ld_in, ld_out);
}

// The fused forward tail: ReLU on `out` (its mask when training), then the hidden Dropout
// (training), both skipped as modules for this pass.  mode 0 when `g` cannot take an epilogue.
GsEpilogue GraphSum::forward_epilogue(bool training, const Stream &s, const DevGraph *g) const {
  GsEpilogue e;
  if (!fwd_relu || !tail_ok(g, in->ld, out->ld)) return e;
  e.mode = 1;
  e.relu_mask = training ? fwd_relu->mask_ptr() : nullptr;
  e.relu_ld = out->ld;
  if (training && fwd_drop) {
    fwd_drop->draw_fused(s.get());
    const DropoutRng &r = fwd_drop->state();
    e.drop_mask = r.mask.get();
    e.drop_base = r.mask_base;
    e.drop_cols = out->cols;
    e.drop_scale = fwd_drop->scale();
  }
  fwd_relu->skip_forward = true;
  if (fwd_next) stage_next(e, fwd_next, fwd_next->forward_table_graph(), true);
  return e;
}

// The fused backward tail: the Dropout backward on in.grad (mask of the last training
// forward), then the ReLU backward, both skipped as modules for this pass.
GsEpilogue GraphSum::backward_epilogue(const DevGraph *g) const {
  GsEpilogue e;
  if (!bwd_relu || !tail_ok(g, out->ld, in->ld)) return e;
  e.mode = 2;
  e.relu_mask = bwd_relu->mask_ptr();
  e.relu_ld = in->ld;
  if (bwd_drop) {
    const DropoutRng &r = bwd_drop->state();
    e.drop_mask = r.mask.get();
    e.drop_base = r.mask_base;
    e.drop_cols = in->cols;
    e.drop_scale = bwd_drop->scale();
    bwd_drop->skip_backward = true;
  }
  bwd_relu->skip_backward = true;
  if (bwd_next) stage_next(e, bwd_next, bwd_next->backward_table_graph(), false);
  return e;
}

void GraphSum::run(const float *src, float *dst, const Stream &s, int mode,
                   const GsEpilogue *epi, bool prestaged) const {
  if (ctx->comm && !ctx->tail_stream) {
    // the last eval pass's tail (eval_tail) still reads the partial buffer and its slots: every
    // collective entry waits for it (Comm::enter; the weight-gradient all-reduce and the loss
    // pair's too)
    ctx->comm->enter(s.get());
    ctx->tail_pending = false;
  }
  Event e0, e1;
  if (ctx->profile) {
    e0 = Event::create(true);
    e1 = Event::create(true);
    e0.record(s.get());
  }
  double bytes = 0;
  const std::vector<DevGraph *> &cgs = mode == 2 ? ctx->chunk_col_graphs : ctx->chunk_graphs;
  if (ctx->comm && ctx->comm->world() == 1 && cgs.size() == 1 && mode != 1) {
    // one rank: its column block is all of Â and the reduce-scatter would be a copy -- the
    // block's sums are final, formed with the tail in the combine as on one GPU
    cgs[0]->graphsum(src, in->ld, dst, out->ld, dim, s.get(), false, epi, prestaged);
    bytes = cgs[0]->algorithmic_bytes(dim);
    if (ctx->profile) e1.record(s.get());
  } else if (ctx->comm && partial.empty()) {
    // one rank, the split's rows only (split_rows): their sums scattered straight into `out`
    // (the other rows keep their last values, as the partials' do at world > 1)
    DevGraph *sk = ctx->chunk_split_graphs[0];
    if (sk->rows() > 0) {
      const size_t need = (size_t)sk->rows() * out->ld;
      if (compact.size() < need) compact.allocate(need);
      sk->graphsum(src, in->ld, compact.get(), out->ld, dim, s.get());
      launch_scatter_rows(compact.get(), ctx->chunk_split_rows[0], sk->rows(), out->ld, dst,
                          s.get());
      bytes = sk->algorithmic_bytes(dim);
    }
    if (ctx->profile) e1.record(s.get());
  } else if (ctx->comm && mode != 1 && ctx->chunk_graphs.size() == 1 &&
             dynamic_cast<PeerComm *>(ctx->comm) && cgs[0]->uses_lds(dim)) {
    // Peer-mapped exchange (PeerComm, k_peer.hip): the ring sums of every padded row from this
    // rank's columns, combined over the column blocks and pushed straight into each owner's
    // receive slot of this rank (k_gs_lds_combine's push mode, over xGMI); then the wait for
    // every rank's push and one kernel that sums the W slots of this rank's rows in rank order
    // and applies the fused tail (k_gs_gather_finish).  No partial buffer, no reduce-scatter.
    auto *pc = static_cast<PeerComm *>(ctx->comm);
    DevGraph *gk = cgs[0];
    const int h = out->rows;  // padded rows per rank (one chunk)
    // eval_tail: this call's push, wait and sum on the tail stream (the eval pass's last
    // GraphSum); any other call first waits for the last tail (partial buffer, slot parity)
    hipStream_t ts = s.get();
    if (ctx->tail_stream && dim <= 16) {
      ts = ctx->tail_stream;
      ctx->tail_used = true;
    }
    PeerSink k = pc->sink(h, (size_t)out->ld);
    pc->note((size_t)h * out->ld * ctx->comm->world() * sizeof(float), 1.0);
    gk->graphsum(src, in->ld, nullptr, out->ld, dim, s.get(), false, nullptr, prestaged, false, &k,
                 ts != s.get() ? ts : nullptr, ctx->tail_fork.get());
    bytes = gk->algorithmic_bytes(dim);
    pc->wait(ts);
    launch_gs_gather_finish(dst, out->ld, ctx->local_rows, (dim + 3) / 4 * 4,
                            epi && epi->mode ? *epi : GsEpilogue{}, pc->recv(), ts);
    if (ctx->profile) e1.record(ts);
  } else if (ctx->comm) {
    // Per row chunk: partial sums of the chunk's (padded) rows from this rank's columns on
    // the compute stream, then its reduce-scatter on the comm stream, which hands every rank
    // its own rows of the chunk while the next chunk is summed.  The chunks share one
    // prescaled table of this rank's columns (DevGraph::share_tables): prescaled once, by
    // the producer's epilogue (prestaged) or by chunk 0's call.
    const size_t h = (size_t)out->rows / ctx->chunk_graphs.size();
    for (size_t k = 0; k < ctx->chunk_graphs.size(); k++) {
      if (mode == 1) {
        // only the split's rows of the chunk; the chunk's other partial rows keep their last
        // values (finite), which reach only rows the loss skips and whose loss gradient is 0
        DevGraph *sk = ctx->chunk_split_graphs[k];
        if (sk->rows() > 0) {
          const size_t need = (size_t)sk->rows() * out->ld;
          if (compact.size() < need) compact.allocate(need);
          sk->graphsum(src, in->ld, compact.get(), out->ld, dim, s.get());
          launch_scatter_rows(compact.get(), ctx->chunk_split_rows[k], sk->rows(), out->ld,
                              partial[k].get(), s.get());
          bytes += sk->algorithmic_bytes(dim);
        }
      } else {
        DevGraph *gk = cgs[k];
        const bool shared = k > 0 && gk->table_owner() == cgs[0] && gk->can_share_tables(dim, in->ld);
        gk->graphsum(src, in->ld, partial[k].get(), out->ld, dim, s.get(), false, nullptr,
                     k == 0 && prestaged, shared);
        bytes += gk->algorithmic_bytes(dim);
      }
      if (ctx->chunk_graphs.size() == 1) {
        // one chunk: nothing to overlap -- the reduce-scatter follows on the compute stream
        // (two cross-stream hand-offs per GraphSum cost ~10 us each on the rank epoch)
        ctx->comm->reduce_scatter_sum(partial[k].get(), dst, h * out->ld, s.get());
        continue;
      }
      computed[k].record(s.get());
      computed[k].wait_on(ctx->comm_stream);
      ctx->comm->reduce_scatter_sum(partial[k].get(), dst + k * h * out->ld, h * out->ld,
                                    ctx->comm_stream);
    }
    if (ctx->chunk_graphs.size() > 1) {
      reduced.record(ctx->comm_stream);
      reduced.wait_on(s.get());  // dst complete, partials free for the next call
    }
    // the fused tail on this rank's rows of the summed output (padding rows stay zero)
    if (epi && epi->mode) launch_gs_finish(dst, out->ld, ctx->local_rows, dim, *epi, s.get());
    if (ctx->profile) e1.record(s.get());
  } else {
    graph->graphsum(src, in->ld, dst, out->ld, dim, s.get(), false, epi, prestaged);
    bytes = graph->algorithmic_bytes(dim);
    if (ctx->profile) e1.record(s.get());
  }
  if (ctx->profile) {
    ctx->gs_events->emplace_back(e0, e1);
    ctx->gs_bytes->push_back(bytes);
  }
}

void GraphSum::forward(bool training, const Stream &s) const {
  const bool pre = prestaged_fwd;  // this call's input table was written by the producer
  prestaged_fwd = false;
  PGCN_CHECK(!pre || ((training || !first_layer) &&
                      !(last_layer && ctx->comm && !ctx->chunk_split_graphs.empty())),
             PGCN_E_INVALID, "graphsum: prestaged input on a path that does not read it");
  if (!training && first_layer) return;  // eval_ax: SparseMatmul wrote Â X W1 already
  if (last_layer && ctx->comm && !ctx->chunk_split_graphs.empty()) {
    run(in->dev_data.get(), out->dev_data.get(), s, 1);
    return;
  }
  DevGraph *sg = last_layer && !ctx->comm ? ctx->split_graph : nullptr;
  if (!sg) {
    const GsEpilogue epi = forward_epilogue(training, s, graph);
    run(in->dev_data.get(), out->dev_data.get(), s, 0, &epi, pre);
    return;
  }
  // output layer: only the split's labelled rows, summed compactly and scattered to their
  // rows; the other rows keep their last (finite) values, which meet only zero loss-gradient
  // rows in Matmul::backward and are skipped by the loss
  float *dst;
  if (ctx->compact_n) {  // the output Matmul and the loss read the compact rows themselves
    dst = ctx->compact_z->dev_data.get();
  } else {
    const size_t need = (size_t)std::max(sg->rows(), 1) * out->ld;
    if (compact.size() < need) compact.allocate(need);
    dst = compact.get();
  }
  Event e0, e1;
  if (ctx->profile) {
    e0 = Event::create(true);
    e1 = Event::create(true);
    e0.record(s.get());
  }
  sg->graphsum(in->dev_data.get(), in->ld, dst, out->ld, dim, s.get(), false, nullptr, pre);
  if (ctx->profile) {
    e1.record(s.get());
    ctx->gs_events->emplace_back(e0, e1);
    ctx->gs_bytes->push_back(sg->algorithmic_bytes(dim));
  }
  if (!ctx->compact_n)
    launch_scatter_rows(dst, ctx->split_rows, sg->rows(), out->ld, out->dev_data.get(), s.get());
}

void GraphSum::backward(const Stream &s) const {
  // the same gather on grads (Â symmetric): in.grad = Â out.grad (module.cpp:98-111)
  const bool pre = prestaged_bwd;  // out.grad's input table was written by its producer
  prestaged_bwd = false;
  if (last_layer && ctx->comm && !ctx->chunk_col_graphs.empty()) {
    // edge-cut: out.grad is zero outside the training split's rows, so each chunk graph keeps
    // only the edges from those columns (all rows stay: the partials are written whole)
    const GsEpilogue epi = backward_epilogue(ctx->chunk_col_graphs[0]);
    run(out->dev_grad.get(), in->dev_grad.get(), s, 2, &epi, pre);
    return;
  }
  DevGraph *cg = last_layer && !ctx->comm ? ctx->split_colgraph : nullptr;
  if (!cg) {
    const GsEpilogue epi = backward_epilogue(graph);
    run(out->dev_grad.get(), in->dev_grad.get(), s, 0, &epi, pre);
    return;
  }
  // output layer: out.grad is the loss gradient, zero outside the split's labelled rows, so
  // only the edges into those rows contribute (the column-subset graph gathers them itself)
  Event e0, e1;
  if (ctx->profile) {
    e0 = Event::create(true);
    e1 = Event::create(true);
    e0.record(s.get());
  }
  // (compact: the Matmul left out.grad in compact rows, which the column-subset graph reads
  // as its columns directly; else it gathers them from the full rows)
  const float *g_in = ctx->compact_n ? ctx->compact_z->dev_grad.get() : out->dev_grad.get();
  const GsEpilogue epi = backward_epilogue(cg);
  cg->graphsum(g_in, out->ld, in->dev_grad.get(), in->ld, dim, s.get(), ctx->compact_n > 0, &epi,
               pre);
  if (ctx->profile) {
    e1.record(s.get());
    ctx->gs_events->emplace_back(e0, e1);
    ctx->gs_bytes->push_back(cg->algorithmic_bytes(dim));
  }
}

// ------------------------------------------------------------------------------------------
// ReLU (src/module.cu:215-265)
// ------------------------------------------------------------------------------------------
ReLU::ReLU(shared_ptr<Variable> in_) : in(std::move(in_)) {
  mask.allocate((size_t)in->rows * in->ld);
  mask.zero();
}

void ReLU::forward(bool training, const Stream &s) const {
  if (skip_forward) {  // applied by the GraphSum before it (epilogue)
    skip_forward = false;
    return;
  }
  launch_relu_fwd(in->dev_data.get(), (long long)in->rows * in->ld, mask.get(), training, s.get());
}

void ReLU::backward(const Stream &s) const {
  if (skip_backward) {  // applied by the GraphSum backward before it (epilogue)
    skip_backward = false;
    return;
  }
  launch_relu_bwd(in->dev_grad.get(), (long long)in->rows * in->ld, mask.get(), s.get());
}

// ------------------------------------------------------------------------------------------
// Matmul (src/module.cu:270-472; hpdga module.cpp:13-38)
// ------------------------------------------------------------------------------------------
Matmul::Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               int m_, int n_, int p_, ModuleContext *ctx_)
    : a(std::move(a_)), b(std::move(b_)), c(std::move(c_)), m(m_), n(n_), p(p_), ctx(ctx_) {}

void Matmul::forward(bool training, const Stream &s) const {
  if (fused_forward && !(last_layer && ctx->compact_n)) return;  // CrossEntropyLoss::forward
  const bool cmp = last_layer && ctx->compact_n;  // compact output layer: the split's rows
  const Variable &A = cmp ? *ctx->compact_z : *a, &C = cmp ? *ctx->compact_out : *c;
  MmProfile prof(ctx, s.get(), 2.0 * (cmp ? ctx->compact_n : m) * p * n);
  launch_gemm_nn(cmp ? ctx->compact_n : m, p, n, A.dev_data.get(), A.ld, b->dev_data.get(), b->ld,
                 0, C.dev_data.get(), C.ld, nullptr, 0, 0, 1.0f, s.get());
}

void Matmul::backward_input(const Stream &s) const {
  launch_gemm_nn(m, n, p, c->dev_grad.get(), c->ld, b->dev_data.get(), b->ld, 1, a->dev_grad.get(),
                 a->ld, nullptr, 0, 0, 1.0f, s.get());
}

void Matmul::backward_weight(hipStream_t s, void *ws) const {
  launch_gemm_tn(m, p, n, a->dev_data.get(), a->ld, c->dev_grad.get(), c->ld, b->dev_grad.get(),
                 b->ld, nullptr, 0, 0, 1.0f, ws, s);
}

void Matmul::backward(const Stream &s) const {
  const bool cmp = last_layer && ctx->compact_n;
  const bool a_done = input_grad_done && !cmp;  // a.grad written by the loss kernel (forward)
  const bool b_done = weight_grad_done && !cmp;  // b.grad too
  input_grad_done = weight_grad_done = false;
  const Variable &A = cmp ? *ctx->compact_z : *a, &C = cmp ? *ctx->compact_out : *c;
  const int rows = cmp ? ctx->compact_n : m;
  const bool side = ctx->mm_side && ctx->side_stream && ctx->gemm_workspace_side && !ctx->profile;
  // (the contractions the loss kernel did are profiled there; a side-stream b.grad is not)
  MmProfile prof(ctx, s.get(), 2.0 * rows * p * n * ((a_done ? 0 : 1) + (side || b_done ? 0 : 1)));
  if (side) {
    // b.grad = a^T * c.grad on the side stream, from here (a.data and c.grad are final; nothing
    // later in the backward pass writes them), joined before the optimizer (GCN)
    ctx->mm_fork.record(s.get());
    ctx->mm_fork.wait_on(ctx->side_stream);
    launch_gemm_tn(rows, p, n, A.dev_data.get(), A.ld, C.dev_grad.get(), C.ld, b->dev_grad.get(),
                   b->ld, nullptr, 0, 0, 1.0f, ctx->gemm_workspace_side, ctx->side_stream);
    ctx->side_pending = true;
  }
  // a.grad = c.grad * b^T   (b stored [n][p] => trans_b); the Dropout / ReLU backward on a
  // in its final write when gemm_nn would take k_xstream_nn anyway (same product, same bits)
  if (!a_done && bwd_relu && !cmp && A.ld == n && xstream_ok(n, p) && !xstream_ring_ok(p, C.ld)) {
    XsEpilogue e;
    if (bwd_drop) {
      e.bwd_drop = bwd_drop->state().mask.get();
      e.drop_base = bwd_drop->state().mask_base;
      e.drop_scale = bwd_drop->scale();
      bwd_drop->skip_backward = true;
    }
    e.bwd_relu = bwd_relu->mask_ptr();
    bwd_relu->skip_backward = true;
    launch_xstream_nn(rows, n, p, C.dev_grad.get(), C.ld, b->dev_data.get(), b->ld, 1,
                      A.dev_grad.get(), A.ld, nullptr, 1.0f, s.get(), nullptr, &e);
  } else if (!a_done) {
    launch_gemm_nn(rows, n, p, C.dev_grad.get(), C.ld, b->dev_data.get(), b->ld, 1,
                   A.dev_grad.get(), A.ld, nullptr, 0, 0, 1.0f, s.get());
  }
  // b.grad = a^T * c.grad (deterministic split-M reduction)
  if (!side && !b_done)
    launch_gemm_tn(rows, p, n, A.dev_data.get(), A.ld, C.dev_grad.get(), C.ld, b->dev_grad.get(),
                   b->ld, nullptr, 0, 0, 1.0f, ctx->gemm_workspace, s.get());
}

// ------------------------------------------------------------------------------------------
// CrossEntropyLoss (src/module.cu:477-562; hpdga module.cpp:122-156)
// ------------------------------------------------------------------------------------------
CrossEntropyLoss::CrossEntropyLoss(shared_ptr<Variable> logits_, int num_classes_,
                                   ModuleContext *ctx_)
    : logits(std::move(logits_)), num_classes(num_classes_), ctx(ctx_) {}

// The fused loss kernel also writes the output layer's input grad (on MFMA in k_xstream_nn's
// sequence: bit-identical; reddit A/B 517.7 -> 520.1 epochs/s) and, at fuse_output >= 2,
// per-block partials of the Matmul's weight grad, reduced in block order right after it
// (deterministic; the same sums as k_gemm_tn's in another grouping): 2 on graphs of >= 65,536
// rows (small graphs keep k_gemm_tn's order: nothing to gain there), 3 on any graph

void CrossEntropyLoss::forward(bool training, const Stream &s) const {
  if (fused && !ctx->compact_n) {
    const Variable &Hv = *fused->input(), &Wv = *fused->weight();
    // the fused output layer's contractions (logits = H W; training: dH = dOut W^T and the
    // W.grad partials) over the fused kernel's time, which includes the loss itself
    const double mm = 2.0 * logits->rows * num_classes * fused->inner();
    MmProfile prof(ctx, s.get(), training ? 3.0 * mm : mm);
    float *dH = Hv.dev_grad ? Hv.dev_grad.get() : nullptr;
    const int nb = xent_blocks(logits->rows);
    float *dWp = nullptr;
    bool deferred = false;
    // (an edge-cut rank's rows are a slice of a large graph: the block partials too)
    if (training && g_fuse_output >= 2 &&
        (g_fuse_output == 3 || logits->rows >= 65536 || ctx->comm) &&
        Wv.dev_grad && logits->ld <= 48 &&
        !ctx->mm_side &&
        tn_reduce_blocks_workspace(nb, fused->inner(), 48) <= ctx->gemm_workspace_bytes)
      dWp = static_cast<float *>(ctx->gemm_workspace);
    // r06: a small graph's partials straight into the deferred-reduction pool when tn_fold is
    // on (the Adam launch sums them in block order): the output layer's W.grad needs no launch
    // of its own (k_xstream_tn before; the same sums in another grouping)
    // (tn_fold 0, or no room: the same one ordered pass as its own launch -- the same bits)
    bool one_pass = false;
    if (training && !dWp && g_fuse_output >= 2 && g_defer_small_wgrad && !ctx->comm &&
        nb <= kDeferWgradMaxBlocks && Wv.dev_grad && logits->ld <= 48 && !ctx->mm_side) {
      dWp = tn_defer_blocks(nb, fused->inner(), num_classes, 48, Wv.dev_grad.get(), Wv.ld);
      deferred = dWp != nullptr;
      if (!dWp && (size_t)nb * fused->inner() * 48 * sizeof(float) <= ctx->gemm_workspace_bytes) {
        dWp = static_cast<float *>(ctx->gemm_workspace);
        one_pass = true;
      }
    }
    // training: dH also to the ring table of the GraphSum backward that reads it
    XentTable tb;
    const bool staged = training && dH && dh_reader && fused->inner() == 16 &&
                        dh_reader->claim_backward_table(Hv.rows, Hv.ld, &tb);
    launch_out_xent(Hv.dev_data.get(), Hv.ld, fused->inner(), Wv.dev_data.get(), Wv.ld,
                    logits->dev_data.get(), logits->ld, training ? logits->dev_grad.get() : nullptr,
                    ctx->truth, logits->rows, num_classes, ctx->count, training ? 1 : 0,
                    ctx->xent_partials, s.get(), dH, Hv.ld, dWp, staged ? &tb : nullptr, ctx->fin);
    ctx->fin_taken = ctx->fin != nullptr;
    if (one_pass)
      launch_tn_reduce_one_pass(dWp, nb, fused->inner(), num_classes, 48, Wv.dev_grad.get(),
                                Wv.ld, s.get());
    else if (dWp && !deferred)
      launch_tn_reduce_blocks(dWp, nb, fused->inner(), num_classes, 48, Wv.dev_grad.get(), Wv.ld,
                              s.get());
    fused->input_grad_done = training && dH;
    fused->weight_grad_done = dWp != nullptr;
    return;
  }
  const Variable &L = ctx->compact_n ? *ctx->compact_out : *logits;
  launch_xent_fwd(L.dev_data.get(), L.ld, training ? L.dev_grad.get() : nullptr,
                  ctx->compact_n ? ctx->compact_truth : ctx->truth,
                  ctx->compact_n ? ctx->compact_n : logits->rows, num_classes, ctx->count,
                  training ? 1 : 0, ctx->xent_partials, s.get(), ctx->compact_n ? 0 : 1,
                  ctx->fin);
  ctx->fin_taken = ctx->fin != nullptr;
}

void CrossEntropyLoss::backward(const Stream &) const {}  // module.cpp:155-156

}  // namespace pgcn
