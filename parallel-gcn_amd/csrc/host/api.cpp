// parallel-gcn_amd/csrc/host/api.cpp -- the reference-shaped C++ API (include/pgcn.hpp) on top
// of the engine's modules (host/module.*), GCN (host/gcn.*) and loader (host/data.*).
//
// One process-wide context plays the part of the reference's static state (Variable's random
// states, include/variable.cuh:13-14) and of the per-GCN buffers its modules share: the
// xorshift128+ stream (glorot draws, then the dropouts' positions), the CE partials, the GEMM
// workspace and the engine's ModuleContext.
#include "../../../include/pgcn.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "../kernels.hpp"
#include "../rng.hpp"
#include "data.hpp"
#include "gcn.hpp"
#include "graph.hpp"
#include "module.hpp"

namespace pgcn {
namespace api {

namespace {

std::vector<int> to_int(const std::vector<natural> &v) { return std::vector<int>(v.begin(), v.end()); }

struct Context {
  ModuleContext ctx;
  Stream stream;  // default stream of Adam::step() and of host-side helpers
  DeviceBuffer<float> xent_partials, sums, out2;
  int xent_rows = 0;
  DeviceBuffer<float> gemm_ws;
  size_t ws_bytes = 0;
  DeviceBuffer<uint8_t> jump_table;
  uint64_t seed[2] = {0, 0};  // the stream's initial state (initialize_random)
  uint64_t state[2] = {0, 0};  // its current state (glorot draws advance it)
  bool seeded = false;
  unsigned long long glorot_draws = 0;
  std::vector<Dropout::Impl *> dropouts;  // construction order = the stream's dropout order
  bool frozen = false;

  Context() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
      throw Error(PGCN_E_NODEVICE, "no HIP device visible: the engine has no CPU fallback");
    stream = Stream::create();
    sums.allocate(4);
    out2.allocate(2);
    ctx.train_ahead = false;
  }
  void ensure_seeded() {
    if (seeded) return;
    pgcn_rng_seed(seed);
    state[0] = seed[0];
    state[1] = seed[1];
    seeded = true;
  }
  void ensure_ws(size_t bytes) {
    if (bytes <= ws_bytes) return;
    gemm_ws.allocate(bytes / sizeof(float) + 64);
    ws_bytes = bytes;
    ctx.gemm_workspace = gemm_ws.get();
  }
  void ensure_xent(int rows) {
    if (rows <= xent_rows) return;
    xent_partials.allocate((size_t)xent_blocks(rows) * 2 + 2);
    xent_rows = rows;
  }
  void freeze();
};

Context &context() {
  static Context *c = new Context();  // lives to process exit (modules hold pointers into it)
  return *c;
}

}  // namespace

// ---------------------------------------------------------------------- streams, events
smart_stream::smart_stream() {
  auto st = std::make_shared<Stream>(Stream::create());
  s_ = st->get();
  own_ = st;
}
smart_stream::smart_stream(hipStream_t borrowed) : s_(borrowed) {}
void smart_stream::sync() const { PGCN_HIP(hipStreamSynchronize(s_)); }

smart_event::smart_event() {
  auto ev = std::make_shared<Event>(Event::create());
  e_ = ev->get();
  own_ = ev;
}
void smart_event::record(const smart_stream &s) const {
  hipEvent_t ev = e_;  // (PGCN_HIP declares its own e_)
  PGCN_HIP(hipEventRecord(ev, s.get()));
}
void smart_event::wait(const smart_stream &s) const {
  hipEvent_t ev = e_;
  PGCN_HIP(hipStreamWaitEvent(s.get(), ev, 0));
}

// ---------------------------------------------------------------------- Variable
struct VariableAccess {
  // node matrix [rows][round_up4(cols)] (modules), or exactly [rows][cols] (weights)
  static void bind(Variable &v, int rows, int cols, bool padded) {
    const int ld = padded ? round_up4(cols) : cols;
    if (v.impl_) {
      PGCN_CHECK(v.impl_->rows == rows && v.impl_->cols == cols, PGCN_E_INVALID,
                 "Variable: used with two different shapes");
      return;
    }
    PGCN_CHECK((long long)rows * cols == (long long)v.size, PGCN_E_INVALID,
               "Variable: rows * cols != size");
    v.impl_ = std::make_shared<pgcn::Variable>(rows, cols, v.requires_grad_, ld);
    v.rows = (natural)rows;
    v.cols = (natural)cols;
    v.ld = (natural)ld;
    v.dev_data.p = v.impl_->dev_data.get();
    v.dev_grad.p = v.impl_->dev_grad.get();
  }
  static void bind_flat(Variable &v) {  // a variable no module has shaped: [1][size]
    if (!v.impl_) bind(v, 1, (int)v.size, false);
  }
};

Variable::Variable(natural size_, bool requires_grad, bool rand, natural rows_, natural cols_)
    : size(size_), requires_grad_(requires_grad) {
  (void)rand;  // the reference's flag allocates curand states; masks here come from the
               // shared xorshift stream
  (void)context();
  if (rows_ && cols_) VariableAccess::bind(*this, (int)rows_, (int)cols_, false);
}

void Variable::zero(const smart_stream &stream) const {
  VariableAccess::bind_flat(const_cast<Variable &>(*this));
  impl_->zero(stream.get());
}
void Variable::zero_grad(const smart_stream &stream) const {
  VariableAccess::bind_flat(const_cast<Variable &>(*this));
  impl_->zero_grad(stream.get());
}

void Variable::glorot() const {
  Context &c = context();
  PGCN_CHECK(!c.frozen, PGCN_E_INVALID,
             "Variable::glorot after the first training forward: the dropout stream positions "
             "are already fixed");
  PGCN_CHECK(rows && cols, PGCN_E_INVALID, "Variable::glorot needs rows and cols");
  c.ensure_seeded();
  std::vector<float> h((size_t)size);
  glorot_fill(h, (int)rows, (int)cols, c.state);
  c.glorot_draws += size;
  from_host(h);
}

void Variable::set_value(real value, const smart_stream &stream) const {
  VariableAccess::bind_flat(const_cast<Variable &>(*this));
  std::vector<float> h((size_t)impl_->rows * impl_->ld, 0.0f);
  for (int r = 0; r < impl_->rows; r++)
    for (int k = 0; k < impl_->cols; k++) h[(size_t)r * impl_->ld + k] = value;
  PGCN_HIP(hipMemcpyAsync(impl_->dev_data.get(), h.data(), h.size() * sizeof(float),
                          hipMemcpyHostToDevice, stream.get()));
  PGCN_HIP(hipStreamSynchronize(stream.get()));
}

std::vector<real> Variable::to_host(bool grad) const {
  VariableAccess::bind_flat(const_cast<Variable &>(*this));
  PGCN_HIP(hipDeviceSynchronize());
  return impl_->to_host(grad ? 1 : 0);
}

void Variable::from_host(const std::vector<real> &v) const {
  VariableAccess::bind_flat(const_cast<Variable &>(*this));
  PGCN_CHECK(v.size() == (size_t)size, PGCN_E_INVALID, "Variable::from_host: size");
  std::vector<float> h((size_t)impl_->rows * impl_->ld, 0.0f);
  for (int r = 0; r < impl_->rows; r++)
    std::memcpy(&h[(size_t)r * impl_->ld], &v[(size_t)r * impl_->cols],
                sizeof(float) * (size_t)impl_->cols);
  impl_->dev_data.upload(h);
}

void Variable::print(const std::string &what, natural col) const {
  const std::vector<real> h = to_host(what == "grad");
  for (size_t i = 0; i < h.size(); i++) {
    printf("%.5f ", h[i]);
    if (col && (i + 1) % col == 0) printf("\n");
  }
  printf("\n");
}

void Variable::save(const std::string &file_name, const std::string &what, natural col) const {
  const std::vector<real> h = to_host(what == "grad");
  std::ofstream f(file_name);
  PGCN_CHECK(f.good(), PGCN_E_IO, "Variable::save: cannot open " + file_name);
  for (size_t i = 0; i < h.size(); i++) {
    f << h[i] << ((col && (i + 1) % col == 0) ? "\n" : " ");
  }
}

void Variable::initialize_random(unsigned seed) {
  Context &c = context();
  PGCN_CHECK(!c.frozen, PGCN_E_INVALID, "initialize_random after the first training forward");
  if (seed) pgcn_rng_seed_glibc(seed, c.seed);
  else pgcn_rng_seed(c.seed);
  c.state[0] = c.seed[0];
  c.state[1] = c.seed[1];
  c.seeded = true;
  c.glorot_draws = 0;
}

// ---------------------------------------------------------------------- sparse index
DevSparseIndex::DevSparseIndex(const SparseIndex &sparse_index) : host_(sparse_index) {
  (void)context();
  indices_size = (natural)host_.indices.size();
  indptr_size = (natural)host_.indptr.size();
  struct Bufs {
    DeviceBuffer<int> indices, indptr;
  };
  auto b = std::make_shared<Bufs>();
  b->indices.allocate(std::max<size_t>(1, host_.indices.size()));
  b->indptr.allocate(std::max<size_t>(1, host_.indptr.size()));
  b->indices.upload(to_int(host_.indices));
  b->indptr.upload(to_int(host_.indptr));
  dev_indices.p = reinterpret_cast<natural *>(b->indices.get());
  dev_indptr.p = reinterpret_cast<natural *>(b->indptr.get());
  dev_ = b;
}

// One device graph per distinct value array (compared bit for bit, so NaNs compare equal to
// themselves), shared by the GraphSums built on it and freed with the last of them: the index
// keeps only weak references (entries whose graph is gone are dropped on lookup), so a
// program rebuilding GraphSums with changing values does not accumulate device graphs.
std::shared_ptr<DevGraph> DevSparseIndex::graph(const std::vector<real> &values) const {
  graphs_.erase(std::remove_if(graphs_.begin(), graphs_.end(),
                               [](const auto &gv) { return gv.second.expired(); }),
                graphs_.end());
  for (const auto &gv : graphs_)
    if (gv.first.size() == values.size() &&
        std::memcmp(gv.first.data(), values.data(), values.size() * sizeof(real)) == 0)
      if (auto g = gv.second.lock()) return g;
  const int n = (int)indptr_size - 1;
  PGCN_CHECK(n > 0 && values.size() == host_.indices.size(), PGCN_E_INVALID,
             "GraphSum: graph values must match the pattern");
  const std::vector<int> ip = to_int(host_.indptr), ix = to_int(host_.indices);
  auto g = std::make_shared<DevGraph>(n, n, ip.data(), ix.data(), values.data());
  // Â = D^-1/2 A D^-1/2 exactly (the parser's coefficients): the LDS path's factorisation
  // s_i s_j applies; any other values keep the per-edge kernels
  if (values == graph_coefs(n, ip.data(), ix.data())) {
    const std::vector<float> s = degree_scales(n, ip.data());
    g->set_scales(s, s);
  }
  graphs_.emplace_back(values, g);
  return g;
}

// ---------------------------------------------------------------------- modules
Module::~Module() {}

struct Dropout::Impl {
  shared_ptr<Variable> in;
  float p;
  long long elems;
  bool input = false;  // the input features' dropout (SparseMatmul applies its mask)
  shared_ptr<DropoutRng> rng = std::make_shared<DropoutRng>();
  std::unique_ptr<pgcn::Dropout> mod;
  pgcn::Dropout *module() {
    if (!mod) {
      if (!input) {
        PGCN_CHECK(in->impl() && in->impl()->ld == in->impl()->cols, PGCN_E_INVALID,
                   "Dropout: its variable needs a shape with cols % 4 == 0 (a module producing it "
                   "must be built first)");
      }
      mod = std::make_unique<pgcn::Dropout>(input ? nullptr : in->impl(), p, rng, &context().ctx);
    }
    return mod.get();
  }
};

// The first training forward fixes every Dropout's stream position: hpdga draws the glorot
// weights first, then per training pass one number per element of each dropout in module order.
void Context::freeze() {
  if (frozen) return;
  ensure_seeded();
  unsigned long long period = 0;
  for (auto *d : dropouts) period += (unsigned long long)d->elems;
  std::vector<uint64_t> table(16 * 256 * 2);
  xs_byte_tables(xs_jump_matrix(period), table.data());
  jump_table.allocate(table.size() * sizeof(uint64_t));
  jump_table.upload(reinterpret_cast<const uint8_t *>(table.data()), table.size() * sizeof(uint64_t));
  ctx.jump_table = jump_table.get();
  unsigned long long offset = glorot_draws;
  for (auto *d : dropouts) {
    init_dropout_rng_range(*d->rng, seed, offset, 0, d->elems);
    offset += (unsigned long long)d->elems;
  }
  frozen = true;
}

Dropout::Dropout(shared_ptr<Variable> in_, real p_) : impl_(std::make_shared<Impl>()) {
  Context &c = context();
  PGCN_CHECK(!c.frozen, PGCN_E_INVALID, "Dropout built after the first training forward");
  PGCN_CHECK(p_ >= 0.0f && p_ < 1.0f, PGCN_E_INVALID, "Dropout: p must be in [0, 1)");
  impl_->in = std::move(in_);
  impl_->p = p_;
  impl_->elems = (long long)impl_->in->size;
  c.dropouts.push_back(impl_.get());
}
Dropout::~Dropout() {
  auto &v = context().dropouts;
  for (size_t i = 0; i < v.size(); i++)
    if (v[i] == impl_.get()) v.erase(v.begin() + (long)i);
}
void Dropout::forward(bool training, const smart_stream &stream) const {
  if (!training) return;  // hpdga module.cpp:209
  context().freeze();
  impl_->module()->forward(true, Stream::wrap(stream.get()));
}
void Dropout::backward(const smart_stream &stream) const {
  if (impl_->input) return;  // the input has no gradient (module.cpp:222)
  impl_->module()->backward(Stream::wrap(stream.get()));
}

struct SparseMatmul::Impl {
  shared_ptr<Variable> a, b, c;
  DevSparseIndex *sp;
  int m, n, p;
  Dropout::Impl *drop = nullptr;
  // src/module.cu:124-160: the forward waits for the weight's optimizer step, the backward
  // signals that the input may be reset (set_input)
  bool events = false;
  smart_event start_matmul_forward, start_set_input;
  DevFeatures feats;
  std::unique_ptr<pgcn::SparseMatmul> mod;
  pgcn::SparseMatmul *module() {
    if (mod) return mod.get();
    // X from the input variable's values and the feature index (X is never rewritten here:
    // the dropout mask is applied on the fly)
    const std::vector<real> vals = a->to_host();
    const std::vector<int> ip = to_int(sp->host().indptr), ix = to_int(sp->host().indices);
    PGCN_CHECK((int)ip.size() == m + 1 && vals.size() == ix.size(), PGCN_E_INVALID,
               "SparseMatmul: feature index and values do not match m");
    bool dense = true;
    for (int i = 0; i < m && dense; i++) {
      dense = ip[(size_t)i + 1] - ip[(size_t)i] == n;
      for (int k = ip[(size_t)i]; k < ip[(size_t)i + 1] && dense; k++)
        dense = ix[(size_t)k] == k - ip[(size_t)i];
    }
    build_dev_features(feats, ip.data(), ix.data(), vals.data(), 0, m, n, dense, p);
    mod = std::make_unique<pgcn::SparseMatmul>(&feats, b->impl(), c->impl(), drop->module(),
                                               &context().ctx);
    return mod.get();
  }
};

SparseMatmul::SparseMatmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_,
                           shared_ptr<Variable> c_, DevSparseIndex *sp_, natural m_, natural n_,
                           natural p_, smart_event &start_matmul_forward_,
                           smart_event &start_set_input_)
    : SparseMatmul(std::move(a_), std::move(b_), std::move(c_), sp_, m_, n_, p_) {
  impl_->events = true;
  impl_->start_matmul_forward = start_matmul_forward_;
  impl_->start_set_input = start_set_input_;
}

SparseMatmul::SparseMatmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_,
                           shared_ptr<Variable> c_, DevSparseIndex *sp_, natural m_, natural n_,
                           natural p_)
    : impl_(std::make_shared<Impl>()) {
  Context &cx = context();
  Impl &I = *impl_;
  I.a = std::move(a_);
  I.b = std::move(b_);
  I.c = std::move(c_);
  I.sp = sp_;
  I.m = (int)m_;
  I.n = (int)n_;
  I.p = (int)p_;
  for (auto *d : cx.dropouts)
    if (d->in.get() == I.a.get()) I.drop = d;
  PGCN_CHECK(I.drop, PGCN_E_INVALID, "SparseMatmul: build the input features' Dropout first");
  I.drop->input = true;
  VariableAccess::bind(*I.b, I.n, I.p, false);
  VariableAccess::bind(*I.c, I.m, I.p, true);
  cx.ensure_ws(gemm_tn_workspace(I.m, I.p, I.n));
}
void SparseMatmul::forward(bool training, const smart_stream &stream) const {
  if (impl_->events) impl_->start_matmul_forward.wait(stream);
  impl_->module()->forward(training, Stream::wrap(stream.get()));
}
void SparseMatmul::backward(const smart_stream &stream) const {
  impl_->module()->backward(Stream::wrap(stream.get()));
  if (impl_->events) impl_->start_set_input.record(stream);
}

struct GraphSum::Impl {
  std::shared_ptr<pgcn::DevGraph> graph;  // kept alive as long as the module
  std::unique_ptr<pgcn::GraphSum> mod;
  // src/module.cu:200-207: the backward signals that the Matmul before it may compute its
  // weight gradient (its c.grad is complete)
  bool generate_event = false;
  smart_event start_matmul_backward;
};

GraphSum::GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevSparseIndex *graph_,
                   const real *dev_graph_value_, natural dim_, bool generate_event_,
                   smart_event &start_matmul_backward_)
    : GraphSum(std::move(in_), std::move(out_), graph_, dev_graph_value_, dim_) {
  impl_->generate_event = generate_event_;
  impl_->start_matmul_backward = start_matmul_backward_;
}

GraphSum::GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevSparseIndex *graph_,
                   const real *dev_graph_value_, natural dim_)
    : impl_(std::make_shared<Impl>()) {
  Context &cx = context();
  const int n = (int)graph_->indptr_size - 1, d = (int)dim_;
  VariableAccess::bind(*in_, n, d, true);
  VariableAccess::bind(*out_, n, d, true);
  std::vector<real> vals(graph_->indices_size);
  PGCN_HIP(hipMemcpy(vals.data(), dev_graph_value_, vals.size() * sizeof(real),
                     hipMemcpyDeviceToHost));
  impl_->graph = graph_->graph(vals);
  impl_->mod = std::make_unique<pgcn::GraphSum>(in_->impl(), out_->impl(), impl_->graph.get(), d,
                                                &cx.ctx);
}
void GraphSum::forward(bool training, const smart_stream &stream) const {
  impl_->mod->forward(training, Stream::wrap(stream.get()));
}
void GraphSum::backward(const smart_stream &stream) const {
  impl_->mod->backward(Stream::wrap(stream.get()));
  if (impl_->generate_event) impl_->start_matmul_backward.record(stream);
}

struct ReLU::Impl {
  std::unique_ptr<pgcn::ReLU> mod;
};
ReLU::ReLU(shared_ptr<Variable> in_) : impl_(std::make_shared<Impl>()) {
  PGCN_CHECK(in_->impl(), PGCN_E_INVALID, "ReLU: its variable has no shape yet (build the module "
                                          "producing it first)");
  impl_->mod = std::make_unique<pgcn::ReLU>(in_->impl());
}
void ReLU::forward(bool training, const smart_stream &stream) const {
  impl_->mod->forward(training, Stream::wrap(stream.get()));
}
void ReLU::backward(const smart_stream &stream) const {
  impl_->mod->backward(Stream::wrap(stream.get()));
}

struct Matmul::Impl {
  std::unique_ptr<pgcn::Matmul> mod;
  // src/module.cu:319-324, 431-472: the forward waits for the weight's optimizer step; the
  // backward computes a.grad on the backward stream and b.grad on the module's own stream once
  // event_backward (c.grad complete) has fired, through a workspace of its own
  bool events = false;
  smart_event event_forward, event_backward;
  smart_stream my_stream;
  DeviceBuffer<float> ws;
};
Matmul::Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               natural m_, natural n_, natural p_, smart_event &event_forward_,
               smart_event &event_backward_, const smart_stream &stream_)
    : Matmul(std::move(a_), std::move(b_), std::move(c_), m_, n_, p_) {
  Impl &I = *impl_;
  I.events = true;
  I.event_forward = event_forward_;
  I.event_backward = event_backward_;
  I.my_stream = stream_;
  I.ws.allocate(gemm_tn_workspace((int)m_, (int)p_, (int)n_) / sizeof(float) + 64);
}
Matmul::Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               natural m_, natural n_, natural p_)
    : impl_(std::make_shared<Impl>()) {
  Context &cx = context();
  const int m = (int)m_, n = (int)n_, p = (int)p_;
  VariableAccess::bind(*a_, m, n, true);
  VariableAccess::bind(*b_, n, p, false);
  VariableAccess::bind(*c_, m, p, true);
  cx.ensure_ws(gemm_tn_workspace(m, p, n));
  impl_->mod = std::make_unique<pgcn::Matmul>(a_->impl(), b_->impl(), c_->impl(), m, n, p, &cx.ctx);
}
void Matmul::forward(bool training, const smart_stream &stream) const {
  if (impl_->events) impl_->event_forward.wait(stream);
  impl_->mod->forward(training, Stream::wrap(stream.get()));
}
void Matmul::backward(const smart_stream &stream) const {
  Impl &I = *impl_;
  if (!I.events) {
    I.mod->backward(Stream::wrap(stream.get()));
    return;
  }
  I.mod->backward_input(Stream::wrap(stream.get()));
  I.event_backward.wait(I.my_stream);
  I.mod->backward_weight(I.my_stream.get(), I.ws.get());
}

struct CrossEntropyLoss::Impl {
  shared_ptr<Variable> logits;
  const integer *truth;
  real *loss;
  int classes;
  std::unique_ptr<pgcn::CrossEntropyLoss> mod;
  PinnedBuffer<float> res{2};
  // src/module.cu:526-548: a training forward signals start_backward once the loss gradient is
  // written; the backward stream waits for it
  bool events = false;
  smart_event start_backward;
};
CrossEntropyLoss::CrossEntropyLoss(shared_ptr<Variable> logits_, const integer *dev_truth_,
                                   real *loss_, natural num_classes_, smart_event &event)
    : CrossEntropyLoss(std::move(logits_), dev_truth_, loss_, num_classes_) {
  impl_->events = true;
  impl_->start_backward = event;
}
CrossEntropyLoss::CrossEntropyLoss(shared_ptr<Variable> logits_, const integer *dev_truth_,
                                   real *loss_, natural num_classes_)
    : impl_(std::make_shared<Impl>()) {
  Context &cx = context();
  PGCN_CHECK(logits_->impl() && logits_->impl()->cols == (int)num_classes_, PGCN_E_INVALID,
             "CrossEntropyLoss: logits need their [rows][num_classes] shape (build the module "
             "producing them first)");
  impl_->logits = std::move(logits_);
  impl_->truth = dev_truth_;
  impl_->loss = loss_;
  impl_->classes = (int)num_classes_;
  cx.ensure_xent(impl_->logits->impl()->rows);
  impl_->mod = std::make_unique<pgcn::CrossEntropyLoss>(impl_->logits->impl(), impl_->classes,
                                                        &cx.ctx);
}
void CrossEntropyLoss::set_num_samples(natural n) { num_samples = n; }
natural CrossEntropyLoss::get_num_samples() const { return num_samples; }
void CrossEntropyLoss::forward(bool training, const smart_stream &stream) const {
  Context &cx = context();
  const int rows = impl_->logits->impl()->rows;
  int count = (int)num_samples;
  if (count == 0) {  // as hpdga's loss (module.cpp:122-156): the rows whose truth is >= 0
    std::vector<int> t((size_t)rows);
    PGCN_HIP(hipStreamSynchronize(stream.get()));
    PGCN_HIP(hipMemcpy(t.data(), impl_->truth, t.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int x : t) count += x >= 0;
  }
  PGCN_CHECK(count > 0, PGCN_E_INVALID, "CrossEntropyLoss: no labelled rows");
  ModuleContext &m = cx.ctx;
  m.truth = impl_->truth;
  m.count = count;
  m.xent_partials = cx.xent_partials.get();
  m.xent_blocks = xent_blocks(rows);
  m.compact_n = 0;
  impl_->mod->forward(training, Stream::wrap(stream.get()));
  if (training && impl_->events) impl_->start_backward.record(stream);
  // mean loss and accuracy of the labelled rows (no weight decay term: GCN adds it)
  launch_reduce_scalars(cx.xent_partials.get(), m.xent_blocks, nullptr, 0, cx.sums.get(),
                        stream.get(), count, 0.0f, cx.out2.get());
  PGCN_HIP(hipMemcpyAsync(impl_->res.get(), cx.out2.get(), 2 * sizeof(float),
                          hipMemcpyDeviceToHost, stream.get()));
  if (impl_->loss)
    PGCN_HIP(hipMemcpyAsync(impl_->loss, cx.out2.get(), sizeof(float), hipMemcpyDeviceToHost,
                            stream.get()));
}
void CrossEntropyLoss::backward(const smart_stream &stream) const {
  // the gradient itself was written by the forward (hpdga module.cpp:155-156)
  if (impl_->events) impl_->start_backward.wait(stream);
}
real CrossEntropyLoss::accuracy() const { return impl_->res.get()[1]; }

// ---------------------------------------------------------------------- Adam
Adam::Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
           AdamParams const *params_)
    : stream_(context().stream.get()) {
  std::vector<shared_ptr<pgcn::Variable>> w;
  for (const auto &v : weights) {
    PGCN_CHECK(v->impl(), PGCN_E_INVALID, "Adam: weights need their rows and cols");
    w.push_back(v->impl());
  }
  pgcn::AdamParams a;
  a.learning_rate = params_->learning_rate;
  a.beta1 = params_->beta1;
  a.beta2 = params_->beta2;
  a.eps = params_->eps;
  a.weight_decay = params_->weight_decay;
  impl_ = std::make_shared<pgcn::Adam>(w, decays, a);
}
Adam::Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
           AdamParams const *params_, const std::vector<smart_stream> &backward_streams_,
           std::vector<smart_event> &start_matmul_forward_, smart_stream &forward_training_stream_)
    : Adam(weights, decays, params_) {
  PGCN_CHECK(backward_streams_.size() >= 2 && start_matmul_forward_.size() == weights.size(),
             PGCN_E_INVALID, "Adam: two backward streams and one event per weight");
  stream_ = forward_training_stream_;
  // src/optim.cu:57-95: the first weight on backward_streams[0], the others on [1], each
  // followed by its start_matmul_forward event
  for (size_t i = 0; i < weights.size(); i++) {
    schedule_.push_back(backward_streams_[i == 0 ? 0 : 1]);
    events_.push_back(start_matmul_forward_[i]);
  }
}
void Adam::step(const smart_stream &stream) { impl_->step(Stream::wrap(stream.get())); }
void Adam::step() {
  if (schedule_.empty()) {
    step(stream_);
    return;
  }
  std::vector<hipStream_t> st;
  std::vector<hipEvent_t> ev;
  for (size_t i = 0; i < schedule_.size(); i++) {
    st.push_back(schedule_[i].get());
    ev.push_back(events_[i].get());
  }
  impl_->step_each(st, ev);
}

// ---------------------------------------------------------------------- Parser
Parser::Parser(GCNParams *gcnParams, GCNData *gcnData, const std::string &graph_name,
               const std::string &root)
    : params_(gcnParams), data_(gcnData), name_(graph_name), root_(root) {}

bool Parser::parse() {
  pgcn::GCNData d;
  pgcn::Parser p(&d, name_, root_);
  if (!p.parse()) return false;
  data_->graph.indptr.assign(d.graph.indptr.begin(), d.graph.indptr.end());
  data_->graph.indices.assign(d.graph.indices.begin(), d.graph.indices.end());
  data_->feature_index.indptr.assign(d.feature_index.indptr.begin(), d.feature_index.indptr.end());
  data_->feature_index.indices.assign(d.feature_index.indices.begin(),
                                      d.feature_index.indices.end());
  data_->feature_value = d.feature_value;
  data_->split.assign(d.split.begin(), d.split.end());
  data_->label = d.label;
  data_->graph_value = graph_coefs(d.num_nodes, d.graph.indptr.data(), d.graph.indices.data());
  params_->num_nodes = (natural)d.num_nodes;
  params_->input_dim = (natural)d.input_dim;
  params_->output_dim = (natural)d.output_dim;
  params_->train_dim = params_->val_dim = params_->test_dim = 0;
  for (int i = 0; i < d.num_nodes; i++) {
    if (d.split[(size_t)i] == 1) params_->train_dim++;
    else if (d.split[(size_t)i] == 2) params_->val_dim++;
    else if (d.split[(size_t)i] == 3) params_->test_dim++;
  }
  return true;
}

// ---------------------------------------------------------------------- GCN
GCN::GCN(GCNParams const *params_, AdamParams const *adam_params_, GCNData const *data_)
    : params(params_), adam_params(adam_params_) {
  pgcn::GCNParams q;
  q.num_nodes = (int)params_->num_nodes;
  q.input_dim = (int)params_->input_dim;
  q.output_dim = (int)params_->output_dim;
  q.n_layers = (int)params_->n_layers;
  q.hidden_dims = to_int(params_->hidden_dims);
  q.dropouts = params_->dropouts;
  q.epochs = (int)params_->epochs;
  q.early_stopping = (int)params_->early_stopping;
  q.reassociate_last = true;
  q.seed = params_->seed;
  pgcn::AdamParams a;
  a.learning_rate = adam_params_->learning_rate;
  a.beta1 = adam_params_->beta1;
  a.beta2 = adam_params_->beta2;
  a.eps = adam_params_->eps;
  a.weight_decay = adam_params_->weight_decay;
  pgcn::GCNData d;
  d.num_nodes = q.num_nodes;
  d.input_dim = q.input_dim;
  d.output_dim = q.output_dim;
  d.graph.indptr = to_int(data_->graph.indptr);
  d.graph.indices = to_int(data_->graph.indices);
  d.feature_index.indptr = to_int(data_->feature_index.indptr);
  d.feature_index.indices = to_int(data_->feature_index.indices);
  d.feature_value = data_->feature_value;
  d.split = to_int(data_->split);
  d.label = data_->label;
  // the engine computes Â's coefficients itself (bit-exact with the parser's, hpdga
  // module.cpp:88-90); a graph_value array holding anything else is refused, not ignored
  if (!data_->graph_value.empty()) {
    const std::vector<float> want =
        graph_coefs(d.num_nodes, d.graph.indptr.data(), d.graph.indices.data());
    PGCN_CHECK(data_->graph_value.size() == want.size() &&
                   std::memcmp(data_->graph_value.data(), want.data(),
                               want.size() * sizeof(float)) == 0,
               PGCN_E_INVALID,
               "GCN: graph_value must be empty or Â's coefficients 1/sqrtf(deg_i deg_j) (the "
               "engine's GraphSum computes them; other values need the Module API)");
  }
  int dev = 0;
  PGCN_HIP(hipGetDevice(&dev));
  impl_ = std::make_unique<pgcn::GCN>(q, a, d, dev);
}
GCN::~GCN() = default;

void GCN::run() {
  const auto t0 = std::chrono::high_resolution_clock::now();
  impl_->run(true);
  total_time = std::chrono::duration<float>(std::chrono::high_resolution_clock::now() - t0).count();
  const long long e = impl_->epochs_run();
  avg_epoch_time = e > 0 ? total_time / (float)e : 0.0f;
  const std::vector<float> r = impl_->results(1);
  if (r.size() >= 4) last_val_accuracy = r[3];
}
std::pair<real, real> GCN::train_epoch() { return impl_->train_epoch(); }
std::pair<real, real> GCN::eval(natural current_split) { return impl_->eval((int)current_split); }

}  // namespace api
}  // namespace pgcn
