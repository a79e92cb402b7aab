/* include/pgcn.hpp -- the reference-shaped C++ API of the MI355X GCN engine.
 *
 * The same classes, constructor shapes and forward/backward contract as the reference's
 * C++ interface, for code written against it:
 *   Variable                      include/variable.cuh:11-29
 *   Module, Dropout, SparseMatmul,
 *   GraphSum, ReLU, Matmul,
 *   CrossEntropyLoss              include/module.cuh:21-145
 *   AdamParams, Adam              include/optim.cuh:16-50
 *   SparseIndex, DevSparseIndex   include/sparse.cuh:11-29
 *   GCNParams, GCNData, GCN       include/gcn.cuh:40-122
 *   smart_stream, smart_event     include/smart_object.cuh:13-52
 *   Parser                        hpdga-spring23/include/parser.h:10-24
 * `using namespace pgcn::api;` makes reference code read unchanged.  Everything runs on the
 * current HIP device through libpgcn.so (HIP kernels for gfx950); there is no CPU fallback.
 *
 * Numerics follow the sequential CPU reference (hpdga-spring23), like the C ABI (pgcn.h):
 * dropout masks and glorot weights come from one process-wide xorshift128+ stream
 * (Variable::initialize_random), CrossEntropyLoss normalises by the labelled count.
 *
 * Differences from the reference, by design:
 *   * device pointers are plain `real *` behind .get() (dev_data.get() reads as before);
 *     a Variable given rows and cols (the weights) is dense [rows][cols]; one given only a size
 *     (the node matrices, as the reference's GCN builds them) takes its shape from the first
 *     module constructed on it and is stored [rows][ld], ld = cols rounded up to a multiple of
 *     4 (padding columns zero); to_host()/from_host() move the logical rows * cols;
 *   * dropout stream positions are assigned in Dropout construction order, which is the
 *     forward order of the reference's GCN (insert_first_layer .. insert_last_layer): the
 *     k-th training forward of a Dropout draws stream positions
 *       glorot draws + (sizes of the Dropouts built before it) + (k - 1) * (sum of all sizes),
 *     i.e. exactly hpdga's sequence when every Dropout runs once per training pass;
 *   * the scheduling arguments of the reference constructors are honoured as the reference
 *     uses them (src/module.cu, src/optim.cu): SparseMatmul / Matmul forwards wait for their
 *     weight's start_matmul_forward event, SparseMatmul's backward records start_set_input,
 *     a GraphSum built with generate_event records start_matmul_backward after its backward,
 *     Matmul's backward computes b.grad on its own stream after event_backward (through a
 *     workspace of its own), CrossEntropyLoss records start_backward after a training forward
 *     and its backward waits for it, and Adam::step() runs the first weight on
 *     backward_streams[0] and the others on [1], each followed by its start_matmul_forward
 *     event.  The constructors without those arguments enqueue everything in order on the
 *     stream passed to forward/backward;
 *   * a GraphSum reads dev_graph_value once, at construction (the reference reads it at every
 *     launch); GCN takes Â's coefficients from the pattern and refuses a graph_value array
 *     holding anything else;
 *   * CrossEntropyLoss::forward also counts the wrong predictions (accuracy());
 *   * a Dropout on the input features must exist before the SparseMatmul reading them.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace pgcn {
class Variable;
class Module;
class DevGraph;
struct DevFeatures;
class GCN;
class Adam;
struct ModuleContext;

namespace api {

using real = float;
using natural = unsigned;
using integer = int;
using std::shared_ptr;

// include/smart_object.cuh: a stream / event owned by the object (shared on copy)
class smart_stream {
 public:
  smart_stream();                           // a new non-blocking stream
  explicit smart_stream(hipStream_t borrowed);  // wraps a stream owned elsewhere
  hipStream_t get() const { return s_; }
  void sync() const;

 private:
  std::shared_ptr<void> own_;
  hipStream_t s_ = nullptr;
};

class smart_event {
 public:
  smart_event();
  hipEvent_t get() const { return e_; }
  void record(const smart_stream &s) const;
  void wait(const smart_stream &s) const;  // s waits for the recorded point

 private:
  std::shared_ptr<void> own_;
  hipEvent_t e_ = nullptr;
};

template <class T>
struct dev_ptr {  // the reference's dev_shared_ptr<T>::get()
  T *p = nullptr;
  T *get() const { return p; }
};

// include/variable.cuh:11-29
class Variable {
 public:
  dev_ptr<real> dev_data, dev_grad;
  natural size = 0, rows = 0, cols = 0;
  natural ld = 0;  // row stride: cols, or cols rounded up to 4 for node matrices

  Variable(natural size_, bool requires_grad = true, bool rand = false, natural rows_ = 0,
           natural cols_ = 0);
  void zero(const smart_stream &stream) const;
  void zero_grad(const smart_stream &stream) const;
  void glorot() const;  // hpdga variable.cpp:15-19 from the shared xorshift stream
  void set_value(real value, const smart_stream &stream) const;
  std::vector<real> to_host(bool grad = false) const;  // logical rows * cols (or size)
  void from_host(const std::vector<real> &v) const;
  void print(const std::string &what, natural col) const;
  void save(const std::string &file_name, const std::string &what, natural col) const;
  // restarts the shared xorshift128+ stream: seed 0 = hpdga's unseeded rand() state, else the
  // state of srand(seed) (the PART2 `seed` key)
  static void initialize_random(unsigned seed = 0);

  // the engine's variable (null until a shape is known: a Variable built from a size alone
  // takes its node-matrix shape [rows][ld] from the first module constructed on it)
  const shared_ptr<pgcn::Variable> &impl() const { return impl_; }

 private:
  friend struct VariableAccess;
  bool requires_grad_ = true;
  shared_ptr<pgcn::Variable> impl_;
};

// include/sparse.cuh:11-29
class SparseIndex {
 public:
  std::vector<natural> indices;
  std::vector<natural> indptr;
};

class DevSparseIndex {
 public:
  explicit DevSparseIndex(const SparseIndex &sparse_index);
  dev_ptr<natural> dev_indices, dev_indptr;
  natural indices_size = 0, indptr_size = 0;
  const SparseIndex &host() const { return host_; }
  // the device adjacency of this pattern with these values (built once per distinct value
  // array, shared by the modules that use it)
  std::shared_ptr<pgcn::DevGraph> graph(const std::vector<real> &values) const;

 private:
  SparseIndex host_;
  std::shared_ptr<void> dev_;
  // device graphs by value array; weak: a graph lives as long as a GraphSum holding it
  mutable std::vector<std::pair<std::vector<real>, std::weak_ptr<pgcn::DevGraph>>> graphs_;
};

// include/module.cuh:21-30
class Module {
 public:
  virtual void forward(bool training, const smart_stream &stream) const = 0;
  virtual void backward(const smart_stream &stream) const = 0;
  virtual void set_num_samples(natural) {}
  virtual natural get_num_samples() const { return 0; }
  virtual ~Module();
};

// include/module.cuh:33-43
class Dropout : public Module {
 public:
  Dropout(shared_ptr<Variable> in_, real p_);
  ~Dropout() override;
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/module.cuh:47-68: c = dropout(a) * b, a = the input features (values of sp)
class SparseMatmul : public Module {
 public:
  SparseMatmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               DevSparseIndex *sp_, natural m_, natural n_, natural p_,
               smart_event &start_matmul_forward_, smart_event &start_set_input_);
  SparseMatmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               DevSparseIndex *sp_, natural m_, natural n_, natural p_);
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/module.cuh:72-86: out = Â in (graph values = Â's coefficients, hpdga
// parser.cpp:164-181 / src/parser.cpp:164-181; dev_graph_value on the device)
class GraphSum : public Module {
 public:
  GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevSparseIndex *graph_,
           const real *dev_graph_value_, natural dim_, bool generate_event_,
           smart_event &start_matmul_backward_);
  GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevSparseIndex *graph_,
           const real *dev_graph_value_, natural dim_);
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/module.cuh:90-99
class ReLU : public Module {
 public:
  explicit ReLU(shared_ptr<Variable> in_);
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/module.cuh:103-124: c = a * b  (a [m][n], b [n][p])
class Matmul : public Module {
 public:
  Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_, natural m_,
         natural n_, natural p_, smart_event &event_forward_, smart_event &event_backward_,
         const smart_stream &stream_);
  Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_, natural m_,
         natural n_, natural p_);
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/module.cuh:128-145: the mean cross-entropy over the rows whose dev_truth >= 0
// (num_samples of them; 0 = count them, with a host sync) lands in *loss (host memory, valid
// after the stream syncs); training forwards leave its gradient in logits.grad (hpdga
// module.cpp:122-156)
class CrossEntropyLoss : public Module {
 public:
  natural num_samples = 0;
  CrossEntropyLoss(shared_ptr<Variable> logits_, const integer *dev_truth_, real *loss_,
                   natural num_classes_, smart_event &event);
  CrossEntropyLoss(shared_ptr<Variable> logits_, const integer *dev_truth_, real *loss_,
                   natural num_classes_);
  void set_num_samples(natural num_samples_) override;
  natural get_num_samples() const override;
  void forward(bool training, const smart_stream &stream) const override;
  void backward(const smart_stream &stream) const override;
  real accuracy() const;  // of the last forward (after the stream syncs)
  struct Impl;

 private:
  shared_ptr<Impl> impl_;
};

// include/optim.cuh:16-50
struct AdamParams {
  real learning_rate{0.01f}, beta1{0.9f}, beta2{0.999f}, eps{1e-8f}, weight_decay{5e-4f};
};

class Adam {
 public:
  Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
       AdamParams const *params_);
  Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
       AdamParams const *params_, const std::vector<smart_stream> &backward_streams_,
       std::vector<smart_event> &start_matmul_forward_, smart_stream &forward_training_stream_);
  void step(const smart_stream &stream);  // every weight on `stream`
  // the reference's schedule when built with its streams and events (src/optim.cu:57-95): the
  // first weight on backward_streams[0], the others on [1], each followed by its
  // start_matmul_forward event; else every weight on the default API stream
  void step();

 private:
  shared_ptr<pgcn::Adam> impl_;
  smart_stream stream_;
  std::vector<smart_stream> schedule_;
  std::vector<smart_event> events_;
};

// include/gcn.cuh:40-58
struct GCNParams {
  natural num_nodes = 0, input_dim = 0, output_dim = 0;
  std::vector<natural> hidden_dims = {16};
  std::vector<real> dropouts = {0.5f, 0.5f};
  natural epochs{100}, early_stopping{0};
  natural train_dim{0}, val_dim{0}, test_dim{0};
  natural n_layers{2};
  unsigned seed{0};  // PART2 `seed` (0: hpdga's unseeded stream)
};

struct GCNData {
  SparseIndex feature_index, graph;
  std::vector<natural> split;
  std::vector<integer> label;
  std::vector<real> graph_value;
  std::vector<real> feature_value;
};

// hpdga-spring23/include/parser.h:10-24: reads <root>/data/<name>.{graph,split,svmlight},
// fills the data and the dataset's sizes in params (num_nodes, input_dim, output_dim,
// train/val/test_dim) and Â's coefficients (graph_value)
class Parser {
 public:
  Parser(GCNParams *gcnParams, GCNData *gcnData, const std::string &graph_name,
         const std::string &root = ".");
  bool parse();

 private:
  GCNParams *params_;
  GCNData *data_;
  std::string name_, root_;
};

// include/gcn.cuh:79-122: the whole model, built and run by the engine (fused kernels, the
// reorganisations of DESIGN.md §1 at their reference-equivalent defaults)
class GCN {
 public:
  real avg_epoch_time = 0, total_time = 0, last_val_accuracy = 0;
  const GCNParams *params;
  const AdamParams *adam_params;
  GCN(GCNParams const *params_, AdamParams const *adam_params_, GCNData const *data_);
  ~GCN();
  void run();
  std::pair<real, real> train_epoch();
  std::pair<real, real> eval(natural current_split);

 private:
  std::unique_ptr<pgcn::GCN> impl_;
};

}  // namespace api
}  // namespace pgcn
