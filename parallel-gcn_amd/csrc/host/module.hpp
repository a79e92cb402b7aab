// parallel-gcn_amd/csrc/host/module.hpp -- Variable and the Module family.
//
// Same classes, constructor shapes and forward/backward contract as the reference's
// include/variable.cuh:11-29 and include/module.cuh:21-145:
//   virtual void forward(bool training, const Stream &) const;
//   virtual void backward(const Stream &) const;
// Each module launches its HIP kernels asynchronously on the stream it is given; data
// stays on the device.  Differences from the reference, by design:
//   * the input features X are never rewritten: the input Dropout only produces the mask
//     bits that SparseMatmul applies on the fly (the reference mutates X in place and
//     restores it with set_input_kernel every pass, src/gcn.cu:181-200);
//   * dropout masks are the CPU reference's xorshift128+ masks, bit for bit;
//   * weight gradients are reduced deterministically (no float atomics);
//   * with an edge-cut communicator, GraphSum combines partial sums with an RCCL
//     reduce-scatter and weight grads are all-reduced by the optimizer.
#pragma once
#include <memory>
#include <vector>

#include "comm.hpp"
#include "graph.hpp"
#include "runtime.hpp"

namespace pgcn {

using std::shared_ptr;

// include/variable.cuh:11-29. Node-sized variables are [rows][ld] with ld = round_up(cols,4)
// (padding columns are kept zero); weights are dense [rows][cols].
class Variable {
 public:
  DeviceBuffer<float> dev_data, dev_grad;
  int rows = 0, cols = 0, ld = 0;
  long long size = 0;  // logical rows * cols
  Variable(int rows_, int cols_, bool requires_grad, int ld_ = -1);
  Variable() = default;
  void zero(hipStream_t s) const { dev_data.zero_async(s); }
  void zero_grad(hipStream_t s) const {
    if (dev_grad) dev_grad.zero_async(s);
  }
  // logical (unpadded) copy to host, which: 0 data, 1 grad
  std::vector<float> to_host(int which) const;
};

// Input features on the device (the feature half of DevGCNData, src/gcn.cu:30-43).
struct DevFeatures {
  bool dense = false;
  int rows = 0, cols = 0;  // local rows, input_dim
  long long nnz = 0;
  // dense: [rows][ldx] fp32, CSR order == row-major order
  DeviceBuffer<float> x;
  int ldx = 0;
  // eval_ax: Â X ([rows][ldx], computed once at engine build; Â and X are constants), so
  // eval's first layer is (Â X) W1 -- one GEMM pass instead of X W1 and a GraphSum
  DeviceBuffer<float> ax;
  // dense + X-stream kernels: the input dropout's keep bits in the nibble layout
  // (k_mask_nibbles, [rows][16] words), rebuilt by every training forward
  DeviceBuffer<uint64_t> maskT;
  // dense + wide first layer (k_gemm_wide.hip, 33..128 outputs, F <= 1024): the same nibble
  // layout for the wide kernels' dropout bits, rebuilt by every training forward
  DeviceBuffer<uint64_t> maskW;
  // sparse: CSR (+ transposed index for the weight gradient)
  DeviceBuffer<int> indptr, indices, csc_ptr, csc_row, csc_pos;
  DeviceBuffer<int> csc_order;  // features by descending column length (weight-gradient order)
  DeviceBuffer<float> values;
  std::vector<float> host_values;  // for reporting the dropped input (API parity)
};

// Dropout mask + xorshift chunk states for one Dropout module on this rank.
struct DropoutRng {
  DeviceBuffer<uint64_t> states;  // 2 per chunk
  DeviceBuffer<uint64_t> mask;    // 1 word per chunk: the last training forward's mask
  DeviceBuffer<uint64_t> mask_ahead;  // the next one, when drawn ahead (input dropout)
  long long chunk_lo = 0, n_chunks = 0;
  // 64-draw mask words per stored state (k_dropout_mask's PER; one state per 128 draws;
  // "mask_per" knob, read at engine build)
  int per = 2;
  long long elem_begin = 0, elem_end = 0;  // global element range of this rank
  long long mask_base = 0;                 // bit of local element 0 in `mask`
};

class Module {
 public:
  virtual void forward(bool training, const Stream &s) const = 0;
  virtual void backward(const Stream &s) const = 0;
  virtual void set_num_samples(int) {}
  virtual int get_num_samples() const { return 0; }
  virtual ~Module() {}
};

class ReLU;
class GraphSum;
class Dropout;

// "fuse_epilogue" bits (host/gcn.cpp g_fuse_epilogue) and "fuse_output" (g_fuse_output)
constexpr int kFuseTails = 1, kFusePrestage = 2, kFuseXstream = 4, kFuseMatmulTails = 8;
extern int g_fuse_epilogue;
extern int g_fuse_output;
extern int g_sparse_dual;

// Shared per-GCN state the modules read (current split, comm, profiling, RNG table).
extern int g_csc_tree;  // "csc_tree" (module.cpp)

struct ModuleContext {
  bool train_ahead = true;     // eval computes the next training forward's first product too
  // (measured and removed, r01/r02: drawing the next input mask on a side stream beside the
  // weight-gradient pass, the eval forward's X-stream product or its output layer -- the RNG
  // kernel and the pass beside it slow each other down, DESIGN.md §3 "Streams")
  hipStream_t side_stream = nullptr;  // mm_side's stream
  // "eval_tail" (edge-cut, peer exchange between processes): the eval pass's last GraphSum
  // pushes, waits and sums on tail_stream (set by GCN for that call), and the output layer and
  // the loss follow there, beside the next epoch's mask draw and first-layer product on the
  // stream; tail_done is recorded after them, and the next GraphSum on the stream waits for it
  // (tail_pending) -- it reuses the partial buffer and the slots' parity
  hipStream_t tail_stream = nullptr;
  Event tail_fork, tail_done;
  bool tail_pending = false;
  bool tail_used = false;  // the GraphSum given tail_stream ran its exchange there
  // "mm_side": a Matmul's weight gradient (b.grad = a^T c.grad, needed only by the optimizer)
  // runs on side_stream beside the rest of the backward pass (the reference's S2/S3 streams,
  // src/module.cu:445-472); GCN joins it (side_join) before the all-reduce / optimizer
  bool mm_side = false;
  Event mm_fork, side_join;
  void *gemm_workspace_side = nullptr;
  bool side_pending = false;
  // output-layer row restriction (single GPU; the edge-cut engine uses chunk_split_graphs):
  // the last GraphSum's forward computes only the current split's labelled rows -- the only
  // rows the loss, the accuracy and (through the loss gradient, zero elsewhere) the weight
  // gradients depend on
  DevGraph *split_graph = nullptr;  // Â restricted to those rows (null: all rows)
  const int *split_rows = nullptr;  // their row ids (device)
  // ... and its backward: the loss gradient is zero outside those rows, so Â out.grad only
  // needs the edges into them (Â's columns of the split)
  DevGraph *split_colgraph = nullptr;
  // compact output layer (reassociated order + row restriction): the last GraphSum writes the
  // split's rows compactly ([compact_n][ld]) and the output Matmul and the loss work on those
  // rows only; compact_n = 0: all rows
  int compact_n = 0;
  const int *compact_truth = nullptr;  // the split's labels in compact row order
  Variable *compact_z = nullptr;       // last GraphSum output / Matmul input (+ grad)
  Variable *compact_out = nullptr;     // logits (+ grad)
  const int *truth = nullptr;  // current split's truth (device)
  int count = 0;               // labelled rows of the current split (global)
  float *xent_partials = nullptr;
  int xent_blocks = 0;
  // one GPU ("fuse_finish"): the pass's scalars finished by the loss kernel's last block
  // (XentFinal); set by GCN for the pass being enqueued, fin_taken by the loss module that
  // passed it on (GCN::finalize then launches nothing)
  const XentFinal *fin = nullptr;
  bool fin_taken = false;
  Comm *comm = nullptr;        // null on one GPU
  hipStream_t comm_stream = nullptr;      // edge-cut: stream of the reduce-scatters
  int local_rows = 0;                     // edge-cut: this rank's rows (the rest is padding)
  std::vector<DevGraph *> chunk_graphs;   // edge-cut: Â column block per RS row chunk
  // edge-cut output-layer row restriction: per RS chunk, the chunk graph restricted to the
  // current split's labelled rows (padded chunk row ids in chunk_split_rows); empty: off
  std::vector<DevGraph *> chunk_split_graphs;
  std::vector<const int *> chunk_split_rows;
  // ... and its backward: per RS chunk, the chunk graph on the columns (local rows) of the
  // training split, where the loss gradient is non-zero; empty: off
  std::vector<DevGraph *> chunk_col_graphs;
  const void *jump_table = nullptr;  // M^period byte tables (device)
  // mask_xstream: the next training forward's masks, drawn by eval's first-layer product
  // (SparseMatmul, eval_ax) -- xs_draw for the ring NN kernel, xs_draw_md for a separate
  // launch when that product takes another kernel; n = 0: none pending
  XsDraw xs_draw;
  MaskDraw xs_draw_md[2];
  void *gemm_workspace = nullptr;
  size_t gemm_workspace_bytes = 0;
  // profiling of GraphSum calls
  bool profile = false;
  std::vector<std::pair<Event, Event>> *gs_events = nullptr;
  std::vector<double> *gs_bytes = nullptr;
  // ... and of the XW contractions on the MFMA kernels (dense X W, H W, their gradients)
  std::vector<std::pair<Event, Event>> *mm_events = nullptr;
  std::vector<double> *mm_flops = nullptr;
  std::vector<Event> *event_pool = nullptr;
};

// Builders shared by GCN and the public C++ API (host/gcn.cpp)
void build_dev_features(DevFeatures &feats, const int *fptr, const int *indices,
                        const float *values, int first, int rows, int F, bool dense, int hidden0);
void init_dropout_rng_range(DropoutRng &r, const uint64_t seed[2], unsigned long long offset,
                            long long elem_begin, long long elem_end);
void glorot_fill(std::vector<float> &w, int in_size, int out_size, uint64_t s[2]);

// include/module.cuh:33-43
class Dropout : public Module {
  shared_ptr<Variable> in;  // null for the input features
  shared_ptr<DropoutRng> rng;
  float p;
  ModuleContext *ctx;

 public:
  Dropout(shared_ptr<Variable> in_, float p_, shared_ptr<DropoutRng> rng_, ModuleContext *ctx_);
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
  float scale() const { return 1.0f / (1.0f - p); }
  const DropoutRng &state() const { return *rng; }
  // Draws the NEXT training forward's mask now (the xorshift stream position is the same
  // whenever it is drawn); that forward then uses it instead of drawing again.  With `ready`,
  // the draw runs on stream s and `ready` is recorded after it: users of the mask on another
  // stream wait for it (wait_ahead).
  void draw_ahead(hipStream_t s, const Event *ready = nullptr) const;
  // The same draw handed to another launch (the optimizer's, mask_adam): fills out[0] (and
  // out[1]: co_draw's next mask) and marks both drawn; returns how many (0: already drawn)
  int ahead_descs(MaskDraw out[2]) const;
  bool drawn_ahead() const { return ahead; }
  void wait_ahead(hipStream_t s) const;
  const uint64_t *mask_ahead() const { return rng->mask_ahead.get(); }
  // Fused into the GraphSum next to it (GraphSum::forward/backward apply this module's work in
  // their epilogue): the training forward's mask is drawn by draw_fused(), and the next
  // forward / backward call of this module is skipped.
  const Variable *variable() const { return in.get(); }
  void draw_fused(hipStream_t s) const;
  mutable bool skip_forward = false, skip_backward = false;
  // the input dropout's training draw also draws `co_draw`'s mask (one launch: the same stream
  // positions, so the same bits); that module's next forward / fused draw then uses it
  // (GCN::build, "co_draw"; sparse X only: the dense input has its own layouts)
  const Dropout *co_draw = nullptr;
  mutable bool pre_drawn = false;

 private:
  void draw(hipStream_t s, uint64_t *mask, int max_blocks = 0) const;
  mutable bool ahead = false;
  mutable const Event *ahead_ready = nullptr;  // recorded after an ahead draw on a side stream
};

// include/module.cuh:47-68: c = drop(X) * W
class SparseMatmul : public Module {
  const DevFeatures *x;
  shared_ptr<Variable> b, c;
  const Dropout *drop;  // the input Dropout (its mask, when training)
  ModuleContext *ctx;
  mutable bool last_training = false;
  // train-ahead (dense X-stream path): an eval forward also computes the next training
  // forward's drop(X) W into `ahead` (same weights: no optimizer step between them), which
  // that forward then swaps in instead of streaming X again
  mutable DeviceBuffer<float> ahead;
  mutable bool ahead_valid = false;

 public:
  SparseMatmul(const DevFeatures *x_, shared_ptr<Variable> b_, shared_ptr<Variable> c_,
               const Dropout *drop_, ModuleContext *ctx_);
  // eval_ax: the first GraphSum's output, written by an eval forward from Â X
  shared_ptr<Variable> eval_out;
  // the GraphSum reading c (training) / standing for eval_out (eval): the X-stream product's
  // epilogue writes that GraphSum's ring table (training) or applies its fused ReLU and
  // writes the next GraphSum's table (eval), when g_fuse_epilogue & kFuseXstream
  const GraphSum *consumer = nullptr;
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
};

// include/module.cuh:72-86
class GraphSum : public Module {
  shared_ptr<Variable> in, out;
  DevGraph *graph;
  int dim;
  ModuleContext *ctx;
  bool last_layer;                   // the output layer's GraphSum (row restriction applies)
 public:
  bool first_layer = false;          // eval_ax: its eval forward was done by SparseMatmul
 private:
  mutable DeviceBuffer<float> compact;  // restricted forward: [split rows][out->ld]
  // edge-cut: per row chunk, the [world*chunk_rows][ld] partial sums and their events
  std::vector<DeviceBuffer<float>> partial;
  std::vector<Event> computed;
  Event reduced;

 public:
  GraphSum(shared_ptr<Variable> in_, shared_ptr<Variable> out_, DevGraph *graph_, int dim_,
           ModuleContext *ctx_, bool last_layer_ = false);
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
  const Variable *input() const { return in.get(); }
  const Variable *output() const { return out.get(); }
  int width() const { return dim; }
  // Element-wise tails fused into this GraphSum's final writes (GCN::fuse_epilogues; null: the
  // modules run on their own): forward, the ReLU (and Dropout) on `out` that follow it;
  // backward, the Dropout (and ReLU) on `in` whose backward follows it
  ReLU *fwd_relu = nullptr;
  const Dropout *fwd_drop = nullptr;
  ReLU *bwd_relu = nullptr;
  const Dropout *bwd_drop = nullptr;
  // ... and the GraphSum that reads this one's fused output next (forward: `out`; backward:
  // in.grad): the epilogue also writes its prescaled input table (ring schedule), so that
  // GraphSum skips its prescale launch (prestaged_*, consumed by its next call)
  GraphSum *fwd_next = nullptr, *bwd_next = nullptr;
  mutable bool prestaged_fwd = false, prestaged_bwd = false;
  // the graph this module's next forward / backward sums over (single GPU)
  DevGraph *forward_graph() const;
  DevGraph *backward_graph() const;
  // ... and the graph whose prescaled table that call reads (edge-cut: row chunk 0's)
  DevGraph *forward_table_graph() const;
  DevGraph *backward_table_graph() const;
  // for a producer of this GraphSum's next forward input with `rows` rows and 16 columns:
  // the ring table (and its scale) that call reads, marked as written by the producer
  // (prestaged_fwd); null when that call has none
  float4 *claim_forward_table(int rows, int ld, const float **scale) const;
  // for the fused loss kernel writing this GraphSum's next backward input (out.grad, `rows` x
  // 16, ld 16): that call's ring table, scale and row map (XentTable), marked as written by
  // it (prestaged_bwd); false when that call has none (single GPU only)
  bool claim_backward_table(int rows, int ld, XentTable *t) const;

 private:
  // mode (edge-cut output layer): 0 all rows, 1 forward over ctx->chunk_split_graphs (the
  // split's rows), 2 backward over ctx->chunk_col_graphs (the split's columns)
  void run(const float *src, float *dst, const Stream &s, int mode = 0,
           const GsEpilogue *epi = nullptr, bool prestaged = false) const;
  // points the epilogue's next_table at `next`'s input table on graph `ng`, if it has one
  void stage_next(GsEpilogue &e, GraphSum *next, DevGraph *ng, bool fwd) const;
  // the fused tails of this call (mode 0 when none applies)
  bool tail_ok(const DevGraph *g, int ld_in, int ld_out) const;
  GsEpilogue forward_epilogue(bool training, const Stream &s, const DevGraph *g) const;
  GsEpilogue backward_epilogue(const DevGraph *g) const;
};

// include/module.cuh:90-99
class ReLU : public Module {
  shared_ptr<Variable> in;
  DeviceBuffer<uint8_t> mask;

 public:
  explicit ReLU(shared_ptr<Variable> in_);
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
  const Variable *variable() const { return in.get(); }
  uint8_t *mask_ptr() const { return const_cast<uint8_t *>(mask.get()); }
  mutable bool skip_forward = false, skip_backward = false;  // done by a GraphSum epilogue
};

// include/module.cuh:103-124: c = a * b
class Matmul : public Module {
  shared_ptr<Variable> a, b, c;
  int m, n, p;
  ModuleContext *ctx;

 public:
  bool last_layer = false;  // the output layer's Matmul (compact rows apply)
  bool fused_forward = false;  // its forward runs inside the loss's (CrossEntropyLoss::fused)
  mutable bool input_grad_done = false;  // ... which also wrote a.grad (this training pass)
  mutable bool weight_grad_done = false;  // ... and b.grad
  // the Dropout (and ReLU) on `a` whose backward follows this one's: applied in the a.grad
  // product's final write when that product runs on k_xstream_nn (GCN::fuse_epilogues)
  const Dropout *bwd_drop = nullptr;
  ReLU *bwd_relu = nullptr;
  Matmul(shared_ptr<Variable> a_, shared_ptr<Variable> b_, shared_ptr<Variable> c_, int m_,
         int n_, int p_, ModuleContext *ctx_);
  const Variable *input() const { return a.get(); }
  const Variable *weight() const { return b.get(); }
  const Variable *output() const { return c.get(); }
  int inner() const { return n; }
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
  // the two halves of backward(), for callers that schedule them on their own streams (the
  // C++ API's reference schedule, src/module.cu:431-472): a.grad = c.grad b^T on s, and
  // b.grad = a^T c.grad on `ws` (a workspace of gemm_tn_workspace(m, p, n) bytes owned by the
  // caller when the stream is not the module's usual one)
  void backward_input(const Stream &s) const;
  void backward_weight(hipStream_t s, void *ws) const;
};

// include/module.cuh:128-145
class CrossEntropyLoss : public Module {
  shared_ptr<Variable> logits;
  int num_classes;
  ModuleContext *ctx;
  int num_samples = 0;

 public:
  CrossEntropyLoss(shared_ptr<Variable> logits_, int num_classes_, ModuleContext *ctx_);
  // the output layer's Matmul whose forward this loss computes with its own (null: none)
  const Matmul *fused = nullptr;
  // ... and the GraphSum whose backward reads that Matmul's input grad (the reassociated
  // output layer's): the fused kernel also writes its prescaled table (claim_backward_table)
  const GraphSum *dh_reader = nullptr;
  const Variable *input() const { return logits.get(); }
  void forward(bool training, const Stream &s) const override;
  void backward(const Stream &s) const override;
  void set_num_samples(int n) override { num_samples = n; }
  int get_num_samples() const override { return num_samples; }
};

}  // namespace pgcn
