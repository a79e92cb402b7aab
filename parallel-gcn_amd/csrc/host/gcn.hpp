// parallel-gcn_amd/csrc/host/gcn.hpp -- GCNParams / AdamParams / Adam / GCN.
//
// Mirrors include/gcn.cuh:40-122 and include/optim.cuh:16-50 of the reference (and
// hpdga-spring23/include/gcn.h, optim.h): same parameter structs and defaults, the same
// L-layer builders (insert_first_layer / insert_layer / insert_last_layer,
// src/gcn.cu:47-142), the same module and variable order, train_epoch / eval / run.
// Numerics follow the sequential CPU reference (hpdga-spring23), not the CUDA one: CPU
// xorshift128+ dropout masks and glorot init, loss normalised by the labelled count.
#pragma once
#include <memory>
#include <utility>
#include <vector>

#include "comm.hpp"
#include "data.hpp"
#include "graph.hpp"
#include "module.hpp"
#include "runtime.hpp"

namespace pgcn {

// GraphSum row chunks of the edge-cut engine at world > 1 (knob rs_chunks): chunk k's
// reduce-scatter overlaps chunk k+1's local sum.  1 by default (r04, reddit-114M, one rank's
// GraphSum timed on one GPU: 58.7 us at world 8 for the whole column block against 81.3 us
// for two row chunks, whose 30 rowset batches leave half the CUs idle; a 13 MB exchange at
// 300 GB/s then fits in the 22.6 us the second chunk would have hidden, and above that rate
// one chunk is ahead; profiles/r04/rank_graphsum_c1.json, rank_graphsum_c2.json)

struct GCNParams {
  int num_nodes = 0, input_dim = 0, output_dim = 0;
  std::vector<int> hidden_dims = {16};
  std::vector<float> dropouts = {0.5f, 0.5f};
  int epochs = 100, early_stopping = 0;
  int n_layers = 2;
  // compute the last layer as (Â H) W instead of Â (H W) when that narrows the GraphSum
  // (hidden < classes); exact algebra, fp32 rounding order only (see insert_last_layer)
  bool reassociate_last = false;
  unsigned seed = 0;  // PART2 `seed`: 0 = hpdga's unseeded rand(), else srand(seed)
};

struct AdamParams {
  float learning_rate = 0.01f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, weight_decay = 5e-4f;
};

// include/optim.cuh:23-50; hpdga optim.cpp:5-35.  Weight decay on W1 only
// (src/gcn.cu:157-158, hpdga gcn.cpp:127).
class Adam {
  struct Var {
    shared_ptr<Variable> w;
    DeviceBuffer<float> m, v;
    bool decay;
  };
  std::vector<Var> vars;
  AdamParams params;
  int step_count = 0;

 public:
  Adam() = default;
  Adam(const std::vector<shared_ptr<Variable>> &weights, const std::vector<bool> &decays,
       const AdamParams &p);
  // defer (one GPU): the weight gradients' deferred last reduction passes (tn_defer), run by
  // this launch for the tensors whose gradients they write, launched before it otherwise
  // peer (edge-cut, processes): the gradients' all-reduce left its sum to this launch --
  // tensor t's gradient is the rank-order sum of peer's slots at its offset in `arena`
  // draws (mask_adam, one GPU): the next training forward's masks drawn by the same launch
  void step(const Stream &s, TnDeferList *defer = nullptr, const PeerRecv *peer = nullptr,
            const float *arena = nullptr, const MaskDraw *draws = nullptr, int n_draws = 0,
            const void *table = nullptr);
  // the reference's per-tensor schedule (src/optim.cu:57-95): one step, tensor i on
  // streams[i], then events[i] recorded there (null: none); the same arithmetic as step()
  void step_each(const std::vector<hipStream_t> &streams, const std::vector<hipEvent_t> &events);
  size_t size() const { return vars.size(); }
  // epoch graphs: the same launches reading the step size from table[ctr[0] % cap] on the
  // device (the host counts the step with advance() at every replay)
  void step_graph(const Stream &s, const float *table, const int *ctr, int cap,
                  TnDeferList *defer = nullptr, const PeerRecv *peer = nullptr,
                  const float *arena = nullptr) const;
  void advance() { step_count++; }
  int steps() const { return step_count; }
  float step_size(int t) const;  // hpdga optim.cpp:24, step t (1-based)

 private:
  void launch(const Stream &s, float st, const float *table, const int *ctr, int cap,
              TnDeferList *defer, const PeerRecv *peer, const float *arena,
              const MaskDraw *draws = nullptr, int n_draws = 0,
              const void *jump_table = nullptr) const;
};

struct DistSpec {
  int rank = 0, world = 1;
  const void *unique_id = nullptr;  // 128 bytes (RCCL)
  // in-process ranks on one device (PeerComm over raw pointers); world = group->world()
  std::shared_ptr<LoopbackGroup> loopback;
  // one process per GPU over peer-mapped slots (PeerComm over hipIpc handles, exchanged by
  // this host all-gather) instead of RCCL
  PeerComm::AllGather allgather;
  bool solo = false;  // timing only: PeerComm with no peers (every push lands in this rank)
};

class GCN {
 public:
  GCN(const GCNParams &params, const AdamParams &adam, const GCNData &data, int device,
      const DistSpec *dist = nullptr);
  ~GCN();
  std::pair<float, float> train_epoch();
  std::pair<float, float> eval(int split);
  void epoch_async();  // train_epoch + eval(2) without a host sync
  void sync();
  std::vector<float> results(int n);  // last n epochs x {tl, ta, vl, va}
  void run(bool verbose);

  int num_vars() const { return (int)variables.size(); }
  std::vector<float> get_var(int idx, int which);
  void set_profile(bool on);
  void profile_read_mm(double *ms, long long *calls, double *flops);  // XW contractions
  void profile_read(double *ms, long long *calls, double *bytes);
  const Partition &partition() const { return part; }
  const GCNParams &get_params() const { return params; }
  const Comm *communicator() const { return comm.get(); }
  bool symmetric() const { return graph_symmetric; }
  long long epochs_run() const { return epoch_count; }
  // device time of the Â X precompute at build (eval_ax; 0 when off)
  float eval_ax_build_ms() const { return ax_build_ms; }
  // GraphSum calls of width 16 take the LDS-staged kernel (large tables)
  bool graphsum_lds() const;
  // the output layer runs as (Â H) W (reassociate_last requested, hidden < classes, Â symmetric)
  bool reassociated() const { return reassociated_; }
  int fused_tails() const { return fused_tails_; }

 private:
  void build(const GCNData &data);
  void upload_features(const GCNData &data);
  void init_dropout_rng(const GCNData &data, long long glorot_draws);
  void insert_first_layer();
  void insert_layer(int in_dim, int out_dim, float dropout, int layer);
  void insert_last_layer();
  void fuse_epilogues();
  void fuse_matmul_tails();
  void fuse_output_layer();
  void prepare_graphs();
  void check_comm() const;
  void build_eval_ax();
  struct FoldScope;
  void backward_pass(FoldScope &fold, TnDeferList *defer);
  PeerRecv adam_peer;  // the pass's gradient all-reduce left its sum to Adam (world > 0)
  // mask_adam: the next training forward's input (and co-drawn hidden) masks for the Adam
  // launch; returns how many (0: not applicable, or drawn already)
  int mask_with_adam(MaskDraw out[2]);
  // mask_xstream: the next training forward's masks drawn by eval's first-layer product
  bool mask_in_eval() const;
  void join_side();
  int fused_tails_ = 0;  // GraphSum epilogues carrying ReLU / Dropout work (forward + backward)
  void set_split(int split);
  void finalize(int slot_offset, bool graph = false, hipStream_t s = nullptr);
  // the eval forward + finalize of ring slot offset `off` (eval_tail: its last GraphSum's
  // exchange and the output layer on side_stream, ModuleContext::tail_stream)
  void eval_forward(int off, bool graph);
  int tail_gs = -1;  // eval_tail: index in `modules` of the last GraphSum; -1 = off
  void enqueue_epoch(bool graph);
  bool graph_eligible() const;
  void capture_epoch();
  void drop_epoch_graph();

  GCNParams params;
  AdamParams adam_params;
  int device;
  int L;
  Partition part;
  std::unique_ptr<Comm> comm;
  Stream stream;
  Stream comm_stream;  // edge-cut: reduce-scatters run here, overlapping the next chunk's sum
  Stream side_stream;  // the next epoch's input-dropout mask, beside the weight-gradient pass
  ModuleContext ctx;

  std::unique_ptr<DevGraph> graph;                    // one GPU: the whole Â
  std::vector<std::unique_ptr<DevGraph>> chunk_graphs;  // edge-cut: Â's column block per RS chunk
  DevFeatures feats;
  DeviceBuffer<int> truth[4];
  int counts[4] = {0, 0, 0, 0};
  // output-layer row restriction (set_split): per split, its labelled rows and Â on them
  std::vector<int> split_rows_host[4];
  std::vector<int> split_rows_global[4];  // edge-cut: the split's labelled global node ids
  DeviceBuffer<int> split_rows_dev[4];
  std::unique_ptr<DevGraph> split_graphs[4], split_colgraphs[4];
  // edge-cut: per split, per RS chunk, the chunk graph on the split's rows + their row ids
  std::vector<std::unique_ptr<DevGraph>> chunk_split_graphs[4];
  std::vector<DeviceBuffer<int>> chunk_split_rows[4];
  std::vector<std::unique_ptr<DevGraph>> chunk_col_graphs;  // training split's columns
  DeviceBuffer<int> truth_compact[4];                // the split's labels, compact row order
  std::unique_ptr<Variable> compact_z, compact_out;  // compact output layer (ModuleContext)
  long long nnz_x_global = 0;
  // Â equals its transpose (csr_symmetric at build): the reassociated output layer's
  // W.grad = (Â H)^T dOut equals the reference's H^T Â dOut only then
  bool graph_symmetric = false;
  std::vector<int> feat_indptr_global;  // for the input dropout ranges

  std::vector<shared_ptr<Variable>> variables;
  std::vector<std::unique_ptr<Module>> modules;
  std::vector<shared_ptr<Variable>> weights;
  std::vector<bool> decays;
  std::vector<shared_ptr<DropoutRng>> rngs;  // [0] input, then one per hidden layer
  std::vector<const Dropout *> dropouts_;
  Adam optimizer;
  DeviceBuffer<float> tn_pool;  // tn_fold: the deferred reduction passes' inputs
  // fuse_finish: the loss kernel's arrival ticket, per-block partials and the pass descriptor
  DeviceBuffer<unsigned> fin_ticket;
  DeviceBuffer<float> fin_part4;
  DeviceBuffer<unsigned> fin_gticket;  // two-level finish: a ticket per 64-B line per group
  DeviceBuffer<float> fin_gpart4;
  int fin_blocks = 0;
  XentFinal fin_desc;
  void arm_finish(int dst_offset, bool graph);
  DeviceBuffer<float> grad_arena;  // all weight grads, one all-reduce
  DeviceBuffer<uint8_t> jump_table;
  DeviceBuffer<uint4> mask_lut;  // the nibble tables in global memory (mask_xstream)
  DeviceBuffer<float> gemm_ws, gemm_ws_side;
  DeviceBuffer<float> xent_partials, sums, results_ring;
  // edge-cut: per ring slot and pass, the all-reduced {loss sum, wrong, sum W1^2, count}; the
  // host composes loss and accuracy from them (compose_raw), so a pass needs no compose launch
  DeviceBuffer<float> raw_ring;
  void compose_raw(const float *raw4, float *out2) const;
  std::pair<float, float> read_slot(int off);
  PinnedBuffer<float> pinned;
  int ring_cap = 1024;
  long long epoch_count = 0;
  bool last_forward_training = false;
  bool reassociated_ = false;
  float ax_build_ms = 0.0f;
  // the last forward ran the output layer over the split's rows only (split_rows): the
  // variables in restricted_vars hold stale rows
  bool out_restricted = false;
  std::vector<int> restricted_vars;

  // Per-epoch hipGraph: epoch_async() replays one captured
  // train_epoch + eval(2).  Everything that changes between epochs lives on the device:
  // the dropout RNG chunk states advance themselves, the Adam step size comes from a host-
  // computed table indexed by a device step counter, the results-ring slot from a device
  // epoch counter, both advanced by the epoch's last kernel.
  hipGraph_t epoch_graph = nullptr;
  hipGraphExec_t epoch_exec = nullptr;
  DeviceBuffer<int> dev_ctr;          // {Adam steps done, epochs done}
  DeviceBuffer<float> step_table;     // step sizes of steps table_block * cap + 1 ...
  static constexpr int kStepTable = 4096;
  long long table_block = -1;
  bool ctr_valid = false;             // dev_ctr equals the host counters
  bool warm = false;                  // one eager epoch_async ran (lazy buffers exist)

  std::vector<std::pair<Event, Event>> gs_events;
  std::vector<std::pair<Event, Event>> mm_events;
  std::vector<double> mm_flops;
  std::vector<double> gs_bytes;
};

}  // namespace pgcn
