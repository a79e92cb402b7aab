// parallel-gcn_amd/csrc/host/graph.hpp -- device adjacency for GraphSum.
//
// The reference keeps the adjacency as DevSparseIndex (include/sparse.cuh:21-29) plus a
// separately uploaded dev_graph_value array (src/parser.cpp:164-181, src/gcn.cu:30-43).  Here
// DevGraph owns the CSR column ids, the Â coefficients and, per row width, the wavefront
// work schedule of k_graphsum (built once; the graph is static across epochs).
//
// Two device layouts:
//  * plain  -- the CSR as given (row-major); work items are row chunks.
//  * blocked -- for feature tables larger than one XCD's L2: the columns are cut into 8
//    nnz-balanced blocks and the edges stored block-major (all of block 0's row segments,
//    then block 1's, ...), so the index/value stream of one block is contiguous and the
//    workgroups of one XCD gather from one 1/8 slice of the feature table.
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
                  int threads = 0, long long min_parallel = 100000);

// True when the pattern equals its transpose, duplicates counted (the multiset of (i, j) is
// the multiset of (j, i)): Â is then symmetric.  Two independent 64-bit hash sums over the
// slots, O(nnz) on the host threads.
bool csr_symmetric(int n, const int *indptr, const int *indices);

// s[i] = 1/sqrt(deg_i) with deg = row length of the (symmetric) CSR: Â = D^-1/2 A D^-1/2.
std::vector<float> degree_scales(int n, const int *indptr);

// Host image of the d = 16 LDS ring schedule (k_graphsum_ring.hip), before upload.
struct LdsHost {
  int n_batches = 0, t_max = 0, n_blocks = 4, ns = LDS_SLOTS;
  bool pair = false;                    // rowsets 2p, 2p+1 in lockstep (ring_pair)
  int w = RING_W;                       // slices a visit reads (window)
  std::vector<int> nsl;                 // slices per column block
  std::vector<int2> slices;             // [block][t_max] {first column, rows}
  std::vector<int> rows;                // [batch][LDS_CW][ns][16] row | spread
  std::vector<unsigned short> counts;   // [wg][t_max][LDS_CW][ns]
  std::vector<long long> wave_off;      // [wg*LDS_CW + 1] entry-block offsets
  std::vector<unsigned short> entries;  // [kb][16 groups][4 steps] ring-row byte offsets
};
// nnz-balanced column cuts (kGraphBlocks + 1 boundaries)
std::vector<int> column_cuts(int n_cols, const std::vector<int> &indices,
                             int n_blocks = kGraphBlocks);
// column blocks of the LDS GraphSum schedule of an n_rows x n_cols graph (XCD-affine), and
// its rowsets per summing wave (ring_slots_ok; knob "lds_slots")
int lds_blocks(int n_rows, int n_cols);
int lds_slots(int n_rows, int n_cols);
// ring schedule (host/ring.cpp): block cuts on RING_SR multiples, the schedule, and its CPU
// walk as the kernel consumes it: out[row] += sum of in[col] (throws on an inconsistent
// schedule)
std::vector<int> ring_cuts(int n_cols, const std::vector<int> &indices, int n_blocks);
// pair: rowsets 2p and 2p + 1 of a wave run the same step count per visit and their entry
// blocks alternate in the stream (k_graphsum_ring<.., true>: both blocks' table reads in flight
// under one wait); -1 = the "ring_pair" knob
// window: slices a visit reads, 2 or 3 (ring_window_for)
LdsHost build_ring_host(int n_rows, int n_cols, const std::vector<int> &indptr,
                        const std::vector<int> &indices, const std::vector<int> &bcut,
                        int ns = LDS_SLOTS, int pair = -1, int window = RING_W);
extern int g_ring_pair;
// "ring_window" (read at schedule build): 0 = by shape (ring_window_for), 2 or 3
extern int g_ring_window;
int ring_window_for(int n_rows, int n_cols, long long nnz, int n_blocks);
void ring_emulate(const LdsHost &h, int n_rows, const float *in, double *out);

class DevGraph {
 public:
  // CSR with n_rows rows and column ids < n_cols; `vals` aligned with `indices`.
  DevGraph(int n_rows, int n_cols, const int *indptr, const int *indices, const float *vals);
  int rows() const { return n_rows_; }
  int cols() const { return n_cols_; }
  long long nnz() const { return nnz_; }
  // out[i,:dim] = sum_j val_ij * in[col_j,:dim]
  // compact_in (column subsets): `in` holds the subset's columns as its rows (no gather)
  // epi: the element-wise tail applied to every output row as it is formed (one pass only:
  // dim <= 16, or a width with a kernel of its own and no 16-column passes)
  // tables_ready: the prescaled table(s) this call reads were filled by a call of the same
  // input on a graph sharing them (share_tables; can_share_tables(dim, ld_in)): no prescale launch
  void graphsum(const float *in, int ld_in, float *out, int ld_out, int dim, hipStream_t s,
                bool compact_in = false, const GsEpilogue *epi = nullptr, bool prestaged = false,
                bool tables_ready = false, const PeerSink *push = nullptr,
                hipStream_t tail_st = nullptr, hipEvent_t fork = nullptr);
  // The ring schedule reads its prescaled input tables from `owner`'s buffers (same columns,
  // column scales and column map: the edge-cut engine's row chunks of one column block), so
  // one prescale serves every graph of the group.
  void share_tables(DevGraph *owner);
  // a graphsum() of this width prescales into tables a sharing graph can read as they are
  bool can_share_tables(int dim, int ld_in) const;
  const DevGraph *table_owner() const { return table_owner_; }
  // The ring schedule's prescaled-input table of a graphsum() of this width (one 16-column
  // pass, no column map), for a producer's epilogue to fill (then graphsum(.., prestaged));
  // null when this graph does not take that path.  next_scale = the table's column scales.
  float *ring_table(int dim, const float **next_scale);
  // ... of a column subset too: its input rows map to table rows through *pos (input row i ->
  // table row pos[i], -1 outside the subset; *pos_rows input rows; null pos: the identity over
  // the graph's columns), for the fused loss kernel's dH (XentTable)
  float *ring_table_mapped(int dim, const float **next_scale, const int **pos, int *pos_rows);
  // graphsum() of this width can take an epilogue (one pass over the columns)
  bool epilogue_ok(int dim, int ld_in, int ld_out) const;
  // graphsum() of this width runs the LDS ring kernel (k_graphsum_ring)
  bool uses_lds(int dim) const;
  // builds the schedule a graphsum() of this width will use now (host work, kept out of timed
  // device regions)
  void prepare(int dim);
  // bytes the kernel must move at minimum (SURVEY.md §8d formula, per call)
  double algorithmic_bytes(int dim) const;
  // schedule statistics (for tests / reports)
  int column_blocks(int dim);

  // Enables the d = 16 LDS path (k_graphsum_ring): out_i = row_scale_i * sum_j col_scale_j
  // in_j over the CSR pattern, i.e. vals_ij = row_scale_i * col_scale_j.
  void set_scales(std::vector<float> row_scale, std::vector<float> col_scale);
  // The rows `rows` (ascending) of this CSR as a graph of its own: same columns, values and
  // scales, row r of the result = row rows[r] here.
  std::unique_ptr<DevGraph> row_subset(const std::vector<int> &rows) const;
  // The edges into the columns `cols` (ascending) as a graph over those columns only: its
  // graphsum() reads input row cols[c] for column c (no compaction by the caller), so it
  // equals this graph's graphsum on an input that is zero outside `cols`.
  std::unique_ptr<DevGraph> col_subset(const std::vector<int> &cols) const;

  static constexpr int kBlocks = kGraphBlocks;   // one column block per XCD
  static constexpr double kL2Budget = 4.0e6;     // one XCD's L2: tables the plain kernel keeps whole
  static constexpr long long kSmallNnz = 1 << 20;  // g_gs_split 1-3: the small-graph schedules
  static constexpr int kWideCap = 1536;  // g_gs_item_iters 0: workgroup items (6 per CU) at most
  static constexpr long long kLdsMinBytes = 1 << 20;  // d = 16 tables above: LDS GraphSum ...
  static constexpr int kLdsMinRows = 32768;           // ... when the rows fill its workgroups

 private:
  struct Sched {
    GraphSchedule s;
    DeviceBuffer<int4> items, comb, wide;
    DeviceBuffer<int> block_items, slot_comb, comb_ctr;
    DeviceBuffer<float> partial;
  };
  Sched &schedule(int vec);
  void build_blocked();
  void compute_cuts();
  void build_lds();
  struct LdsSched {
    LdsSchedule s;
    DeviceBuffer<uint2> entries;
    DeviceBuffer<long long> wave_off;
    DeviceBuffer<unsigned short> counts;
    DeviceBuffer<int2> slices;
    DeviceBuffer<int> n_slices, rows;
    DeviceBuffer<float> row_scale, col_scale, scratch, partial;
    DeviceBuffer<float> tables;  // every pass's prescaled table of a wide call (lazily)
  };
  std::unique_ptr<LdsSched> lds_;
  DevGraph *table_owner_ = nullptr;  // share_tables: the graph whose table buffers this one reads
  float *table_scratch();            // the one-pass table (own or the owner's)
  float *table_wide(size_t floats);  // the multi-pass tables (own or the owner's), >= floats
  std::vector<float> h_row_scale_, h_col_scale_;
  // column subset: input row of compact column c (device), and the compacted input (plain path)
  DeviceBuffer<int> col_map_;
  DeviceBuffer<int> col_pos_;  // input row -> compact column (-1: outside), col_pos_rows_ rows
  int col_pos_rows_ = 0;
  DeviceBuffer<float> col_in_;
  // column subset, unblocked plain path: every slot's ORIGINAL column id, so the gather kernel
  // reads the caller's full input rows (no compacting launch; the same values, the same bits)
  DeviceBuffer<int> orig_indices_;
  int n_rows_, n_cols_;
  long long nnz_;
  std::vector<int> h_indptr_, h_indices_;
  std::vector<float> h_vals_;
  DeviceBuffer<int> indices_;  // plain layout
  DeviceBuffer<float> vals_;
  // blocked layout
  bool blocked_built_ = false;
  std::vector<int> bcut_;                 // kBlocks + 1 column boundaries
  std::vector<int> lds_cut_;              // LDS schedule: lds_blocks() + 1 boundaries
  std::vector<long long> bseg_;           // (kBlocks) x (n_rows + 1) segment offsets
  long long bnnz_ = 0;                    // blocked slots incl. padding
  DeviceBuffer<int> bindices_;
  DeviceBuffer<float> bvals_;
  std::map<int, std::unique_ptr<Sched>> scheds_;
};

}  // namespace pgcn
