// parallel-gcn_amd/csrc/kernels.hpp -- internal launcher interface of the HIP kernels.
// (C ABI wrappers in capi.cpp; host classes in host/*.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "gs_epilogue.hpp"

namespace pgcn {

// Launch counts of the kernel families (process-wide; pgcn_debug_path_count): tests assert
// which kernels a configuration took
enum KernelPath {
  KP_XS_NN_RING, KP_XS_TN_RING, KP_XS_NN, KP_XS_TN, KP_GS_RING, KP_GS_GATHER, KP_OUT_XENT,
  KP_GEMM_NN, KP_GEMM_TN, KP_GEMM_NN_W, KP_GEMM_TN_W, KP_LAUNCHES, KP_COUNT
};
void note_path(KernelPath p);
// every kernel launch of the library goes through this (counted: "launches")
#define PGCN_LAUNCH(...)                     \
  do {                                       \
    ::pgcn::note_path(::pgcn::KP_LAUNCHES);  \
    hipLaunchKernelGGL(__VA_ARGS__);         \
  } while (0)
// n empty kernels back to back on s (the per-launch floor of the small graphs' epochs)
void launch_empty(int n, hipStream_t s);
// mine[i] = the loss kernel's exp of x[i] <= 0, lib[i] = expf(x[i]) (pgcn_debug_exp_check)
void launch_exp_check(const float *x, long long n, float *mine, float *lib, hipStream_t s);
void launch_div_check(const float *a, const float *b, long long n, float *q, hipStream_t s);

// GraphSum work schedule for one row width (VEC float4 per row); device arrays.
struct GraphSchedule {
  int vec = 0;
  int chunk = 0;          // max slots per work item
  int nbc = 1;            // column blocks (workgroup w serves block w % nbc)
  int n_items = 0;        // int4 {row, begin, end, slot(-1 = direct)}, grouped by block
  int max_block_items = 0;
  int n_comb = 0;         // int4 {row, first_slot, count, 0}
  long long n_slots = 0;  // partial rows (VEC float4 each)
  const int4 *items = nullptr;
  const int *block_items = nullptr;  // nbc + 1 offsets into items
  const int4 *comb = nullptr;
  // in-kernel combine (g_gs_split 1): the comb index of each slot, and one arrival counter per
  // comb row (zero between calls); the last item of a split row to finish sums its slots
  const int *slot_comb = nullptr;
  int *comb_ctr = nullptr;
  // workgroup items (g_gs_split 3): rows one whole workgroup sums ({row, begin, end, -1}),
  // taken by the launch's first n_wide workgroups
  int n_wide = 0;
  const int4 *wide = nullptr;
  // d = 16 on the blocked layout: 0 = k_graphsum16 (an item's 64-slot sub-chunks, a 16-slot run
  // per neighbour sub-group), 1 = k_graphsum<4, 16> (sub-group nb takes slots nb, nb + 4, ...:
  // short segments keep every sub-group busy)
  int gather16 = 0;
};
int graphsum_group_lanes(int vec);

void launch_graphsum(const GraphSchedule &s, const int *indices, const float *vals,
                     const float *in, int ld_in, float *out, int ld_out, float *partial,
                     hipStream_t st, const GsEpilogue *epi = nullptr);
bool graphsum_vec_supported(int vec);

// ---- d = 16 GraphSum with LDS-staged feature slices (k_graphsum_ring.hip) -----------------
constexpr int kGraphBlocks = 8;                      // plain kernel: column blocks (one per XCD)
constexpr int LDS_CW = 15;                           // summing waves per workgroup
constexpr int LDS_SLOTS = 16;                        // rowsets (16 rows) per summing wave (max)
// the ring schedule's rowsets per summing wave (r04: 8, half the rows per workgroup and twice
// the batches, measured slower and removed)
constexpr bool ring_slots_ok(int ns) { return ns == LDS_SLOTS; }
constexpr int LDS_THREADS = 64 * (LDS_CW + 1);       // + one slice loader wave
// Sliding-window ring schedule (k_graphsum_ring.hip, host/ring.cpp): slices of RING_SR rows,
// a ring of RING_K slices in LDS as 4 quarter planes of RING_P rows, visits read RING_W slices
// (PGCN_RING_SR / _K / _W override them for schedule experiments; RING_W <= RING_K - 1: the
// loader may run RING_K - RING_W slices ahead of a visit's last slice)
#ifndef PGCN_RING_SR
#define PGCN_RING_SR 512
#endif
#ifndef PGCN_RING_K
#define PGCN_RING_K 4
#endif
#ifndef PGCN_RING_W
#define PGCN_RING_W (PGCN_RING_K - 1)
#endif
constexpr int RING_SR = PGCN_RING_SR;
constexpr int RING_K = PGCN_RING_K;
constexpr int RING_W = PGCN_RING_W;
static_assert(RING_W >= 1 && RING_W <= RING_K - 1 && RING_SR % 64 == 0, "ring shape");
constexpr int RING_P = RING_K * RING_SR + 4;  // + 4 zero rows; = 4 mod 16 (bank quarters)
constexpr int kRingWindow = 5;                // the schedule kind reported by pgcn_debug_lds_counts
// ring schedule rows[]: row id | log2(spread) << 28; kRingEmpty = no row (spread kept)
constexpr int kRingRowMask = 0x0fffffff;
constexpr int kRingEmpty = 0x0fffffff;
static_assert(RING_P % 16 == 4, "plane stride: lane v's chunk = 4v + row (mod 16)");
struct LdsSchedule {
  int n_rows = 0, n_cols = 0;
  int n_batches = 0;  // workgroups = n_batches * n_blocks
  int n_blocks = 4;   // column blocks (workgroup w serves block w % n_blocks)
  int t_max = 0;      // max slices per column block
  int ns = LDS_SLOTS;  // rowsets per summing wave (ring_slots_ok)
  bool pair = false;   // rowsets in lockstep pairs, their blocks alternating (host/ring.cpp)
  int w = RING_W;      // slices a visit reads (2 or 3; k_graphsum_ring's WIN)
  const uint2 *entries = nullptr;            // [kb][16 lane groups] x 4 uint16 row offsets
  const long long *wave_off = nullptr;       // [wg][LDS_CW] first kb of each wave's stream
  const unsigned short *counts = nullptr;    // [wg][t_max][LDS_CW][ns] steps
  const int2 *slices = nullptr;              // [block][t_max] {first column, rows}
  const int *n_slices = nullptr;             // [block]
  const int *rows = nullptr;                 // [batch][LDS_CW][ns][16] row | spread
  const float *row_scale = nullptr;          // 1/sqrt(deg) of output rows
  const float *col_scale = nullptr;          // 1/sqrt(deg) of input rows
};
// prescale (skipped when `prestaged`: scratch_in already holds this call's prescaled input,
// written by the epilogue of the kernel that produced `in`) + ring kernel + combine (+ epi);
// scratch_in holds ceil(n_cols / RING_SR) slices
// the column offsets of a wide GraphSum's 16-column passes (<= 8: d <= 128)
struct RingPasses {
  int n = 0;
  int c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};
// every pass's prescaled table in one launch: tables + p * table_floats = pass p's scratch
void launch_ring_prescale_wide(const LdsSchedule &s, const float *in, int ld_in, int width,
                               const RingPasses &passes, float *tables, long long table_floats,
                               hipStream_t st);
void launch_graphsum_ring(const LdsSchedule &s, const float *in, int ld_in, float *out,
                          int ld_out, float *scratch_in, float *partial, hipStream_t st,
                          const int *col_map = nullptr, const GsEpilogue *epi = nullptr,
                          bool prestaged = false, const struct PeerSink *push = nullptr,
                          hipStream_t tail_st = nullptr, hipEvent_t fork = nullptr);
// The edge-cut engine's GraphSum tail: after the reduce-scatter has summed every rank's
// partials into this rank's rows y [n][ld] (ld % 4 == 0, dim % 4 == 0), the fused
// element-wise epilogue (gs_epilogue.hpp: ReLU / Dropout, the next GraphSum's table) in place
void launch_gs_finish(float *y, int ld, int n, int dim, const GsEpilogue &epi, hipStream_t st);

// maskT (optional): the same dropout bits in the nibble layout, read by the wide kernels
void launch_gemm_nn(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                    int trans_b, float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                    long long mask_ld, float a_scale, hipStream_t s,
                    const uint64_t *maskT = nullptr);
size_t gemm_tn_workspace(int M, int N, int K);
// wide outputs (k_gemm_wide.hip): N in 33..128 (the hidden-128 layers and their output layer),
// register-blocked MFMA; maskT: A's dropout bits in the nibble layout (k_mask_nibbles, K <=
// 1024) instead of the flat bitmap a_mask
bool gemm_wide_ok(int N);
void launch_gemm_nn_wide(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                         int trans_b, float *C, int ldc, const uint64_t *a_mask,
                         long long mask_base, long long mask_ld, float a_scale, hipStream_t s,
                         int nst, const uint64_t *maskT = nullptr);
size_t gemm_tn_wide_workspace(int M, int N, int K);
void launch_gemm_tn_wide(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                         long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                         int nst, const uint64_t *maskT = nullptr);
// ordered reduce of n_slabs partials [K][ldp] (k_gemm.hip): slab order, deterministic
void launch_slab_reduce(float *partial, int n_slabs, int K, int N, int ldp, float *C, int ldc,
                        int nst, hipStream_t s);
// X-stream kernels (k_gemm.hip): N <= 16, K <= 640, dropout bits in the nibble layout
bool xstream_ok(int N, int K);
void launch_mask_nibbles(const uint64_t *mask, long long mask_base, long long mask_ld, int M,
                         int K, uint64_t *out, hipStream_t s);
// What the first layer's X-stream product feeds (single C output, N <= 16): relu = the ReLU
// of the GraphSum it stands for (eval from Â X; no mask: eval only), next_table = that
// GraphSum's or the next one's prescaled ring table (next_scale[r] * value at the ring
// layout of k_ring_prescale), so neither the ReLU nor the prescale needs a launch
// One variable's mask draw (k_dropout_mask's segment; mask_draw.hpp draws it)
struct MaskSeg {
  uint64_t *states = nullptr;
  long long n_chunks = 0, elem0 = 0, elem_end = 0;
  int threshold = 0;
  uint64_t *mask = nullptr;
  int per = 1;  // 64-draw words per stored state (MaskDraw::per)
};
// masks drawn by extra waves of the X-stream NN kernel (`mask_xstream`): up to two segments,
// the nibble tables (32 x 16 uint4, launch_mask_lut) in global memory
struct XsDraw {
  MaskSeg seg[2];
  int n = 0;
  const uint4 *lut = nullptr;
};
struct XsEpilogue {
  int relu = 0;
  // backward tails of the product's rows [M][ldc] (Matmul input grad): element e = r*ldc + j
  // times Dropout's keep-bit (base + e) ? scale : 0, then 0 where the ReLU's mask byte e is 0
  // (k_dropout_apply then k_relu_bwd: the same bits)
  const uint64_t *bwd_drop = nullptr;
  long long drop_base = 0;
  float drop_scale = 0.0f;
  const uint8_t *bwd_relu = nullptr;
  float4 *next_table = nullptr;
  const float *next_scale = nullptr;
  int next_sr = 0;
  const XsDraw *draw = nullptr;  // (host) masks the ring NN kernel draws beside its product
};
// The flat dropout bitmap of X [M][K] (keep bit of X[m][k] at bit base + m * ld + k, the
// element order rng.cpp draws), which the X-stream ring kernels read in place of the nibble
// layout: their loader waves stage each 16-row group's bits beside its X (no nibble pass)
struct XsMask {
  const uint64_t *bits = nullptr;
  long long base = 0, ld = 0;
  long long words = 0;  // uint64 words at bits, even (staged in whole 16-B pieces inside them)
};
// flat: the mask as a flat bitmap instead of maskT (the ring kernels only: xstream_ring_ok)
void launch_xstream_nn(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                       int trans_b, float *C, int ldc, const uint64_t *maskT, float a_scale,
                       hipStream_t s, float *C2 = nullptr,  // C2: drop(X) W beside C = X W
                       const XsEpilogue *epi = nullptr, const XsMask *flat = nullptr);
// k_xstream_lds.hip: the X-stream products with loader and MFMA waves split (the default
// form, g_xstream_ring; the launchers above dispatch to them)
bool xstream_ring_ok(int K, int lda);
void launch_xstream_nn_ring(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                            int trans_b, float *C, int ldc, const uint64_t *maskT, float a_scale,
                            hipStream_t s, float *C2, const XsEpilogue &e,
                            const XsMask *flat = nullptr);
// partial[n_blocks][K][16] (the workgroups' sums; reduced in block order by the caller)
void launch_xstream_tn_ring(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                            const uint64_t *maskT, float a_scale, float *partial, int n_blocks,
                            hipStream_t s, const XsMask *flat = nullptr);
// out[r][0:ld] = src[rows[r]][0:ld]  (ld % 4 == 0)
void launch_gather_rows(const float *src, const int *rows, int n, int ld, float *out,
                        hipStream_t s);
// ---- peer-mapped exchange (k_peer.hip, host/comm.cpp PeerComm) -----------------------------
constexpr int kPeerMaxRanks = 16;
// a wait gives up after this many ticks of the 100 MHz s_memrealtime clock (20 s)
constexpr unsigned long long kPeerTimeoutTicks = 2000000000ull;
// where one collective's pushes of this rank go: receiver q's slot of this rank (dst[q], in q's
// memory or, q == rank, this rank's own) and q's flag word of this rank
struct PeerSink {
  float *dst[kPeerMaxRanks];
  unsigned *flag[kPeerMaxRanks];
  unsigned *arrive = nullptr;  // this rank's arrival counter (zero between launches)
  long long slot_bytes = 0;    // bytes from dst[q] to the end of q's slot
  unsigned gen = 0;            // the collective's generation, stored into the flags
  int world = 0;               // 0: not pushing
  int rows_per_rank = 0;       // GraphSum push: padded rows per owner (row r -> owner r / this)
  int signal = 1;              // 0: an earlier pass of a multi-pass push (no flags yet)
  // the wait fused into the push (separate processes): the signalling launch's last workgroup
  // then polls this rank's flags wait_flags[q < nwait] for gen (bounded as k_peer_wait); 0: the
  // receiver launches k_peer_wait itself
  const unsigned *wait_flags = nullptr;
  int nwait = 0;
  unsigned *err = nullptr;
};
// this rank's received slots of one collective: slot[q] = what rank q pushed
struct PeerRecv {
  const float *slot[kPeerMaxRanks];
  int world = 0;
};
// one small all-reduce done inside one workgroup (peer_allreduce_block, peer_sync.hpp): push,
// signal, wait for waited[q < nwait], sum the received slots in rank order
struct PeerSmall {
  PeerSink k;
  PeerRecv r;
  const unsigned *waited = nullptr;
  int nwait = 0;
  unsigned *err = nullptr;
};
// send [world][count] -> sink.dst[q] (same_for_all: send [count] to every q); then the flags
// (the launch's last workgroup)
void launch_peer_push(const float *send, size_t count, const PeerSink &k, hipStream_t s,
                      bool same_for_all);
// one wave until flags[q] == gen for every q < world (err: set on a timeout, then no waiting)
void launch_peer_wait(const unsigned *flags, int world, unsigned gen, unsigned *err,
                      hipStream_t s);
// one workgroup: push buf [n] to every receiver, signal, wait for waited[q < nwait], sum the
// received slots in rank order back into buf (separate processes only: see k_peer.hip).
// Up to 1,024 floats (the loss / wrong-count pairs): the weight gradients (10.3 k floats on
// reddit) took 51 us in one workgroup at W = 8 (its write-through pushes run at one
// workgroup's rate, profiles/r05/g/rank8_breakdown.txt) against ~15 us for the three-kernel
// form's whole-grid push, wait and sum
constexpr int kPeerSmallAllreduce = 1 << 10;
void launch_peer_allreduce_small(float *buf, int n, const PeerSink &k, const PeerRecv &r,
                                 const unsigned *waited, int nwait, unsigned *err, hipStream_t s);
// dst[i] = sum over q (rank order) of r.slot[q][i]
void launch_peer_sum(const PeerRecv &r, float *dst, size_t count, hipStream_t s);
// the GraphSum exchange's receiving end: y[j] (j < n local rows, [ld] floats, dim columns) =
// sum over q (rank order) of r.slot[q] row j, then the fused element-wise epilogue (as
// launch_gs_finish)
void launch_gs_gather_finish(float *y, int ld, int n, int dim, const GsEpilogue &epi,
                             const PeerRecv &r, hipStream_t st);

// out[rows[r]][0:ld] = src[r][0:ld]  (ld % 4 == 0)
void launch_scatter_rows(const float *src, const int *rows, int n, int ld, float *out,
                         hipStream_t s);
void launch_xstream_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                       float *C, int ldc, const uint64_t *maskT, float a_scale, void *workspace,
                       hipStream_t s, const XsMask *flat = nullptr);
void launch_gemm_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                    float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                    long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                    const uint64_t *maskT = nullptr);

void launch_spmm_csr(int m, int p, int ldc, const int *indptr, const int *indices,
                     const float *a, const uint64_t *mask, long long mask_base, float scale,
                     const float *b, float *c, hipStream_t s);
// c = X b and c2 = drop(X) b from one pass over X (the sparse form of the X-stream dual)
void launch_spmm_csr_dual(int m, int p, int ldc, const int *indptr, const int *indices,
                          const float *a, const uint64_t *mask, long long mask_base, float scale,
                          const float *b, float *c, float *c2, hipStream_t s);
// nnz: the entries of all nf columns (picks the chunk size; 0 = unknown: 256); order (optional):
// the nf feature ids in the order their workgroups launch (descending column length)
void launch_spmm_csc_bwd(int nf, int p, int ldg, const int *csc_ptr, const int *csc_row,
                         const int *csc_pos, const float *a, const uint64_t *mask,
                         long long mask_base, float scale, const float *cgrad, float *bgrad,
                         hipStream_t s, long long nnz = 0, const int *order = nullptr,
                         bool tree = false);  // tree: k_spmm_csc_tree (not the chain's bits)

void launch_dropout_mask(uint64_t *states, long long n_chunks, long long elem0,
                         long long elem_end, float p, uint64_t *mask, const void *table,
                         hipStream_t s, int max_blocks = 0, int per = 1);
// two variables' draws (each as launch_dropout_mask's arguments) in one launch
// per: 64-draw mask words per stored state (1, or 2: one state per 128 draws -- half the state
// traffic and half the period jumps per draw, the engine's layout; the C ABI's is 1)
struct MaskDraw {
  uint64_t *states;
  long long n_chunks, elem0, elem_end;
  float p;
  uint64_t *mask;
  int per = 1;
};
void launch_dropout_mask2(const MaskDraw &d0, const MaskDraw &d1, const void *table,
                          hipStream_t s);
// the segment k_dropout_mask draws for d (launch_dropout_mask's threshold)
MaskSeg mask_seg_of(const MaskDraw &d);
// lut [32 * 16] uint4 = the nibble tables k_dropout_mask stages in LDS, from the byte tables
void launch_mask_lut(const void *table, void *lut, hipStream_t s);
void launch_dropout_apply_based(float *x, long long n, const uint64_t *mask, long long base,
                                float scale, hipStream_t s);
void launch_relu_fwd(float *x, long long n, uint8_t *mask, int training, hipStream_t s);
void launch_relu_bwd(float *g, long long n, const uint8_t *mask, hipStream_t s);
int xent_blocks(int n);
// the output layer's product and the loss in one pass (k_xent_fwd<true>): logits = H W
// (H [n][ldh], kh <= 16 columns; W [kh][ldw]) written max-shifted like launch_xent_fwd's
// write_back, then its loss / grad / wrong count; bit-identical to launch_gemm_nn + xent.
// Training with dH: also dH [n][lddh] = grad W^T (columns >= kh zero), bit-identical to the
// Matmul backward's launch_gemm_nn(trans_b)
// Training with tb.table: dH row i also goes, prescaled, to the ring table of the GraphSum
// backward that reads dH -- tb.scale[p] * dH[i][0:16] at table row p = tb.pos[i] (skipped when
// p < 0; null pos: p = i for i < tb.rows), k_ring_prescale's products in its slice-plane
// layout, so that call skips its prescale launch
struct XentTable {
  float *table = nullptr;
  const float *scale = nullptr;
  const int *pos = nullptr;
  int rows = 0;
};
// One GPU (r06): the pass's scalars finished inside the loss kernel -- k_reduce_scalars' work
// done by its last-arriving block.  Every block writes {loss, wrong, its slice of sum w^2, 0}
// to part4[block] write-through (sc1) and adds one to *ticket; the block whose add returns
// gridDim - 1 reads every part4 write-through, sums them in block order (a fixed tree), writes
// out2 = {loss / count + wd * l2 / 2, (count - wrong) / count} (slot 4 * (ctr[1] % ring_cap)
// with ctr) and the optional sums {loss, wrong}, and zeroes the ticket for the next launch
struct XentFinal {
  const float *w = nullptr;  // W1 (the l2 term), n_w floats
  long long n_w = 0;
  float wd = 0.0f;
  float *out2 = nullptr;
  const int *ctr = nullptr;
  int ring_cap = 1;
  float *sums = nullptr;
  unsigned *ticket = nullptr;  // zero between launches
  float4 *part4 = nullptr;     // [blocks]
  // two levels (large grids, r06): blocks arrive on their group's ticket (gticket[16 g]: one
  // 64-B line each) and the group's last block sums the group's partials into gpart4[g], then
  // arrives on `ticket`; group = 0: every block on `ticket`
  int group = 0;
  unsigned *gticket = nullptr;  // [groups * 16], zero between launches
  float4 *gpart4 = nullptr;     // [groups]
};
void launch_out_xent(const float *H, int ldh, int kh, const float *W, int ldw, float *logits,
                     int ld, float *grad, const int *truth, int n, int c, int count, int training,
                     float *partials, hipStream_t s, float *dH = nullptr, int lddh = 0,
                     float *dWp = nullptr, const XentTable *tb = nullptr,
                     const XentFinal *fin = nullptr);
// with dWp (training, <= 48 classes): per-block partials [xent_blocks(n)][kh][48] of W.grad =
// H^T grad, reduced in block order into C [kh][ldc] (N = c columns) by:
void launch_tn_reduce_blocks(float *partial, int n_blocks, int K, int N, int ldp, float *C, int ldc,
                             hipStream_t s);
// tn_defer active (the Adam launch sums deferred passes): room in its pool for n_blocks
// per-block partials [K][ldp] of C [K][N] (ldc == N) and the deferred entry that sums them in
// block order (one ordered pass, k_gemm_tn_reduce's loads and adds), or null
float *tn_defer_blocks(int n_blocks, int K, int N, int ldp, float *C, int ldc);
// C [K][N] = the n partials [K][ldp] summed in order by one k_gemm_tn_reduce pass (the sum
// a tn_defer_blocks entry makes in the Adam launch)
void launch_tn_reduce_one_pass(const float *partial, int n, int K, int N, int ldp, float *C,
                               int ldc, hipStream_t s);
size_t tn_reduce_blocks_workspace(int n_blocks, int K, int ldp);
void launch_xent_fwd(float *logits, int ld, float *grad, const int *truth, int n, int c,
                     int count, int training, float *partials, hipStream_t s, int write_back = 1,
                     const XentFinal *fin = nullptr);
// sums (optional): {loss sum, wrong}; out2 (optional): the composed {loss + l2, accuracy};
// raw4 (optional): {loss sum, wrong, sum w^2, count} for a composition after an all-reduce
void launch_reduce_scalars(const float *partials, int n_blocks, const float *w, long long n_w,
                           float *sums, hipStream_t s, int count = 0, float wd = 0.0f,
                           float *out2 = nullptr, const int *ctr = nullptr, int ring_cap = 1,
                           float *raw4 = nullptr, const PeerSmall *peer = nullptr);
// ctr (epoch graphs, device {Adam step, epoch} counters): out2 is slot 4 * (ctr[1] % ring_cap)
// step_table (epoch graphs): step_size = step_table[ctr[0] % table_cap]
void launch_adam(float *w, const float *g, float *m, float *v, long long n, float step_size,
                 float beta1, float beta2, float eps, float wd, int decay, hipStream_t s,
                 const float *step_table = nullptr, const int *ctr = nullptr, int table_cap = 1);
// all weights of the model in one launch (<= kAdamBatch tensors; tensor t = grid row t)
constexpr int kAdamBatch = 8;
// The last ordered pass of a weight gradient's split reduction (k_gemm_tn_reduce), deferred
// into the Adam launch: grad[k][j] = sum over groups q < n_groups, in order, of
// src[q * K * ldp + k * ldp + j] (the same loads and adds: the same bits), stored to C and used
// by the update (one GPU; an edge-cut rank all-reduces the finished gradients in between)
struct TnDeferred {
  const float *src = nullptr;
  int n_groups = 0, K = 0, N = 0, ldp = 0;
  float *C = nullptr;
};
struct TnDeferList {
  int n = 0;
  TnDeferred d[4];
  // the deferred passes' inputs (the first pass's group sums) go here, not to the GEMM
  // workspace that later products of the same backward pass reuse
  float *pool = nullptr;
  size_t pool_floats = 0, used = 0;
};
// while set (this host thread), tn_reduce records its last pass here instead of launching it
// when that pass writes a whole [K][N] gradient (ldc = nst = N) from two passes and the list's
// pool has room for the first pass's output
void tn_defer(TnDeferList *list);
// launches every recorded pass not taken by an Adam launch (k_gemm_tn_reduce), empties the list
void tn_defer_flush(TnDeferList &list, hipStream_t s);

struct AdamBatch {
  float *w[kAdamBatch];
  const float *g[kAdamBatch];
  float *m[kAdamBatch], *v[kAdamBatch];
  long long n[kAdamBatch];
  int decay[kAdamBatch];
  int count;
  TnDeferred red[kAdamBatch];  // red[t].src: tensor t's gradient reduced first (into g[t])
  // peer.world > 0 (edge-cut, processes): tensor t's all-reduced gradient is the rank-order sum
  // of the received slots at arena_off[t] (stored into g[t] first; k_peer_sum's sum)
  PeerRecv peer;
  long long arena_off[kAdamBatch];
};
// The weight gradients' all-reduce push between processes (PeerComm::allreduce_grads): element
// i of the arena, or -- inside deferred region r (arena offset offs[r]) -- the deferred pass's
// sum, stored to every receiver's slot of this rank; the push's last workgroup signals and waits
// (peer_arrive).  k_peer_push's job with the TN reductions' last passes folded in.
struct GradRegions {
  int n = 0;
  long long off[4];
  TnDeferred d[4];
};
void launch_peer_push_grads(const float *arena, long long n, const GradRegions &r,
                            const PeerSink &k, hipStream_t s);
// draws (optional, eager one-GPU steps): up to two masks drawn by the same launch (k_adam_mask;
// MaskDraw and `table` as launch_dropout_mask2)
void launch_adam_multi(const AdamBatch &b, float step_size, float beta1, float beta2, float eps,
                       float wd, hipStream_t s, const float *step_table = nullptr,
                       const int *ctr = nullptr, int table_cap = 1,
                       const MaskDraw *draws = nullptr, int n_draws = 0,
                       const void *table = nullptr);
// set: ctr = {step, epoch}; else both += 1 (the end of a graph-replayed epoch)
void launch_counters(int *ctr, int set, int step, int epoch, hipStream_t s);

}  // namespace pgcn
