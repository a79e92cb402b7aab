// parallel-gcn_amd/csrc/host/graph.cpp
#include "graph.hpp"

#include <atomic>

#include <algorithm>
#include <cmath>
#include <functional>
#include <numeric>
#include <thread>

namespace pgcn {

float graph_coef(int deg_src, int deg_dst) {
  // hpdga-spring23/src/module.cpp:88-90: int product -> float for sqrtf, double division,
  // stored to float.  (src/parser.cpp:164-181 precomputes the same expression.)
  return (float)(1.0 / (double)sqrtf((float)(deg_src * deg_dst)));
}

void parallel_for(long long n, const std::function<void(long long, long long)> &f, int threads,
                  long long min_parallel) {
  if (threads <= 0) {
    threads = (int)std::thread::hardware_concurrency();
    if (threads > 16) threads = 16;  // the GPU box grants 16 CPUs per GPU
    if (threads < 1) threads = 1;
  }
  if (n < min_parallel || threads == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const long long step = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    const long long b = t * step, e = std::min(n, b + step);
    if (b >= e) break;
    ts.emplace_back([=, &f] { f(b, e); });
  }
  for (auto &t : ts) t.join();
}

std::vector<float> graph_coefs(int n, const int *indptr, const int *indices) {
  std::vector<float> v((size_t)indptr[n]);
  parallel_for(n, [&](long long b, long long e) {
    for (long long src = b; src < e; src++) {
      const int ds = indptr[src + 1] - indptr[src];
      for (int i = indptr[src]; i < indptr[src + 1]; i++) {
        const int dst = indices[i];
        v[i] = graph_coef(ds, indptr[dst + 1] - indptr[dst]);
      }
    }
  });
  return v;
}

namespace {
inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
}  // namespace

bool csr_symmetric(int n, const int *indptr, const int *indices) {
  const int nt = 16;
  std::vector<uint64_t> acc((size_t)nt * 4, 0);
  std::atomic<int> slot{0};
  parallel_for(n, [&](long long b, long long e) {
    const int t = slot++;
    uint64_t f0 = 0, f1 = 0, r0 = 0, r1 = 0;
    for (long long i = b; i < e; i++)
      for (int k = indptr[i]; k < indptr[i + 1]; k++) {
        const uint64_t a = (uint64_t)(uint32_t)i, c = (uint64_t)(uint32_t)indices[k];
        f0 += mix64(a << 32 | c);
        f1 += mix64((a << 32 | c) ^ 0x5851f42d4c957f2dull);
        r0 += mix64(c << 32 | a);
        r1 += mix64((c << 32 | a) ^ 0x5851f42d4c957f2dull);
      }
    acc[(size_t)t * 4] = f0;
    acc[(size_t)t * 4 + 1] = f1;
    acc[(size_t)t * 4 + 2] = r0;
    acc[(size_t)t * 4 + 3] = r1;
  }, nt);
  uint64_t s[4] = {0, 0, 0, 0};
  for (int t = 0; t < nt; t++)
    for (int q = 0; q < 4; q++) s[q] += acc[(size_t)t * 4 + q];
  return s[0] == s[2] && s[1] == s[3];
}

std::vector<float> degree_scales(int n, const int *indptr) {
  std::vector<float> s((size_t)n);
  for (int i = 0; i < n; i++) {
    const int d = indptr[i + 1] - indptr[i];
    s[(size_t)i] = d > 0 ? (float)(1.0 / std::sqrt((double)d)) : 0.0f;
  }
  return s;
}

DevGraph::DevGraph(int n_rows, int n_cols, const int *indptr, const int *indices,
                   const float *vals)
    : n_rows_(n_rows), n_cols_(n_cols), nnz_(indptr[n_rows]), h_indptr_(indptr, indptr + n_rows + 1),
      h_indices_(indices, indices + indptr[n_rows]), h_vals_(vals, vals + indptr[n_rows]) {
  indices_.allocate((size_t)nnz_ + 64);  // slack: unrolled loads never step past the end
  vals_.allocate((size_t)nnz_ + 64);
  indices_.upload(h_indices_);
  vals_.upload(h_vals_);
  PGCN_HIP(hipMemset(indices_.get() + nnz_, 0, 64 * sizeof(int)));
  PGCN_HIP(hipMemset(vals_.get() + nnz_, 0, 64 * sizeof(float)));
}

// d = 16 feature tables above this byte count take the LDS GraphSum ("lds_min_kb"; the
// plain path blocks its columns per XCD above DevGraph::kL2Budget: below it one XCD's 4 MB L2
// holds the whole table).  The LDS path also wants rows to fill its workgroups (kLdsMinRows).
// r02, the edge-cut engine's per-rank graphs of reddit-114M (tools/rank_graphsum.py, 118 k
// padded rows): 3.7 MB table (4 ranks) LDS 0.123 vs plain 0.249 ms, 1.9 MB (8 ranks) 0.083 vs
// 0.114 ms; 15 MB (1 rank) 0.33 vs 1.04 ms
long long g_lds_min_bytes = DevGraph::kLdsMinBytes;


// "gs_split" (read at schedule build), the rows of the plain unblocked path longer than one
// work item: 0 = their items write slots that a combine launch sums; 1 = the last of a row's
// items to finish sums them in the same launch (an arrival counter per row, the combine's
// order: the same bits), on graphs of <= kSmallNnz slots (each arrival writes its XCD's L2
// back: costly when many rows split -- pubmed_synth lost 4 % at 8-iteration items); 2 = on
// those graphs, rows up to 8 items long stay one item (no slots; another summation order);
// 3 = as 1, but rows of up to 8 workgroup-wide iterations are summed by one whole workgroup
// (4 waves, an LDS reduce in wave order: no cross-workgroup hand-off; another summation
// order), power-of-two row widths
int g_gs_split = 3;
// "gs_item_iters" (read at schedule build): group iterations per work item of the plain
// unblocked path on graphs of <= kSmallNnz slots with gs_split 1 / 3 (32 elsewhere).  A small
// graph's GraphSum lasts as long as its longest item (one index -> gather round trip per
// iteration), so its long rows are cut short and summed in-kernel or by workgroup items.
// 0 (default) = by shape with gs_split 3: the shortest of 2, 4, 8, 16, 32 that leaves at most
// kWideCap workgroup items (r04 late: cora 224 rows at 2 iterations, 11.5k vs 11.1k epochs/s
// at 8; pubmed_synth 3,215 rows at 2 lost 2 %, 1,321 at 4 gained 1 %: profiles/r04/ab_item_iters.txt)
int g_gs_item_iters = 0;
// "gs_orig_cols" (read per call): a column subset's unblocked plain GraphSum gathers the
// input's own rows through the original column ids (1) instead of compacting them first (0)
int g_gs_orig_cols = 1;
// "gs16_gather" (read at schedule build): the blocked d = 16 path's kernel (GraphSchedule::
// gather16): 0 = by shape -- the interleaved k_graphsum<4, 16> when a row's segment in a column
// block averages under 16 slots (r05 late, one call: reddit-11.6M, ~12 slots, 341 vs 595 us;
// reddit-114M, ~60 slots, k_graphsum16 1,016 vs 1,089 us; profiles/r05/y, z), 1 = k_graphsum16,
// 2 = the interleaved kernel
int g_gs16_gather = 0;

int DevGraph::column_blocks(int dim) {
  const int vec = (dim + 3) / 4;
  const double table = (double)n_cols_ * vec * 16.0;
  return (graphsum_group_lanes(vec) < 64 && table > kL2Budget) ? kBlocks : 1;
}

// Cut the columns into kBlocks nnz-balanced ranges.
void DevGraph::compute_cuts() {
  if (bcut_.empty()) bcut_ = column_cuts(n_cols_, h_indices_);
}

// Store the edges block-major (per column block, rows in order).
void DevGraph::build_blocked() {
  if (blocked_built_) return;
  const int B = kBlocks;
  compute_cuts();
  auto block_of = [&](int col) {
    return (int)(std::upper_bound(bcut_.begin(), bcut_.end(), col) - bcut_.begin()) - 1;
  };
  // per-row counts per block
  std::vector<int> cnt((size_t)n_rows_ * B, 0);
  parallel_for(n_rows_, [&](long long b0, long long b1) {
    for (long long i = b0; i < b1; i++)
      for (int k = h_indptr_[(size_t)i]; k < h_indptr_[(size_t)i + 1]; k++)
        cnt[(size_t)i * B + block_of(h_indices_[(size_t)k])]++;
  });
  // block-major segment offsets; every segment padded to a multiple of 4 slots so that the
  // d=16 kernel reads 4 (index, value) pairs with one aligned 16-byte load per lane.  Padding
  // slots carry value 0 and the block's first column (an L2-hot row).
  bseg_.assign((size_t)B * (n_rows_ + 1), 0);
  long long base = 0;
  for (int b = 0; b < B; b++) {
    long long *seg = &bseg_[(size_t)b * (n_rows_ + 1)];
    seg[0] = base;
    for (int i = 0; i < n_rows_; i++) seg[i + 1] = seg[i] + ((cnt[(size_t)i * B + b] + 3) & ~3);
    base = seg[n_rows_];
  }
  bnnz_ = base;
  std::vector<int> bi((size_t)bnnz_);
  std::vector<float> bv((size_t)bnnz_, 0.0f);
  parallel_for(n_rows_, [&](long long b0, long long b1) {
    for (long long i = b0; i < b1; i++) {
      long long o[kBlocks];
      for (int b = 0; b < B; b++) o[b] = bseg_[(size_t)b * (n_rows_ + 1) + i];
      for (int k = h_indptr_[(size_t)i]; k < h_indptr_[(size_t)i + 1]; k++) {
        const int b = block_of(h_indices_[(size_t)k]);
        bi[(size_t)o[b]] = h_indices_[(size_t)k];
        bv[(size_t)o[b]] = h_vals_[(size_t)k];
        o[b]++;
      }
      for (int b = 0; b < B; b++)
        for (long long p = o[b]; p < bseg_[(size_t)b * (n_rows_ + 1) + i + 1]; p++)
          bi[(size_t)p] = bcut_[(size_t)b] < n_cols_ ? bcut_[(size_t)b] : 0;
    }
  });
  bindices_.allocate((size_t)bnnz_ + 64);
  bvals_.allocate((size_t)bnnz_ + 64);
  bindices_.upload(bi);
  bvals_.upload(bv);
  PGCN_HIP(hipMemset(bindices_.get() + bnnz_, 0, 64 * sizeof(int)));
  PGCN_HIP(hipMemset(bvals_.get() + bnnz_, 0, 64 * sizeof(float)));
  blocked_built_ = true;
}

DevGraph::Sched &DevGraph::schedule(int vec) {
  auto it = scheds_.find(vec);
  if (it != scheds_.end()) return *it->second;
  PGCN_CHECK(graphsum_vec_supported(vec), PGCN_E_INVALID,
             "graphsum: row width not supported: " + std::to_string(4 * vec));
  auto sp = std::make_unique<Sched>();
  const int G = graphsum_group_lanes(vec);
  const int nb = G / vec;
  const int nbc = column_blocks(4 * vec);
  std::vector<int4> items, comb;
  std::vector<int> block_items(1, 0);
  long long slots = 0;
  int chunk;
  std::vector<int> slot_comb;
  std::vector<int4> wide;
  if (nbc == 1) {
    const bool small = nnz_ <= kSmallNnz;
    const bool arrive = (g_gs_split == 1 || g_gs_split == 3) && small;
    chunk = nb * 32;  // 32 group iterations per work item
    const int wide_max = g_gs_split == 3 && small && (vec & (vec - 1)) == 0 ? 256 / vec * 8 : 0;
    if (arrive && g_gs_item_iters > 0) {
      chunk = nb * g_gs_item_iters;
    } else if (arrive) {
      int it = 2;
      for (; it < 32; it *= 2) {
        long long wide_rows = 0;
        for (int r = 0; r < n_rows_; r++) {
          const int len = h_indptr_[(size_t)r + 1] - h_indptr_[(size_t)r];
          wide_rows += len > nb * it && len <= wide_max;
        }
        if (wide_rows <= kWideCap) break;
      }
      chunk = nb * (wide_max ? it : 8);
    }
    const int whole = g_gs_split == 2 && small ? 8 * chunk : chunk;
    items.reserve((size_t)n_rows_ + (size_t)(nnz_ / chunk) + 1);
    for (int r = 0; r < n_rows_; r++) {
      const int b = h_indptr_[(size_t)r], e = h_indptr_[(size_t)r + 1];
      if (e - b <= whole) {
        items.push_back(make_int4(r, b, e, -1));
      } else if (e - b <= wide_max) {
        wide.push_back(make_int4(r, b, e, -1));
      } else {
        const int first = (int)slots;
        int cnt = 0;
        for (int p = b; p < e; p += chunk) {
          items.push_back(make_int4(r, p, std::min(e, p + chunk), (int)slots++));
          if (arrive) slot_comb.push_back((int)comb.size());
          cnt++;
        }
        comb.push_back(make_int4(r, first, cnt, 0));
      }
    }
    // longest items first: the tail of the launch is short items
    std::stable_sort(items.begin(), items.end(),
                     [](const int4 &a, const int4 &b) { return (a.z - a.y) > (b.z - b.y); });
    block_items.push_back((int)items.size());
  } else {
    build_blocked();
    chunk = nb * 64;
    const int B = kBlocks;
    // slots: row-major, then block, then chunk -> a row's slots are contiguous and ordered
    std::vector<long long> rslot((size_t)n_rows_ + 1, 0);
    for (int i = 0; i < n_rows_; i++) {
      long long s = 0;
      for (int b = 0; b < B; b++) {
        const long long len = bseg_[(size_t)b * (n_rows_ + 1) + i + 1] - bseg_[(size_t)b * (n_rows_ + 1) + i];
        s += (len + chunk - 1) / chunk;
      }
      rslot[(size_t)i + 1] = rslot[(size_t)i] + s;
    }
    slots = rslot[(size_t)n_rows_];
    PGCN_CHECK(slots < (1LL << 31) && nnz_ < (1LL << 31), PGCN_E_INVALID, "graph too large");
    std::vector<long long> used((size_t)n_rows_, 0);
    for (int b = 0; b < B; b++) {
      const size_t start = items.size();
      const long long *seg = &bseg_[(size_t)b * (n_rows_ + 1)];
      for (int i = 0; i < n_rows_; i++) {
        for (long long p = seg[i]; p < seg[i + 1]; p += chunk) {
          const long long slot = rslot[(size_t)i] + used[(size_t)i]++;
          items.push_back(make_int4(i, (int)p, (int)std::min(seg[i + 1], p + chunk), (int)slot));
        }
      }
      std::stable_sort(items.begin() + (long)start, items.end(),
                       [](const int4 &a, const int4 &c) { return (a.z - a.y) > (c.z - c.y); });
      block_items.push_back((int)items.size());
    }
    comb.reserve((size_t)n_rows_);
    for (int i = 0; i < n_rows_; i++)
      comb.push_back(make_int4(i, (int)rslot[(size_t)i], (int)(rslot[(size_t)i + 1] - rslot[(size_t)i]), 0));
  }
  int max_block = 0;
  for (size_t b = 0; b + 1 < block_items.size(); b++)
    max_block = std::max(max_block, block_items[b + 1] - block_items[b]);
  sp->s.vec = vec;
  if (nbc > 1 && vec == 4) {
    const bool short_segments = nnz_ < 16LL * kBlocks * std::max(n_rows_, 1);
    sp->s.gather16 = g_gs16_gather == 2 || (g_gs16_gather == 0 && short_segments) ? 1 : 0;
  }
  sp->s.chunk = chunk;
  sp->s.nbc = nbc;
  sp->s.n_items = (int)items.size();
  sp->s.max_block_items = max_block;
  sp->s.n_comb = (int)comb.size();
  sp->s.n_slots = slots;
  sp->items.allocate(std::max<size_t>(items.size(), 1));
  sp->items.upload(items);
  sp->block_items.allocate(block_items.size());
  sp->block_items.upload(block_items);
  if (!comb.empty()) {
    sp->comb.allocate(comb.size());
    sp->comb.upload(comb);
  }
  if (slots) sp->partial.allocate((size_t)slots * vec * 4);
  sp->s.items = sp->items.get();
  sp->s.block_items = sp->block_items.get();
  sp->s.comb = sp->comb.get();
  if (!wide.empty()) {
    // longest first: they start in the launch's first workgroups
    std::stable_sort(wide.begin(), wide.end(),
                     [](const int4 &a, const int4 &c) { return (a.z - a.y) > (c.z - c.y); });
    sp->wide.allocate(wide.size());
    sp->wide.upload(wide);
    sp->s.n_wide = (int)wide.size();
    sp->s.wide = sp->wide.get();
  }
  if (!slot_comb.empty()) {
    sp->slot_comb.allocate(slot_comb.size());
    sp->slot_comb.upload(slot_comb);
    sp->comb_ctr.allocate(comb.size());
    sp->comb_ctr.zero();
    sp->s.slot_comb = sp->slot_comb.get();
    sp->s.comb_ctr = sp->comb_ctr.get();
  }
  auto &ref = *sp;
  scheds_[vec] = std::move(sp);
  return ref;
}

std::unique_ptr<DevGraph> DevGraph::row_subset(const std::vector<int> &rows) const {
  std::vector<int> ip(rows.size() + 1, 0), ix;
  std::vector<float> v;
  for (size_t r = 0; r < rows.size(); r++) {
    const int i = rows[r];
    PGCN_CHECK(i >= 0 && i < n_rows_, PGCN_E_INVALID, "row_subset: row id");
    ip[r + 1] = ip[r] + (h_indptr_[(size_t)i + 1] - h_indptr_[(size_t)i]);
  }
  ix.reserve((size_t)ip.back());
  v.reserve((size_t)ip.back());
  for (int i : rows) {
    ix.insert(ix.end(), h_indices_.begin() + h_indptr_[(size_t)i], h_indices_.begin() + h_indptr_[(size_t)i + 1]);
    v.insert(v.end(), h_vals_.begin() + h_indptr_[(size_t)i], h_vals_.begin() + h_indptr_[(size_t)i + 1]);
  }
  auto g = std::make_unique<DevGraph>((int)rows.size(), n_cols_, ip.data(), ix.data(), v.data());
  if (!h_row_scale_.empty()) {
    std::vector<float> rs(rows.size());
    for (size_t r = 0; r < rows.size(); r++) rs[r] = h_row_scale_[(size_t)rows[r]];
    g->set_scales(std::move(rs), h_col_scale_);
  }
  return g;
}

std::unique_ptr<DevGraph> DevGraph::col_subset(const std::vector<int> &cols) const {
  std::vector<int> pos((size_t)n_cols_, -1);
  for (size_t c = 0; c < cols.size(); c++) {
    PGCN_CHECK(cols[c] >= 0 && cols[c] < n_cols_ && (c == 0 || cols[c] > cols[c - 1]),
               PGCN_E_INVALID, "col_subset: columns must be ascending ids");
    pos[(size_t)cols[c]] = (int)c;
  }
  std::vector<int> ip((size_t)n_rows_ + 1, 0), ix;
  std::vector<float> v;
  for (int i = 0; i < n_rows_; i++) {
    for (int k = h_indptr_[(size_t)i]; k < h_indptr_[(size_t)i + 1]; k++) {
      const int c = pos[(size_t)h_indices_[(size_t)k]];
      if (c < 0) continue;
      ix.push_back(c);
      v.push_back(h_vals_[(size_t)k]);
    }
    ip[(size_t)i + 1] = (int)ix.size();
  }
  if (ix.empty()) {  // keep a valid (empty) CSR
    ix.push_back(0);
    v.push_back(0.0f);
  }
  auto g = std::make_unique<DevGraph>(n_rows_, std::max((int)cols.size(), 1), ip.data(), ix.data(),
                                      v.data());
  if (!h_col_scale_.empty() && !cols.empty()) {
    std::vector<float> cs(cols.size());
    for (size_t c = 0; c < cols.size(); c++) cs[c] = h_col_scale_[(size_t)cols[c]];
    g->set_scales(h_row_scale_, std::move(cs));
  }
  g->col_map_.allocate(std::max<size_t>(cols.size(), 1));
  g->col_map_.upload(cols.empty() ? std::vector<int>{0} : cols);
  g->col_pos_.allocate(pos.size());
  g->col_pos_.upload(pos);
  g->col_pos_rows_ = n_cols_;
  std::vector<int> ox(ix.size());
  for (size_t k = 0; k < ix.size(); k++) ox[k] = cols.empty() ? 0 : cols[(size_t)ix[k]];
  g->orig_indices_.allocate(ox.size() + 64);  // the same slack as indices_
  g->orig_indices_.upload(ox);
  PGCN_HIP(hipMemset(g->orig_indices_.get() + ox.size(), 0, 64 * sizeof(int)));
  return g;
}

void DevGraph::set_scales(std::vector<float> row_scale, std::vector<float> col_scale) {
  PGCN_CHECK((int)row_scale.size() == n_rows_ && (int)col_scale.size() == n_cols_,
             PGCN_E_INVALID, "set_scales: sizes");
  h_row_scale_ = std::move(row_scale);
  h_col_scale_ = std::move(col_scale);
  lds_.reset();
}

// "lds_blocks": column blocks of the LDS schedule; 0 = by shape (r01, reddit): 4 blocks when the
// graph has about as many rows as columns (the full graph and its column subsets: one round of
// 256 workgroups, half the partials; the same kernel time, combine 18 -> 11 us), 8 for a small
// row subset (its 256 workgroups then stream half the table each: val rows 0.11 vs 0.22 ms)
int g_lds_blocks = 0;

int lds_slots(int n_rows, int n_cols) {
  (void)n_rows;
  (void)n_cols;
  return LDS_SLOTS;
}

int lds_blocks(int n_rows, int n_cols) {
  if (g_lds_blocks) return g_lds_blocks;
  const long long cap = (long long)LDS_CW * lds_slots(n_rows, n_cols);
  if ((double)n_rows >= 0.9 * (double)n_cols) {
    // square-ish: 4 blocks, or 8 when the rowset batches fill the chip only then and every
    // block keeps >= 20 slices of 512 columns (r02, edge-cut chunk graphs of reddit-114M,
    // tools/rank_graphsum.py: 1 rank 0.336 vs 0.400 ms, 2 ranks 0.202 vs 0.223; 4 ranks
    // (14 slices per block at 8) 0.130 vs 0.125)
    const long long nrs = ((long long)n_rows + 15) / 16;
    const long long nb = std::max(1LL, (nrs + cap - 1) / cap);
    if (nb * 8 <= kCUs && n_cols / 8 >= 20 * RING_SR) return 8;
    // tall (an edge-cut rank's column block at W = 8: 233 k rows x 29 k columns): 2 blocks,
    // half the partials for the combine to add and push (r05, solo W = 8 rank epoch 0.488 vs
    // 0.512 ms at 4, 0.548 at 1; at W = 4, 4x as tall, 4 blocks stay best: 0.669 vs 0.708 ms;
    // profiles/r05/p)
    if ((long long)n_rows >= 6LL * n_cols) return 2;
    return 4;
  }
  // row subsets: 8 blocks, or more when few batches of rowsets would leave each workgroup a
  // long sweep over its block's slices with little work per slice (the validation rows: 7
  // batches -> 32 blocks, a quarter of the slices per workgroup)
  const long long nrs = ((long long)n_rows + 15) / 16;
  const long long nb = std::max(1LL, (nrs + cap - 1) / cap);
  int B = 8;
  while (B < 32 && nb * B * 2 <= kCUs) B *= 2;
  return B;
}

std::vector<int> column_cuts(int n_cols, const std::vector<int> &indices, int n_blocks) {
  const int B = n_blocks;
  const long long nnz = (long long)indices.size();
  std::vector<long long> colcnt((size_t)n_cols + 1, 0);
  for (long long k = 0; k < nnz; k++) colcnt[(size_t)indices[(size_t)k] + 1]++;
  for (int c = 0; c < n_cols; c++) colcnt[(size_t)c + 1] += colcnt[(size_t)c];
  std::vector<int> cut((size_t)B + 1, 0);
  cut[(size_t)B] = n_cols;
  for (int b = 1; b < B; b++) {
    const long long target = (long long)((double)nnz * b / B);
    int c = (int)(std::lower_bound(colcnt.begin(), colcnt.end(), target) - colcnt.begin());
    c = std::max(c, cut[(size_t)b - 1]);
    cut[(size_t)b] = std::min(c, n_cols);
  }
  return cut;
}

void DevGraph::build_lds() {
  if (lds_cut_.empty()) lds_cut_ = ring_cuts(n_cols_, h_indices_, lds_blocks(n_rows_, n_cols_));
  auto L = std::make_unique<LdsSched>();
  LdsHost h = build_ring_host(
      n_rows_, n_cols_, h_indptr_, h_indices_, lds_cut_, lds_slots(n_rows_, n_cols_), -1,
      ring_window_for(n_rows_, n_cols_, (long long)h_indices_.size(), (int)lds_cut_.size() - 1));
  // + 2 KB slack: ring refills read whole 512-B chunks (up to 3) past a wave's last block
  L->entries.allocate(h.entries.size() / 4 + 256);
  L->entries.upload(reinterpret_cast<const uint2 *>(h.entries.data()), h.entries.size() / 4);
  L->wave_off.allocate(h.wave_off.size());
  L->wave_off.upload(h.wave_off);
  L->counts.allocate(h.counts.size());
  L->counts.upload(h.counts);
  L->slices.allocate(h.slices.size());
  L->slices.upload(h.slices);
  L->n_slices.allocate(h.nsl.size());
  L->n_slices.upload(h.nsl);
  L->rows.allocate(h.rows.size());
  L->rows.upload(h.rows);
  L->row_scale.allocate(h_row_scale_.size());
  L->row_scale.upload(h_row_scale_);
  L->col_scale.allocate(h_col_scale_.size());
  L->col_scale.upload(h_col_scale_);
  // whole slices of RING_SR rows (the loader copies 8-KB plane pieces); a graph sharing
  // another's tables has none of its own
  if (!table_owner_) L->scratch.allocate((size_t)ceil_div(n_cols_, RING_SR) * RING_SR * 16);
  L->partial.allocate((size_t)h.n_blocks * n_rows_ * 16);
  L->s.n_blocks = h.n_blocks;
  L->s.ns = h.ns;
  L->s.pair = h.pair;
  L->s.w = h.w;
  L->s.n_rows = n_rows_;
  L->s.n_cols = n_cols_;
  L->s.n_batches = h.n_batches;
  L->s.t_max = h.t_max;
  L->s.entries = L->entries.get();
  L->s.wave_off = L->wave_off.get();
  L->s.counts = L->counts.get();
  L->s.slices = L->slices.get();
  L->s.n_slices = L->n_slices.get();
  L->s.rows = L->rows.get();
  L->s.row_scale = L->row_scale.get();
  L->s.col_scale = L->col_scale.get();
  lds_ = std::move(L);
}

void DevGraph::prepare(int dim) {
  if (uses_lds(dim) && !lds_) build_lds();
}

bool DevGraph::uses_lds(int dim) const {
  return dim >= 16 && !h_row_scale_.empty() && (double)n_cols_ * 64.0 > (double)g_lds_min_bytes &&
         n_rows_ >= kLdsMinRows;
}

bool DevGraph::epilogue_ok(int dim, int ld_in, int ld_out) const {
  (void)ld_in;
  (void)ld_out;
  // LDS path: every 16-column pass's combine applies the tail to its columns (a pass that
  // overlaps the one before it recomputes those columns from the input: the same bits)
  if (uses_lds(dim)) return true;
  return !(dim > 16 && !graphsum_vec_supported((dim + 3) / 4));
}

float *DevGraph::ring_table(int dim, const float **next_scale) {
  if (dim > 16 || !uses_lds(dim) || col_map_) return nullptr;
  if (!lds_) build_lds();
  *next_scale = lds_->s.col_scale;
  return table_scratch();
}

float *DevGraph::ring_table_mapped(int dim, const float **next_scale, const int **pos,
                                   int *pos_rows) {
  if (dim > 16 || !uses_lds(dim) || table_owner_ || (col_map_ && !col_pos_rows_)) return nullptr;
  if (!lds_) build_lds();
  *next_scale = lds_->s.col_scale;
  *pos = col_map_ ? col_pos_.get() : nullptr;
  *pos_rows = col_map_ ? col_pos_rows_ : n_cols_;
  return table_scratch();
}

void DevGraph::share_tables(DevGraph *owner) {
  PGCN_CHECK(owner && owner != this && !owner->table_owner_ && owner->n_cols_ == n_cols_ &&
                 owner->h_col_scale_ == h_col_scale_ && !owner->col_map_ == !col_map_,
             PGCN_E_INVALID, "share_tables: the graphs' columns differ");
  table_owner_ = owner;
  lds_.reset();
}

bool DevGraph::can_share_tables(int dim, int ld_in) const {
  if (!uses_lds(dim)) return false;
  // one 16-column pass, or every pass's table from the batched prescale -- graphsum()'s
  // `batch` condition below (ld_in <= 128); wider inputs prescale per pass
  return dim <= 16 || (!col_map_ && ld_in <= 128);
}

float *DevGraph::table_scratch() {
  if (!table_owner_) return lds_->scratch.get();
  if (!table_owner_->lds_) table_owner_->build_lds();
  return table_owner_->lds_->scratch.get();
}

float *DevGraph::table_wide(size_t floats) {
  DevGraph *o = table_owner_ ? table_owner_ : this;
  if (!o->lds_) o->build_lds();
  if (o->lds_->tables.size() < floats) o->lds_->tables.allocate(floats);
  return o->lds_->tables.get();
}

void DevGraph::graphsum(const float *in, int ld_in, float *out, int ld_out, int dim,
                        hipStream_t s, bool compact_in, const GsEpilogue *epi, bool prestaged,
                        bool tables_ready, const PeerSink *push, hipStream_t tail_st,
                        hipEvent_t fork) {
  const int *col_map = compact_in ? nullptr : col_map_.get();
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0 && ld_in >= dim && ld_out >= dim,
             PGCN_E_INVALID, "graphsum: leading dims must be multiples of 4 and >= dim");
  PGCN_CHECK(!epi || epi->mode == 0 || epilogue_ok(dim, ld_in, ld_out), PGCN_E_INVALID,
             "graphsum: epilogue on a multi-pass width");
  PGCN_CHECK(!prestaged || uses_lds(dim), PGCN_E_INVALID, "graphsum: prestaged input, plain path");
  if (uses_lds(dim)) {
    if (!lds_) build_lds();
    // wider rows: one LDS pass per 16 columns (the last pass overlaps the one before it so it
    // stays inside both leading dims; overlapped columns are recomputed to the same bits).
    // d = 128 on reddit: 8 passes ~2.7 ms against ~7 ms for the gather kernel, whose 512-B
    // rows come from the Infinity Cache at ~7.7 TB/s
    const int ldm = std::min(ld_in, ld_out);
    // (a column subset's table prestaged through its row map: ring_table_mapped)
    PGCN_CHECK(!prestaged || dim <= 16, PGCN_E_INVALID,
               "graphsum: prestaged input on a path without a ring table");
    const size_t table = (size_t)ceil_div(n_cols_, RING_SR) * RING_SR * 16;
    const int n_pass = ceil_div(dim, 16);
    PGCN_CHECK(!tail_st || (push && n_pass == 1), PGCN_E_INVALID,
               "graphsum: a tail stream for a one-pass push only");
    auto pass_col = [&](int p) { return std::min(16 * p, ldm - 16); };
    // several passes: one launch prescales all of them (each pass then reads its own table);
    // inputs up to 128 wide (at most 8 passes: RingPasses), wider ones prescale per pass
    const bool batch = n_pass > 1 && !col_map && ld_in <= 128;
    PGCN_CHECK(!tables_ready || (can_share_tables(dim, ld_in) && (n_pass == 1 || batch)),
               PGCN_E_INVALID, "graphsum: shared tables on a call that prescales per pass");
    RingPasses ps;
    if (batch) {
      PGCN_CHECK(n_pass <= 8, PGCN_E_INVALID, "graphsum: batched passes");
      for (int p = 0; p < n_pass; p++) ps.c[ps.n++] = pass_col(p);
    }
    float *tables = batch ? table_wide(table * n_pass) : nullptr;
    if (batch && !tables_ready)
      launch_ring_prescale_wide(lds_->s, in, ld_in, std::min(ld_in, ps.c[ps.n - 1] + 16), ps,
                                tables, (long long)table, s);
    for (int p = 0; p < n_pass; p++) {
      const int c = pass_col(p);
      GsEpilogue ep = epi ? *epi : GsEpilogue{};
      ep.col0 = c;
      PeerSink pk;
      if (push) {  // this pass's columns of every owner's slot; the last pass signals
        pk = *push;
        for (int q = 0; q < pk.world; q++) pk.dst[q] += c;
        pk.slot_bytes -= 4LL * c;
        pk.signal = p == n_pass - 1 ? push->signal : 0;
      }
      launch_graphsum_ring(lds_->s, in + c, ld_in, out ? out + c : nullptr, ld_out,
                           batch ? tables + table * p : table_scratch(), lds_->partial.get(), s,
                           col_map, &ep, prestaged || batch || tables_ready, push ? &pk : nullptr,
                           tail_st, fork);
    }
    return;
  }
  PGCN_CHECK(!push, PGCN_E_INVALID, "graphsum: push on the plain path");
  if (dim > 16 && !graphsum_vec_supported((dim + 3) / 4)) {
    // widths without a kernel instantiation (PART2 hidden 72, 600): 16-column passes, the
    // last one overlapping the one before it (recomputed columns get the same bits)
    const int ldm = std::min(ld_in, ld_out);
    for (int c0 = 0; c0 < dim; c0 += 16) {
      const int c = std::min(c0, ldm - 16);
      graphsum(in + c, ld_in, out + c, ld_out, 16, s, compact_in);
    }
    return;
  }
  const int vec = (dim + 3) / 4;
  Sched &sc = schedule(vec);
  const bool blocked = sc.s.nbc > 1;
  const bool orig = col_map && !blocked && g_gs_orig_cols;
  if (col_map && !orig) {  // plain path of a column subset: compact the input rows first
    const size_t need = (size_t)n_cols_ * ld_in;
    if (col_in_.size() < need) col_in_.allocate(need);
    launch_gather_rows(in, col_map, n_cols_, ld_in, col_in_.get(), s);
    in = col_in_.get();
  }
  launch_graphsum(sc.s, blocked ? bindices_.get() : (orig ? orig_indices_.get() : indices_.get()),
                  blocked ? bvals_.get() : vals_.get(), in, ld_in, out, ld_out, sc.partial.get(), s,
                  epi);
}

double DevGraph::algorithmic_bytes(int dim) const {
  // 4(N+1) indptr + 8 nnz (index + value) + 4 N_in d (read) + 4 N d (write)
  return 4.0 * (n_rows_ + 1) + 8.0 * (double)nnz_ + 4.0 * (double)n_cols_ * dim +
         4.0 * (double)n_rows_ * dim;
}

}  // namespace pgcn
