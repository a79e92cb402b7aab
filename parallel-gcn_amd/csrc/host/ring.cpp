// parallel-gcn_amd/csrc/host/ring.cpp -- host builder of the sliding-window ("ring") schedule
// of the d = 16 LDS GraphSum (k_graphsum_ring, csrc/k_graphsum_ring.hip).
//
// Replaces, for GraphSum (hpdga module.cpp:82-111, src/module.cu:172-210), the window-1
// schedule of build_lds_host.  Same work split (column blocks x batches of rowsets, one
// workgroup per CU, 15 summing waves holding 16 rowsets x 16 rows of accumulators in
// registers), different slice pipeline:
//
//  * the block's columns are cut into slices of RING_SR = 512 rows; LDS holds a ring of
//    RING_K = 4 slices and a visit v reads the RING_W = 3 resident slices v, v+1, v+2 while
//    the loader stages slice v+3 into the buffer slice v-1 left;
//  * per (visit, rowset) the wave runs n steps in lockstep (lane group g = row g of the
//    rowset), n = the most edges any of the 16 rows still has in slice v (they must be done
//    before slice v leaves the ring), rounded up to a 4-step entry block; rows with fewer
//    such edges fill the spare steps with edges of slices v+1 and v+2.  Lockstep padding:
//    1.9 step slots per edge on reddit-114M against 2.85 for one slice at a time (33 % fewer
//    entry blocks, the kernel's unit of work);
//  * the table sits in LDS as 4 quarter planes (lane v of a lane group reads columns 4v..4v+3
//    of the row from plane v), so a 16-bit entry (ring row x 16 B) addresses any row of the
//    4-slice ring from a per-lane constant base: one VALU add per step, as before;
//  * plane rows RING_P = 2052 (= 4 mod 16): the 4 lane groups of one ds_read_b128 LDS cycle
//    are conflict-free when their rows differ mod 4; the builder orders each step's picks so
//    (bank-quarter residue = column mod 4, slices start at multiples of 4); padding steps read
//    one of 4 zero rows (ring rows 2048 + r).
#include <algorithm>
#include <numeric>

#include "graph.hpp"

namespace pgcn {

namespace {
// lane groups served in one LDS cycle of ds_read_b128 (MI355X_MICROARCH.md §LDS)
const int kQuad[4][4] = {{0, 3, 5, 6}, {1, 2, 4, 7}, {8, 11, 13, 14}, {9, 10, 12, 15}};

const int kPerm[24][4] = {
    {0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {0, 3, 2, 1},
    {1, 0, 2, 3}, {1, 0, 3, 2}, {1, 2, 0, 3}, {1, 2, 3, 0}, {1, 3, 0, 2}, {1, 3, 2, 0},
    {2, 0, 1, 3}, {2, 0, 3, 1}, {2, 1, 0, 3}, {2, 1, 3, 0}, {2, 3, 0, 1}, {2, 3, 1, 0},
    {3, 0, 1, 2}, {3, 0, 2, 1}, {3, 1, 0, 2}, {3, 1, 2, 0}, {3, 2, 0, 1}, {3, 2, 1, 0}};

struct Edge {
  int slice;  // visit index inside the column block
  int col;    // global column
};

// Per lane group: admitted edges (slice <= v + W - 1, not yet consumed), one FIFO per bank
// residue; each FIFO is nondecreasing in slice (edges are admitted in column order).
struct Lane {
  std::vector<Edge> q[4];
  size_t head[4] = {0, 0, 0, 0};
  int due = 0;        // admitted edges of the current visit's slice not yet consumed
  int next = 0;       // next sidx position to admit
  int stride = 1;     // every stride-th edge of the row (its piece of a spread row)
  int end = 0;        // past the row's last edge of this column block
  bool empty_res(int r) const { return head[r] == q[r].size(); }
  const Edge &front(int r) const { return q[r][head[r]]; }
  int pending() const {
    int n = 0;
    for (int r = 0; r < 4; r++) n += (int)(q[r].size() - head[r]);
    return n;
  }
};
}  // namespace

// x10 mean edges per slice above which a row is spread over 2, 4, 8 or 16 lane groups (r02
// sweep on reddit-114M: 60 best; pulling extra blocks into waves below a visit's slowest
// measured no faster and was removed)
constexpr int kRingSpread = 60;

std::vector<int> ring_cuts(int n_cols, const std::vector<int> &indices, int n_blocks) {
  std::vector<int> cut = column_cuts(n_cols, indices, n_blocks);
  for (int b = 1; b < n_blocks; b++) {
    int c = (cut[(size_t)b] + RING_SR / 2) / RING_SR * RING_SR;
    c = std::max(c, cut[(size_t)b - 1]);
    cut[(size_t)b] = std::min(c, n_cols);
  }
  return cut;
}

// "ring_pair" (read at schedule build): rowsets in lockstep pairs (build_ring_host)
int g_ring_pair = 0;

int g_ring_window = 0;

// The window by shape: 3 (the reddit graph's), or 2 where a visit's work is too short to cover
// the loader's one-slice-ahead LDS-DMA (~1.3 us per 32-KB slice): r06 tall edge-cut rank
// graphs and sparse graphs, decided on the mean entry blocks a summing wave runs per visit
// (about rows x (nnz / rows / slices + 1) / 64 per wave at 4-step blocks)
int ring_window_for(int n_rows, int n_cols, long long nnz, int n_blocks) {
  if (g_ring_window) return g_ring_window;
  (void)n_rows;
  (void)n_cols;
  (void)nnz;
  (void)n_blocks;
  return RING_W;
}

LdsHost build_ring_host(int n_rows, int n_cols, const std::vector<int> &indptr,
                        const std::vector<int> &indices, const std::vector<int> &bcut, int ns,
                        int pair_arg, int window) {
  (void)n_cols;
  PGCN_CHECK(window == 2 || window == 3, PGCN_E_INVALID, "graphsum_ring: window 2 or 3");
  const int B = (int)bcut.size() - 1, SR = RING_SR, W = window, K = RING_K;
  const int CW = LDS_CW, NS = ns;
  const bool pair = pair_arg < 0 ? g_ring_pair != 0 : pair_arg != 0;
  PGCN_CHECK(ring_slots_ok(ns), PGCN_E_INVALID, "graphsum_ring: rowsets per wave");
  PGCN_CHECK(B >= 1 && kCUs % B == 0, PGCN_E_INVALID, "graphsum_ring: column blocks");
  for (int b = 0; b < B; b++)
    PGCN_CHECK(bcut[(size_t)b] % SR == 0, PGCN_E_INVALID, "graphsum_ring: block cut alignment");
  std::vector<int> nsl((size_t)B);
  int t_max = 1;
  for (int b = 0; b < B; b++) {
    nsl[(size_t)b] = (bcut[(size_t)b + 1] - bcut[(size_t)b] + SR - 1) / SR;
    t_max = std::max(t_max, nsl[(size_t)b]);
  }
  std::vector<int2> slices((size_t)B * t_max, make_int2(0, 0));
  std::vector<int> vis_first((size_t)B + 1, 0);
  for (int b = 0; b < B; b++) {
    for (int t = 0; t < nsl[(size_t)b]; t++) {
      const int c0 = bcut[(size_t)b] + t * SR;
      slices[(size_t)b * t_max + t] = make_int2(c0, std::min(SR, bcut[(size_t)b + 1] - c0));
    }
    vis_first[(size_t)b + 1] = vis_first[(size_t)b] + nsl[(size_t)b];
  }
  const int n_vis = vis_first[(size_t)B];
  // Units: a row takes m = 2^s lane groups ("spread"), each summing every m-th of its edges
  // in this column block; the wave adds the m partial sums at the end (k_graphsum_ring's
  // partial write).  m doubles while the row's mean edges per slice over m exceed
  // kRingSpread / 10 (hub rows would otherwise pace their rowset, their wave and, through
  // the visits' hand-offs, their workgroup).  Rowsets hold 16 units of one m, rows by m, then
  // degree, descending; rowsets are dealt round-robin to batches.
  std::vector<int> order((size_t)n_rows);
  std::iota(order.begin(), order.end(), 0);
  const double per_slice = (double)SR / std::max(1, n_cols);
  auto spread_of = [&](int row) {
    const double lam = (indptr[(size_t)row + 1] - indptr[(size_t)row]) * per_slice;
    int s = 0;
    while (s < 4 && lam / (1 << s) > kRingSpread / 10.0) s++;
    return s;
  };
  std::vector<int> spread((size_t)n_rows);
  for (int r = 0; r < n_rows; r++) spread[(size_t)r] = spread_of(r);
  std::stable_sort(order.begin(), order.end(), [&](int a, int c) {
    if (spread[(size_t)a] != spread[(size_t)c]) return spread[(size_t)a] > spread[(size_t)c];
    return indptr[(size_t)a + 1] - indptr[(size_t)a] > indptr[(size_t)c + 1] - indptr[(size_t)c];
  });
  // unit_row[16 * rowset + g] = row | s << 28 (kRingEmpty | s << 28: no row); piece = g % m
  std::vector<int> unit_row;
  for (size_t i = 0; i < order.size();) {
    const int s = spread[(size_t)order[i]], m = 1 << s;
    for (int g = 0; g < 16; g += m) {
      const bool have = i < order.size() && spread[(size_t)order[i]] == s;
      for (int p = 0; p < m; p++) unit_row.push_back((have ? order[i] : kRingEmpty) | s << 28);
      if (have) i++;
    }
  }
  const long long nrs = (long long)unit_row.size() / 16;
  const long long cap = (long long)CW * NS;
  const int per_round = kCUs / B;
  const int nbat = (int)(((nrs + cap - 1) / cap + per_round - 1) / per_round * per_round);
  const long long n_wg = (long long)nbat * B;
  std::vector<int> sidx(indices);
  parallel_for(n_rows, [&](long long b0, long long b1) {
    for (long long i = b0; i < b1; i++)
      std::sort(sidx.begin() + indptr[(size_t)i], sidx.begin() + indptr[(size_t)i + 1]);
  });
  // per (rowset, visit): entry blocks under the window rule with first-in-first-out lanes
  // (an estimate for balancing the waves; the emitted schedule below orders for banks)
  std::vector<unsigned short> rs_blocks((size_t)nrs * n_vis, 0);
  parallel_for(nrs, [&](long long r0, long long r1) {
    std::vector<int> cnt((size_t)16 * t_max);
    for (long long r = r0; r < r1; r++)
      for (int b = 0; b < B; b++) {
        const int T = nsl[(size_t)b];
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int g = 0; g < 16; g++) {
          const int u = unit_row[(size_t)(16 * r + g)], row = u & kRingRowMask, m = 1 << (u >> 28);
          if (row == kRingEmpty) continue;
          const int *rb = &sidx[(size_t)indptr[(size_t)row]], *re = &sidx[(size_t)indptr[(size_t)row + 1]];
          const int *lo = std::lower_bound(rb, re, bcut[(size_t)b]);
          for (const int *p = lo + g % m; p < re && *p < bcut[(size_t)b + 1]; p += m)
            cnt[(size_t)g * t_max + (*p - bcut[(size_t)b]) / SR]++;
        }
        for (int v = 0; v < T; v++) {
          int n = 0;
          for (int g = 0; g < 16; g++) n = std::max(n, cnt[(size_t)g * t_max + v]);
          const int nb = (n + 3) / 4;
          rs_blocks[(size_t)r * n_vis + vis_first[(size_t)b] + v] = (unsigned short)std::min(nb, 65535);
          for (int g = 0; g < 16; g++) {
            int c = 4 * nb;
            for (int u = v; u < std::min(T, v + W) && c > 0; u++) {
              int &x = cnt[(size_t)g * t_max + u];
              const int take = std::min(c, x);
              x -= take;
              c -= take;
            }
          }
        }
      }
  }, 0, 64);
  // rowsets of a batch to waves (heaviest first): the wave whose per-visit loads grow the sum
  // over visits of the per-visit maximum least (visits end in hand-offs the slowest wave paces)
  std::vector<int> rows((size_t)nbat * CW * NS * 16, kRingEmpty);
  parallel_for(nbat, [&](long long b0, long long b1) {
    std::vector<int> load((size_t)CW * n_vis), cur_max((size_t)n_vis);
    for (long long bat = b0; bat < b1; bat++) {
      std::vector<long long> mine;
      for (long long r = bat; r < nrs; r += nbat) mine.push_back(r);
      std::vector<long long> tot(mine.size(), 0);
      for (size_t a = 0; a < mine.size(); a++)
        for (int s = 0; s < n_vis; s++) tot[a] += rs_blocks[(size_t)mine[a] * n_vis + s];
      std::vector<size_t> idx(mine.size());
      std::iota(idx.begin(), idx.end(), 0);
      std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return tot[x] > tot[y]; });
      std::fill(load.begin(), load.end(), 0);
      std::fill(cur_max.begin(), cur_max.end(), 0);
      std::vector<int> used((size_t)CW, 0);
      for (size_t a : idx) {
        const unsigned short *x = &rs_blocks[(size_t)mine[a] * n_vis];
        long long best = -1;
        int bw = -1;
        for (int w = 0; w < CW; w++) {
          if (used[(size_t)w] >= NS) continue;
          long long inc = 0;
          const int *lw = &load[(size_t)w * n_vis];
          for (int s = 0; s < n_vis; s++) {
            const int nl = lw[s] + x[s];
            if (nl > cur_max[(size_t)s]) inc += nl - cur_max[(size_t)s];
          }
          if (bw < 0 || inc < best || (inc == best && used[(size_t)w] < used[(size_t)bw])) {
            best = inc;
            bw = w;
          }
        }
        PGCN_CHECK(bw >= 0, PGCN_E_INVALID, "graphsum_ring: batch over capacity");
        int *lw = &load[(size_t)bw * n_vis];
        for (int s = 0; s < n_vis; s++) {
          lw[s] += x[s];
          cur_max[(size_t)s] = std::max(cur_max[(size_t)s], lw[s]);
        }
        const int j = used[(size_t)bw]++;
        for (int g = 0; g < 16; g++)
          rows[(size_t)(((bat * CW + bw) * NS + j) * 16 + g)] = unit_row[(size_t)(16 * mine[a] + g)];
      }
    }
  }, 0, 1);
  std::vector<unsigned short> counts((size_t)n_wg * t_max * CW * NS, 0);
  // walks workgroup wg: per visit, per wave, per rowset, the steps of its 16 lane groups;
  // appends each wave's entry blocks to out[wave].
  //
  // Visits end in hand-offs (a slice leaves the ring once every wave is done with it), so
  // the slowest wave of a visit paces the workgroup.
  auto walk_wg = [&](long long wg, std::vector<std::vector<unsigned short>> &out) {
    const int b = (int)(wg % B), bat = (int)(wg / B), T = nsl[(size_t)b];
    const int base_col = bcut[(size_t)b];
    std::vector<Lane> lanes((size_t)CW * NS * 16);
    for (int w = 0; w < CW; w++) {
      const int *rw = &rows[(size_t)(((long long)bat * CW + w) * NS) * 16];
      for (int k = 0; k < NS * 16; k++) {
        Lane &L = lanes[(size_t)w * NS * 16 + k];
        const int r = rw[k] & kRingRowMask;
        if (r == kRingEmpty) continue;
        L.stride = 1 << ((unsigned)rw[k] >> 28);
        const int *rb = &sidx[(size_t)indptr[(size_t)r]], *re = &sidx[(size_t)indptr[(size_t)r + 1]];
        L.next = (int)(std::lower_bound(rb, re, bcut[(size_t)b]) - sidx.data()) + (k % 16) % L.stride;
        L.end = (int)(std::lower_bound(rb, re, bcut[(size_t)b + 1]) - sidx.data());
      }
    }
    auto admit = [&](Lane &L, int upto_slice) {  // edges of slices <= upto_slice
      const int c1 = base_col + (upto_slice + 1) * SR;
      while (L.next < L.end && sidx[(size_t)L.next] < c1) {
        const int c = sidx[(size_t)L.next];
        L.next += L.stride;
        L.q[c & 3].push_back(Edge{(c - base_col) / SR, c});
      }
    };
    for (auto &L : lanes) admit(L, W - 2);  // slices resident before visit 0's window completes
    std::vector<int> nb((size_t)CW * NS);
    for (int v = 0; v < T; v++) {
      // forced blocks per (wave, rowset)
      for (int w = 0; w < CW; w++) {
        for (int j = 0; j < NS; j++) {
          int n = 0;
          for (int g = 0; g < 16; g++) {
            Lane &L = lanes[((size_t)w * NS + j) * 16 + g];
            admit(L, v + W - 1);
            L.due = 0;
            for (int r = 0; r < 4; r++)
              for (size_t h = L.head[r]; h < L.q[r].size() && L.q[r][h].slice == v; h++) L.due++;
            n = std::max(n, L.due);
          }
          nb[(size_t)w * NS + j] = (n + 3) / 4;
        }
        // pairs: both rowsets take the longer run (the shorter one fills the extra steps with
        // its later slices' edges, or padding)
        if (pair)
          for (int j = 0; j < NS; j += 2) {
            int &a = nb[(size_t)w * NS + j], &c = nb[(size_t)w * NS + j + 1];
            a = c = std::max(a, c);
          }
      }
      for (int w = 0; w < CW; w++) {
        size_t pair_base = 0;
        for (int j = 0; j < NS; j++) {
          const int S = 4 * nb[(size_t)w * NS + j];
          PGCN_CHECK(S < 65536, PGCN_E_INVALID, "graphsum_ring: visit run too long");
          counts[(size_t)(((wg * t_max + v) * CW + w) * NS + j)] = (unsigned short)S;
          Lane *lj = &lanes[((size_t)w * NS + j) * 16];
          std::vector<unsigned short> &ow = out[(size_t)w];
          // block k of this rowset's run: kb + bstride * k (pairs: rowset 2p's blocks at the
          // even places of the pair's run, 2p + 1's at the odd ones)
          size_t kb;
          const size_t bstride = pair ? 2 : 1;
          if (!pair) {
            kb = ow.size() / 64;
            ow.resize(ow.size() + (size_t)S * 16);
          } else if (j % 2 == 0) {
            pair_base = kb = ow.size() / 64;
            ow.resize(ow.size() + (size_t)S * 32);
          } else {
            kb = pair_base + 1;
          }
          for (int st = 0; st < S; st++) {
            for (int q = 0; q < 4; q++) {
              const int *grp = kQuad[q];
              // one residue (bank quarter) per member: the permutation of the 4 residues that
              // serves every forced member (as many due edges left as steps) a due edge, then
              // the most due edges, then the most later edges (earliest slices first); members
              // left without an edge of their residue read that residue's zero row
              Lane *M[4];
              bool forced[4];
              for (int a2 = 0; a2 < 4; a2++) {
                M[a2] = &lj[grp[a2]];
                forced[a2] = M[a2]->due > 0 && M[a2]->due >= S - st;
              }
              auto value = [&](int a2, int r) -> int {
                const Lane &L = *M[a2];
                if (L.empty_res(r)) return forced[a2] ? -100000 : 0;
                const int sl = L.front(r).slice;
                if (sl == v) return forced[a2] ? 10000 : 1000;
                return forced[a2] ? -100000 : 100 - (sl - v);
              };
              int best = 0, best_v = -(1 << 30);
              for (int pi = 0; pi < 24; pi++) {
                int tot = 0;
                for (int a2 = 0; a2 < 4; a2++) tot += value(a2, kPerm[pi][a2]);
                if (tot > best_v) {
                  best_v = tot;
                  best = pi;
                }
              }
              for (int a2 = 0; a2 < 4; a2++) {
                const int g = grp[a2];
                Lane &L = *M[a2];
                int pick = kPerm[best][a2];
                const int zero = pick;
                if (L.empty_res(pick) || (L.front(pick).slice != v && forced[a2])) {
                  pick = -1;
                  if (forced[a2])  // no permutation serves it: a due edge, accepting a conflict
                    for (int r = 0; r < 4; r++)
                      if (!L.empty_res(r) && L.front(r).slice == v) {
                        pick = r;
                        break;
                      }
                }
                int val;
                if (pick >= 0) {
                  const Edge e = L.front(pick);
                  L.head[pick]++;
                  if (e.slice == v) L.due--;
                  const int col0 = base_col + e.slice * SR;
                  val = ((e.slice % K) * SR + (e.col - col0)) * 16;
                } else {  // padding: the zero row of this member's residue
                  val = (K * SR + zero) * 16;
                }
                ow[(kb + bstride * (size_t)(st / 4)) * 64 + (size_t)(g * 4 + (st % 4))] =
                    (unsigned short)val;
              }
            }
          }
          for (int g = 0; g < 16; g++)
            PGCN_CHECK(lj[g].due == 0, PGCN_E_INVALID, "graphsum_ring: edge past its slice's visit");
        }
      }
    }
    for (auto &L : lanes)
      PGCN_CHECK(L.pending() == 0 && L.next >= L.end, PGCN_E_INVALID,
                 "graphsum_ring: edges left after the last visit");
  };
  std::vector<std::vector<std::vector<unsigned short>>> ent_w((size_t)n_wg);
  parallel_for(n_wg, [&](long long a, long long e) {
    for (long long x = a; x < e; x++) {
      ent_w[(size_t)x].resize((size_t)CW);
      walk_wg(x, ent_w[(size_t)x]);
    }
  }, 0, 2);
  std::vector<long long> off((size_t)n_wg * CW + 1, 0);
  for (long long x = 0; x < n_wg * CW; x++)
    off[(size_t)x + 1] = off[(size_t)x] + (long long)(ent_w[(size_t)(x / CW)][(size_t)(x % CW)].size() / 64);
  std::vector<unsigned short> ent((size_t)std::max<long long>(off.back(), 1) * 64, 0);
  parallel_for(n_wg, [&](long long a, long long e) {
    for (long long x = a; x < e; x++)
      for (int w = 0; w < CW; w++) {
        auto &src = ent_w[(size_t)x][(size_t)w];
        std::copy(src.begin(), src.end(), ent.begin() + off[(size_t)(x * CW + w)] * 64);
        std::vector<unsigned short>().swap(src);
      }
  }, 0, 2);
  LdsHost h;
  h.ns = NS;
  h.pair = pair;
  h.w = W;
  h.n_blocks = B;
  h.n_batches = nbat;
  h.t_max = t_max;
  h.nsl = std::move(nsl);
  h.slices = std::move(slices);
  h.rows = std::move(rows);
  h.counts = std::move(counts);
  h.wave_off = std::move(off);
  h.entries = std::move(ent);
  return h;
}

// Walks a ring schedule as k_graphsum_ring consumes it: per visit the resident slices v..v+2
// (ring buffer t % 4 holds slice t), entry blocks in wave order, zero rows; adds each row's
// sum of in[col] into out[row].  Throws on anything the kernel would turn into a wrong sum.
void ring_emulate(const LdsHost &h, int n_rows, const float *in, double *out) {
  const int B = h.n_blocks, CW = LDS_CW, NS = h.ns, SR = RING_SR, K = RING_K, W = h.w;
  const long long n_wg = (long long)h.n_batches * B;
  std::vector<double> acc((size_t)NS * 16);
  for (long long wg = 0; wg < n_wg; wg++) {
    const int b = (int)(wg % B), bat = (int)(wg / B), T = h.nsl[(size_t)b];
    for (int w = 0; w < CW; w++) {
      long long kb = h.wave_off[(size_t)(wg * CW + w)];
      std::fill(acc.begin(), acc.end(), 0.0);
      for (int v = 0; v < T; v++) {
        const unsigned short *cn = &h.counts[(size_t)(((wg * h.t_max + v) * CW + w) * NS)];
        std::vector<int> seq;  // the rowset of each block, in stream order
        for (int j = 0; j < NS; j++)
          PGCN_CHECK(cn[j] % 4 == 0, PGCN_E_INVALID, "ring schedule: steps not whole blocks");
        if (h.pair) {  // pairs: blocks of rowsets 2p, 2p + 1 alternate
          for (int j = 0; j < NS; j += 2) {
            PGCN_CHECK(cn[j] == cn[j + 1], PGCN_E_INVALID, "ring schedule: unequal pair runs");
            for (int k = 0; k < cn[j] / 4; k++) {
              seq.push_back(j);
              seq.push_back(j + 1);
            }
          }
        } else {
          for (int j = 0; j < NS; j++)
            for (int k = 0; k < cn[j] / 4; k++) seq.push_back(j);
        }
        for (const int j : seq) {
          {
            for (int st = 0; st < 4; st++)
              for (int g = 0; g < 16; g++) {
                const int e = h.entries[(size_t)kb * 64 + g * 4 + st];
                PGCN_CHECK(e % 16 == 0, PGCN_E_INVALID, "ring schedule: entry not a row");
                const int idx = e / 16;
                if (idx >= K * SR) {
                  PGCN_CHECK(idx < K * SR + 4, PGCN_E_INVALID, "ring schedule: past the zero rows");
                  continue;
                }
                const int buf = idx / SR, row = idx % SR;
                // the slice in buffer `buf` during visit v: the one of v..v+W-1 congruent to it
                int t = -1;
                for (int u = v; u < std::min(T, v + W); u++)
                  if (u % K == buf) t = u;
                PGCN_CHECK(t >= 0, PGCN_E_INVALID, "ring schedule: buffer not resident");
                const int2 sc = h.slices[(size_t)b * h.t_max + t];
                PGCN_CHECK(row < sc.y, PGCN_E_INVALID, "ring schedule: entry past the slice");
                acc[(size_t)j * 16 + g] += (double)in[sc.x + row];
              }
          }
          kb++;
        }
      }
      PGCN_CHECK(kb == h.wave_off[(size_t)(wg * CW + w) + 1], PGCN_E_INVALID,
                 "ring schedule: wave stream length");
      for (int j = 0; j < NS; j++)
        for (int g = 0; g < 16; g++) {
          const int u = h.rows[(size_t)(((long long)bat * CW + w) * NS + j) * 16 + g];
          const int r = u & kRingRowMask, m = 1 << ((unsigned)u >> 28);
          PGCN_CHECK(((unsigned)h.rows[(size_t)(((long long)bat * CW + w) * NS + j) * 16] >> 28) ==
                         ((unsigned)u >> 28),
                     PGCN_E_INVALID, "ring schedule: mixed spreads in a rowset");
          if (r != kRingEmpty) {
            PGCN_CHECK(r < n_rows, PGCN_E_INVALID, "ring schedule: row id");
            PGCN_CHECK(g % m != 0 || g + m <= 16, PGCN_E_INVALID, "ring schedule: spread pieces");
            out[r] += acc[(size_t)j * 16 + g];
          } else {
            PGCN_CHECK(acc[(size_t)j * 16 + g] == 0.0, PGCN_E_INVALID,
                       "ring schedule: edges on an empty slot");
          }
        }
    }
  }
}

}  // namespace pgcn
