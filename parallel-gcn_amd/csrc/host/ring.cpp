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

std::vector<int> ring_cuts(int n_cols, const std::vector<int> &indices, int n_blocks) {
  std::vector<int> cut = column_cuts(n_cols, indices, n_blocks);
  for (int b = 1; b < n_blocks; b++) {
    int c = (cut[(size_t)b] + RING_SR / 2) / RING_SR * RING_SR;
    c = std::max(c, cut[(size_t)b - 1]);
    cut[(size_t)b] = std::min(c, n_cols);
  }
  return cut;
}

LdsHost build_ring_host(int n_rows, int n_cols, const std::vector<int> &indptr,
                        const std::vector<int> &indices, const std::vector<int> &bcut) {
  (void)n_cols;
  const int B = (int)bcut.size() - 1, SR = RING_SR, W = RING_W, K = RING_K;
  const int CW = LDS_CW, NS = LDS_SLOTS;
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
  // rowsets: rows by degree (descending), 16 per rowset, dealt round-robin to batches
  std::vector<int> order((size_t)n_rows);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int c) {
    return indptr[(size_t)a + 1] - indptr[(size_t)a] > indptr[(size_t)c + 1] - indptr[(size_t)c];
  });
  const long long nrs = ((long long)n_rows + 15) / 16;
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
          const long long i = 16 * r + g;
          if (i >= n_rows) break;
          const int row = order[(size_t)i];
          const int *rb = &sidx[(size_t)indptr[(size_t)row]], *re = &sidx[(size_t)indptr[(size_t)row + 1]];
          for (const int *p = std::lower_bound(rb, re, bcut[(size_t)b]); p < re && *p < bcut[(size_t)b + 1]; p++)
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
  std::vector<int> rows((size_t)nbat * CW * NS * 16, -1);
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
        for (int g = 0; g < 16; g++) {
          const long long i = 16 * mine[a] + g;
          rows[(size_t)(((bat * CW + bw) * NS + j) * 16 + g)] = i < n_rows ? order[(size_t)i] : -1;
        }
      }
    }
  }, 0, 1);
  std::vector<unsigned short> counts((size_t)n_wg * t_max * CW * NS, 0);
  // walks (wg, wave): per visit, per rowset, the steps of its 16 lane groups.  Returns the
  // wave's entry blocks (and writes them when out != nullptr).
  auto walk = [&](long long wg, int w, unsigned short *out) -> long long {
    const int b = (int)(wg % B), bat = (int)(wg / B), T = nsl[(size_t)b];
    const int *rw = &rows[(size_t)(((long long)bat * CW + w) * NS) * 16];
    std::vector<Lane> lanes((size_t)NS * 16);
    for (int k = 0; k < NS * 16; k++) {
      Lane &L = lanes[(size_t)k];
      const int r = rw[k];
      if (r < 0) continue;
      const int *rb = &sidx[(size_t)indptr[(size_t)r]], *re = &sidx[(size_t)indptr[(size_t)r + 1]];
      L.next = (int)(std::lower_bound(rb, re, bcut[(size_t)b]) - sidx.data());
      L.end = (int)(std::lower_bound(rb, re, bcut[(size_t)b + 1]) - sidx.data());
    }
    auto admit = [&](Lane &L, int upto_slice) {  // edges of slices <= upto_slice
      const int c1 = bcut[(size_t)b] + (upto_slice + 1) * SR;
      while (L.next < L.end && sidx[(size_t)L.next] < c1) {
        const int c = sidx[(size_t)L.next++];
        L.q[c & 3].push_back(Edge{(c - bcut[(size_t)b]) / SR, c});
      }
    };
    for (auto &L : lanes) admit(L, W - 2);  // slices resident before visit 0's window completes
    long long kb = 0;
    for (int v = 0; v < T; v++) {
      const int base_col = bcut[(size_t)b];
      for (int j = 0; j < NS; j++) {
        int n = 0;
        for (int g = 0; g < 16; g++) {
          Lane &L = lanes[(size_t)j * 16 + g];
          admit(L, v + W - 1);
          L.due = 0;
          for (int r = 0; r < 4; r++)
            for (size_t h = L.head[r]; h < L.q[r].size() && L.q[r][h].slice == v; h++) L.due++;
          n = std::max(n, L.due);
        }
        const int S = (n + 3) / 4 * 4;
        PGCN_CHECK(S < 65536, PGCN_E_INVALID, "graphsum_ring: visit run too long");
        counts[(size_t)(((wg * t_max + v) * CW + w) * NS + j)] = (unsigned short)S;
        for (int st = 0; st < S; st++) {
          for (int q = 0; q < 4; q++) {
            const int *grp = kQuad[q];
            // one residue (bank quarter) per member: the permutation of the 4 residues that
            // serves every forced member (as many due edges left as steps) a due edge, then
            // the most due edges, then the most later edges (earliest slices first); members
            // left without an edge of their residue read that residue's zero row
            Lane *M[4];
            bool forced[4];
            for (int a = 0; a < 4; a++) {
              M[a] = &lanes[(size_t)j * 16 + grp[a]];
              forced[a] = M[a]->due > 0 && M[a]->due >= S - st;
            }
            auto value = [&](int a, int r) -> int {
              const Lane &L = *M[a];
              if (L.empty_res(r)) return forced[a] ? -100000 : 0;
              const int sl = L.front(r).slice;
              if (sl == v) return forced[a] ? 10000 : 1000;
              return forced[a] ? -100000 : 100 - (sl - v);
            };
            static const int kPerm[24][4] = {
                {0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {0, 3, 2, 1},
                {1, 0, 2, 3}, {1, 0, 3, 2}, {1, 2, 0, 3}, {1, 2, 3, 0}, {1, 3, 0, 2}, {1, 3, 2, 0},
                {2, 0, 1, 3}, {2, 0, 3, 1}, {2, 1, 0, 3}, {2, 1, 3, 0}, {2, 3, 0, 1}, {2, 3, 1, 0},
                {3, 0, 1, 2}, {3, 0, 2, 1}, {3, 1, 0, 2}, {3, 1, 2, 0}, {3, 2, 0, 1}, {3, 2, 1, 0}};
            int best = 0, best_v = -1 << 30;
            for (int pi = 0; pi < 24; pi++) {
              int tot = 0;
              for (int a = 0; a < 4; a++) tot += value(a, kPerm[pi][a]);
              if (tot > best_v) {
                best_v = tot;
                best = pi;
              }
            }
            for (int a = 0; a < 4; a++) {
              const int g = grp[a];
              Lane &L = *M[a];
              int pick = kPerm[best][a];
              const int zero = pick;
              if (L.empty_res(pick) || (L.front(pick).slice != v && forced[a])) {
                pick = -1;
                if (forced[a])  // no permutation serves it: a due edge, accepting a conflict
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
              if (out) out[(size_t)(kb + st / 4) * 64 + g * 4 + (st % 4)] = (unsigned short)val;
            }
          }
        }
        for (int g = 0; g < 16; g++)
          PGCN_CHECK(lanes[(size_t)j * 16 + g].due == 0, PGCN_E_INVALID,
                     "graphsum_ring: edge past its slice's visit");
        kb += S / 4;
      }
    }
    for (auto &L : lanes)
      PGCN_CHECK(L.pending() == 0 && L.next == L.end, PGCN_E_INVALID,
                 "graphsum_ring: edges left after the last visit");
    return kb;
  };
  std::vector<long long> kbs((size_t)n_wg * CW, 0);
  parallel_for(n_wg * CW, [&](long long a, long long e) {
    for (long long x = a; x < e; x++) kbs[(size_t)x] = walk(x / CW, (int)(x % CW), nullptr);
  }, 0, 64);
  std::vector<long long> off((size_t)n_wg * CW + 1, 0);
  for (size_t x = 0; x < kbs.size(); x++) off[x + 1] = off[x] + kbs[x];
  std::vector<unsigned short> ent((size_t)std::max<long long>(off.back(), 1) * 64, 0);
  parallel_for(n_wg * CW, [&](long long a, long long e) {
    for (long long x = a; x < e; x++) walk(x / CW, (int)(x % CW), &ent[(size_t)off[(size_t)x] * 64]);
  }, 0, 64);
  LdsHost h;
  h.n_blocks = B;
  h.window = kRingWindow;
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
  const int B = h.n_blocks, CW = LDS_CW, NS = LDS_SLOTS, SR = RING_SR, K = RING_K, W = RING_W;
  const long long n_wg = (long long)h.n_batches * B;
  std::vector<double> acc((size_t)NS * 16);
  for (long long wg = 0; wg < n_wg; wg++) {
    const int b = (int)(wg % B), bat = (int)(wg / B), T = h.nsl[(size_t)b];
    for (int w = 0; w < CW; w++) {
      long long kb = h.wave_off[(size_t)(wg * CW + w)];
      std::fill(acc.begin(), acc.end(), 0.0);
      for (int v = 0; v < T; v++) {
        const unsigned short *cn = &h.counts[(size_t)(((wg * h.t_max + v) * CW + w) * NS)];
        for (int j = 0; j < NS; j++) {
          PGCN_CHECK(cn[j] % 4 == 0, PGCN_E_INVALID, "ring schedule: steps not whole blocks");
          for (int k = 0; k < cn[j] / 4; k++, kb++)
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
      }
      PGCN_CHECK(kb == h.wave_off[(size_t)(wg * CW + w) + 1], PGCN_E_INVALID,
                 "ring schedule: wave stream length");
      for (int j = 0; j < NS; j++)
        for (int g = 0; g < 16; g++) {
          const int r = h.rows[(size_t)(((long long)bat * CW + w) * NS + j) * 16 + g];
          if (r >= 0) {
            PGCN_CHECK(r < n_rows, PGCN_E_INVALID, "ring schedule: row id");
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
