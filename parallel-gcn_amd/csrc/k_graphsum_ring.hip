// parallel-gcn_amd/csrc/k_graphsum_ring.hip -- GraphSum for 16-wide rows over a sliding
// window of LDS-resident feature slices (the reddit hot path; schedule: host/ring.cpp).
//
// Replaces graphsum_kernel (src/module.cu:172-210) / hpdga GraphSum::forward/backward
// (module.cpp:82-111) for d = 16 on graphs whose feature table exceeds an XCD's L2.
//
// Algebra as k_graphsum_lds: Â = D^-1/2 A D^-1/2, out_i = s_i * sum_{j in N(i)} (s_j in_j);
// k_ring_prescale forms s ⊙ in once per call (or the producing kernel's epilogue does),
// k_gs_lds_combine adds a row's column-block partials in block order, applies s_i and the
// fused element-wise tail (deterministic).
//
// Workgroup (batch, block b), one per CU: 15 summing waves + 1 loader wave, 159 KB of LDS:
//   [4 quarter planes x RING_P rows x 16 B]  the ring of RING_K = 4 slices of RING_SR = 512
//                                            rows (plane v = columns 4v..4v+3), + 4 zero rows
//   [2 x 512 B]                              step counts of visits v (v & 1), hand-off words
//   [15 x 2 KB]                              per-wave entry rings (LDS-DMA refilled)
// Visit v (one per slice of the block) reads slices v, v+1, v+2 (ring buffers t % 4); the
// loader stages slice v+3 into buffer (v+3) % 4 once every summing wave has finished visit
// v-1 (the last reader of the slice that buffer held), with the counts of visit v+1.  Entries
// are 16-bit plane offsets (ring row x 16 B): lane (g, v) reads plane v at entry + plane base.
#include "common.hpp"
#include "gs_epilogue.hpp"
#include "kernels.hpp"
#include "lds_dma.hpp"
#include "peer_sync.hpp"

namespace pgcn {

constexpr int RING_PLANE_B = RING_P * 16;                   // 32,832 B per quarter plane
constexpr int RING_TABLE_B = 4 * RING_PLANE_B;              // 131,328 B
constexpr int RING_CNT_USED = LDS_CW * LDS_SLOTS * 2;       // <= 480 B of counts per visit
constexpr int RING_CNT_B = 512;
// counts buffers: visit v's counts land with slice v + W - 1, up to K - W visits ahead of the
// slowest wave's visit (K - W + 1 buffers; room for the 2-slice window's 3)
constexpr int RING_NCB_MAX = RING_K - 1;
constexpr int RING_CNT_OFF = RING_TABLE_B;
// loaded, done[K] in the tail of counts buffer 0 (past the largest counts block)
constexpr int RING_FLAG_OFF = RING_CNT_OFF + RING_CNT_USED;
constexpr int RING_NFLAGS = 1 + RING_K;
constexpr int RING_ERING_OFF = RING_CNT_OFF + RING_NCB_MAX * RING_CNT_B;
constexpr int RING_CHUNK = 512;                             // 4 entry blocks of 128 B
constexpr int RING_ESLOTS = 4;                              // chunks: 3 in flight + 1 read
constexpr int RING_ERING_B = RING_ESLOTS * RING_CHUNK;
constexpr int RING_TOTAL_B = RING_ERING_OFF + LDS_CW * RING_ERING_B;  // 163,584 B
static_assert(RING_TOTAL_B <= 160 * 1024, "LDS budget");
static_assert(RING_FLAG_OFF + RING_NFLAGS * 4 <= RING_CNT_OFF + RING_CNT_B,
              "hand-off words fit");
static_assert(RING_SR * 16 % 1024 == 0, "a slice's plane piece is whole 1-KB LDS-DMA pieces");
static_assert(RING_K * RING_SR * 16 + 4 * 16 <= 65536, "ring rows addressable by 16 bits");

// in'[r] = scale[r] * in[col_map ? col_map[r] : r], written to the slice-plane layout:
// float4 (r / SR) * 4 SR + v SR + r % SR   (slice, plane v, row) -- the loader then copies each
// of a slice's four 8-KB planes with contiguous LDS-DMA pieces.
__global__ __launch_bounds__(256) void k_ring_prescale(const float4 *__restrict__ in, int ld4_in,
                                                       const float *__restrict__ scale, int n,
                                                       float4 *__restrict__ out,
                                                       const int *__restrict__ col_map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t >> 2;
  if (r >= n) return;
  const int v = (int)(t & 3);
  const float s = scale[r];
  const long long src = col_map ? (long long)col_map[r] : r;
  float4 x = in[src * ld4_in + v];
  x.x *= s;
  x.y *= s;
  x.z *= s;
  x.w *= s;
  out[(r / RING_SR) * (4 * RING_SR) + v * RING_SR + r % RING_SR] = x;
}

// Every 16-column pass of a wide GraphSum prescaled by one launch (r03): table p = the
// k_ring_prescale output for input columns c[p] .. c[p] + 15.  A block stages 64 rows x up to
// 128 columns through LDS (coalesced row reads, rows padded to 132 floats so 16 consecutive
// rows' float4s are bank-distinct) and writes each (pass, plane) as 64 consecutive float4s
// (1 KB) of its slice plane.  The same products as the per-pass prescale: same bits.
constexpr int RPW_ROWS = 64;
constexpr int RPW_LD = 132;
static_assert(RING_SR % RPW_ROWS == 0, "a block's rows stay inside one slice");
__global__ __launch_bounds__(256) void k_ring_prescale_wide(const float *__restrict__ in, int ld_in,
                                                            int width, const float *__restrict__ scale,
                                                            int n, RingPasses passes,
                                                            float4 *__restrict__ out,
                                                            long long table_f4) {
  __shared__ float rows[RPW_ROWS * RPW_LD];
  const int r0 = blockIdx.x * RPW_ROWS;
  const int w4 = width / 4;  // float4s per row staged (width: multiple of 4, <= 128)
  for (int e = threadIdx.x; e < RPW_ROWS * w4; e += 256) {
    const int r = e / w4, q = e - r * w4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < n) {
      x = *reinterpret_cast<const float4 *>(in + (long long)(r0 + r) * ld_in + 4 * q);
      const float s = scale[r0 + r];
      x.x *= s;
      x.y *= s;
      x.z *= s;
      x.w *= s;
    }
    *reinterpret_cast<float4 *>(&rows[r * RPW_LD + 4 * q]) = x;
  }
  __syncthreads();
  const long long slot0 = (long long)(r0 / RING_SR) * (4 * RING_SR) + r0 % RING_SR;
  for (int e = threadIdx.x; e < passes.n * 4 * RPW_ROWS; e += 256) {
    const int r = e % RPW_ROWS, pv = e / RPW_ROWS, p = pv >> 2, v = pv & 3;
    if (r0 + r >= n) continue;
    const float4 x = *reinterpret_cast<const float4 *>(&rows[r * RPW_LD + passes.c[p] + 4 * v]);
    out[p * table_f4 + slot0 + v * RING_SR + r] = x;
  }
}

// out[r] = scale[r] * sum_{b < nb} partial[b][r]   (block order => deterministic), then the
// fused element-wise tail (gs_epilogue.hpp)
//
// Push mode (PUSH, the edge-cut engine's peer exchange, k_peer.hip): row r belongs to rank
// q = r / rows_per_rank, and its sum goes straight into q's receive slot of this rank (over
// xGMI when q is a peer) instead of `out`; the launch's last workgroup then signals the
// receivers (peer_arrive).  No epilogue: the receiver applies it after summing the ranks.
template <bool PUSH>
__global__ __launch_bounds__(PUSH ? 1024 : 256) void k_gs_lds_combine(
    const float4 *__restrict__ partial, long long part_stride, int nb,
    const float *__restrict__ scale, int n, float4 *__restrict__ out, int ld4_out,
    GsEpilogue epi, PeerSink push) {
  if (PUSH) {
    // 64-row tiles; consecutive tiles serve different owners (tile b: owner b % world, its rows
    // 64 (b / world) ..), so the pushes in flight at any time spread over every peer's link
    // instead of draining the owners one after another.  A bounded grid of 1,024-thread
    // workgroups walks the tiles (4 at a time per workgroup): each workgroup ends with one
    // system-scope release (peer_arrive), and few workgroups keep those L2 write-backs few.
    const long long n_tiles = (long long)push.world * ((push.rows_per_rank + 63) / 64);
    // Two tiles per thread and iteration, both tiles' loads issued before either's adds.
    const int v = (int)(threadIdx.x & 3);
    const long long step = (long long)gridDim.x * 4;
    for (long long tile = (long long)blockIdx.x * 4 + (threadIdx.x >> 8); tile < n_tiles;
         tile += 2 * step) {
      int q[2];
      long long j[2], r[2];
      bool ok[2];
      float s[2];
      float4 p[2][4];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const long long t = tile + u * step;
        q[u] = (int)(t % push.world);                                 // the owner
        j[u] = (t / push.world) * 64 + ((threadIdx.x & 255) >> 2);    // its row
        r[u] = (long long)q[u] * push.rows_per_rank + j[u];
        ok[u] = t < n_tiles && j[u] < push.rows_per_rank && r[u] < n;
        if (ok[u]) {
          s[u] = scale[r[u]];
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (b < nb) p[u][b] = partial[((long long)b * part_stride + r[u]) * 4 + v];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        if (!ok[u]) continue;
        float4 a = p[u][0];
#pragma unroll
        for (int b = 1; b < 4; b++)
          if (b < nb) f4_acc(a, p[u][b]);
        for (int b = 4; b < nb; b++)
          f4_acc(a, partial[((long long)b * part_stride + r[u]) * 4 + v]);
        a.x *= s[u];
        a.y *= s[u];
        a.z *= s[u];
        a.w *= s[u];
        peer_store16(push.dst[q[u]], push.slot_bytes, j[u] * ld4_out + v, a);
      }
    }
    peer_arrive(push);
    return;
  }
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t >> 2;
  if (r >= n) return;
  const int v = (int)(t & 3);
  // the row scale and the epilogue's inputs with the partials: one round trip, not one each
  const float s = scale[r];
  GsEpiIn ein;
  gs_epi_load(ein, r, 4 * v, epi);
  float4 a;
  if (nb <= 8) {  // every block's partial loaded before the (ordered) adds
    float4 p[8];
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (b < nb) p[b] = partial[((long long)b * part_stride + r) * 4 + v];
    a = p[0];
#pragma unroll
    for (int b = 1; b < 8; b++)
      if (b < nb) f4_acc(a, p[b]);
  } else {
    a = partial[r * 4 + v];
    for (int b = 1; b < nb; b++) f4_acc(a, partial[((long long)b * part_stride + r) * 4 + v]);
  }
  a.x *= s;
  a.y *= s;
  a.z *= s;
  a.w *= s;
  gs_epilogue(a, r, 4 * v, epi, ein);
  out[r * ld4_out + v] = a;
}

// y[r] = epilogue(y[r]) for the n rows of a reduce-scattered GraphSum output (edge-cut engine:
// the tail a one-GPU GraphSum applies in its combine, applied once the partial sums of every
// rank have been added; the same operations on the same sums: bit-identical to the modules)
__global__ __launch_bounds__(256) void k_gs_finish(float4 *__restrict__ y, int ld4, int n, int vec,
                                                   GsEpilogue epi) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t / vec;
  if (r >= n) return;
  const int v = (int)(t - r * vec);
  GsEpiIn ein;
  gs_epi_load(ein, r, 4 * v, epi);
  float4 a = y[r * ld4 + v];
  gs_epilogue(a, r, 4 * v, epi, ein);
  y[r * ld4 + v] = a;
}

// The receiving end of a pushed GraphSum (k_peer.hip): y[r] = the sum over ranks q (rank
// order) of slot q's row r, then the fused tail as k_gs_finish (the same operations on the
// same sums as the reduce-scattered form with a rank-order sum)
__global__ __launch_bounds__(256) void k_gs_gather_finish(float4 *__restrict__ y, int ld4, int n,
                                                          int vec, GsEpilogue epi, PeerRecv rv) {
  acquire_system_workgroup();  // the peers' pushes (peer_sync.hpp)
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t / vec;
  if (r >= n) return;
  const int v = (int)(t - r * vec);
  GsEpiIn ein;
  gs_epi_load(ein, r, 4 * v, epi);
  float4 p[kPeerMaxRanks];
#pragma unroll
  for (int q = 0; q < kPeerMaxRanks; q++)
    if (q < rv.world) p[q] = reinterpret_cast<const float4 *>(rv.slot[q])[r * ld4 + v];
  float4 a = p[0];
#pragma unroll
  for (int q = 1; q < kPeerMaxRanks; q++)
    if (q < rv.world) f4_acc(a, p[q]);
  gs_epilogue(a, r, 4 * v, epi, ein);
  y[r * ld4 + v] = a;
}

// NS: rowsets per summing wave (LDS_SLOTS).  PAIR (ring_pair, host/ring.cpp): rowsets 2p and
// 2p + 1 run the same step count per visit and their entry blocks alternate, so a wave issues
// both blocks' eight table reads before it waits (the adds of 2p's block wait only for its own
// four): two blocks in flight per wave instead of one, the same adds in the same order per row
// WIN: slices a visit reads (the schedule's window, LdsSchedule::w): 3, or 2 -- the loader
// then runs two slices ahead of the visits, for schedules whose visits are shorter than a
// slice's LDS-DMA (tall edge-cut rank graphs, sparse graphs)
template <int NS, bool PAIR, int WIN>
__global__ __launch_bounds__(LDS_THREADS) void k_graphsum_ring(
    const uint2 *__restrict__ entries, const long long *__restrict__ wave_off,
    const unsigned short *__restrict__ counts, int t_max, const int2 *__restrict__ slices,
    const int *__restrict__ n_slices, const int *__restrict__ rows, const char *__restrict__ table,
    float4 *__restrict__ partial, long long part_stride, int n_blocks) {
  static_assert(NS == 16, "rowsets per wave");
  static_assert(WIN >= 2 && WIN <= RING_K - 1, "ring window");
  constexpr int RING_NCB = RING_K - WIN + 1;
  constexpr int CNT_USED = LDS_CW * NS * 2;  // counts of one visit (bytes)
  __shared__ float4 lds[RING_TOTAL_B / 16];
  const int nb = n_blocks;
  const int b = blockIdx.x % nb, batch = blockIdx.x / nb;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = lane >> 2, v = lane & 3;
  const int T = n_slices[b];
  char *const lb = reinterpret_cast<char *>(lds);
  const unsigned lds_base = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<size_t>((__attribute__((address_space(3))) float4 *)lds));
  // zero rows: ring rows K*SR .. K*SR+3 of every plane (padding entries read them)
  if (threadIdx.x < 16)
    lds[((threadIdx.x >> 2) * RING_PLANE_B + (RING_K * RING_SR + (threadIdx.x & 3)) * 16) / 16] =
        make_float4(0.f, 0.f, 0.f, 0.f);
  unsigned *const flags = reinterpret_cast<unsigned *>(lb + RING_FLAG_OFF);
  unsigned *const loaded = flags, *const done = flags + 1;
  if (threadIdx.x < RING_NFLAGS) flags[threadIdx.x] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // zero rows and hand-off words set (the only barrier)
  asm volatile("" ::: "memory");

  if (wave == LDS_CW) {  // ------------------------------------------------ loader wave
    __builtin_amdgcn_s_setprio(3);
    const int2 *sl = slices + (long long)b * t_max;
    const char *cnt_src =
        reinterpret_cast<const char *>(counts) + (long long)blockIdx.x * t_max * CNT_USED;
    const int iters = T + WIN - 1;
    for (int s = 0; s < iters; s++) {
      // buffer s % K (and counts buffer (s - W + 1) & 1) free: visit s - K done everywhere
      if (s >= RING_K)
        lds_wait_ge(done + (s - RING_K) % RING_K, (unsigned)(LDS_CW * ((s - RING_K) / RING_K + 1)));
      if (s < T) {
        const char *src = table + (long long)sl[s].x * 64 + lane * 16;
        const unsigned dst = lds_base + (unsigned)((s % RING_K) * RING_SR * 16);
#pragma unroll
        for (int p = 0; p < 4; p++) {  // plane p of the slice: RING_SR * 16 B
#pragma unroll
          for (int q = 0; q + 4096 <= RING_SR * 16; q += 4096)
            glds16x4(src + p * (RING_SR * 16) + q, dst + (unsigned)(p * RING_PLANE_B + q));
#pragma unroll
          for (int q = RING_SR * 16 / 4096 * 4096; q < RING_SR * 16; q += 1024)
            glds16(src + p * (RING_SR * 16) + q, dst + (unsigned)(p * RING_PLANE_B + q));
        }
      }
      const int cv = s - (WIN - 1);  // the visit whose last slice this is
      if (cv >= 0 && lane * 16 < CNT_USED)
        glds16(cnt_src + (long long)cv * CNT_USED + lane * 16,
               lds_base + (unsigned)(RING_CNT_OFF + (cv % RING_NCB) * RING_CNT_B));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slice s and counts landed
      if (lane == 0) __atomic_store_n(loaded, (unsigned)(s + 1), __ATOMIC_RELAXED);
      asm volatile("" ::: "memory");
    }
    return;
  }

  // ------------------------------------------------------------------------- summing waves
  const long long wid = (long long)blockIdx.x * LDS_CW + wave;
  const long long kb0 = wave_off[wid];
  // the wave's entry stream, 512-B chunks (4 entry blocks) into a 4-slot LDS ring; refills
  // run up to 3 chunks past the stream's end (the entries array has 2 KB of slack)
  const char *esrc = reinterpret_cast<const char *>(entries) + kb0 * 128 + lane * 16;
  const unsigned ring_dst = lds_base + (unsigned)(RING_ERING_OFF + wave * RING_ERING_B);
  auto refill = [&](int c) {  // chunk c -> ring slot c % 4
    if (lane < 32) glds16(esrc, ring_dst + (unsigned)((c & (RING_ESLOTS - 1)) * RING_CHUNK));
    esrc += RING_CHUNK;
  };
  refill(0);
  refill(1);
  refill(2);
  refill(3);
  asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // chunk 0

  f4v acc[NS];
#pragma unroll
  for (int j = 0; j < NS; j++) acc[j] = f4v{0.f, 0.f, 0.f, 0.f};
  // Entry ring cursor: this lane's LDS byte address of the next block's entries, and the
  // blocks left in the current 4-block chunk (r03: per block one VALU add and a scalar
  // count-down, where the ring offset arithmetic and the chunk test took six scalar ops)
  unsigned ecur = ring_dst + (unsigned)(g * 8);
  const unsigned ering_end = ring_dst + (unsigned)RING_ERING_B;
  constexpr int UNIT = PAIR ? 256 : 128;  // bytes of entries per step of the loop
  int left = RING_CHUNK / UNIT;
  int chunk = 0;
  u2v e_next = ds_rd64(ecur);
  u2v e_next1 = PAIR ? ds_rd64(ecur + 128) : u2v{0u, 0u};
  // lane (g, v) reads plane v: entry (ring row x 16 B) + this constant
  const unsigned tb = lds_base + (unsigned)(v * RING_PLANE_B);
  // One entry block: its four table addresses from the landed entries, then the next block's
  // entry read (into the same registers: in-order issue reads them first), its chunk's refill
  // when a chunk is entered (the slot refilled held the chunk before, whose last entries were
  // waited for with the previous block), the four table reads, one wait, the adds.
  auto block = [&](f4v &a) {
    const unsigned a0 = tb + (e_next.x & 0xffffu), a1 = tb + (e_next.x >> 16),
                   a2 = tb + (e_next.y & 0xffffu), a3 = tb + (e_next.y >> 16);
    ecur += 128;
    if (--left == 0) {
      left = RING_CHUNK / 128;
      ++chunk;
      if (ecur >= ering_end) ecur -= RING_ERING_B;
      refill(chunk + 3);
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // chunk `chunk` landed
    }
    ds_rd64_into(e_next, ecur);
    f4v x0 = ds_rd128(a0), x1 = ds_rd128(a1), x2 = ds_rd128(a2), x3 = ds_rd128(a3);
    lgkm_wait<0>(x0, x1, x2, x3, e_next);
    a += x0;
    a += x1;
    a += x2;
    a += x3;
  };
  // PAIR: block k of rowset 2p then block k of rowset 2p + 1 (256 B of entries): both blocks'
  // addresses from the landed entries, the next pair's two entry reads, the eight table reads,
  // 2p's adds once its four have returned (lgkmcnt(4): LDS operations complete in order), then
  // 2p + 1's
  auto pair_block = [&](f4v &a, f4v &b) {
    const unsigned a0 = tb + (e_next.x & 0xffffu), a1 = tb + (e_next.x >> 16),
                   a2 = tb + (e_next.y & 0xffffu), a3 = tb + (e_next.y >> 16);
    const unsigned b0 = tb + (e_next1.x & 0xffffu), b1 = tb + (e_next1.x >> 16),
                   b2 = tb + (e_next1.y & 0xffffu), b3 = tb + (e_next1.y >> 16);
    ecur += 256;
    if (--left == 0) {
      left = RING_CHUNK / 256;
      ++chunk;
      if (ecur >= ering_end) ecur -= RING_ERING_B;
      refill(chunk + 3);
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // chunk `chunk` landed
    }
    ds_rd64_into(e_next, ecur);
    ds_rd64_into(e_next1, ecur + 128);
    f4v x0 = ds_rd128(a0), x1 = ds_rd128(a1), x2 = ds_rd128(a2), x3 = ds_rd128(a3);
    f4v y0 = ds_rd128(b0), y1 = ds_rd128(b1), y2 = ds_rd128(b2), y3 = ds_rd128(b3);
    lgkm_wait<4>(x0, x1, x2, x3, e_next, e_next1);
    a += x0;
    a += x1;
    a += x2;
    a += x3;
    lgkm_wait<0>(y0, y1, y2, y3);
    b += y0;
    b += y1;
    b += y2;
    b += y3;
  };
  for (int t = 0; t < T; t++) {
    lds_wait_ge(loaded, (unsigned)(t + WIN));  // slices t .. t+WIN-1 and visit t's counts
    // lane l reads rowset (l % 16)'s step count; two ballots give the rowsets with blocks this
    // visit and those with more than one: per rowset a scalar bit test (the sign bit of the
    // mask shifted), the count itself only for the few longer runs (r03 late: per visit 8
    // readfirstlanes and 16 extract-compare-branch sequences were ~40 of the wave's SALU
    // instructions; 254.8 -> 250.4 us per call, 536-538 -> 541-542 epochs/s).  Per (rowset,
    // visit): 0 blocks (half the pairs on reddit), 1 (92 % of the blocks) or more
    const unsigned short *c16 = reinterpret_cast<const unsigned short *>(
        lb + RING_CNT_OFF + (t % RING_NCB) * RING_CNT_B + wave * (2 * NS));
    const unsigned cl = c16[lane & (NS - 1)];
    const unsigned nz = (unsigned)__ballot(cl != 0u), big = (unsigned)__ballot(cl > 4u);
    if constexpr (PAIR) {
#pragma unroll
      for (int j = 0; j < NS; j += 2) {
        if (__builtin_amdgcn_readfirstlane((int)(nz << (31 - j))) < 0) {  // the pair's run
          pair_block(acc[j], acc[j + 1]);
          if ((big >> j) & 1u) {
            const unsigned n = (unsigned)__builtin_amdgcn_readlane((int)cl, j);
            for (unsigned k = 4; k < n; k += 4) pair_block(acc[j], acc[j + 1]);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NS; j++) {
        if (__builtin_amdgcn_readfirstlane((int)(nz << (31 - j))) < 0) {  // bit j: the sign bit
          block(acc[j]);
          if ((big >> j) & 1u) {
            const unsigned n = (unsigned)__builtin_amdgcn_readlane((int)cl, j);
            for (unsigned k = 4; k < n; k += 4) block(acc[j]);
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of slice t returned
    // the visit's done count += 1 by lane 0 alone (exec = lane 0 inside the asm; hipcc's
    // atomic optimizer made the C++ form a 25-instruction ballot / mbcnt / nested-exec
    // sequence; r03 late: 253.5 -> 247.5 us per call); the returned value is read from lane 0
    unsigned rank;
    {
      unsigned long long saved;
      const unsigned daddr = lds_base + (unsigned)(RING_FLAG_OFF + 4 * (1 + t % RING_K));
      asm volatile(
          "s_mov_b64 %1, exec\n\t"
          "s_mov_b64 exec, 1\n\t"
          "ds_add_rtn_u32 %0, %2, %3\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "s_mov_b64 exec, %1"
          : "=&v"(rank), "=&s"(saved)
          : "v"(daddr), "v"(1u)
          : "memory");
    }
    // The arbiter favours older waves, so the youngest waves of a workgroup fall behind and
    // the visits' hand-offs make everyone wait for them (r02 stamps: 395 vs 576 cycles per
    // block from the oldest to the youngest wave).  The last third of the waves to finish a
    // visit run the next one at raised priority, the first third at the lowest (hand-off
    // waits 22 % -> 6 %).
    rank = (unsigned)__builtin_amdgcn_readfirstlane((int)rank) - (unsigned)(LDS_CW * (t / RING_K));
    if (rank >= (unsigned)(2 * LDS_CW / 3)) __builtin_amdgcn_s_setprio(2);
    else if (rank >= (unsigned)(LDS_CW / 3)) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the dummy ring refills
  // rows[] = row | log2(m) << 28: a row spread over m lane groups (host/ring.cpp) has its m
  // partial sums added across lane groups g ^ 1, g ^ 2, .. (xor butterfly, fixed order for the
  // writing lane group g % m == 0); m is uniform per rowset
  // (every rowset's row word first, one wait for all: loaded at its use, each load waited
  // behind the store before it, NS round trips at the kernel's end)
  const int *rw = rows + (((long long)batch * LDS_CW + wave) * NS) * 16 + g;
  float4 *pb = partial + (long long)b * part_stride * 4 + v;
  int uw[NS];
#pragma unroll
  for (int j = 0; j < NS; j++) uw[j] = rw[j * 16];
#pragma unroll
  for (int j = 0; j < NS; j++) {
    const int u = uw[j];
    const int sp = __builtin_amdgcn_readfirstlane((int)((unsigned)u >> 28));
    float4 a = make_float4(acc[j].x, acc[j].y, acc[j].z, acc[j].w);
    for (int k = 0; k < sp; k++) {
      const int d = 4 << k;
      a.x += __shfl_xor(a.x, d);
      a.y += __shfl_xor(a.y, d);
      a.z += __shfl_xor(a.z, d);
      a.w += __shfl_xor(a.w, d);
    }
    const int r = u & kRingRowMask;
    if (r != kRingEmpty && (g & ((1 << sp) - 1)) == 0) pb[(long long)r * 4] = a;
  }
}

// Measured and removed (r02): the batch's last workgroup combining the block partials itself
// (an sc1 write-through hand-off, bit-identical, 0.263 vs 0.230 ms per call: the combine of
// all 61 batches then runs at the kernel's end on 61 CUs), one prescale / combine launch for
// all 16-column passes of a wide row (1.677 vs 1.594 ms per d = 128 call: the 8 passes'
// partials no longer stay in the Infinity Cache), fixed issue priority (hand-off waits 22 %).

void launch_gs_finish(float *y, int ld, int n, int dim, const GsEpilogue &epi, hipStream_t st) {
  PGCN_CHECK(ld % 4 == 0 && dim % 4 == 0 && dim <= ld && n >= 0, PGCN_E_INVALID,
             "gs_finish: shape");
  PGCN_CHECK(!epi.next_table || dim == 16, PGCN_E_INVALID, "gs_finish: next table of a wide row");
  if (n == 0 || epi.mode == 0) return;
  const long long t = (long long)n * (dim / 4);
  PGCN_LAUNCH(k_gs_finish, dim3((unsigned)ceil_div(t, 256)), dim3(256), 0, st,
              reinterpret_cast<float4 *>(y), ld / 4, n, dim / 4, epi);
  PGCN_HIP(hipGetLastError());
}

void launch_gs_gather_finish(float *y, int ld, int n, int dim, const GsEpilogue &epi,
                             const PeerRecv &r, hipStream_t st) {
  PGCN_CHECK(ld % 4 == 0 && dim % 4 == 0 && dim <= ld && n >= 0 && r.world >= 1 &&
                 r.world <= kPeerMaxRanks,
             PGCN_E_INVALID, "gs_gather_finish: shape");
  PGCN_CHECK(!epi.next_table || dim == 16, PGCN_E_INVALID,
             "gs_gather_finish: next table of a wide row");
  if (n == 0) return;
  const long long t = (long long)n * (dim / 4);
  PGCN_LAUNCH(k_gs_gather_finish, dim3((unsigned)ceil_div(t, 256)), dim3(256), 0, st,
              reinterpret_cast<float4 *>(y), ld / 4, n, dim / 4, epi, r);
  PGCN_HIP(hipGetLastError());
}

void launch_ring_prescale_wide(const LdsSchedule &s, const float *in, int ld_in, int width,
                               const RingPasses &passes, float *tables, long long table_floats,
                               hipStream_t st) {
  PGCN_CHECK(ld_in % 4 == 0 && width % 4 == 0 && width <= 128 && passes.n >= 1 && passes.n <= 8,
             PGCN_E_INVALID, "ring_prescale_wide: shape");
  for (int p = 0; p < passes.n; p++)
    PGCN_CHECK(passes.c[p] % 4 == 0 && passes.c[p] + 16 <= width, PGCN_E_INVALID,
               "ring_prescale_wide: pass columns");
  PGCN_LAUNCH(k_ring_prescale_wide, dim3((unsigned)ceil_div(s.n_cols, RPW_ROWS)), dim3(256), 0, st,
              in, ld_in, width, s.col_scale, s.n_cols, passes, reinterpret_cast<float4 *>(tables),
              table_floats / 4);
  PGCN_HIP(hipGetLastError());
}

void launch_graphsum_ring(const LdsSchedule &s, const float *in, int ld_in, float *out,
                          int ld_out, float *scratch_in, float *partial, hipStream_t st,
                          const int *col_map, const GsEpilogue *epi, bool prestaged,
                          const PeerSink *push, hipStream_t tail_st, hipEvent_t fork) {
  note_path(KP_GS_RING);
  PGCN_CHECK(!tail_st || (push && fork), PGCN_E_INVALID, "graphsum_ring: tail stream of a push");
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0, PGCN_E_INVALID, "graphsum_ring: ld % 4");
  const long long pre = (long long)s.n_cols * 4;
  if (!prestaged)
    PGCN_LAUNCH(k_ring_prescale, dim3((unsigned)ceil_div(pre, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float4 *>(in), ld_in / 4, s.col_scale, s.n_cols,
                       reinterpret_cast<float4 *>(scratch_in), col_map);
  const long long n_wg = (long long)s.n_batches * s.n_blocks;
#define RING_LAUNCH(NS_, PAIR_, WIN_)                                                           \
  PGCN_LAUNCH((k_graphsum_ring<NS_, PAIR_, WIN_>), dim3((unsigned)n_wg), dim3(LDS_THREADS), 0, st, s.entries, \
              s.wave_off, s.counts, s.t_max, s.slices, s.n_slices, s.rows,                      \
              reinterpret_cast<const char *>(scratch_in), reinterpret_cast<float4 *>(partial), \
              (long long)s.n_rows, s.n_blocks)
  PGCN_CHECK(ring_slots_ok(s.ns), PGCN_E_INVALID, "graphsum_ring: rowsets per wave");
  PGCN_CHECK((s.w == 2 || s.w == 3) && (!s.pair || s.w == 3), PGCN_E_INVALID,
             "graphsum_ring: window (pairs: 3 only)");
  if (s.pair)
    RING_LAUNCH(16, true, 3);
  else if (s.w == 2)
    RING_LAUNCH(16, false, 2);
  else
    RING_LAUNCH(16, false, 3);
#undef RING_LAUNCH
  const GsEpilogue none{};
  const long long post = (long long)s.n_rows * 4;
  if (push) {
    PGCN_CHECK((!epi || epi->mode == 0) && push->world >= 1 && push->world <= kPeerMaxRanks &&
                   push->rows_per_rank > 0 && (long long)push->rows_per_rank * push->world >= s.n_rows,
               PGCN_E_INVALID, "graphsum_ring: push shape");
    const long long tiles = (long long)push->world * ceil_div(push->rows_per_rank, 64);
    // one workgroup per CU: 2 / 4 / 8 per CU measured 0.542 / 0.590 / 0.586 ms per W = 8 rank
    // epoch against 0.511 (profiles/r05/k): every workgroup's release writes back its L2
    const long long blocks = std::min<long long>(ceil_div(tiles, 4), (long long)kCUs);
    if (tail_st) {  // the push (and what follows it) on another stream, after the ring
      PGCN_HIP(hipEventRecord(fork, st));
      PGCN_HIP(hipStreamWaitEvent(tail_st, fork, 0));
      st = tail_st;
    }
    PGCN_LAUNCH(k_gs_lds_combine<true>, dim3((unsigned)blocks), dim3(1024), 0, st,
                reinterpret_cast<const float4 *>(partial), (long long)s.n_rows, s.n_blocks,
                s.row_scale, s.n_rows, nullptr, ld_out / 4, none, *push);
  } else {
    PGCN_LAUNCH(k_gs_lds_combine<false>, dim3((unsigned)ceil_div(post, 256)), dim3(256), 0, st,
                reinterpret_cast<const float4 *>(partial), (long long)s.n_rows, s.n_blocks,
                s.row_scale, s.n_rows, reinterpret_cast<float4 *>(out), ld_out / 4,
                epi ? *epi : none, PeerSink{});
  }
  PGCN_HIP(hipGetLastError());
}

}  // namespace pgcn
