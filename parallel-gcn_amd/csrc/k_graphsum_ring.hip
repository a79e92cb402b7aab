// parallel-gcn_amd/csrc/k_graphsum_ring.hip -- GraphSum for 16-wide rows over a sliding
// window of LDS-resident feature slices (the reddit hot path; schedule: host/ring.cpp).
//
// Replaces graphsum_kernel (src/module.cu:172-210) / hpdga GraphSum::forward/backward
// (module.cpp:82-111) for d = 16 on graphs whose feature table exceeds an XCD's L2.
//
// Algebra as k_graphsum_lds: Â = D^-1/2 A D^-1/2, out_i = s_i * sum_{j in N(i)} (s_j in_j);
// k_ring_prescale forms s ⊙ in once per call, k_gs_lds_combine adds a row's column-block
// partials in block order and applies s_i (deterministic).
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

namespace pgcn {

constexpr int RING_PLANE_B = RING_P * 16;                   // 32,832 B per quarter plane
constexpr int RING_TABLE_B = 4 * RING_PLANE_B;              // 131,328 B
constexpr int RING_CNT_USED = LDS_CW * LDS_SLOTS * 2;       // 480 B of counts per visit
constexpr int RING_CNT_B = 512;
// counts buffers: visit v's counts land with slice v + W - 1, up to K - W visits ahead of the
// slowest wave's visit
constexpr int RING_NCB = RING_K - RING_W + 1;
constexpr int RING_CNT_OFF = RING_TABLE_B;
// loaded, done[K], last (fused combine) in the tail of counts buffer 0
constexpr int RING_FLAG_OFF = RING_CNT_OFF + RING_CNT_USED;
constexpr int RING_LAST_FLAG = 1 + RING_K;
constexpr int RING_ERING_OFF = RING_CNT_OFF + RING_NCB * RING_CNT_B;
constexpr int RING_CHUNK = 512;                             // 4 entry blocks of 128 B
constexpr int RING_ESLOTS = 4;                              // chunks: 3 in flight + 1 read
constexpr int RING_ERING_B = RING_ESLOTS * RING_CHUNK;
constexpr int RING_TOTAL_B = RING_ERING_OFF + LDS_CW * RING_ERING_B;  // 163,072 B
static_assert(RING_TOTAL_B <= 160 * 1024, "LDS budget");
static_assert(RING_FLAG_OFF + (RING_LAST_FLAG + 1) * 4 <= RING_CNT_OFF + RING_CNT_B,
              "hand-off + arrival words fit");
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

// Rows wider than 16 (host/graph.cpp): one launch forms every 16-column pass's table.  Pass p
// holds columns 4 c4(p) .. 4 c4(p) + 15, c4(p) = 4p except the last pass, which starts at
// last_c4 (it overlaps the one before it so it stays inside the leading dims).  Thread order:
// row fastest, so each (pass, quarter) plane is written contiguously.
__global__ __launch_bounds__(256) void k_ring_prescale_wide(const float4 *__restrict__ in,
                                                            int ld4_in,
                                                            const float *__restrict__ scale, int n,
                                                            float4 *__restrict__ tables,
                                                            long long table4, int n_pass,
                                                            int last_c4,
                                                            const int *__restrict__ col_map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long pv = t / n;
  const int r = (int)(t - pv * n);
  if (pv >= 4LL * n_pass) return;
  const int p = (int)(pv >> 2), v = (int)(pv & 3);
  const int c4 = p < n_pass - 1 ? 4 * p : last_c4;
  const float s = scale[r];
  const long long src = col_map ? (long long)col_map[r] : r;
  float4 x = in[src * ld4_in + c4 + v];
  x.x *= s;
  x.y *= s;
  x.z *= s;
  x.w *= s;
  tables[p * table4 + (r / RING_SR) * (4 * RING_SR) + v * RING_SR + r % RING_SR] = x;
}

// ... and one launch adds every pass's block partials (block order, as k_gs_lds_combine), scales
// by s_i, applies the epilogue and writes whole rows: out float4 q of row r comes from pass
// p = min(q / 4, n_pass - 1) (the last pass's overlap is recomputed to the same bits).
__global__ __launch_bounds__(256) void k_gs_lds_combine_wide(
    const float4 *__restrict__ partial, long long pass4, long long part_stride, int nb,
    const float *__restrict__ scale, int n, float4 *__restrict__ out, int ld4_out, int q_end,
    int n_pass, int last_c4, GsEpilogue epi) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t / q_end;
  if (r >= n) return;
  const int q = (int)(t - r * q_end);
  const int p = min(q >> 2, n_pass - 1);
  const int v = q - (p < n_pass - 1 ? 4 * p : last_c4);
  const float4 *pp = partial + p * pass4 + v;
  float4 a = pp[r * 4];
  for (int b = 1; b < nb; b++) f4_acc(a, pp[((long long)b * part_stride + r) * 4]);
  const float s = scale[r];
  a.x *= s;
  a.y *= s;
  a.z *= s;
  a.w *= s;
  gs_epilogue(a, r, 4 * q, epi);
  out[r * ld4_out + q] = a;
}

void launch_graphsum_ring_wide(const LdsSchedule &s, const float *in, int ld_in, float *out,
                               int ld_out, int dim, float *tables, long long table_floats,
                               float *partials, long long partial_floats, hipStream_t st,
                               const int *col_map, const GsEpilogue *epi) {
  const int ldm = ld_in < ld_out ? ld_in : ld_out;
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0 && ldm >= 16 && dim > 16 && dim <= ldm,
             PGCN_E_INVALID, "graphsum_ring_wide: leading dims");
  const int n_pass = (dim + 15) / 16, last_c4 = (ldm - 16) / 4 < 4 * (n_pass - 1) ? (ldm - 16) / 4
                                                                                 : 4 * (n_pass - 1);
  const long long pre = 4LL * n_pass * s.n_cols;
  hipLaunchKernelGGL(k_ring_prescale_wide, dim3((unsigned)ceil_div(pre, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(in), ld_in / 4, s.col_scale, s.n_cols,
                     reinterpret_cast<float4 *>(tables), table_floats / 4, n_pass, last_c4,
                     col_map);
  for (int p = 0; p < n_pass; p++)
    launch_graphsum_ring(s, nullptr, ld_in, nullptr, ld_out, tables + p * table_floats,
                         partials + p * partial_floats, st, nullptr, nullptr, true, false);
  const GsEpilogue none{};
  const int q_end = (4 * (last_c4 + 4) < ldm ? 4 * (last_c4 + 4) : ldm) / 4;
  const long long post = (long long)s.n_rows * q_end;
  hipLaunchKernelGGL(k_gs_lds_combine_wide, dim3((unsigned)ceil_div(post, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(partials), partial_floats / 4,
                     (long long)s.n_rows, s.n_blocks, s.row_scale, s.n_rows,
                     reinterpret_cast<float4 *>(out), ld_out / 4, q_end, n_pass, last_c4,
                     epi ? *epi : none);
  PGCN_HIP(hipGetLastError());
}

// diagnostics ("graphsum_lds_diag", k_graphsum_lds.hip): 4 = per-wave cycle stamps into
// stamps[wg][wave][8] (summing: 0 loop, 1 hand-off wait, 2 ring wait, 3 entry blocks, 4 visits;
// loader: 1 wait for a free buffer, 2 wait for its pieces to land, 4 slices); 1 = no table reads;
// 2 = the loader stages 1/8 of each slice (both timing only)
extern int g_graphsum_lds_diag;
unsigned long long *lds_stamps(long long n_wg);
__device__ __forceinline__ unsigned long long ring_clk() { return __builtin_amdgcn_s_memtime(); }


// Fused combine (arrive != null): the last of a batch's n_blocks workgroups to finish adds the
// batch's rows' block partials in block order, scales them by s_i, applies the epilogue and
// writes the output -- k_gs_lds_combine's arithmetic, bit for bit, without its launch.
// Hand-off (MI355X_MICROARCH.md "visibility", valid-forms table row 1; no fences):
//   * the partials are stored write-through (16-B sc1 stores) and every storing wave drains
//     them (vmcnt(0)) before the workgroup barrier;
//   * then ONE lane adds 1 to the batch's counter (agent-scope atomic); the workgroup whose add
//     returns n_blocks - 1 is the last, tells its waves through an LDS word behind a second
//     barrier, and resets the counter for the next call (kernels on one stream are ordered);
//   * every load of the partials there is an sc1 load (bypasses the CU's L1).
// No workgroup waits for another: a workgroup that is not last exits.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_part_rsrc(const float4 *partial,
                                                                 long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(partial), 0, (int)bytes,
                                           0x00020000);
}
typedef unsigned ring_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ring_st_sc1(__amdgpu_buffer_rsrc_t rs, unsigned off, float4 a) {
  const ring_u4 u = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(a.z),
                     __float_as_uint(a.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);  // aux 16 = sc1
}
__device__ __forceinline__ float4 ring_ld_sc1(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  const ring_u4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                     __uint_as_float(u.w));
}

__device__ __forceinline__ void ring_combine_tail(int *__restrict__ arrive, int batch, int nb,
                                                  unsigned *flags, int wave, int g, int v,
                                                  const int *__restrict__ rows,
                                                  __amdgpu_buffer_rsrc_t prs, long long part_stride,
                                                  const float *__restrict__ row_scale,
                                                  float4 *__restrict__ out, int ld4_out,
                                                  const GsEpilogue &epi) {
  if (!arrive) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores drained
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(arrive + batch, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = old == nb - 1;
    if (last) __hip_atomic_store(arrive + batch, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flags[RING_LAST_FLAG] = last;
  }
  __syncthreads();
  if (!flags[RING_LAST_FLAG] || wave == LDS_CW) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // loads stay below the barrier
  const int *rw = rows + (((long long)batch * LDS_CW + wave) * LDS_SLOTS) * 16 + g;
  const unsigned bstride = (unsigned)part_stride * 64u;
  // 4 rowsets at a time, 4 blocks' partials of each in flight (16 loads), added in block order
  for (int j0 = 0; j0 < LDS_SLOTS; j0 += 4) {
    int rr[4];
    bool ok[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int u = rw[(j0 + q) * 16];
      const int sp = (int)((unsigned)u >> 28);
      rr[q] = u & kRingRowMask;
      ok[q] = rr[q] != kRingEmpty && (g & ((1 << sp) - 1)) == 0;
    }
    float4 acc[4];
    for (int b0 = 0; b0 < nb; b0 += 4) {
      float4 t[4][4];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++)
          t[q][bb] = ok[q] && b0 + bb < nb
                         ? ring_ld_sc1(prs, (unsigned)(b0 + bb) * bstride +
                                                ((unsigned)rr[q] * 4u + (unsigned)v) * 16u)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
          if (b0 + bb >= nb) continue;
          if (b0 + bb == 0) acc[q] = t[q][0];
          else f4_acc(acc[q], t[q][bb]);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (!ok[q]) continue;
      float4 a = acc[q];
      const float s = row_scale[rr[q]];
      a.x *= s;
      a.y *= s;
      a.z *= s;
      a.w *= s;
      gs_epilogue(a, rr[q], 4 * v, epi);
      out[(long long)rr[q] * ld4_out + v] = a;
    }
  }
}

template <int DIAG>
__global__ __launch_bounds__(LDS_THREADS) void k_graphsum_ring(
    const uint2 *__restrict__ entries, const long long *__restrict__ wave_off,
    const unsigned short *__restrict__ counts, int t_max, const int2 *__restrict__ slices,
    const int *__restrict__ n_slices, const int *__restrict__ rows, const char *__restrict__ table,
    float4 *__restrict__ partial, long long part_stride, int n_blocks,
    unsigned long long *__restrict__ stamps, int prio, int *__restrict__ arrive,
    const float *__restrict__ row_scale, float4 *__restrict__ out, int ld4_out, GsEpilogue epi) {
  __shared__ float4 lds[RING_TOTAL_B / 16];
  unsigned long long st_loop = 0, st_wait = 0, st_ring = 0;
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
  if (threadIdx.x < RING_LAST_FLAG) flags[threadIdx.x] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // zero rows and hand-off words set (the only barrier)
  asm volatile("" ::: "memory");

  if (wave == LDS_CW) {  // ------------------------------------------------ loader wave
    __builtin_amdgcn_s_setprio(3);
    const int2 *sl = slices + (long long)b * t_max;
    const char *cnt_src =
        reinterpret_cast<const char *>(counts) + (long long)blockIdx.x * t_max * RING_CNT_USED;
    const int iters = T + RING_W - 1;
    for (int s = 0; s < iters; s++) {
      // buffer s % K (and counts buffer (s - W + 1) & 1) free: visit s - K done everywhere
      if (s >= RING_K) {
        unsigned long long c0 = 0;
        if constexpr (DIAG == 4) c0 = ring_clk();
        lds_wait_ge(done + (s - RING_K) % RING_K, (unsigned)(LDS_CW * ((s - RING_K) / RING_K + 1)));
        if constexpr (DIAG == 4) st_wait += ring_clk() - c0;
      }
      if (s < T) {
        const char *src = table + (long long)sl[s].x * 64 + lane * 16;
        const unsigned dst = lds_base + (unsigned)((s % RING_K) * RING_SR * 16);
        if constexpr (DIAG == 2) {  // timing only: 1/8 of the slice
          glds16x4(src, dst);
        } else {
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
      }
      const int cv = s - (RING_W - 1);  // the visit whose last slice this is
      if (cv >= 0 && lane * 16 < RING_CNT_USED)
        glds16(cnt_src + (long long)cv * RING_CNT_USED + lane * 16,
               lds_base + (unsigned)(RING_CNT_OFF + (cv % RING_NCB) * RING_CNT_B));
      unsigned long long c1 = 0;
      if constexpr (DIAG == 4) c1 = ring_clk();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slice s and counts landed
      if constexpr (DIAG == 4) st_ring += ring_clk() - c1;
      if (lane == 0) __atomic_store_n(loaded, (unsigned)(s + 1), __ATOMIC_RELAXED);
      asm volatile("" ::: "memory");
    }
    if constexpr (DIAG == 4) {
      if (lane == 0) {
        unsigned long long *o = stamps + ((long long)blockIdx.x * 16 + wave) * 8;
        o[1] = st_wait;
        o[2] = st_ring;
        o[4] = T;
      }
    }
    ring_combine_tail(arrive, batch, nb, flags, wave, g, v, rows,
                      ring_part_rsrc(partial, (long long)nb * part_stride * 64), part_stride,
                      row_scale, out, ld4_out, epi);
    return;
  }

  // ------------------------------------------------------------------------- summing waves
  const long long wid = (long long)blockIdx.x * LDS_CW + wave;
  const long long kb0 = wave_off[wid];
  // the wave's entry stream, 512-B chunks (4 entry blocks) into a 4-slot LDS ring; refills
  // run up to 3 chunks past the stream's end (the entries array has 2 KB of slack)
  const char *esrc = reinterpret_cast<const char *>(entries) + kb0 * 128 + lane * 16;
  const unsigned ring_dst = lds_base + (unsigned)(RING_ERING_OFF + wave * RING_ERING_B);
  const char *ring = lb + RING_ERING_OFF + wave * RING_ERING_B + g * 8;
  auto refill = [&](int c) {  // chunk c -> ring slot c % 4
    if (DIAG != 5 && DIAG != 6 && lane < 32)  // DIAG 5/6: no entry stream (timing only)
      glds16(esrc, ring_dst + (unsigned)((c & (RING_ESLOTS - 1)) * RING_CHUNK));
    esrc += RING_CHUNK;
  };
  refill(0);
  refill(1);
  refill(2);
  refill(3);
  asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // chunk 0

  float4 acc[LDS_SLOTS];
#pragma unroll
  for (int j = 0; j < LDS_SLOTS; j++) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  int chunk = 0;
  int roff = 0;
  static_assert((RING_ERING_B & (RING_ERING_B - 1)) == 0, "ring wraps by masking");
  uint2 e_next = *reinterpret_cast<const uint2 *>(ring);
  // next entry block (its refill when a chunk is entered).  The slot refilled holds the chunk
  // before this one: the read of its last entry block (the caller's current entry, which
  // hipcc waits for only where it is first used) must have returned before the DMA lands.
  auto next_block = [&]() {
    roff = (roff + 128) & (RING_ERING_B - 1);
    if ((roff & (RING_CHUNK - 1)) == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ++chunk;
      refill(chunk + 3);
      unsigned long long c0 = 0;
      if constexpr (DIAG == 4) c0 = ring_clk();
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      if constexpr (DIAG == 4) st_ring += ring_clk() - c0;
    }
    e_next = *reinterpret_cast<const uint2 *>(ring + roff);
  };
  if constexpr (DIAG == 4) st_loop = ring_clk();
  long long nblk = 0;
  // lane (g, v) reads plane v: entry (ring row x 16 B) + this constant
  const char *tb = lb + v * RING_PLANE_B;
  auto rd = [&](unsigned off) { return *reinterpret_cast<const float4 *>(tb + off); };
  for (int t = 0; t < T; t++) {
    unsigned long long hw0 = 0;
    if constexpr (DIAG == 4) hw0 = ring_clk();
    lds_wait_ge(loaded, (unsigned)(t + RING_W));  // slices t .. t+2 and visit t's counts
    if constexpr (DIAG == 4) st_wait += ring_clk() - hw0;
    const uint4 *c4 = reinterpret_cast<const uint4 *>(lb + RING_CNT_OFF + (t % RING_NCB) * RING_CNT_B +
                                                      wave * 32);
    const uint4 cw0 = c4[0], cw1 = c4[1];
    const unsigned cw[8] = {
        (unsigned)__builtin_amdgcn_readfirstlane(cw0.x), (unsigned)__builtin_amdgcn_readfirstlane(cw0.y),
        (unsigned)__builtin_amdgcn_readfirstlane(cw0.z), (unsigned)__builtin_amdgcn_readfirstlane(cw0.w),
        (unsigned)__builtin_amdgcn_readfirstlane(cw1.x), (unsigned)__builtin_amdgcn_readfirstlane(cw1.y),
        (unsigned)__builtin_amdgcn_readfirstlane(cw1.z), (unsigned)__builtin_amdgcn_readfirstlane(cw1.w)};
#pragma unroll
    for (int j = 0; j < LDS_SLOTS; j++) {
      int n = (cw[j >> 1] >> (16 * (j & 1))) & 0xffff;  // steps of rowset j (x 4)
      if constexpr (DIAG == 7) n = 0;  // timing only: visits without blocks
      for (int k = 0; k < n; k += 4) {
        const uint2 e = e_next;
        next_block();
        // the next entry read goes out before this block's table reads: it returns first
        // (LDS reads complete in order), so the next block finds it landed
        asm volatile("" ::: "memory");
        if constexpr (DIAG == 4) nblk++;
        if constexpr (DIAG == 1 || DIAG == 6) {  // timing only: no table reads
          acc[j].x += __uint_as_float(e.x);
          acc[j].y += __uint_as_float(e.y);
        } else {
          const float4 x0 = rd(e.x & 0xffffu), x1 = rd(e.x >> 16), x2 = rd(e.y & 0xffffu),
                       x3 = rd(e.y >> 16);
          __builtin_amdgcn_s_waitcnt(0xC07F);  // one lgkmcnt(0) wait, then the adds
          f4_acc(acc[j], x0);
          f4_acc(acc[j], x1);
          f4_acc(acc[j], x2);
          f4_acc(acc[j], x3);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of slice t returned
    unsigned rank = 0;
    if (lane == 0)
      rank = __hip_atomic_fetch_add(done + t % RING_K, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    if (prio) {
      // The arbiter favours older waves, so the youngest waves of a workgroup fall behind
      // and the visits' hand-offs make everyone wait for them (r02 stamps: 395 vs 576 cycles
      // per block from the oldest to the youngest wave).  The last third of the waves to
      // finish a visit run the next one at raised priority, the first third at the lowest.
      rank = (unsigned)__builtin_amdgcn_readfirstlane((int)rank) - (unsigned)(LDS_CW * (t / RING_K));
      if (rank >= (unsigned)(2 * LDS_CW / 3)) __builtin_amdgcn_s_setprio(2);
      else if (rank >= (unsigned)(LDS_CW / 3)) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
  }
  if constexpr (DIAG == 4) {
    st_loop = ring_clk() - st_loop;
    if (lane == 0) {
      unsigned long long *o = stamps + ((long long)blockIdx.x * 16 + wave) * 8;
      o[0] = st_loop;
      o[1] = st_wait;
      o[2] = st_ring;
      o[3] = (unsigned long long)nblk;
      o[4] = T;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the dummy ring refills
  // rows[] = row | log2(m) << 28: a row spread over m lane groups (host/ring.cpp) has its m
  // partial sums added across lane groups g ^ 1, g ^ 2, .. (xor butterfly, fixed order for the
  // writing lane group g % m == 0); m is uniform per rowset
  const int *rw = rows + (((long long)batch * LDS_CW + wave) * LDS_SLOTS) * 16 + g;
  float4 *pb = partial + (long long)b * part_stride * 4 + v;
  const __amdgpu_buffer_rsrc_t prs = ring_part_rsrc(partial, (long long)n_blocks * part_stride * 64);
  const unsigned pb_off = ((unsigned)b * (unsigned)part_stride * 4u + (unsigned)v) * 16u;
#pragma unroll
  for (int j = 0; j < LDS_SLOTS; j++) {
    const int u = rw[j * 16];
    const int sp = __builtin_amdgcn_readfirstlane((int)((unsigned)u >> 28));
    float4 a = acc[j];
    for (int k = 0; k < sp; k++) {
      const int d = 4 << k;
      a.x += __shfl_xor(a.x, d);
      a.y += __shfl_xor(a.y, d);
      a.z += __shfl_xor(a.z, d);
      a.w += __shfl_xor(a.w, d);
    }
    const int r = u & kRingRowMask;
    if (r != kRingEmpty && (g & ((1 << sp) - 1)) == 0) {
      if (arrive) ring_st_sc1(prs, pb_off + (unsigned)r * 64u, a);  // read by another XCD
      else pb[(long long)r * 4] = a;
    }
  }
  ring_combine_tail(arrive, batch, nb, flags, wave, g, v, rows, prs, part_stride, row_scale,
                    out, ld4_out, epi);
}

// "graphsum_ring_prio": 1 = waves that finished a visit last run the next one at raised
// issue priority (see the summing loop), 0 = fixed priority
int g_graphsum_ring_prio = 1;
// "graphsum_ring_fused": 1 = the batch's last workgroup combines the block partials (no
// k_gs_lds_combine launch), 0 = separate combine kernel.  Off: correct (bit-identical, tested)
// but slower on reddit-114M, 0.263 vs 0.230 ms per call (r02): the combine of all 61 batches
// then runs at the kernel's end on 61 CUs instead of over the whole chip
int g_graphsum_ring_fused = 0;

void launch_graphsum_ring(const LdsSchedule &s, const float *in, int ld_in, float *out,
                          int ld_out, float *scratch_in, float *partial, hipStream_t st,
                          const int *col_map, const GsEpilogue *epi, bool prestaged,
                          bool combine) {
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0, PGCN_E_INVALID, "graphsum_ring: ld % 4");
  PGCN_CHECK(s.window == kRingWindow, PGCN_E_INVALID, "graphsum_ring: not a ring schedule");
  const long long pre = (long long)s.n_cols * 4;
  if (!prestaged)
    hipLaunchKernelGGL(k_ring_prescale, dim3((unsigned)ceil_div(pre, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float4 *>(in), ld_in / 4, s.col_scale, s.n_cols,
                       reinterpret_cast<float4 *>(scratch_in), col_map);
  const long long n_wg = (long long)s.n_batches * s.n_blocks;
  const GsEpilogue none{};
  // (an epilogue that stages the next GraphSum's input may write this call's own table: that
  // needs the separate combine, after every workgroup has read it)
  int *arrive = g_graphsum_ring_fused && s.arrive && combine && !(epi && epi->next_table)
                   ? s.arrive : nullptr;
#define GS_RING(D)                                                                            \
  hipLaunchKernelGGL((k_graphsum_ring<D>), dim3((unsigned)n_wg), dim3(LDS_THREADS), 0, st,   \
                     s.entries, s.wave_off, s.counts, s.t_max, s.slices, s.n_slices, s.rows,      \
                     reinterpret_cast<const char *>(scratch_in),                                 \
                     reinterpret_cast<float4 *>(partial), (long long)s.n_rows, s.n_blocks,         \
                     D == 4 ? lds_stamps(n_wg) : nullptr, g_graphsum_ring_prio, arrive,          \
                     s.row_scale, reinterpret_cast<float4 *>(out), ld_out / 4, epi ? *epi : none)
  switch (g_graphsum_lds_diag) {
    case 1: GS_RING(1); break;
    case 2: GS_RING(2); break;
    case 4: GS_RING(4); break;
    case 5: GS_RING(5); break;  // no entry stream (zero entries: every step reads row 0)
    case 6: GS_RING(6); break;  // no entry stream, no table reads
    case 7: GS_RING(7); break;  // visits and hand-offs only
    default: GS_RING(0); break;
  }
#undef GS_RING
  if (!arrive && combine) launch_gs_lds_combine(s, partial, out, ld_out, st, epi);
  PGCN_HIP(hipGetLastError());
}

}  // namespace pgcn
