// parallel-gcn_amd/csrc/k_graphsum_lds.hip -- GraphSum for 16-wide rows with the gathered
// feature table staged in LDS (the reddit hot path).
//
// Replaces graphsum_kernel (src/module.cu:172-210) / hpdga GraphSum::forward/backward
// (module.cpp:82-111) for d = 16 on graphs whose feature table exceeds an XCD's L2.
//
// Why: a random 64-B row gathered through the vector-memory pipeline costs ~2.3 CU-cycles per
// row (tools/ta_micro.hip), which puts a TA-gather kernel at >= 0.43 ms per reddit call.  An
// LDS ds_read_b128 moves 1 KB in 4-8 cycles.  So every neighbour row is read from LDS, and
// the vector-memory pipeline only carries contiguous slice copies and a 2-byte-per-slot edge
// stream.
//
// Algebra: Â = D^-1/2 A D^-1/2 (hpdga coefficient 1/sqrtf(d_i d_j), module.cpp:88-90), so
//   out_i = s_i * sum_{j in N(i)} (s_j * in_j),  s = 1/sqrt(deg)
// -- no per-edge coefficient: k_gs_prescale forms in' = s ⊙ in once per call, the edge
// stream holds only 16-bit slice-local row offsets, k_gs_lds_combine applies s_i.  Exact in
// real arithmetic; the fp32 rounding differs from the reference's per-edge product by ~1 ulp
// per term (covered by the 1e-4 parity tolerance, like the summation order).
//
// Schedule (host, DevGraph::build_lds):
//  * columns are cut into kBlocks = 8 nnz-balanced blocks (one per XCD: workgroup w serves
//    block w % 8, so a block's slices are re-read from that XCD's L2) and each block into
//    slices of LDS_SR = 1024 rows (64 KB);
//  * rows are sorted by degree and grouped into rowsets of 16 (similar degree => the 16 rows
//    of a rowset have similar per-slice edge counts); rowsets are dealt round-robin to
//    batches; a workgroup (batch, block) owns up to LDS_CW x LDS_SLOTS rowsets;
//  * wave w of a workgroup holds the accumulators of its LDS_SLOTS rowsets in registers
//    (lane 4g+v: row g of the rowset, float4 v of the row) for the whole sweep over the
//    block's slices; per (rowset, slice) the wave runs max_g(count_g) steps, reading its
//    entries as [step/4][g][step%4] uint16 (one 8-byte load per lane per 4 steps, 128 B per
//    wave); missing entries point at a zero row.
//  * one loader wave per workgroup copies slice t+1 into the other LDS buffer with
//    global_load_lds (no VGPRs) while the LDS_CW compute waves sum slice t.
// Each workgroup writes its rows' partial sums for its column block; k_gs_lds_combine adds
// the 8 partials of a row in block order and scales by s_i => deterministic.
#include "common.hpp"
#include "kernels.hpp"
#include "lds_dma.hpp"

namespace pgcn {

typedef __attribute__((address_space(3))) void lds_void;

// in'[r, 0:16] = scale[r] * in[r, 0:16]   (rows of 4 float4; ld4 = row stride in float4)
// (col_map: the table's rows are rows col_map[r] of `in` -- a column-subset graph)
__global__ __launch_bounds__(256) void k_gs_prescale(const float4 *__restrict__ in, int ld4_in,
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
  out[r * 4 + v] = x;
}

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// Window-2 step: lanes in `m` (slot J+1) add x into acc1, the others (slot J, or a padding
// zero row) into acc0.  Exec is set by hand around four packed adds (the summing waves run
// with all 64 lanes active, so exec is restored to all ones).
__device__ __forceinline__ void win_add(f2v &a0l, f2v &a0h, f2v &a1l, f2v &a1h, const f4v &x,
                                        uint64_t m) {
  const f2v xl = __builtin_shufflevector(x, x, 0, 1), xh = __builtin_shufflevector(x, x, 2, 3);
  asm volatile(
      "s_mov_b64 exec, %[m]\n\t"
      "v_pk_add_f32 %[a1l], %[a1l], %[xl]\n\t"
      "v_pk_add_f32 %[a1h], %[a1h], %[xh]\n\t"
      "s_not_b64 exec, %[m]\n\t"
      "v_pk_add_f32 %[a0l], %[a0l], %[xl]\n\t"
      "v_pk_add_f32 %[a0h], %[a0h], %[xh]\n\t"
      "s_mov_b64 exec, -1"
      : [a0l] "+v"(a0l), [a0h] "+v"(a0h), [a1l] "+v"(a1l), [a1h] "+v"(a1h)
      : [m] "s"(m), [xl] "v"(xl), [xh] "v"(xh)
      : "scc");  // s_not_b64 writes SCC (the loop branches on it)
}

// The 4 step masks of one entry block (32 B at p, uniform) into SGPRs.  A scalar load issued
// from inline asm (the kernel's asm memory clobbers would otherwise turn a plain uniform load
// into a vector load that upsets the hand-counted vmcnt of the entry ring); it waits for
// itself (lgkmcnt(0): call it when no LDS read is outstanding) and touches the line two
// blocks ahead, so the next loads hit the scalar cache.
typedef unsigned u32x8 __attribute__((ext_vector_type(8)));
template <bool g_touch>
__device__ __forceinline__ void load_masks(const uint64_t *p, uint64_t (&m)[4]) {
  u32x8 v;
  unsigned touch;
  if (g_touch)
    asm volatile(
        "s_load_dwordx8 %0, %2, 0x0\n\t"
        "s_load_dword %1, %2, 0x40\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(v), "=&s"(touch)
        : "s"(p)
        : "memory");
  else
    asm volatile(
        "s_load_dwordx8 %0, %1, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(v)
        : "s"(p)
        : "memory");
  (void)touch;
#pragma unroll
  for (int s = 0; s < 4; s++) m[s] = (uint64_t)v[2 * s] | ((uint64_t)v[2 * s + 1] << 32);
}

constexpr int LDS_TABLE_F4 = 2 * LDS_ROWS * 4;       // two slice buffers (float4 units)
constexpr int LDS_RING_CHUNK = 512;                  // bytes: 4 entry blocks of 128 B
constexpr int LDS_RING_SLOTS = 4;                    // chunks per wave: 3 in flight + 1 read
constexpr int LDS_RING_BYTES = LDS_RING_SLOTS * LDS_RING_CHUNK;
constexpr int LDS_CNT_BYTES = 512;                   // one slice's step counts (480 B used)
static_assert(LDS_CW * LDS_SLOTS * 2 <= LDS_CNT_BYTES, "counts area");
constexpr int LDS_RING_F4 = LDS_TABLE_F4 + 2 * LDS_CNT_BYTES / 16;  // after 2 counts areas
constexpr int LDS_TOTAL_F4 = LDS_RING_F4 + LDS_CW * LDS_RING_BYTES / 16;

// Wave roles: waves 0 .. LDS_CW-1 sum (each owns LDS_SLOTS rowsets and an entry ring); wave
// LDS_CW copies slice t+1 into the other buffer while slice t is summed.  The copies and the
// ring refills are LDS-DMA issued from inline asm, invisible to hipcc's waitcnt bookkeeping;
// each wave counts its own: a summing wave only ever has ring refills outstanding (constant
// vmcnt(3) = "the chunk refilled three chunks ago has landed"), the loader waits vmcnt(0) once
// per slice.  Slices are handed over through LDS words (lds_wait_ge), not barriers.
// DIAG 4: per-wave cycle stamps (s_memtime) -> stamps[wg][wave][8]:
//   0 loop cycles, 1 hand-off wait cycles, 2 ring-wait cycles, 3 entry blocks, 4 slices
__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

// Slice hand-off words in LDS (the spare tail of counts area 0): loaded[b] = t + 1 once slice t
// sits in buffer b; done[b] counts summing-wave completions of the slices held in buffer b.
// Replaces a workgroup barrier per slice, so summing waves may drift up to one slice apart
// (per-slice imbalance between waves no longer stalls everyone; r01 stamps: 18 % of the loop).
constexpr int LDS_FLAG_BYTE = LDS_CW * LDS_SLOTS * 2;  // 480: first byte past the counts
static_assert(LDS_FLAG_BYTE + 16 <= 512, "flag words fit the counts area tail");
template <int DIAG, int WIN, int SYNC>
__global__ __launch_bounds__(LDS_THREADS) void k_graphsum_lds(
    const uint2 *__restrict__ entries, const uint64_t *__restrict__ masks,
    const long long *__restrict__ wave_off,
    const unsigned short *__restrict__ counts, int t_max, const int2 *__restrict__ slices,
    const int *__restrict__ n_slices, const int *__restrict__ rows, const float4 *__restrict__ in,
    int n_cols, float4 *__restrict__ partial, long long part_stride,
    unsigned long long *__restrict__ stamps, int opt, int n_blocks) {
  unsigned long long st_loop = 0, st_bar = 0, st_ring = 0;
  // ONE __shared__ object: [2][LDS_ROWS][4] float4 slice buffers, then the entry rings
  __shared__ float4 lds[LDS_TOTAL_F4];
  const int nb = n_blocks;
  const int b = blockIdx.x % nb, batch = blockIdx.x / nb;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = lane >> 2, v = lane & 3;
  const int T = n_slices[b];
  const unsigned lds_base = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<size_t>((__attribute__((address_space(3))) float4 *)lds));
  // zero rows LDS_SR .. LDS_SR+3 of both buffers (padding entries point at them)
  if (threadIdx.x < 32) {
    const int buf = threadIdx.x >> 4, q = threadIdx.x & 15;
    lds[(buf * LDS_ROWS + LDS_SR) * 4 + q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  unsigned *const flags = reinterpret_cast<unsigned *>(
      reinterpret_cast<char *>(lds + LDS_TABLE_F4) + LDS_FLAG_BYTE);
  unsigned *const loaded = flags, *const done = flags + 2;
  if (threadIdx.x < 4) flags[threadIdx.x] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // zero rows and hand-off words set (the only barrier)
  asm volatile("" ::: "memory");

  if (wave == LDS_CW) {  // ------------------------------------------------ loader wave
    // the loader's few instructions go first on its SIMD (the summing waves there would
    // otherwise delay every piece it issues; r01 stamps: slices landed late 21 % of the loop)
    if (opt & 2) __builtin_amdgcn_s_setprio(3);
    const int2 *sl = slices + (long long)b * t_max;
    const int last = n_cols - 1;
    const char *cnt_src = reinterpret_cast<const char *>(counts) +
                          (long long)blockIdx.x * t_max * (LDS_CW * LDS_SLOTS * 2);
    int2 sc_next = T > 0 ? sl[0] : make_int2(0, 0);
    for (int t = 0; t < T; t++) {
      // slice t -> buffer t & 1 once every summing wave is done with slice t - 2, with the
      // summing waves' step counts for slice t
      if (SYNC == 1 && t >= 2) {
        unsigned long long cw0 = 0;
        if constexpr (DIAG == 4) cw0 = clk();
        lds_wait_ge(done + (t & 1), (unsigned)(LDS_CW * (t / 2)));
        if constexpr (DIAG == 4) st_bar += clk() - cw0;
      }
      const int2 sc = sc_next;
      if (t + 1 < T) sc_next = sl[t + 1];
      if (lane * 16 < LDS_CW * LDS_SLOTS * 2)
        glds16(cnt_src + (long long)t * (LDS_CW * LDS_SLOTS * 2) + lane * 16,
               lds_base + (unsigned)(LDS_TABLE_F4 * 16 + (t & 1) * LDS_CNT_BYTES));
      const unsigned dst = lds_base + (unsigned)((t & 1) * LDS_ROWS * 64);
      // The slice is LDS_SR consecutive 64-B rows of `in` (the prescaled table, allocated with
      // LDS_ROWS rows of slack past n_cols: rows past a slice's end are copied, never read),
      // so piece i (16 rows, 1 KB) sits 1 KB past piece i-1 in the table and in LDS.
      const char *src = reinterpret_cast<const char *>(in + (long long)sc.x * 4) + lane * 16;
      constexpr int full = LDS_SR / 16;
      if (opt & 1) {
        constexpr bool stage16 = DIAG == 1 || DIAG == 5 || DIAG >= 7;
        const int pieces4 = stage16 ? 1 : full / 4;  // DIAG 1/5/7: stage 1/16 (timing only)
#pragma unroll 4
        for (int i = 0; i < pieces4; i++) glds16x4(src + i * 4096, dst + (unsigned)(i * 4096));
        if (!stage16)
          for (int i = full / 4 * 4; i < full; i++) glds16(src + i * 1024, dst + (unsigned)(i * 1024));
      } else {
        const int pieces = DIAG == 1 ? 4 : full;
#pragma unroll 8
        for (int i = 0; i < pieces; i++) {
          int r = sc.x + 16 * i + g;
          r = r < last ? r : last;
          glds16(in + (long long)r * 4 + v, dst + (unsigned)(i * 1024));
        }
      }
      if (LDS_SR % 16 && g < LDS_SR % 16)  // last partial piece (keeps the zero rows)
        glds16(src + full * 1024, dst + (unsigned)(full * 1024));
      unsigned long long c0 = 0;
      if constexpr (DIAG == 4) c0 = clk();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slice t and its counts landed
      if constexpr (DIAG == 4) st_ring += clk() - c0;   // loader: staging wait
      if constexpr (SYNC == 1) {
        if (lane == 0) __atomic_store_n(loaded + (t & 1), (unsigned)(t + 1), __ATOMIC_RELAXED);
        asm volatile("" ::: "memory");
      } else {  // SYNC 0: one workgroup barrier per slice
        unsigned long long c1 = 0;
        if constexpr (DIAG == 4) c1 = clk();
        __builtin_amdgcn_s_barrier();  // slice t ready (t = 0) / slice t-1 summed
        asm volatile("" ::: "memory");
        if constexpr (DIAG == 4) st_bar += clk() - c1;
      }
    }
    if constexpr (SYNC == 0) __builtin_amdgcn_s_barrier();  // the summing waves' last slice
    if constexpr (DIAG == 4) {
      if (lane == 0) {
        unsigned long long *o = stamps + ((long long)blockIdx.x * 16 + wave) * 8;
        o[1] = st_bar;
        o[2] = st_ring;
        o[4] = T;
      }
    }
    return;
  }

  // ------------------------------------------------------------------------- summing waves
  const long long wid = (long long)blockIdx.x * LDS_CW + wave;
  const long long kb0 = wave_off[wid], kb1 = wave_off[wid + 1];
  // entry blocks: 128 B (4 steps), window 4: 256 B (8 steps); a ring chunk is 512 B
  constexpr int BLKB = WIN == 4 ? 256 : 128, BPC = LDS_RING_CHUNK / BLKB;
  const long long nchunk = (kb1 - kb0 + BPC - 1) / BPC;
  const char *ebytes = reinterpret_cast<const char *>(entries) + kb0 * BLKB;
  const unsigned ring_dst = lds_base + LDS_RING_F4 * 16 + (unsigned)(wave * LDS_RING_BYTES);
  const char *ring = reinterpret_cast<const char *>(lds + LDS_RING_F4) + wave * LDS_RING_BYTES +
                     g * (BLKB / 16);
  auto refill = [&](long long c) {  // chunk c -> ring slot c % 4 (clamped: dummy past the end)
    long long cc = c < nchunk ? c : nchunk - 1;
    cc = cc > 0 ? cc : 0;
    if (DIAG < 7 && lane < 32)  // DIAG 7-9: no entry stream (timing only)
      glds16(ebytes + cc * LDS_RING_CHUNK + lane * 16,
             ring_dst + (unsigned)((c % LDS_RING_SLOTS) * LDS_RING_CHUNK));
  };
  refill(0);
  refill(1);
  refill(2);
  if constexpr (WIN == 3) {  // window 3 keeps two chunks in flight (see ahead())
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // chunk 0
  } else {
    refill(3);
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // chunk 0
  }

  float4 acc[LDS_SLOTS];
#pragma unroll
  for (int j = 0; j < LDS_SLOTS; j++) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  int chunk = 0;  // ring chunk being read
  int roff = 0;   // byte offset of the current entry block in the ring (power-of-two ring)
  static_assert((LDS_RING_BYTES & (LDS_RING_BYTES - 1)) == 0, "ring wraps by masking");
  uint2 e_next = *reinterpret_cast<const uint2 *>(ring);

  if constexpr (DIAG == 4) st_loop = clk();
  // slice t staged (counts included) / this wave is done with slice t
  auto slice_ready = [&](int t) {
    unsigned long long cw0 = 0;
    if constexpr (DIAG == 4) cw0 = clk();
    if constexpr (SYNC == 1) {
      lds_wait_ge(loaded + (t & 1), (unsigned)(t + 1));
    } else if (t == 0) {
      __builtin_amdgcn_s_barrier();  // slice 0 staged
      asm volatile("" ::: "memory");
    }
    if constexpr (DIAG == 4) st_bar += clk() - cw0;
  };
  auto slice_done = [&](int t) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of slice t returned
    if constexpr (SYNC == 1) {
      if (lane == 0)
        __hip_atomic_fetch_add(done + (t & 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");
    } else {
      unsigned long long cb = 0;
      if constexpr (DIAG == 4) cb = clk();
      __builtin_amdgcn_s_barrier();  // slice t summed; slice t+1 staged
      asm volatile("" ::: "memory");
      if constexpr (DIAG == 4) st_bar += clk() - cb;
    }
  };
  // next entry block of the ring (and its refill when a chunk is entered)
  auto next_block = [&]() {
    roff = (roff + 128) & (LDS_RING_BYTES - 1);
    if ((roff & (LDS_RING_CHUNK - 1)) == 0) {  // entering the next chunk: refill the slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before, wait for it
      ++chunk;
      refill(chunk + 3);
      unsigned long long c0 = 0;
      if constexpr (DIAG == 4) c0 = clk();
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      if constexpr (DIAG == 4) st_ring += clk() - c0;
    }
    e_next = *reinterpret_cast<const uint2 *>(ring + roff);  // (past the end: unused)
  };
  if constexpr (WIN == 4) {
    // 8-step blocks (256 B: lane group g's 8 uint16 offsets at 16 g), exact step counts: a
    // run of n steps takes n / 8 full blocks and one block of n % 8 steps.  Half the blocks
    // (and the per-block loop / ring work) of window 1, and LDS reads only for real steps.
    uint4 e4 = *reinterpret_cast<const uint4 *>(ring);
    auto next4 = [&]() {
      roff = (roff + BLKB) & (LDS_RING_BYTES - 1);
      if ((roff & (LDS_RING_CHUNK - 1)) == 0) {  // entering the next chunk: refill the slot
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ++chunk;
        refill(chunk + 3);
        unsigned long long c0 = 0;
        if constexpr (DIAG == 4) c0 = clk();
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        if constexpr (DIAG == 4) st_ring += clk() - c0;
      }
      e4 = *reinterpret_cast<const uint4 *>(ring + roff);
    };
    for (int t = 0; t < T; t++) {
      slice_ready(t);
      const char *tb = reinterpret_cast<const char *>(lds + (t & 1) * LDS_ROWS * 4 + v);
      auto rd = [&](unsigned off) { return *reinterpret_cast<const float4 *>(tb + off); };
      const uint4 *c4 = reinterpret_cast<const uint4 *>(
          reinterpret_cast<const char *>(lds + LDS_TABLE_F4) + (t & 1) * LDS_CNT_BYTES + wave * 32);
      const uint4 cw0 = c4[0], cw1 = c4[1];
      const unsigned cw[8] = {
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.x), (unsigned)__builtin_amdgcn_readfirstlane(cw0.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.z), (unsigned)__builtin_amdgcn_readfirstlane(cw0.w),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.x), (unsigned)__builtin_amdgcn_readfirstlane(cw1.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.z), (unsigned)__builtin_amdgcn_readfirstlane(cw1.w)};
#pragma unroll
      for (int j = 0; j < LDS_SLOTS; j++) {
        int n = (cw[j >> 1] >> (16 * (j & 1))) & 0xffff;  // steps of rowset j
        for (; n >= 8; n -= 8) {
          const uint4 e = e4;
          next4();
          const float4 x0 = rd(e.x & 0xffffu), x1 = rd(e.x >> 16), x2 = rd(e.y & 0xffffu),
                       x3 = rd(e.y >> 16), x4 = rd(e.z & 0xffffu), x5 = rd(e.z >> 16),
                       x6 = rd(e.w & 0xffffu), x7 = rd(e.w >> 16);
          f4_acc(acc[j], x0);
          f4_acc(acc[j], x1);
          f4_acc(acc[j], x2);
          f4_acc(acc[j], x3);
          f4_acc(acc[j], x4);
          f4_acc(acc[j], x5);
          f4_acc(acc[j], x6);
          f4_acc(acc[j], x7);
        }
        if (n) {  // the last 1..7 steps (uniform branches)
          const uint4 e = e4;
          next4();
          unsigned w0 = e.x, w1 = e.y;
          if (n >= 4) {
            const float4 x0 = rd(w0 & 0xffffu), x1 = rd(w0 >> 16), x2 = rd(w1 & 0xffffu),
                         x3 = rd(w1 >> 16);
            f4_acc(acc[j], x0);
            f4_acc(acc[j], x1);
            f4_acc(acc[j], x2);
            f4_acc(acc[j], x3);
            w0 = e.z;
            w1 = e.w;
            n -= 4;
          }
          if (n >= 1) f4_acc(acc[j], rd(w0 & 0xffffu));
          if (n >= 2) f4_acc(acc[j], rd(w0 >> 16));
          if (n >= 3) f4_acc(acc[j], rd(w1 & 0xffffu));
        }
      }
      slice_done(t);
    }
  } else if constexpr (WIN == 3) {
    // Slot pairs (2p, 2p+1) interleaved block by block (host order: A0 B0 A1 B1 ..., then the
    // longer slot's rest), so every iteration has 8 ds_read_b128 (two blocks) in flight where
    // window 1 had 4: a slot runs ~1.4 blocks per slice on reddit, so pipelining inside one
    // slot would not find a second block.  Two entry blocks are read ahead (q0, q1); the
    // lookahead pointer drives the ring: entering chunk c refills chunk c + 2 into the slot of
    // chunk c - 2, whose reads were all consumed (waited for) two blocks ago -- no drain.
    uint2 q0 = e_next, q1;
    auto ahead = [&]() -> uint2 {
      roff = (roff + 128) & (LDS_RING_BYTES - 1);
      if ((roff & (LDS_RING_CHUNK - 1)) == 0) {
        ++chunk;
        refill(chunk + 2);
        unsigned long long c0 = 0;
        if constexpr (DIAG == 4) c0 = clk();
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        if constexpr (DIAG == 4) st_ring += clk() - c0;
      }
      return *reinterpret_cast<const uint2 *>(ring + roff);
    };
    q1 = ahead();
    for (int t = 0; t < T; t++) {
      slice_ready(t);
      const char *tb = reinterpret_cast<const char *>(lds + (t & 1) * LDS_ROWS * 4 + v);
      auto rd = [&](unsigned off) { return *reinterpret_cast<const float4 *>(tb + off); };
      const uint4 *c4 = reinterpret_cast<const uint4 *>(
          reinterpret_cast<const char *>(lds + LDS_TABLE_F4) + (t & 1) * LDS_CNT_BYTES + wave * 32);
      const uint4 cw0 = c4[0], cw1 = c4[1];
      const unsigned cw[8] = {
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.x), (unsigned)__builtin_amdgcn_readfirstlane(cw0.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.z), (unsigned)__builtin_amdgcn_readfirstlane(cw0.w),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.x), (unsigned)__builtin_amdgcn_readfirstlane(cw1.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.z), (unsigned)__builtin_amdgcn_readfirstlane(cw1.w)};
      // the longer slot's rest: two blocks per iteration, then one
      auto rest = [&](float4 &a, int r) {
        for (; r >= 2; r -= 2) {
          const uint2 e0 = q0, e1 = q1;
          const float4 x0 = rd(e0.x & 0xffffu), x1 = rd(e0.x >> 16), x2 = rd(e0.y & 0xffffu),
                       x3 = rd(e0.y >> 16), x4 = rd(e1.x & 0xffffu), x5 = rd(e1.x >> 16),
                       x6 = rd(e1.y & 0xffffu), x7 = rd(e1.y >> 16);
          q0 = ahead();
          q1 = ahead();
          f4_acc(a, x0);
          f4_acc(a, x1);
          f4_acc(a, x2);
          f4_acc(a, x3);
          f4_acc(a, x4);
          f4_acc(a, x5);
          f4_acc(a, x6);
          f4_acc(a, x7);
        }
        if (r) {
          const uint2 e0 = q0;
          const float4 x0 = rd(e0.x & 0xffffu), x1 = rd(e0.x >> 16), x2 = rd(e0.y & 0xffffu),
                       x3 = rd(e0.y >> 16);
          q0 = q1;
          q1 = ahead();
          f4_acc(a, x0);
          f4_acc(a, x1);
          f4_acc(a, x2);
          f4_acc(a, x3);
        }
      };
#pragma unroll
      for (int p = 0; p < LDS_SLOTS / 2; p++) {
        const int na = ((cw[p] & 0xffffu) + 3) >> 2, nb2 = ((cw[p] >> 16) + 3) >> 2;
        const int both = na < nb2 ? na : nb2;
        for (int i = 0; i < both; i++) {
          const uint2 e0 = q0, e1 = q1;
          const float4 x0 = rd(e0.x & 0xffffu), x1 = rd(e0.x >> 16), x2 = rd(e0.y & 0xffffu),
                       x3 = rd(e0.y >> 16), x4 = rd(e1.x & 0xffffu), x5 = rd(e1.x >> 16),
                       x6 = rd(e1.y & 0xffffu), x7 = rd(e1.y >> 16);
          q0 = ahead();
          q1 = ahead();
          f4_acc(acc[2 * p], x0);
          f4_acc(acc[2 * p], x1);
          f4_acc(acc[2 * p], x2);
          f4_acc(acc[2 * p], x3);
          f4_acc(acc[2 * p + 1], x4);
          f4_acc(acc[2 * p + 1], x5);
          f4_acc(acc[2 * p + 1], x6);
          f4_acc(acc[2 * p + 1], x7);
        }
        if (na > nb2) rest(acc[2 * p], na - nb2);
        else if (nb2 > na) rest(acc[2 * p + 1], nb2 - na);
      }
      slice_done(t);
    }
  } else if constexpr (WIN == 2) {
    // accumulators as packed halves (v_pk_add_f32 operands)
    f2v al[LDS_SLOTS], ah[LDS_SLOTS];
#pragma unroll
    for (int j = 0; j < LDS_SLOTS; j++) al[j] = ah[j] = f2v{0.f, 0.f};
    // this wave's per-step lane masks (uniform: scalar loads)
    const uint64_t *mk = masks + kb0 * 4;
    for (int t = 0; t < T; t++) {
      slice_ready(t);
      const char *tb = reinterpret_cast<const char *>(lds + (t & 1) * LDS_ROWS * 4 + v);
      const uint4 *c4 = reinterpret_cast<const uint4 *>(
          reinterpret_cast<const char *>(lds + LDS_TABLE_F4) + (t & 1) * LDS_CNT_BYTES + wave * 32);
      const uint4 cw0 = c4[0], cw1 = c4[1];
      const unsigned cw[8] = {
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.x), (unsigned)__builtin_amdgcn_readfirstlane(cw0.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw0.z), (unsigned)__builtin_amdgcn_readfirstlane(cw0.w),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.x), (unsigned)__builtin_amdgcn_readfirstlane(cw1.y),
          (unsigned)__builtin_amdgcn_readfirstlane(cw1.z), (unsigned)__builtin_amdgcn_readfirstlane(cw1.w)};
#pragma unroll
      for (int j = 0; j < LDS_SLOTS; j++) {
        const int n = (cw[j >> 1] >> (16 * (j & 1))) & 0xffff;  // entry blocks of run j
        for (int k = 0; k < n; k++) {
          const uint2 e = e_next;
          uint64_t m[4];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (e_next has landed anyway)
          load_masks<DIAG != 6>(mk, m);
          mk += 4;
          next_block();
          const f4v x0 = *reinterpret_cast<const f4v *>(tb + (e.x & 0xffffu));
          const f4v x1 = *reinterpret_cast<const f4v *>(tb + (e.x >> 16));
          const f4v x2 = *reinterpret_cast<const f4v *>(tb + (e.y & 0xffffu));
          const f4v x3 = *reinterpret_cast<const f4v *>(tb + (e.y >> 16));
          if (j + 1 < LDS_SLOTS) {
            win_add(al[j], ah[j], al[j + 1], ah[j + 1], x0, m[0]);
            win_add(al[j], ah[j], al[j + 1], ah[j + 1], x1, m[1]);
            win_add(al[j], ah[j], al[j + 1], ah[j + 1], x2, m[2]);
            win_add(al[j], ah[j], al[j + 1], ah[j + 1], x3, m[3]);
          } else {  // the last slot has no successor: all lanes add into it
            al[j] += __builtin_shufflevector(x0, x0, 0, 1) + __builtin_shufflevector(x1, x1, 0, 1) +
                     __builtin_shufflevector(x2, x2, 0, 1) + __builtin_shufflevector(x3, x3, 0, 1);
            ah[j] += __builtin_shufflevector(x0, x0, 2, 3) + __builtin_shufflevector(x1, x1, 2, 3) +
                     __builtin_shufflevector(x2, x2, 2, 3) + __builtin_shufflevector(x3, x3, 2, 3);
          }
        }
      }
      slice_done(t);
    }
#pragma unroll
    for (int j = 0; j < LDS_SLOTS; j++) acc[j] = make_float4(al[j].x, al[j].y, ah[j].x, ah[j].y);
  } else {
  for (int t = 0; t < T; t++) {
    slice_ready(t);
    // edge entries are byte offsets of slice rows: address = entry + (buffer base + 16 v)
    const char *tb = reinterpret_cast<const char *>(lds + (t & 1) * LDS_ROWS * 4 + v);
    // this wave's 16 step counts for slice t, staged by the loader (uniform: broadcast read)
    const uint4 *c4 = reinterpret_cast<const uint4 *>(
        reinterpret_cast<const char *>(lds + LDS_TABLE_F4) + (t & 1) * LDS_CNT_BYTES + wave * 32);
    const uint4 cw0 = c4[0], cw1 = c4[1];
    const unsigned cw[8] = {
        (unsigned)__builtin_amdgcn_readfirstlane(cw0.x), (unsigned)__builtin_amdgcn_readfirstlane(cw0.y),
        (unsigned)__builtin_amdgcn_readfirstlane(cw0.z), (unsigned)__builtin_amdgcn_readfirstlane(cw0.w),
        (unsigned)__builtin_amdgcn_readfirstlane(cw1.x), (unsigned)__builtin_amdgcn_readfirstlane(cw1.y),
        (unsigned)__builtin_amdgcn_readfirstlane(cw1.z), (unsigned)__builtin_amdgcn_readfirstlane(cw1.w)};
    if constexpr (DIAG == 9) {  // timing only: the slice's blocks as ONE loop (no slot visits)
      int nb = 0;
#pragma unroll
      for (int j = 0; j < LDS_SLOTS; j++) nb += (((cw[j >> 1] >> (16 * (j & 1))) & 0xffff) + 3) >> 2;
      for (int k = 0; k < nb; k++) {
        const uint2 e = e_next;
        next_block();
        acc[0].x += __uint_as_float(e.x);
        acc[0].y += __uint_as_float(e.y);
      }
      slice_done(t);
      continue;
    }
#pragma unroll
    for (int j = 0; j < LDS_SLOTS; j++) {
      int n = (cw[j >> 1] >> (16 * (j & 1))) & 0xffff;  // steps of rowset j
      if constexpr (DIAG == 8) n = n < 4 ? n : 4;  // timing only: one block per visit
      for (int k = 0; k < n; k += 4) {
        const uint2 e = e_next;
        next_block();
        // all 4 entries are valid: steps past a row's run point at a zero row
        if constexpr (DIAG == 2 || DIAG == 5 || DIAG == 7 || DIAG == 8) {  // no table reads
          acc[j].x += __uint_as_float(e.x);
          acc[j].y += __uint_as_float(e.y);
        } else {
          const float4 x0 = *reinterpret_cast<const float4 *>(tb + (e.x & 0xffffu));
          const float4 x1 = *reinterpret_cast<const float4 *>(tb + (e.x >> 16));
          const float4 x2 = *reinterpret_cast<const float4 *>(tb + (e.y & 0xffffu));
          const float4 x3 = *reinterpret_cast<const float4 *>(tb + (e.y >> 16));
          if constexpr (DIAG == 3) {  // diagnostic: one add per read
            acc[j].x += x0.x;
            acc[j].y += x1.y;
            acc[j].z += x2.z;
            acc[j].w += x3.w;
          } else if constexpr (DIAG == 10) {  // timing only: every row read twice (LDS load x2)
            const float4 y0 = *reinterpret_cast<const float4 *>(tb + (e.x & 0xffffu) + 16384);
            const float4 y1 = *reinterpret_cast<const float4 *>(tb + (e.x >> 16) + 16384);
            const float4 y2 = *reinterpret_cast<const float4 *>(tb + (e.y & 0xffffu) + 16384);
            const float4 y3 = *reinterpret_cast<const float4 *>(tb + (e.y >> 16) + 16384);
            f4_acc(acc[j], x0);
            f4_acc(acc[j], x1);
            f4_acc(acc[j], x2);
            f4_acc(acc[j], x3);
            f4_acc(acc[j], y0);
            f4_acc(acc[j], y1);
            f4_acc(acc[j], y2);
            f4_acc(acc[j], y3);
          } else if constexpr (DIAG == 11) {  // timing only: twice the adds (VALU load x2)
            float4 z = x0;
            f4_acc(z, x1);
            f4_acc(z, x2);
            f4_acc(z, x3);
            f4_acc(acc[j], x0);
            f4_acc(acc[j], x1);
            f4_acc(acc[j], x2);
            f4_acc(acc[j], x3);
            f4_acc(acc[(j + 1) % LDS_SLOTS], z);
            asm volatile("" ::"v"(z.x), "v"(z.y), "v"(z.z), "v"(z.w));
          } else {
            f4_acc(acc[j], x0);
            f4_acc(acc[j], x1);
            f4_acc(acc[j], x2);
            f4_acc(acc[j], x3);
          }
        }
      }
    }
    slice_done(t);
  }
  }
  if constexpr (DIAG == 4) {
    st_loop = clk() - st_loop;
    if (lane == 0) {
      unsigned long long *o = stamps + ((long long)blockIdx.x * 16 + wave) * 8;
      o[0] = st_loop;
      o[1] = st_bar;
      o[2] = st_ring;
      o[3] = (unsigned long long)chunk * 4 + (roff & (LDS_RING_CHUNK - 1)) / 128;
      o[4] = T;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the dummy ring refills
  const int *rw = rows + (((long long)batch * LDS_CW + wave) * LDS_SLOTS) * 16 + g;
  float4 *pb = partial + (long long)b * part_stride * 4 + v;
#pragma unroll
  for (int j = 0; j < LDS_SLOTS; j++) {
    const int r = rw[j * 16];
    if (r >= 0) pb[(long long)r * 4] = acc[j];
  }
}

// out[r] = scale[r] * sum_{b < nb} partial[b][r]   (block order => deterministic)
__global__ __launch_bounds__(256) void k_gs_lds_combine(const float4 *__restrict__ partial,
                                                        long long part_stride, int nb,
                                                        const float *__restrict__ scale, int n,
                                                        float4 *__restrict__ out, int ld4_out,
                                                        GsEpilogue epi) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t >> 2;
  if (r >= n) return;
  const int v = (int)(t & 3);
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
  const float s = scale[r];
  a.x *= s;
  a.y *= s;
  a.z *= s;
  a.w *= s;
  gs_epilogue(a, r, 4 * v, epi);
  out[r * ld4_out + v] = a;
}

int g_graphsum_lds_diag = 0;  // diagnostics only ("graphsum_lds_diag")
int g_graphsum_lds_sync = 1;  // diagnostics ("graphsum_lds_sync"): 0 = a barrier per slice
// "graphsum_lds_opt": bit 0 = slice copies as 4-piece runs from one address VGPR (needs the
// table's row slack), bit 1 = loader wave at raised issue priority
int g_graphsum_lds_opt = 3;

// DIAG 4 stamp buffer (diagnostics; read back with pgcn_debug_read("graphsum_lds_stamps"))
static unsigned long long *g_stamps = nullptr;
static long long g_stamps_n = 0;
unsigned long long *lds_stamps(long long n_wg) {
  if (g_graphsum_lds_diag != 4) return nullptr;
  const long long n = n_wg * 16 * 8;
  if (n > g_stamps_n) {
    if (g_stamps) PGCN_HIP(hipFree(g_stamps));
    PGCN_HIP(hipMalloc(&g_stamps, n * sizeof(unsigned long long)));
    g_stamps_n = n;
  }
  PGCN_HIP(hipMemset(g_stamps, 0, n * sizeof(unsigned long long)));
  return g_stamps;
}
long long lds_stamps_read(void *dst, long long max_elems) {
  const long long n = g_stamps_n < max_elems ? g_stamps_n : max_elems;
  if (dst && n > 0) PGCN_HIP(hipMemcpy(dst, g_stamps, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return g_stamps_n;
}

void launch_graphsum_lds(const LdsSchedule &s, const float *in, int ld_in, float *out,
                         int ld_out, float *scratch_in, float *partial, hipStream_t st,
                         const int *col_map, const GsEpilogue *epi) {
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0, PGCN_E_INVALID, "graphsum_lds: ld % 4");
  const long long pre = (long long)s.n_cols * 4;
  hipLaunchKernelGGL(k_gs_prescale, dim3((unsigned)ceil_div(pre, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(in), ld_in / 4, s.col_scale, s.n_cols,
                     reinterpret_cast<float4 *>(scratch_in), col_map);
#define GS_LDS(D, W, Y)                                                                     \
  hipLaunchKernelGGL((k_graphsum_lds<D, W, Y>), dim3((unsigned)(s.n_batches * s.n_blocks)),    \
                     dim3(LDS_THREADS), 0, st, s.entries, s.masks, s.wave_off, s.counts,        \
                     s.t_max, s.slices, s.n_slices, s.rows,                                    \
                     reinterpret_cast<const float4 *>(scratch_in), s.n_cols,                   \
                     reinterpret_cast<float4 *>(partial), (long long)s.n_rows,                 \
                     lds_stamps(s.n_batches * s.n_blocks), g_graphsum_lds_opt, s.n_blocks)
  const int diag = g_graphsum_lds_diag;
  if (s.window == 4) {
    if (diag == 4) GS_LDS(4, 4, 1);
    else GS_LDS(0, 4, 1);
  } else if (s.window == 3) {
    if (diag == 4) GS_LDS(4, 3, 1);
    else GS_LDS(0, 3, 1);
  } else if (s.window == 2) {
    if (diag == 4) GS_LDS(4, 2, 1);
    else if (diag == 6) GS_LDS(6, 2, 1);  // no next-line touch
    else GS_LDS(0, 2, 1);
  } else if (g_graphsum_lds_sync == 0) {  // r01: a workgroup barrier per slice
    if (diag == 4) GS_LDS(4, 1, 0);
    else GS_LDS(0, 1, 0);
  } else {
    switch (diag) {
      case 1: GS_LDS(1, 1, 1); break;
      case 2: GS_LDS(2, 1, 1); break;
      case 3: GS_LDS(3, 1, 1); break;
      case 5: GS_LDS(5, 1, 1); break;  // no table reads, 1/16 staged
      case 7: GS_LDS(7, 1, 1); break;  // as 5, no entry stream either
      case 8: GS_LDS(8, 1, 1); break;  // as 7, one block per slot visit
      case 9: GS_LDS(9, 1, 1); break;  // as 7, one loop over a slice's blocks
      case 10: GS_LDS(10, 1, 1); break;  // every row read twice (LDS load x2)
      case 11: GS_LDS(11, 1, 1); break;  // twice the adds (VALU load x2)
      case 4: GS_LDS(4, 1, 1); break;
      default: GS_LDS(0, 1, 1); break;
    }
  }
#undef GS_LDS
  launch_gs_lds_combine(s, partial, out, ld_out, st, epi);
}

void launch_gs_lds_combine(const LdsSchedule &s, const float *partial, float *out, int ld_out,
                           hipStream_t st, const GsEpilogue *epi) {
  const GsEpilogue none{};
  const long long post = (long long)s.n_rows * 4;
  hipLaunchKernelGGL(k_gs_lds_combine, dim3((unsigned)ceil_div(post, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(partial), (long long)s.n_rows,
                     s.n_blocks, s.row_scale, s.n_rows, reinterpret_cast<float4 *>(out),
                     ld_out / 4, epi ? *epi : none);
  PGCN_HIP(hipGetLastError());
}

}  // namespace pgcn
