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

namespace pgcn {

typedef __attribute__((address_space(3))) void lds_void;

// in'[r, 0:16] = scale[r] * in[r, 0:16]   (rows of 4 float4; ld4 = row stride in float4)
__global__ __launch_bounds__(256) void k_gs_prescale(const float4 *__restrict__ in, int ld4_in,
                                                     const float *__restrict__ scale, int n,
                                                     float4 *__restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t >> 2;
  if (r >= n) return;
  const int v = (int)(t & 3);
  const float s = scale[r];
  float4 x = in[r * ld4_in + v];
  x.x *= s;
  x.y *= s;
  x.z *= s;
  x.w *= s;
  out[r * 4 + v] = x;
}

__device__ __forceinline__ void f4_acc(float4 &a, const float4 &x) {
  a.x += x.x;
  a.y += x.y;
  a.z += x.z;
  a.w += x.w;
}

// One LDS-DMA piece: 16 B per active lane to LDS byte address lds_dst + 16 * lane.  Inline
// asm keeps the DMA out of hipcc's waitcnt bookkeeping (it would otherwise drain it with
// vmcnt(0) before unrelated LDS reads); completion is counted by hand (s_waitcnt vmcnt).
__device__ __forceinline__ void glds16(const void *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

constexpr int LDS_TABLE_F4 = 2 * LDS_ROWS * 4;       // two slice buffers (float4 units)
constexpr int LDS_RING_CHUNK = 512;                  // bytes: 4 entry blocks of 128 B
constexpr int LDS_RING_SLOTS = 3;                    // chunks per wave: 2 in flight + 1 read
constexpr int LDS_RING_BYTES = LDS_RING_SLOTS * LDS_RING_CHUNK;
constexpr int LDS_TOTAL_F4 = LDS_TABLE_F4 + LDS_CW * LDS_RING_BYTES / 16;

// Wave roles: waves 0 .. LDS_CW-1 sum (each owns LDS_SLOTS rowsets and an entry ring); wave
// LDS_CW copies slice t+1 into the other buffer while slice t is summed.  The copies and the
// ring refills are LDS-DMA issued from inline asm, invisible to hipcc's waitcnt bookkeeping;
// each wave counts its own: a summing wave only ever has ring refills outstanding (constant
// vmcnt(2) = "the chunk refilled two chunks ago has landed"), the loader waits vmcnt(0) once
// per slice.  One barrier per slice (raw s_barrier: no compiler-inserted vmcnt(0)).
__global__ __launch_bounds__(LDS_THREADS) void k_graphsum_lds(
    const uint2 *__restrict__ entries, const long long *__restrict__ wave_off,
    const unsigned short *__restrict__ counts, int t_max, const int2 *__restrict__ slices,
    const int *__restrict__ n_slices, const int *__restrict__ rows, const float4 *__restrict__ in,
    int n_cols, float4 *__restrict__ partial, long long part_stride) {
  // ONE __shared__ object: [2][LDS_ROWS][4] float4 slice buffers, then the entry rings
  __shared__ float4 lds[LDS_TOTAL_F4];
  const int nb = kGraphBlocks;
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

  if (wave == LDS_CW) {  // ------------------------------------------------ loader wave
    const int2 *sl = slices + (long long)b * t_max;
    const int last = n_cols - 1;
    for (int t = 0; t < T; t++) {
      // slice t -> buffer t & 1 (free: every wave passed the barrier after slice t - 2)
      const int2 sc = sl[t];
      const unsigned dst = lds_base + (unsigned)((t & 1) * LDS_ROWS * 64);
#pragma unroll 8
      for (int i = 0; i < LDS_SR / 16; i++) {
        int r = sc.x + 16 * i + g;
        r = r < last ? r : last;  // rows past the slice end are never referenced
        glds16(in + (long long)r * 4 + v, dst + (unsigned)(i * 1024));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // slice t ready (t = 0) / slice t-1 summed
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // matches the summing waves' last slice
    return;
  }

  // ------------------------------------------------------------------------- summing waves
  const long long wid = (long long)blockIdx.x * LDS_CW + wave;
  const long long kb0 = wave_off[wid], kb1 = wave_off[wid + 1];
  const long long nchunk = (kb1 - kb0 + 3) >> 2;
  const char *ebytes = reinterpret_cast<const char *>(entries) + kb0 * 128;
  const unsigned ring_dst = lds_base + LDS_TABLE_F4 * 16 + (unsigned)(wave * LDS_RING_BYTES);
  const char *ring = reinterpret_cast<const char *>(lds + LDS_TABLE_F4) + wave * LDS_RING_BYTES +
                     g * 8;
  auto refill = [&](long long c) {  // chunk c -> ring slot c % 3 (clamped: dummy past the end)
    long long cc = c < nchunk ? c : nchunk - 1;
    cc = cc > 0 ? cc : 0;
    if (lane < 32)
      glds16(ebytes + cc * LDS_RING_CHUNK + lane * 16,
             ring_dst + (unsigned)((c % LDS_RING_SLOTS) * LDS_RING_CHUNK));
  };
  refill(0);
  refill(1);
  refill(2);
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // chunk 0

  float4 acc[LDS_SLOTS];
#pragma unroll
  for (int j = 0; j < LDS_SLOTS; j++) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  const unsigned short *cnt = counts + ((long long)blockIdx.x * t_max) * (LDS_CW * LDS_SLOTS) +
                              wave * LDS_SLOTS;
  int blk = 0;    // entry blocks consumed (ring position = blk % 12 blocks)
  int roff = 0;   // byte offset of block `blk` in the ring
  uint2 e_next = *reinterpret_cast<const uint2 *>(ring);

  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // zero rows written
  __builtin_amdgcn_s_barrier();                       // slice 0 staged
  asm volatile("" ::: "memory");
  for (int t = 0; t < T; t++) {
    const float4 *tb = lds + (t & 1) * LDS_ROWS * 4 + v;
    const uint4 *c4 = reinterpret_cast<const uint4 *>(cnt + (long long)t * (LDS_CW * LDS_SLOTS));
    const uint4 cw0 = c4[0], cw1 = c4[1];  // 16 step counts (scalar loads)
    const unsigned cw[8] = {cw0.x, cw0.y, cw0.z, cw0.w, cw1.x, cw1.y, cw1.z, cw1.w};
#pragma unroll
    for (int j = 0; j < LDS_SLOTS; j++) {
      const int n = (cw[j >> 1] >> (16 * (j & 1))) & 0xffff;  // steps of rowset j
      for (int k = 0; k < n; k += 4) {
        const uint2 e = e_next;
        ++blk;
        roff = roff + 128 == LDS_RING_BYTES ? 0 : roff + 128;
        if ((blk & 3) == 0) {  // entering chunk blk/4: refill the slot read before, wait for it
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          refill((blk >> 2) + 2);
          asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
        e_next = *reinterpret_cast<const uint2 *>(ring + roff);  // (past the end: unused)
        // all 4 entries are valid: steps past a row's run point at a zero row
        const float4 x0 = tb[e.x & 0xffffu], x1 = tb[e.x >> 16];
        const float4 x2 = tb[e.y & 0xffffu], x3 = tb[e.y >> 16];
        f4_acc(acc[j], x0);
        f4_acc(acc[j], x1);
        f4_acc(acc[j], x2);
        f4_acc(acc[j], x3);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // slice t summed; slice t+1 staged
    asm volatile("" ::: "memory");
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
                                                        float4 *__restrict__ out, int ld4_out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long r = t >> 2;
  if (r >= n) return;
  const int v = (int)(t & 3);
  float4 a = partial[r * 4 + v];
  for (int b = 1; b < nb; b++) f4_acc(a, partial[((long long)b * part_stride + r) * 4 + v]);
  const float s = scale[r];
  a.x *= s;
  a.y *= s;
  a.z *= s;
  a.w *= s;
  out[r * ld4_out + v] = a;
}

void launch_graphsum_lds(const LdsSchedule &s, const float *in, int ld_in, float *out,
                         int ld_out, float *scratch_in, float *partial, hipStream_t st) {
  PGCN_CHECK(ld_in % 4 == 0 && ld_out % 4 == 0, PGCN_E_INVALID, "graphsum_lds: ld % 4");
  const long long pre = (long long)s.n_cols * 4;
  hipLaunchKernelGGL(k_gs_prescale, dim3((unsigned)ceil_div(pre, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(in), ld_in / 4, s.col_scale, s.n_cols,
                     reinterpret_cast<float4 *>(scratch_in));
  hipLaunchKernelGGL(k_graphsum_lds, dim3((unsigned)(s.n_batches * kGraphBlocks)),
                     dim3(LDS_THREADS), 0, st, s.entries, s.wave_off, s.counts, s.t_max,
                     s.slices, s.n_slices, s.rows, reinterpret_cast<const float4 *>(scratch_in),
                     s.n_cols, reinterpret_cast<float4 *>(partial), (long long)s.n_rows);
  const long long post = (long long)s.n_rows * 4;
  hipLaunchKernelGGL(k_gs_lds_combine, dim3((unsigned)ceil_div(post, 256)), dim3(256), 0, st,
                     reinterpret_cast<const float4 *>(partial), (long long)s.n_rows,
                     kGraphBlocks, s.row_scale, s.n_rows, reinterpret_cast<float4 *>(out),
                     ld_out / 4);
  PGCN_HIP(hipGetLastError());
}

}  // namespace pgcn
