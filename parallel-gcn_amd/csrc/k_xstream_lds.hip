// parallel-gcn_amd/csrc/k_xstream_lds.hip -- the X-stream GEMMs with loader and MFMA waves
// split (the default form of k_xstream_nn / k_xstream_tn, csrc/k_gemm.hip, for reddit's
// feature width).
//
// Same products as those kernels (Z = drop(X) W and W.grad = drop(X)^T dZ over the dense
// feature matrix X [M][lda], N <= 16; src/module.cu:108-163 in the reference), same per-lane
// MFMA feed.  What changes is who waits for memory.  In the register-streamed kernels every
// wave both streams X and runs its MFMAs; on reddit (X = 563 MB) they move X at 3.4-4.1 TB/s
// although a bare read of X with the same lane map reaches 6.1 TB/s here, because the
// 0.05 ms of fp32 MFMA per pass (64 FLOP/clk/SIMD) does not overlap the stream
// (tools/xs_micro.hip: read alone 91 us, read + MFMA in the same waves 122 us, MFMA alone
// 50 us; loader + MFMA waves as below 90-98 us).
//
// One workgroup per CU, 6 waves (NN: 2 loaders, 4 consumers) or 4 (TN: 1 loader, 3 consumers):
//   loader waves          copy whole 16-row groups of X (16 * lda contiguous floats) into an
//                         LDS ring of up to 4 slots by LDS-DMA (global_load_lds_dwordx4,
//                         nontemporal, 1 KB per instruction, no VGPRs, NI instructions per
//                         group: a compile-time count, so hipcc sees a straight-line issue),
//                         one group in flight each (option: two): wait for the slot to be
//                         handed back, issue, s_waitcnt, publish;
//   consumer waves        take the groups in turn, copy the group's MFMA operands from the
//                         slot to registers (ds_read_b128), hand the slot back and run the
//                         MFMAs, with their state (B of the NN product, the TN accumulators)
//                         in registers.
// The slot is the group's bytes as they lie in X (row stride lda / 4 chunks, lda = K rounded
// up to 4), plus the bytes after it up to NI KB, then (flat mask, r05 late) the group's keep
// bits from the dropout bitmap as drawn (FLATM: no nibble-layout pass over the mask).  In the last group of X, lanes past the end
// of X copy the group's first chunk instead, so every value in a slot is finite data except
// the ld padding (k in [K, lda), possibly NaN): NN zeroes it in the slot before use (B is 0
// for k >= K, so the finite values past K add exact zeros); in TN it reaches only output rows
// k >= K, which are not written.
// NN results are bit-identical to k_xstream_nn (same MFMA sequence per row group); TN sums
// each workgroup's row groups in group order into one [K][16] partial per workgroup (the
// ordered k_slab_reduce1 / k_gemm_tn_reduce pass follows): deterministic.
#include <cmath>

#include "common.hpp"
#include "kernels.hpp"
#include "lds_dma.hpp"
#include "mask_draw.hpp"

#ifndef PGCN_XS_CHAINS
#define PGCN_XS_CHAINS 1
#endif

namespace pgcn {

// "xstream_ring": 1 = these kernels for the X-stream products where they apply (default),
// 0 = the register-streamed k_xstream_nn / k_xstream_tn (the oracle-tested fallback of every
// other width).  Measured and removed (r02): two groups in flight per loader wave with fewer
// slots (r04 keeps two in flight at the same slot count, publishing group t-1 after group t's
// DMAs are issued: xl_load), and a TN split in which every consumer takes a share of K of every group (173 vs 137
// us on reddit: every consumer then waits on every group).
int g_xstream_ring = 1;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// NN: 2 loaders + 4 consumers (two waves on two SIMDs: 2 x ~220 registers fit); TN: 1 loader +
// 3 consumers (its accumulators need a SIMD per consumer)
constexpr int XL_NN_LOADERS = 2, XL_NN_CONSUMERS = 4;
// mask_xstream (r06): two more waves that draw the next training forward's dropout masks
// beside an unmasked NN pass (eval's (A X) W1: HBM-bound, its VALU mostly idle); they share
// SIMDs 2 and 3 with a consumer each (2 x ~220 VGPRs per SIMD, as the loaders do)
constexpr int XL_NN_DRAWERS = 2;
#ifndef PGCN_XS_TN_ABLATE
#define PGCN_XS_TN_ABLATE 0
#endif
#ifndef PGCN_XS_TN_LOADERS
#define PGCN_XS_TN_LOADERS 1
#endif
constexpr int XL_TN_LOADERS = PGCN_XS_TN_LOADERS, XL_TN_CONSUMERS = 4 - PGCN_XS_TN_LOADERS;
constexpr int XL_LDS = 159 * 1024;  // ring + hand-off words (one workgroup per CU)
constexpr int XL_FLAGS = 64;        // ready[8], freed[8] at the end
constexpr int XL_KC = 10;           // the instantiated width: K in (576, 640] (reddit: 602)
constexpr int XL_S0 = 4 * (XL_KC - 1) + 1;  // NN steps (16 k each) inside every such K
constexpr int XL_BS = 648;          // B^T row stride in floats (== 8 mod 16: conflict-free)
constexpr int XL_BT_BYTES = 16 * XL_BS * 4 / 1024 * 1024 + 1024;  // NN: B^T ahead of the ring

struct XlRing {
  int off;    // LDS byte offset of slot 0 (NN: past B^T)
  int st;     // row stride in 16-B chunks (lda / 4 = ceil(K / 4))
  int nslot;  // slots in the ring (<= 4)
  int sb;     // bytes per slot: the group's NI KB of X, then mb bytes of its keep bits
  int mb;     // (flat mask) the group's bitmap bytes from a 16-B boundary, 256-B multiple; or 0
};

// DMA instructions (1 KB) per group for a row of lda floats: the group's 64 * lda bytes
__host__ __device__ constexpr int xl_ni(int lda) { return (64 * lda + 1023) / 1024; }

// mask_ld > 0: the keep bits come as the flat bitmap (XsMask, mask_ld bits per row), staged
// with the group: 16 rows' bits from the 16-B boundary below the first (<= 15 B ahead), 1 B
// of slack, rounded up to 256 B (reddit: 1,220 -> 1,280 B)
XlRing xl_ring(int lda, int ni, int off, long long mask_ld = 0) {
  XlRing r;
  r.off = off;
  r.st = lda / 4;
  r.mb = mask_ld > 0 ? (int)((15 + (16 * mask_ld + 7) / 8 + 1 + 255) / 256 * 256) : 0;
  r.sb = ni * 1024 + r.mb;
  r.nslot = std::min(4, (XL_LDS - XL_FLAGS - off) / r.sb);
  return r;
}

// byte offset (16-B aligned) in the bitmap of the first keep bit of group row0's rows
__device__ __forceinline__ long long xl_mask_byte0(const XsMask &mk, long long row0) {
  return ((mk.base + row0 * mk.ld) >> 3) & ~15LL;
}

// keep bit t of `bits` (as 0 / all ones by a 1-bit signed field extract) masks element t, then
// the scale: x * scale or +0 (k_gemm.hip's apply4 gives x * 0, a zero of x's sign: the sums
// are the same).  FOLD: the scale is a power of two and is applied to the finished sums (NN)
// or to dZ (TN) instead -- exact scalings, so the same bits with one multiply per product less.
template <bool FOLD>
__device__ __forceinline__ void xl_apply4(float4 &a, uint32_t bits, float scale) {
  a.x = __uint_as_float(__float_as_uint(a.x) & (uint32_t)__builtin_amdgcn_sbfe((int)bits, 0, 1));
  a.y = __uint_as_float(__float_as_uint(a.y) & (uint32_t)__builtin_amdgcn_sbfe((int)bits, 1, 1));
  a.z = __uint_as_float(__float_as_uint(a.z) & (uint32_t)__builtin_amdgcn_sbfe((int)bits, 2, 1));
  a.w = __uint_as_float(__float_as_uint(a.w) & (uint32_t)__builtin_amdgcn_sbfe((int)bits, 3, 1));
  if constexpr (!FOLD) {
    a.x *= scale;
    a.y *= scale;
    a.z *= scale;
    a.w *= scale;
  }
}

// groups of this workgroup: blockIdx.x + t * gridDim.x, t < T
__device__ __forceinline__ int xl_groups(long long M) {
  const long long n_rg = (M + 15) / 16;
  return blockIdx.x < n_rg ? (int)((n_rg - blockIdx.x + gridDim.x - 1) / gridDim.x) : 0;
}

// nontemporal LDS-DMA of four consecutive 1-KB pieces (one address, offsets 0..3 KB)
__device__ __forceinline__ void xl_dma4(const char *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024 nt\n\t"
      "global_load_lds_dwordx4 %1, off offset:2048 nt\n\t"
      "global_load_lds_dwordx4 %1, off offset:3072 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// Loader wave `wave` of NL: groups wave, wave + NL, ... into slot t % nslot, NI pieces
// each; a consumer per group releases the slot by storing t + 1 into freed.
// FLATM: then the group's keep bits (rg.mb bytes of the flat bitmap from xl_mask_byte0) behind
// its X in the slot, by up to two more LDS-DMA instructions (lanes past the bitmap's end copy
// its first chunk: bits of rows past M, which no output reads)
template <int NI, int NL, bool FLATM>
__device__ __forceinline__ void xl_load(const float *__restrict__ A, int lda, long long M, int T,
                                        int wave, int lane, const XlRing &rg, char *lds,
                                        unsigned *ready, unsigned *freed, const XsMask &mk) {
  constexpr int NM = FLATM ? 2 : 0;  // mask pieces per group (rg.mb <= 2 KB)
  static_assert(NI + NM < 64, "vmcnt counts at most 63");
  __builtin_amdgcn_s_setprio(3);
  wave = __builtin_amdgcn_readfirstlane(wave);  // uniform (the LDS-DMA destination is an SGPR)
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<size_t>((__attribute__((address_space(3))) char *)lds));
  const unsigned slot_bytes = (unsigned)rg.sb;
  const long long x_bytes = M * (long long)lda * 4;
  auto publish = [&](int u) {
    if (lane == 0) __atomic_store_n(ready + u % rg.nslot, (unsigned)(u + 1), __ATOMIC_RELAXED);
    asm volatile("" ::: "memory");
  };
  int pend = -1;  // the group issued last, not yet published (its DMAs may still land)
  for (int t = wave; t < T; t += NL) {
    const int slot = t % rg.nslot;
    // the slot's last group is this wave's own unpublished one when nslot <= NL (NN at lda
    // 628..640: 2 slots for 2 loaders): land and publish it first, or its consumers never
    // free the slot this wave waits for
    if (pend >= 0 && t - rg.nslot >= pend) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      publish(pend);
      pend = -1;
    }
    if (t >= rg.nslot) lds_wait_ge(freed + slot, (unsigned)(t - rg.nslot + 1));
    const long long b0 = (blockIdx.x + (long long)t * gridDim.x) * 16 * (long long)lda * 4;
    const char *blk = reinterpret_cast<const char *>(A) + b0;
    const unsigned dst = __builtin_amdgcn_readfirstlane(base + (unsigned)(rg.off + slot * slot_bytes));
    if (b0 + NI * 1024 <= x_bytes) {  // the whole NI KB lies inside X
      const char *src = blk + lane * 16;
#pragma unroll
      for (int q = 0; q + 4 <= NI; q += 4) xl_dma4(src + q * 1024, dst + (unsigned)(q * 1024));
#pragma unroll
      for (int q = NI / 4 * 4; q < NI; q++) glds16_nt(src + q * 1024, dst + (unsigned)(q * 1024));
    } else {  // the last group of X: lanes past its end copy the group's first chunk
      const long long left = x_bytes - b0;
#pragma unroll
      for (int q = 0; q < NI; q++) {
        const long long off = q * 1024 + lane * 16;
        glds16_nt(blk + (off < left ? off : 0), dst + (unsigned)(q * 1024));
      }
    }
    if constexpr (FLATM) {
      const long long byte0 = xl_mask_byte0(mk, (blockIdx.x + (long long)t * gridDim.x) * 16);
      const char *mb = reinterpret_cast<const char *>(mk.bits);
      const long long mbytes = mk.words * 8;
#pragma unroll
      for (int q = 0; q < NM; q++) {
        const long long off = byte0 + q * 1024 + lane * 16;
        const char *src = mb + (off + 16 <= mbytes ? off : 0);
        // (the second piece: only the lanes inside rg.mb; one instruction either way)
        if (q * 1024 + lane * 16 < rg.mb) glds16_nt(src, dst + (unsigned)(NI * 1024 + q * 1024));
      }
    }
    // two groups in flight: the previous one lands while this one's DMAs are issued (at most
    // NI (+ NM) of this group's pieces still counted; r04: X-stream passes 339 -> 329 us per
    // epoch, most of it on TN, whose single loader had one group in flight)
    if (pend >= 0) {
      asm volatile("s_waitcnt vmcnt(%c0)" ::"n"(NI + NM) : "memory");
      publish(pend);
    }
    pend = t;
  }
  if (pend >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    publish(pend);
  }
}

// a consumer's release of a slot once every read of it returned
__device__ __forceinline__ void xl_release(unsigned *freed, int slot, int t, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __atomic_store_n(freed + slot, (unsigned)(t + 1), __ATOMIC_RELAXED);
  asm volatile("" ::: "memory");
}

// NN: C[M][N<=16] = drop(X) W (DUAL: C = X W and C2 = drop(X) W); consumer lane (i, g) of a
// group holds B[16 s + 4 g + t][i] for every step s (registers) and feeds MFMA t of step s with
// X[row i][16 s + 4 g + t] -- k_xstream_nn's feed and order, so the same bits (up to the sign
// of zero products: see xl_apply4).  B^T sits in LDS ahead of the ring (as in k_xstream_nn).
// FLATM (with MASKED): the keep bits from the flat bitmap `mk`, staged in the slot by the loader
// (no nibble-layout pass): lane (i, g) forms its row's bits as ten 64-bit words W[c] = row bits
// 64 c .. 64 c + 63 (v_alignbit from the slot's dwords), and step s's nibble is bits
// 16 (s & 3) + 4 g .. + 3 of W[s >> 2] -- the nibble maskT[row][4 (s & 3) + g] holds at 4 (s >> 2)
template <int NI, bool MASKED, bool DUAL, bool FOLD, bool FLATM, bool DRAW = false>
__global__ __launch_bounds__(64 * (XL_NN_LOADERS + XL_NN_CONSUMERS + (DRAW ? XL_NN_DRAWERS : 0)),
                             1) void k_xs_nn_ring(
    int M, int N, int K, const float *__restrict__ A, int lda, const float *__restrict__ B,
    int ldb, int trans_b, float *__restrict__ C, int ldc, const uint64_t *__restrict__ maskT,
    float a_scale, float *__restrict__ C2, XsEpilogue epi, XlRing rg, XsMask mk, XsDraw dr) {
  static_assert(!DUAL || MASKED, "dual: the second product is the masked one");
  static_assert(!FLATM || MASKED, "a flat mask is a mask");
  constexpr int NS = 4 * XL_KC;
  __shared__ __attribute__((aligned(1024))) char lds[XL_LDS];
  unsigned *const ready = reinterpret_cast<unsigned *>(lds + XL_LDS - XL_FLAGS);
  unsigned *const freed = ready + 8;
  if (threadIdx.x < 16) ready[threadIdx.x] = 0u;
  {  // B^T [16][XL_BS] (zero outside [K, N]) ahead of the ring: every load of the thread's
     // elements issued before their stores (one round trip, not one per element)
    float *bt = reinterpret_cast<float *>(lds);
    constexpr int NT = 64 * (XL_NN_LOADERS + XL_NN_CONSUMERS + (DRAW ? XL_NN_DRAWERS : 0)),
                  PER = (16 * NS * 16 + NT - 1) / NT;
    float v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int e = threadIdx.x + u * NT, k = e >> 4, j = e & 15;
      v[u] = 0.0f;
      if (e < 16 * NS * 16 && k < K && j < N)
        v[u] = trans_b ? B[(long long)j * ldb + k] : B[(long long)k * ldb + j];
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
      const int e = threadIdx.x + u * NT, k = e >> 4, j = e & 15;
      if (e < 16 * NS * 16) bt[j * XL_BS + k] = v[u];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = xl_groups(M);
  if constexpr (DRAW) {
    if (wave >= XL_NN_LOADERS + XL_NN_CONSUMERS) {  // the drawing waves: k_dropout_mask's work
      constexpr int DT = 64 * XL_NN_DRAWERS;
      const long long t0 = (long long)blockIdx.x * DT +
                           (threadIdx.x - 64 * (XL_NN_LOADERS + XL_NN_CONSUMERS));
      const long long G = (long long)gridDim.x * DT;
      for (int q = 0; q < dr.n; q++) {
        if (dr.seg[q].per == 2)
          dropout_mask_seg<2>(dr.seg[q], dr.lut, t0, G);
        else
          dropout_mask_seg<1>(dr.seg[q], dr.lut, t0, G);
      }
      return;
    }
  }
  if (wave < XL_NN_LOADERS) {
    xl_load<NI, XL_NN_LOADERS, FLATM>(A, lda, M, T, wave, lane, rg, lds, ready, freed, mk);
    return;
  }
  const int cid = wave - XL_NN_LOADERS, g = lane >> 4, i = lane & 15;
  constexpr bool NIB = MASKED && !FLATM;  // keep bits from maskT (prefetched a group ahead)
  const float *bl = reinterpret_cast<const float *>(lds) + i * XL_BS + 4 * g;
  auto load_mask = [&](int t, uint64_t(&m)[4]) {  // keep bits of the lane's row of group t
    long long row = (blockIdx.x + (long long)t * gridDim.x) * 16 + i;
    row = row < M ? row : M - 1;
#pragma unroll
    for (int q = 0; q < 4; q++) m[q] = maskT[row * 16 + 4 * q + g];
  };
  // group t with its keep bits in mw; the next group's go to mwn (two static buffers that
  // alternate: a copy would wait for the prefetch)
  auto group = [&](int t, const uint64_t(&mw)[4], uint64_t(&mwn)[4]) {
    if (NIB && t + XL_NN_CONSUMERS < T) load_mask(t + XL_NN_CONSUMERS, mwn);
    const long long rgi = blockIdx.x + (long long)t * gridDim.x;
    // the epilogue's row scales, loaded before the slot wait (whose memory clobber keeps them
    // here) so they land during the MFMAs: loaded at their use, each load waited for alone
    // behind the stores before it (vmcnt counts stores), four HBM round trips per group
    float nsc[4];  // read only under epi.next_table
    if constexpr (!DUAL) {
      if (epi.next_table) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const long long rr = rgi * 16 + 4 * g + r;
          nsc[r] = epi.next_scale[rr < M ? rr : M - 1];
        }
      }
    }
    const int slot = t % rg.nslot;
    lds_wait_ge(ready + slot, (unsigned)(t + 1));
    char *const sb = lds + rg.off + slot * rg.sb;
    if (K & 3) {  // the ld padding k >= K of each row's last chunk (may be NaN)
      if (lane < 16) {
        float *pc = reinterpret_cast<float *>(sb + (lane * rg.st + rg.st - 1) * 16);
        for (int e = K & 3; e < 4; e++) pc[e] = 0.0f;
      }
      asm volatile("" ::: "memory");
    }
    // the group's fragments into registers, then the slot goes back to the loader
    // (K > 64 (XL_KC - 1) on this kernel: steps s < XL_S0 always lie inside K, so only the
    // last few test it -- no per-step branch for hipcc to schedule around)
    const char *a = sb + i * rg.st * 16 + g * 16;
    float4 xa[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
      xa[s] = (s < XL_S0 || 16 * s < K) ? *reinterpret_cast<const float4 *>(a + 64 * s)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned wl[XL_KC], wh[XL_KC];  // FLATM: the row's keep bits, W[c] = wh[c]:wl[c]
    if constexpr (FLATM) {
      const long long row0 = rgi * 16;
      const long long bit = mk.base + (row0 + i) * mk.ld - 8 * xl_mask_byte0(mk, row0);
      const unsigned *dw = reinterpret_cast<const unsigned *>(sb + NI * 1024) + (bit >> 5);
      const unsigned sh = (unsigned)bit & 31u;
      unsigned d[2 * XL_KC + 1];
#pragma unroll
      for (int e = 0; e < 2 * XL_KC + 1; e++) d[e] = dw[e];
#pragma unroll
      for (int c = 0; c < XL_KC; c++) {
        wl[c] = __builtin_amdgcn_alignbit(d[2 * c + 1], d[2 * c], sh);
        wh[c] = __builtin_amdgcn_alignbit(d[2 * c + 2], d[2 * c + 1], sh);
      }
    }
    xl_release(freed, slot, t, lane);
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f}, acc2 = floatx4{0.f, 0.f, 0.f, 0.f};
#if PGCN_XS_CHAINS == 2
    // experiment: the single product's steps on two accumulators (even / odd steps), added
    // at the end (MFMA dependent latency 40 vs 32 cycles issue)
    floatx4 acch = floatx4{0.f, 0.f, 0.f, 0.f};
#endif
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (s >= XL_S0 && 16 * s >= K) break;  // steps wholly past K add nothing
      float4 x = xa[s];
      const float4 bb = *reinterpret_cast<const float4 *>(bl + 16 * s);
      if constexpr (DUAL) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, bb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, bb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, bb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, bb.w, acc, 0, 0, 0);
      }
      if constexpr (FLATM)
        xl_apply4<FOLD>(x, __builtin_amdgcn_ubfe((s & 2) ? wh[s >> 2] : wl[s >> 2],
                                                 16 * (s & 1) + 4 * g, 4), a_scale);
      else if constexpr (MASKED)
        xl_apply4<FOLD>(x, (uint32_t)(mw[s & 3] >> (4 * (s >> 2))) & 0xfu, a_scale);
#if PGCN_XS_CHAINS == 2
      floatx4 &am = DUAL ? acc2 : ((s & 1) ? acch : acc);
#else
      floatx4 &am = DUAL ? acc2 : acc;
#endif
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, bb.x, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, bb.y, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, bb.z, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, bb.w, am, 0, 0, 0);
    }
#if PGCN_XS_CHAINS == 2
    if constexpr (!DUAL) acc = acc + acch;
#endif
    if constexpr (MASKED && FOLD) {  // the masked product's scale, on its sums
      floatx4 &am = DUAL ? acc2 : acc;
      am = am * a_scale;
    }
    // lane holds C[16 rg + 4 g + r][i] (k_xstream_nn's epilogue)
    float cv[4];
    if (i < ldc) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const long long rr = rgi * 16 + 4 * g + r;
        float c = acc[r];
        if constexpr (!DUAL) {
          if (epi.relu && !(c > 0.0f)) c = 0.0f;  // k_relu_fwd's test (NaN -> 0)
        }
        cv[r] = c;
        if (rr < M) {
          C[rr * ldc + i] = c;
          if constexpr (DUAL) C2[rr * ldc + i] = acc2[r];
        }
      }
    }
    if constexpr (!DUAL) {
      if (epi.next_table) {
        // k_ring_prescale of the stored values, s_r * C[r][4 v .. 4 v + 3], one float4 per
        // lane: lane (g, 4 v + q) takes row 4 g + q's plane v from its quad (ldc = 16: every
        // lane holds a column; a 4 x 4 transpose in four shuffles, as the fused loss kernel's)
        const int q = i & 3, v = i >> 2;
        float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int out_r = (q - k) & 3, in_c = (q + k) & 3;
          const float send = out_r == 0 ? cv[0] : out_r == 1 ? cv[1] : out_r == 2 ? cv[2] : cv[3];
          const float got = __shfl(send, (lane & ~3) | in_c, 64);
#pragma unroll
          for (int m = 0; m < 4; m++) o[m] = in_c == m ? got : o[m];
        }
        const long long rr = rgi * 16 + 4 * g + q;
        const float s = q == 0 ? nsc[0] : q == 1 ? nsc[1] : q == 2 ? nsc[2] : nsc[3];
        if (rr < M) {
          const long long sr = epi.next_sr;
          epi.next_table[(rr / sr) * 4 * sr + v * sr + rr % sr] =
              make_float4(o[0] * s, o[1] * s, o[2] * s, o[3] * s);
        }
      }
    }
  };
  uint64_t mwa[4] = {0, 0, 0, 0}, mwb[4] = {0, 0, 0, 0};
  if (NIB && cid < T) load_mask(cid, mwa);
  for (int t = cid; t < T; t += 2 * XL_NN_CONSUMERS) {
    group(t, mwa, mwb);
    if (t + XL_NN_CONSUMERS < T) group(t + XL_NN_CONSUMERS, mwb, mwa);
  }
}

// TN: partial[blockIdx.x][k][j] = sum over this workgroup's rows m of drop(X)[m][k] G[m][j].
// A group is 4 steps of 4 rows; consumer lane (i, g) feeds MFMA (c, t) of step q with
// X[row 4q + g][64 c + 4 i + t] and G[row 4q + g][i] (k_xstream_tn's feed); the two consumers'
// accumulators (groups t = c mod 3 for consumer c) are added in consumer order at the end.
template <int NI, bool MASKED, bool FOLD, bool FLATM>
__global__ __launch_bounds__(64 * (XL_TN_LOADERS + XL_TN_CONSUMERS), 1) void k_xs_tn_ring(
    int M, int N, int K, const float *__restrict__ A, int lda, const float *__restrict__ G,
    int ldg, const uint64_t *__restrict__ maskT, float a_scale, float *__restrict__ partial,
    XlRing rg, XsMask mk) {
  static_assert(!FLATM || MASKED, "a flat mask is a mask");
  constexpr bool NIB = MASKED && !FLATM;
  constexpr int KC = XL_KC;
  __shared__ __attribute__((aligned(1024))) char lds[XL_LDS];
  unsigned *const ready = reinterpret_cast<unsigned *>(lds + XL_LDS - XL_FLAGS);
  unsigned *const freed = ready + 8;
  if (threadIdx.x < 16) ready[threadIdx.x] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, i = lane & 15;
  const int T = xl_groups(M);
  floatx4 acc[KC][4];
#pragma unroll
  for (int c = 0; c < KC; c++)
#pragma unroll
    for (int t = 0; t < 4; t++) acc[c][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (wave < XL_TN_LOADERS) {
    xl_load<NI, XL_TN_LOADERS, FLATM>(A, lda, M, T, wave, lane, rg, lds, ready, freed, mk);
  } else {
    const int cid = wave - XL_TN_LOADERS;
    // dZ and keep bits of group t, raw: unconditional loads whose values are first used a
    // group later (a select or multiply here made hipcc branch around each load and wait for
    // it on the spot: four HBM round trips per group)
    auto load_rows = [&](int t, float(&bv)[4], uint64_t(&m)[4]) {
      const long long row0 = (blockIdx.x + (long long)t * gridDim.x) * 16;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const long long mr = row0 + 4 * q + g;
        const long long row = mr < M ? mr : M - 1;
        bv[q] = G[row * ldg + (i < N ? i : 0)];
        if constexpr (NIB) m[q] = maskT[row * 16 + i];
      }
    };
    // group t with dZ / keep bits in bj / mw, the next group's into bjn / mwn (alternating
    // static buffers)
    auto group = [&](int t, const float(&bv)[4], const uint64_t(&mw)[4], float(&bjn)[4],
                     uint64_t(&mwn)[4]) {
      if (t + XL_TN_CONSUMERS < T) load_rows(t + XL_TN_CONSUMERS, bjn, mwn);
      const int slot = t % rg.nslot;
      lds_wait_ge(ready + slot, (unsigned)(t + 1));
      float bj[4];  // rows past M and columns past N feed zeros
      const long long row0 = (blockIdx.x + (long long)t * gridDim.x) * 16;
#pragma unroll
      for (int q = 0; q < 4; q++)
        bj[q] = (row0 + 4 * q + g < M && i < N) ? (MASKED && FOLD ? bv[q] * a_scale : bv[q]) : 0.0f;
      // the group's fragments into registers, then the slot goes back to the loader
      const char *sp = lds + rg.off + slot * rg.sb + i * 16;
      float4 xa[4][KC];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int c = 0; c < KC; c++)
          xa[q][c] = *reinterpret_cast<const float4 *>(sp + (4 * q + g) * rg.st * 16 + 256 * c);
      // FLATM: the nibbles maskT[row][i] holds (c: bits 64 c + 4 i .. + 3 of the row), from the
      // keep bits the loader staged behind the group's X
      uint64_t mf[4];
      if constexpr (FLATM) {
        const unsigned *dw = reinterpret_cast<const unsigned *>(lds + rg.off + slot * rg.sb + NI * 1024);
        const long long b0 = mk.base - 8 * xl_mask_byte0(mk, row0) + 4 * i;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const long long bit = b0 + (row0 + 4 * q + g) * mk.ld;
          const unsigned *d = dw + (bit >> 5);
          const unsigned sh = (unsigned)bit & 31u;
          unsigned lo = 0, hi = 0;
#pragma unroll
          for (int c = 0; c < KC; c++) {
            const unsigned nib = __builtin_amdgcn_alignbit(d[2 * c + 1], d[2 * c], sh) & 0xfu;
            if (c < 8)
              lo |= nib << (4 * c);
            else
              hi |= nib << (4 * (c - 8));
          }
          mf[q] = ((uint64_t)hi << 32) | lo;
        }
      }
      xl_release(freed, slot, t, lane);
#if PGCN_XS_TN_ABLATE & 2  // timing-only diagnostic builds: no MFMAs
      if (M > 0) return;
#endif
#pragma unroll
      for (int q = 0; q < 4; q++) {
        // a uniform exit per row step (never taken: nslot >= 2) keeps hipcc from scheduling
        // the four steps as one block, which holds every step's masked operands live at once
        // and spills (r03: 512 VGPRs + scratch, 202 vs 144 us; with it 360 VGPRs, none)
        if (rg.nslot <= 0) break;
#pragma unroll
        for (int c = 0; c < KC; c++) {
          float4 x = xa[q][c];
          if constexpr (FLATM)
            xl_apply4<FOLD>(x, (uint32_t)(mf[q] >> (4 * c)) & 0xfu, a_scale);
          else if constexpr (MASKED)
            xl_apply4<FOLD>(x, (uint32_t)(mw[q] >> (4 * c)) & 0xfu, a_scale);
          acc[c][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, bj[q], acc[c][0], 0, 0, 0);
          acc[c][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, bj[q], acc[c][1], 0, 0, 0);
          acc[c][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, bj[q], acc[c][2], 0, 0, 0);
          acc[c][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, bj[q], acc[c][3], 0, 0, 0);
        }
      }
    };
    float bja[4] = {0.f, 0.f, 0.f, 0.f}, bjb[4] = {0.f, 0.f, 0.f, 0.f};
    uint64_t mwa[4] = {0, 0, 0, 0}, mwb[4] = {0, 0, 0, 0};
    if (cid < T) load_rows(cid, bja, mwa);
    for (int t = cid; t < T; t += 2 * XL_TN_CONSUMERS) {
      group(t, bja, mwa, bjb, mwb);
      if (t + XL_TN_CONSUMERS < T) group(t + XL_TN_CONSUMERS, bjb, mwb, bja, mwa);
    }
  }
#if PGCN_XS_TN_ABLATE & 1  // timing-only diagnostic builds (tools/xs_scale.py): no epilogue
  if (threadIdx.x == 0 && M < 0) partial[0] = acc[0][0][0];
  return;
#endif
  // consumers 1, 2 hand their accumulators to consumer 0 through the (idle) ring; 0 adds them
  // in consumer order and writes the partial
  __syncthreads();
  float *red = reinterpret_cast<float *>(lds);
  constexpr int RED = KC * 4 * 4 * 64;  // floats per consumer
  if (wave > XL_TN_LOADERS) {
    float *rw = red + (wave - XL_TN_LOADERS - 1) * RED;
#pragma unroll
    for (int c = 0; c < KC; c++)
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) rw[((c * 4 + t) * 4 + r) * 64 + lane] = acc[c][t][r];
  }
  __syncthreads();
  if (wave == XL_TN_LOADERS) {
    // per 64-column chunk: the other consumers' 16 values read together, then the adds (in
    // consumer order) and 16 stores through a buffer resource of the partial's K rows, whose
    // range check drops the rows k >= K -- no per-store branch, so no LDS round trip per value
    // (r06: the branch-per-store form waited on each read: ~15 us of every TN launch)
    float *p = partial + (long long)blockIdx.x * K * 16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, K * 16 * 4, 0x00020000);
#pragma unroll
    for (int c = 0; c < KC; c++) {
      float o[16][XL_TN_CONSUMERS > 1 ? XL_TN_CONSUMERS - 1 : 1];
#pragma unroll
      for (int tr = 0; tr < 16; tr++)
#pragma unroll
        for (int q = 0; q < XL_TN_CONSUMERS - 1; q++) o[tr][q] = red[q * RED + (c * 16 + tr) * 64 + lane];
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int k = 64 * c + 4 * (4 * g + r) + t;
          float v = acc[c][t][r];
#pragma unroll
          for (int q = 0; q < XL_TN_CONSUMERS - 1; q++) v += o[t * 4 + r][q];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (k * 16 + i) * 4, 0, 0);
        }
    }
  }
}

}  // namespace

// a_scale = 2^n (dropout 1/2, 3/4, ...): scaling by it is exact, so it can move
static bool xl_pow2(float v) {
  int e;
  return v > 0.0f && std::frexp(v, &e) == 0.5f && std::isnormal(v);
}

// the shapes these kernels take: ten 64-column chunks (K in 577..640), rows packed at lda =
// K rounded up to 4 (the group is contiguous), N <= 16
bool xstream_ring_ok(int K, int lda) {
  return g_xstream_ring && K > 64 * (XL_KC - 1) && K <= 64 * XL_KC && lda == (K + 3) / 4 * 4;
}

void launch_xstream_nn_ring(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                            int trans_b, float *C, int ldc, const uint64_t *maskT, float a_scale,
                            hipStream_t s, float *C2, const XsEpilogue &e, const XsMask *flat) {
  note_path(KP_XS_NN_RING);
  PGCN_CHECK(xstream_ring_ok(K, lda) && N <= 16 && ldc <= 16, PGCN_E_INVALID,
             "xstream ring: K in 577..640, lda = K rounded to 4, N <= 16");
  const XsMask mk = flat && flat->bits ? *flat : XsMask{};
  PGCN_CHECK(!mk.bits || (!maskT && mk.ld >= K && mk.words > 0 && mk.words % 2 == 0),
             PGCN_E_INVALID,
             "xstream ring: one mask, the flat one of >= K bits per row in whole 16-B pieces");
  const int ni = xl_ni(lda);
  const XlRing rg = xl_ring(lda, ni, XL_BT_BYTES, mk.bits ? mk.ld : 0);
  PGCN_CHECK(rg.nslot >= 2, PGCN_E_INVALID, "xstream ring: LDS");
  PGCN_CHECK(!mk.bits || (rg.mb > 1024 && rg.mb <= 2048), PGCN_E_INVALID,
             "xstream ring: the staged keep bits take two LDS-DMA pieces");
  PGCN_CHECK(!e.next_table || ldc == 16, PGCN_E_INVALID,
             "xstream ring: a prescaled table from 16-column rows only");
  const long long n_rg = (M + 15) / 16;
  const dim3 grid((unsigned)std::min<long long>(n_rg, kCUs)),
      block(64 * (XL_NN_LOADERS + XL_NN_CONSUMERS));
  const bool fold = xl_pow2(a_scale);
  const bool masked = maskT || mk.bits;
  const XsDraw dr = e.draw ? *e.draw : XsDraw{};
  PGCN_CHECK(dr.n == 0 || (!masked && dr.n <= 2 && dr.lut), PGCN_E_INVALID,
             "xstream ring: mask draws beside an unmasked product, the nibble tables");
  const dim3 block_d(64 * (XL_NN_LOADERS + XL_NN_CONSUMERS + XL_NN_DRAWERS));
#define XNR_LAUNCH(NI, MS, DU, FO, FL)                                                          \
  PGCN_LAUNCH((k_xs_nn_ring<NI, MS, DU, FO, FL>), grid, block, 0, s, M, N, K, A, lda, B, ldb,   \
              trans_b, C, ldc, maskT, a_scale, C2, e, rg, mk, XsDraw{})
#define XNR_CASE(NI)                                                                           \
  case NI:                                                                                     \
    if (!masked && dr.n > 0)                                                                   \
      PGCN_LAUNCH((k_xs_nn_ring<NI, false, false, false, false, true>), grid, block_d, 0, s, M, \
                  N, K, A, lda, B, ldb, trans_b, C, ldc, maskT, a_scale, C2, e, rg, mk, dr);    \
    else if (!masked)                                                                          \
      XNR_LAUNCH(NI, false, false, false, false);                                              \
    else if (mk.bits) {                                                                        \
      if (C2 && fold) XNR_LAUNCH(NI, true, true, true, true);                                  \
      else if (C2) XNR_LAUNCH(NI, true, true, false, true);                                    \
      else if (fold) XNR_LAUNCH(NI, true, false, true, true);                                  \
      else XNR_LAUNCH(NI, true, false, false, true);                                           \
    } else {                                                                                   \
      if (C2 && fold) XNR_LAUNCH(NI, true, true, true, false);                                 \
      else if (C2) XNR_LAUNCH(NI, true, true, false, false);                                   \
      else if (fold) XNR_LAUNCH(NI, true, false, true, false);                                 \
      else XNR_LAUNCH(NI, true, false, false, false);                                          \
    }                                                                                          \
    break;
  switch (ni) {
    XNR_CASE(37) XNR_CASE(38) XNR_CASE(39) XNR_CASE(40)
    default: PGCN_CHECK(false, PGCN_E_INVALID, "xstream ring: no kernel for this row width");
  }
#undef XNR_CASE
#undef XNR_LAUNCH
}

void launch_xstream_tn_ring(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                            const uint64_t *maskT, float a_scale, float *partial, int n_blocks,
                            hipStream_t s, const XsMask *flat) {
  note_path(KP_XS_TN_RING);
  PGCN_CHECK(xstream_ring_ok(K, lda) && N <= 16, PGCN_E_INVALID,
             "xstream ring: K in 577..640, lda = K rounded to 4, N <= 16");
  const XsMask mk = flat && flat->bits ? *flat : XsMask{};
  PGCN_CHECK(!mk.bits || (!maskT && mk.ld >= K && mk.words > 0 && mk.words % 2 == 0),
             PGCN_E_INVALID,
             "xstream ring: one mask, the flat one of >= K bits per row in whole 16-B pieces");
  const int ni = xl_ni(lda);
  const XlRing rg = xl_ring(lda, ni, 0, mk.bits ? mk.ld : 0);
  PGCN_CHECK(rg.nslot >= 2, PGCN_E_INVALID, "xstream ring: LDS");
  PGCN_CHECK(!mk.bits || (rg.mb > 1024 && rg.mb <= 2048), PGCN_E_INVALID,
             "xstream ring: the staged keep bits take two LDS-DMA pieces");
  const dim3 grid((unsigned)n_blocks),
      block(64 * (XL_TN_LOADERS + XL_TN_CONSUMERS));  // every block writes its partial
  const bool fold = xl_pow2(a_scale);
#define XTR_LAUNCH(NI, MS, FO, FL)                                                              \
  PGCN_LAUNCH((k_xs_tn_ring<NI, MS, FO, FL>), grid, block, 0, s, M, N, K, A, lda, G, ldg,      \
              maskT, a_scale, partial, rg, mk)
#define XTR_CASE(NI)                                                                           \
  case NI:                                                                                     \
    if (mk.bits && fold) XTR_LAUNCH(NI, true, true, true);                                     \
    else if (mk.bits) XTR_LAUNCH(NI, true, false, true);                                       \
    else if (maskT && fold) XTR_LAUNCH(NI, true, true, false);                                 \
    else if (maskT) XTR_LAUNCH(NI, true, false, false);                                        \
    else XTR_LAUNCH(NI, false, false, false);                                                  \
    break;
  switch (ni) {
    XTR_CASE(37) XTR_CASE(38) XTR_CASE(39) XTR_CASE(40)
    default: PGCN_CHECK(false, PGCN_E_INVALID, "xstream ring: no kernel for this row width");
  }
#undef XTR_CASE
#undef XTR_LAUNCH
}

}  // namespace pgcn
