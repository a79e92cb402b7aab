// parallel-gcn_amd/csrc/k_gemm_wide.hip -- the wide "XW" contractions (65..128 output columns:
// the hidden-128 layers of the L-layer model) on fp32 MFMA, register-blocked for gfx950.
//
// Replaces matmul_kernel_forward / matmul_kernel_backward_1 / _2 (src/module.cu:274-472) for
// N in 65..128, where k_gemm_nn / k_gemm_tn (k_gemm.hip: one 16-row group per wave, a B
// operand read from LDS per MFMA) ran at 0.24-0.28 of the fp32 MFMA peak on reddit.
//
// v_mfma_f32_16x16x4_f32 fragment maps as k_gemm.hip: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
// C/D[row=4*(l>>4)+r][col=l&15].  A lane loads 4 consecutive k of one A row as a float4 and
// feeds MFMA t (t = 0..3) with component t, so MFMA t of a 16-wide step reduces k = 4g + t
// over the lane groups g: the same sequence of MFMAs per output tile as k_gemm_nn (steps of
// 16 k ascending, t ascending), i.e. the same sums.
//
//  k_gemm_nn_w : C[M, 16NT] = drop(A)[M, K] B.  Workgroup = 4 waves x 32 rows (128 rows);
//                a wave keeps 2 row tiles x NT column tiles of accumulators, so one A float4
//                feeds 4 NT MFMAs and one B float4 (from LDS) feeds 8.  B^T is staged in LDS in
//                64-k chunks, double-buffered, through registers (the next chunk's global loads
//                fly while the current chunk computes).  2 workgroups per CU.
//  k_gemm_tn_w : partial[slab][K][ldp] = drop(A)[slab rows]^T G.  A wave owns 64 k (one A
//                float4 per lane per 4 rows feeds 4 NT MFMAs); WK waves along k, WR along rows
//                (their partials summed in LDS in wave order); slabs reduced in slab order by
//                the k_gemm.hip reduce (deterministic, no float atomics).
#include "common.hpp"
#include "kernels.hpp"

#include <algorithm>

namespace pgcn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// 4 dropout bits for elements idx..idx+3 of a flat bitmap (may straddle a 64-bit word)
__device__ __forceinline__ uint32_t wmask4(const uint64_t *__restrict__ mask, long long idx) {
  const long long w = idx >> 6;
  const int sh = (int)(idx & 63);
  uint64_t v = mask[w] >> sh;
  if (sh > 60) v |= mask[w + 1] << (64 - sh);
  return (uint32_t)v & 0xfu;
}

// A[row][k .. k+3] (zero past K: the ld padding may hold anything), dropped and scaled
template <bool MASKED>
__device__ __forceinline__ float4 load_a4(const float *__restrict__ arow, long long row, int k,
                                          int K, const uint64_t *__restrict__ a_mask,
                                          long long mask_base, long long mask_ld,
                                          float a_scale) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < K) {
    a = *reinterpret_cast<const float4 *>(arow + k);
    if (k + 4 > K) {
      if (k + 1 >= K) a.y = 0.f;
      if (k + 2 >= K) a.z = 0.f;
      if (k + 3 >= K) a.w = 0.f;
    }
    if constexpr (MASKED) {
      const uint32_t bits = wmask4(a_mask, mask_base + row * mask_ld + k);
      a.x *= (bits & 1) ? a_scale : 0.0f;
      a.y *= (bits & 2) ? a_scale : 0.0f;
      a.z *= (bits & 4) ? a_scale : 0.0f;
      a.w *= (bits & 8) ? a_scale : 0.0f;
    }
  }
  return a;
}

// ------------------------------------------------------------------------------------------
// NN
// ------------------------------------------------------------------------------------------
constexpr int WNN_KC = 64;             // k per LDS chunk of B^T
constexpr int WNN_S = WNN_KC + 4;      // B^T row stride in floats (== 4 mod 64: 2-way at most)
constexpr int WNN_ROWS = 128;          // rows per workgroup (4 waves x 2 tiles x 16)

// Dropout bits of A (MK): 0 none, 1 the flat element-order bitmap (bit mask_base + row *
// mask_ld + k), 2 the nibble layout of k_mask_nibbles (maskT[row][j] nibble c = bits of
// k = 64c + 4j .. +3; K <= 1024).
template <int NT, bool TRANS_B, int MK>
__global__ __launch_bounds__(256, 2) void k_gemm_nn_w(int M, int N, int K,
                                                      const float *__restrict__ A, int lda,
                                                      const float *__restrict__ B, int ldb,
                                                      float *__restrict__ C, int ldc,
                                                      const uint64_t *__restrict__ a_mask,
                                                      long long mask_base, long long mask_ld,
                                                      float a_scale, int nst) {
  constexpr bool MASKED = MK != 0;
  constexpr int NC = 16 * NT;                  // columns of the tile (past N: zero B columns)
  constexpr int NCP = NT <= 4 ? 64 : 128;      // staging width (columns past NC stay unused)
  constexpr int PER = NCP * WNN_KC / 256;      // B elements per thread per chunk
  static_assert(NC <= NCP, "staging covers the tile");
  __shared__ float bt[2][NCP * WNN_S];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i = lane & 15;
  const long long rbase = (long long)blockIdx.x * WNN_ROWS + 32 * w;
  long long row[2];
  const float *arow[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    row[r] = rbase + 16 * r + i;
    const long long rr = row[r] < M ? row[r] : (long long)M - 1;
    row[r] = rr;
    arow[r] = A + rr * (long long)lda;
  }
  floatx4 acc[2][NT];
#pragma unroll
  for (int r = 0; r < 2; r++)
#pragma unroll
    for (int t = 0; t < NT; t++) acc[r][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // B chunk c -> registers, element q of this thread: (j, kk) coalesced along B's rows
  //   B [K][ldb]   : j = tid % NCP, kk = tid / NCP + (256 / NCP) q
  //   B^T [N][ldb] : j = tid / 64 + 4 q, kk = tid % 64
  const int sj = TRANS_B ? tid / 64 : tid % NCP, skk = TRANS_B ? tid % WNN_KC : tid / NCP;
  constexpr int DJ = TRANS_B ? 4 : 0, DK = TRANS_B ? 0 : 256 / NCP;
  // buffer loads: one 32-bit voffset per thread, the q stride in the scalar offset, rows past
  // B's (K rows of B, N rows of B^T) read as 0 by the descriptor's range check
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(B), 0, (int)((long long)(TRANS_B ? N : K) * ldb * 4), 0x00020000);
  float stg[PER];
  auto load_chunk = [&](int c) {
    const int k = c * WNN_KC + skk;
    // a column past N (B) or a k past K (B^T: the ld padding) contributes 0
    const bool ok = TRANS_B ? k < K : sj < N;
    const int voff = 4 * (TRANS_B ? sj * ldb + k : k * ldb + sj);
    const int sq = 4 * (TRANS_B ? DJ * ldb : DK * ldb);
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, voff, sq * q, 0));
      stg[q] = ok ? v : 0.0f;
    }
  };
  auto store_chunk = [&](int buf) {
    float *d = &bt[buf][sj * WNN_S + skk];
#pragma unroll
    for (int q = 0; q < PER; q++) d[(DJ * WNN_S + DK) * q] = stg[q];
  };
  const int nchunks = (K + WNN_KC - 1) / WNN_KC;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  // A: a ring of 4 steps (3 loading while one computes), raw; the K tail and the dropout bits
  // are applied at use.  Dropout bits: per chunk and row tile, the 64-bit window of the flat
  // bitmap at the chunk's first k (loaded a chunk ahead); step s, lane group g takes bits
  // 16 s + 4 g .. +3 of it.
  float4 ar[4][2];
  auto load_raw = [&](int c, int s, float4 (&dst)[2]) {
    const int k = c * WNN_KC + 16 * s + 4 * g;
#pragma unroll
    for (int r = 0; r < 2; r++)
      dst[r] = *reinterpret_cast<const float4 *>(arow[r] + (k < K ? k : 0));  // k >= K: zeroed at use
  };
  // (loads without branches: a value merged with a constant in a divergent branch makes
  // hipcc wait for the load on the spot; the second word's index is clamped to the first
  // when the window does not reach it, i.e. past the bitmap's end, and dropped when combined)
  uint64_t wc[2] = {0, 0}, wn0[2] = {0, 0}, wn1[2] = {0, 0};
  auto load_win = [&](int c) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const long long p0 = mask_base + row[r] * mask_ld;
      const long long p = p0 + (long long)c * WNN_KC;
      const long long lo = p >> 6, last = (p0 + min(K, (c + 1) * WNN_KC) - 1) >> 6;
      wn0[r] = a_mask[lo];
      wn1[r] = a_mask[lo + 1 < last ? lo + 1 : last];
    }
  };
  auto make_win = [&](int c) {  // the window of chunk c from its two words
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const long long p0 = mask_base + row[r] * mask_ld;
      const long long p = p0 + (long long)c * WNN_KC;
      const long long lo = p >> 6, last = (p0 + min(K, (c + 1) * WNN_KC) - 1) >> 6;
      const int sh = (int)(p & 63);
      const uint64_t w1 = lo + 1 <= last ? wn1[r] : 0ull;
      wc[r] = sh ? (wn0[r] >> sh) | (w1 << (64 - sh)) : wn0[r];
    }
  };
  // nibble masks: the lane's words of its two rows, j = 4 s + g (every chunk takes nibble c)
  uint64_t nw[2][4];
  if constexpr (MK == 2) {
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int s = 0; s < 4; s++) nw[r][s] = a_mask[row[r] * 16 + 4 * s + g];
  }
  load_raw(0, 0, ar[0]);
  load_raw(0, 1, ar[1]);
  load_raw(0, 2, ar[2]);
  if constexpr (MK == 1) load_win(0);
  for (int c = 0; c < nchunks; c++) {
    const int buf = c & 1;
    if constexpr (MK == 1) make_win(c);
    if (c + 1 < nchunks) {
      load_chunk(c + 1);  // in flight during this chunk's MFMAs
      if constexpr (MK == 1) load_win(c + 1);
    }
    const bool tail = c * WNN_KC + WNN_KC > K;
    const float *bl = &bt[buf][i * WNN_S + 4 * g];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      // step s + 3 of the stream into the slot step s - 1 left
      {
        const int cc = c + (s + 3) / 4, ss = (s + 3) % 4;
        if (cc < nchunks) load_raw(cc, ss, ar[(s + 3) & 3]);
      }
      float4 av[2] = {ar[s][0], ar[s][1]};
      if (tail) {
        const int k = c * WNN_KC + 16 * s + 4 * g;
#pragma unroll
        for (int r = 0; r < 2; r++) {
          av[r].x = k + 1 > K ? 0.f : av[r].x;
          av[r].y = k + 2 > K ? 0.f : av[r].y;
          av[r].z = k + 3 > K ? 0.f : av[r].z;
          av[r].w = k + 4 > K ? 0.f : av[r].w;
        }
      }
      if constexpr (MASKED) {
#pragma unroll
        for (int r = 0; r < 2; r++) {
          const uint32_t bits = MK == 1 ? (uint32_t)(wc[r] >> (16 * s + 4 * g)) & 0xfu
                                        : (uint32_t)(nw[r][s] >> (4 * c)) & 0xfu;
          av[r].x *= (bits & 1) ? a_scale : 0.0f;
          av[r].y *= (bits & 2) ? a_scale : 0.0f;
          av[r].z *= (bits & 4) ? a_scale : 0.0f;
          av[r].w *= (bits & 8) ? a_scale : 0.0f;
        }
      }
      const float4 a0 = av[0], a1 = av[1];
      if (c * WNN_KC + 16 * s >= K) continue;  // a step wholly past K adds zeros: skipped
      float4 b[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) b[t] = *reinterpret_cast<const float4 *>(bl + 16 * t * WNN_S + 16 * s);
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b[t].x, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b[t].x, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b[t].y, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b[t].y, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b[t].z, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b[t].z, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b[t].w, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b[t].w, acc[1][t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // one step's B reads live at a time
    }
    if (c + 1 < nchunks) store_chunk(buf ^ 1);  // that buffer's last readers passed the barrier
    __syncthreads();
  }
  // lane holds C[rbase + 16 r + 4 g + q][16 t + i]
#pragma unroll
  for (int r = 0; r < 2; r++)
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const int col = 16 * t + i;
      if (col >= nst) continue;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const long long rr = rbase + 16 * r + 4 * g + q;
        if (rr < M) C[rr * ldc + col] = acc[r][t][q];
      }
    }
}

// Persistent NN for K <= 128 (the hidden layers' products and input grads, the output layer):
// all of B^T stays in LDS (one or two 64-k chunks, staged once) and a workgroup walks row
// tiles blockIdx.x, blockIdx.x + gridDim.x, ..; the A ring runs on across tiles, so the next
// tile's first steps load while this tile's last ones compute.  Same MFMA sequence per tile.
template <int NT, bool TRANS_B, int NCH>
__global__ __launch_bounds__(256, 2) void k_gemm_nn_wp(int M, int N, int K,
                                                       const float *__restrict__ A, int lda,
                                                       const float *__restrict__ B, int ldb,
                                                       float *__restrict__ C, int ldc, int nst) {
  constexpr int NCP = NT <= 4 ? 64 : 128;
  constexpr int PER = NCP * WNN_KC / 256;
  constexpr int US = 4 * NCH;  // steps per tile
  __shared__ float bt[NCH][NCP * WNN_S];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i = lane & 15;
  {  // B^T, every chunk, once
    const int sj = TRANS_B ? tid / 64 : tid % NCP, skk = TRANS_B ? tid % WNN_KC : tid / NCP;
    constexpr int DJ = TRANS_B ? 4 : 0, DK = TRANS_B ? 0 : 256 / NCP;
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(B), 0, (int)((long long)(TRANS_B ? N : K) * ldb * 4), 0x00020000);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int k = c * WNN_KC + skk;
      const bool ok = TRANS_B ? k < K : sj < N;
      const int voff = 4 * (TRANS_B ? sj * ldb + k : k * ldb + sj);
      const int sq = 4 * (TRANS_B ? DJ * ldb : DK * ldb);
      float *d = &bt[c][sj * WNN_S + skk];
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, voff, sq * q, 0));
        d[(DJ * WNN_S + DK) * q] = ok ? v : 0.0f;
      }
    }
  }
  const long long ntiles = ((long long)M + WNN_ROWS - 1) / WNN_ROWS;
  auto row_of = [&](long long tile, int r) {
    const long long rr = tile * WNN_ROWS + 32 * w + 16 * r + i;
    return rr < M ? rr : (long long)M - 1;
  };
  float4 ar[4][2];
  // step u of tile `tile` (u < US) into dst
  auto load_step = [&](long long tile, int u, float4 (&dst)[2]) {
    const int k = (u / 4) * WNN_KC + 16 * (u % 4) + 4 * g;
#pragma unroll
    for (int r = 0; r < 2; r++)
      dst[r] = *reinterpret_cast<const float4 *>(A + row_of(tile, r) * (long long)lda +
                                                 (k < K ? k : 0));  // k >= K: zeroed at use
  };
  long long tile = blockIdx.x;
  if (tile < ntiles) {
    load_step(tile, 0, ar[0]);
    load_step(tile, 1, ar[1]);
    load_step(tile, 2, ar[2]);
  }
  __syncthreads();
  for (; tile < ntiles; tile += gridDim.x) {
    floatx4 acc[2][NT];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int t = 0; t < NT; t++) acc[r][t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < US; u++) {
      const int c = u / 4, s = u % 4;
      {  // step u + 3 of the stream (this tile or the next one) into the slot u - 1 left
        const int un = u + 3;
        if (un < US) load_step(tile, un, ar[un & 3]);
        else if (tile + gridDim.x < ntiles) load_step(tile + gridDim.x, un - US, ar[un & 3]);
      }
      float4 av[2] = {ar[u & 3][0], ar[u & 3][1]};
      if (c * WNN_KC + WNN_KC > K) {
        const int k = c * WNN_KC + 16 * s + 4 * g;
#pragma unroll
        for (int r = 0; r < 2; r++) {
          av[r].x = k + 1 > K ? 0.f : av[r].x;
          av[r].y = k + 2 > K ? 0.f : av[r].y;
          av[r].z = k + 3 > K ? 0.f : av[r].z;
          av[r].w = k + 4 > K ? 0.f : av[r].w;
        }
      }
      const float4 a0 = av[0], a1 = av[1];
      const float *bl = &bt[c][i * WNN_S + 4 * g];
      if (c * WNN_KC + 16 * s >= K) continue;  // a step wholly past K adds zeros: skipped
      float4 b[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) b[t] = *reinterpret_cast<const float4 *>(bl + 16 * t * WNN_S + 16 * s);
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b[t].x, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b[t].x, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b[t].y, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b[t].y, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b[t].z, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b[t].z, acc[1][t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b[t].w, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b[t].w, acc[1][t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const long long rbase = tile * WNN_ROWS + 32 * w;
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const int col = 16 * t + i;
        if (col >= nst) continue;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const long long rr = rbase + 16 * r + 4 * g + q;
          if (rr < M) C[rr * ldc + col] = acc[r][t][q];
        }
      }
  }
}

bool gemm_wide_ok(int N) { return N > 32 && N <= 128; }

void launch_gemm_nn_wide(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                         int trans_b, float *C, int ldc, const uint64_t *a_mask,
                         long long mask_base, long long mask_ld, float a_scale, hipStream_t s,
                         int nst, const uint64_t *maskT) {
  PGCN_CHECK(gemm_wide_ok(N), PGCN_E_INVALID, "gemm_nn_wide: N must be in 33..128");
  PGCN_CHECK(!maskT || K <= 1024, PGCN_E_INVALID, "gemm_nn_wide: nibble masks need K <= 1024");
  if (M <= 0) return;
  note_path(KP_GEMM_NN_W);
  const dim3 grid((unsigned)ceil_div(M, WNN_ROWS)), block(256);
  const int nt = (N + 15) / 16;
  if (!a_mask && K <= 2 * WNN_KC) {  // B stays in LDS: persistent row-tile walk
    const long long ntiles = ceil_div(M, WNN_ROWS);
    const dim3 pgrid((unsigned)std::min<long long>(ntiles, 2LL * kCUs));
#define WNP_LAUNCH(T, D, NCH)                                                                \
  PGCN_LAUNCH((k_gemm_nn_wp<T, D, NCH>), pgrid, block, 0, s, M, N, K, A, lda, B, ldb, C, ldc, nst)
#define WNP_CH(T, D) \
  if (K <= WNN_KC) WNP_LAUNCH(T, D, 1); \
  else WNP_LAUNCH(T, D, 2);
#define WNP_T(T) \
  if (trans_b) { WNP_CH(T, true) } else { WNP_CH(T, false) }
    if (nt <= 3) { WNP_T(3) }
    else if (nt == 4) { WNP_T(4) }
    else { WNP_T(8) }
#undef WNP_T
#undef WNP_CH
#undef WNP_LAUNCH
    return;
  }
  const int mk = maskT ? 2 : (a_mask ? 1 : 0);
  const uint64_t *mp = maskT ? maskT : a_mask;
#define WNN_LAUNCH(T, D, MK)                                                                  \
  PGCN_LAUNCH((k_gemm_nn_w<T, D, MK>), grid, block, 0, s, M, N, K, A, lda, B, ldb, C, ldc, mp, \
              mask_base, mask_ld, a_scale, nst)
#define WNN_MK(T, D)                 \
  if (mk == 2) WNN_LAUNCH(T, D, 2);  \
  else if (mk == 1) WNN_LAUNCH(T, D, 1); \
  else WNN_LAUNCH(T, D, 0);
#define WNN_T(T)                \
  if (trans_b) { WNN_MK(T, true) } else { WNN_MK(T, false) }
  if (nt <= 3) { WNN_T(3) }
  else if (nt == 4) { WNN_T(4) }
  else { WNN_T(8) }
#undef WNN_T
#undef WNN_MK
#undef WNN_LAUNCH
}

// ------------------------------------------------------------------------------------------
// TN split-M
// ------------------------------------------------------------------------------------------
// Wave (wk, wr): k = kb .. kb + 63 with kb = 64 (WK * blockIdx.y + wk), rows m = m_begin + 4 wr
// + 4 WR u (u = 0, 1, ..) of the block's slab.  Per step of 4 rows, lane (i, g) loads
// A[m + g][kb + 4i .. +3] and G[m + g][64h + 4i .. +3] (h = 0, 1: two float4), and MFMA (c, t)
// -- output rows k = kb + 4i' + c (i' = the MFMA's row index), columns n = 64 (t / 4) + 4i'' +
// t % 4 (i'' = its column index) -- reduces over the 4 rows g.  A ring of 4 steps: 3 load while
// one computes.
template <int NH, int WK, int MK>
__global__ __launch_bounds__(256, 2) void k_gemm_tn_w(int M, int N, int K, int slab,
                                                      const float *__restrict__ A, int lda,
                                                      const float *__restrict__ G, int ldg,
                                                      const uint64_t *__restrict__ a_mask,
                                                      long long mask_base, long long mask_ld,
                                                      float a_scale, float *__restrict__ partial,
                                                      int ldp) {
  constexpr bool MASKED = MK != 0;
  constexpr int WR = 4 / WK;
  constexpr int NT = 4 * NH;  // NH float4s of G per lane and step: 64 NH columns
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, i = lane & 15;
  const int wk = w % WK, wr = w / WK;
  const int kb = 64 * (WK * (int)blockIdx.y + wk);
  const long long m_begin = (long long)blockIdx.x * slab;
  const long long m_end = m_begin + slab < M ? m_begin + slab : (long long)M;
  floatx4 acc[4][NT];
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int t = 0; t < NT; t++) acc[c][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  // Loads without branches (a value merged with a constant in a divergent branch makes hipcc
  // wait for the load on the spot): clamped addresses, raw values; the row / column / K tails
  // and the dropout bits are applied at compute, when the data has landed.
  struct Step {
    float4 a, b0, b1;
    uint64_t w0, w1;  // mask words of bits p .. p + 3 (w1: the next word, or w0 again)
    int meta;         // row ok (bit 0) | bit offset p % 64 << 1
  };
  const int ka = kb + 4 * i;
  const int n0 = 4 * i, n1 = 64 + 4 * i;  // this lane's G columns (h = 0, 1)
  const int kl = ka < K ? ka : 0;
  const int nl0 = n0 < N ? n0 : 0, nl1 = n1 < N ? n1 : 0;
  auto load = [&](Step &st, long long m) {
    const long long mr = m + g;
    const bool ok = mr < m_end;
    const long long row = ok ? mr : m_end - 1;
    st.a = *reinterpret_cast<const float4 *>(A + row * (long long)lda + kl);
    const float *gr = G + row * (long long)ldg;
    st.b0 = *reinterpret_cast<const float4 *>(gr + nl0);
    if constexpr (NH == 2) st.b1 = *reinterpret_cast<const float4 *>(gr + nl1);
    int sh = 0;
    if constexpr (MK == 2) {
      st.w0 = a_mask[row * 16 + i];  // nibble kb / 64 holds bits ka .. ka + 3
    } else if constexpr (MK == 1) {
      const long long p = mask_base + row * mask_ld + kl;
      const long long lo = p >> 6;
      sh = (int)(p & 63);
      st.w0 = a_mask[lo];
      // the row's last bit's word bounds the second read (past the bitmap's end otherwise)
      const long long last = (mask_base + row * mask_ld + K - 1) >> 6;
      st.w1 = a_mask[lo + 1 < last ? lo + 1 : last];
    }
    st.meta = (ok ? 1 : 0) | sh << 1;
  };
  // full: the step's 4 rows inside the slab (the loop's uniform test) -- then only the K and N
  // tails (uniform per wave) need selects.  Operands are formed before the MFMAs (one write
  // per register: a select rewriting an MFMA's source register while the MFMAs before it
  // read it stalls the issue, r03 counters: 73 % of the wave cycles)
  const bool ktail = kb + 64 > K, ntail = N < 64 * NH;
  auto compute = [&](const Step &st, bool full) {
    float4 a = st.a;
    if (ktail) {
      a.x = ka + 1 <= K ? a.x : 0.f;
      a.y = ka + 2 <= K ? a.y : 0.f;
      a.z = ka + 3 <= K ? a.z : 0.f;
      a.w = ka + 4 <= K ? a.w : 0.f;
    }
    if constexpr (MASKED) {
      const int sh = MK == 2 ? kb / 16 : st.meta >> 1;
      // (bits past K: zero data anyway)
      const uint64_t v =
          (st.w0 >> sh) | (MK == 1 && sh > 60 ? st.w1 << (64 - sh) : 0ull);
      const uint32_t bits = (uint32_t)v & 0xfu;
      a.x *= (bits & 1) ? a_scale : 0.0f;
      a.y *= (bits & 2) ? a_scale : 0.0f;
      a.z *= (bits & 4) ? a_scale : 0.0f;
      a.w *= (bits & 8) ? a_scale : 0.0f;
    }
    float bv[NT];
    bv[0] = st.b0.x;
    bv[1] = st.b0.y;
    bv[2] = st.b0.z;
    bv[3] = st.b0.w;
    if constexpr (NH == 2) {
      bv[4] = st.b1.x;
      bv[5] = st.b1.y;
      bv[6] = st.b1.z;
      bv[7] = st.b1.w;
    }
    if (!full || ntail) {
      const bool ok = st.meta & 1;
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const int col = 64 * (t / 4) + 4 * i + t % 4;
        bv[t] = ok && col < N ? bv[t] : 0.0f;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NT; t++) {
      acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bv[t], acc[0][t], 0, 0, 0);
      acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bv[t], acc[1][t], 0, 0, 0);
      acc[2][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bv[t], acc[2][t], 0, 0, 0);
      acc[3][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bv[t], acc[3][t], 0, 0, 0);
    }
  };
  const long long stride = 4LL * WR;
  long long m = m_begin + 4 * wr;
  if (kb < K && m < m_end) {
    const long long steps = (m_end - m + stride - 1) / stride;
    Step s0, s1, s2, s3;
    load(s0, m);
    load(s1, m + stride);
    load(s2, m + 2 * stride);
    for (long long n = 0; n < steps; n += 4) {
      load(s3, m + 3 * stride);
      __builtin_amdgcn_sched_barrier(0);
      compute(s0, m + 4 <= m_end);
      if (n + 1 >= steps) break;
      load(s0, m + 4 * stride);
      __builtin_amdgcn_sched_barrier(0);
      compute(s1, m + stride + 4 <= m_end);
      if (n + 2 >= steps) break;
      load(s1, m + 5 * stride);
      __builtin_amdgcn_sched_barrier(0);
      compute(s2, m + 2 * stride + 4 <= m_end);
      if (n + 3 >= steps) break;
      load(s2, m + 6 * stride);
      __builtin_amdgcn_sched_barrier(0);
      compute(s3, m + 3 * stride + 4 <= m_end);
      m += 4 * stride;
    }
  }
  // the WR row-waves of one k range meet in LDS (wave order), one column tile at a time
  __shared__ floatx4 red[WR > 1 ? (WR - 1) * WK * 4 * 64 : 1];
  float *p = partial + (long long)blockIdx.x * K * ldp;
#pragma unroll
  for (int t = 0; t < NT; t++) {
    if constexpr (WR > 1) {
      if (wr > 0) {
#pragma unroll
        for (int c = 0; c < 4; c++) red[(((wr - 1) * WK + wk) * 4 + c) * 64 + lane] = acc[c][t];
      }
      __syncthreads();
      if (wr == 0) {
#pragma unroll
        for (int q = 1; q < WR; q++)
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const floatx4 v = red[(((q - 1) * WK + wk) * 4 + c) * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; r++) acc[c][t][r] += v[r];
          }
      }
      __syncthreads();
    }
    if (wr == 0) {
      const int col = 64 * (t / 4) + 4 * i + t % 4;
      if (col < ldp) {
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int k = kb + 4 * (4 * g + r) + c;
            if (k < K) p[(long long)k * ldp + col] = acc[c][t][r];
          }
      }
    }
  }
}

struct TnWidePlan {
  int wk, kgroups, slab, n_slabs, ldp;
};

static TnWidePlan tn_wide_plan(int M, int N, int K) {
  (void)N;
  TnWidePlan p;
  p.ldp = N <= 64 ? 64 : 128;  // the partial's row: all 64 NH columns (zero past N)
  const int nkc = (K + 63) / 64;
  // waves along k: one 64-k chunk each (r03: 4 along k spilled its epilogue, 6.4 vs 0.58 ms)
  p.wk = nkc >= 2 ? 2 : 1;
  p.kgroups = (nkc + p.wk - 1) / p.wk;
  const int wr = 4 / p.wk;
  // ~2 workgroups per CU over all k groups
  long long slab = ceil_div((long long)M * p.kgroups, 2LL * kCUs);
  const int q = 4 * wr;
  slab = (slab + q - 1) / q * q;
  if (slab < 64) slab = 64;
  p.slab = (int)slab;
  p.n_slabs = (int)std::max(1LL, ceil_div((long long)M, slab));
  return p;
}

size_t gemm_tn_wide_workspace(int M, int N, int K) {
  const TnWidePlan p = tn_wide_plan(M, N, K);
  const size_t groups = ((size_t)p.n_slabs + 15) / 16;  // launch_slab_reduce's second level
  return ((size_t)p.n_slabs + groups) * (size_t)K * (size_t)p.ldp * sizeof(float);
}

void launch_gemm_tn_wide(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                         long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                         int nst, const uint64_t *maskT) {
  PGCN_CHECK(gemm_wide_ok(N), PGCN_E_INVALID, "gemm_tn_wide: N must be in 33..128");
  PGCN_CHECK(!maskT || K <= 1024, PGCN_E_INVALID, "gemm_tn_wide: nibble masks need K <= 1024");
  PGCN_CHECK(ldg % 4 == 0 && (reinterpret_cast<size_t>(G) & 15) == 0, PGCN_E_INVALID,
             "gemm_tn_wide: G rows must be 16-B aligned");
  const TnWidePlan p = tn_wide_plan(M, N, K);
  float *partial = static_cast<float *>(workspace);
  if (M > 0) {
    note_path(KP_GEMM_TN_W);
    const dim3 grid((unsigned)p.n_slabs, (unsigned)p.kgroups), block(256);
    const int mk = maskT ? 2 : (a_mask ? 1 : 0);
    const uint64_t *mp = maskT ? maskT : a_mask;
#define WTN_LAUNCH(NH, WK, MK)                                                                 \
  PGCN_LAUNCH((k_gemm_tn_w<NH, WK, MK>), grid, block, 0, s, M, N, K, p.slab, A, lda, G, ldg,   \
              mp, mask_base, mask_ld, a_scale, partial, p.ldp)
#define WTN_MK(NH, WK)                  \
  if (mk == 2) WTN_LAUNCH(NH, WK, 2);     \
  else if (mk == 1) WTN_LAUNCH(NH, WK, 1); \
  else WTN_LAUNCH(NH, WK, 0);
#define WTN_WK(NH)                          \
  if (p.wk == 2) { WTN_MK(NH, 2) } else { WTN_MK(NH, 1) }
    if (N <= 64) { WTN_WK(1) }
    else { WTN_WK(2) }
#undef WTN_WK
#undef WTN_MK
#undef WTN_LAUNCH
  }
  launch_slab_reduce(partial, M > 0 ? p.n_slabs : 0, K, N, p.ldp, C, ldc, nst, s);
}

}  // namespace pgcn
