// parallel-gcn_amd/csrc/k_gemm.hip -- the "XW" contractions on fp32 MFMA for gfx950.
//
// Replaces matmul_kernel_forward / matmul_kernel_backward_1 / matmul_kernel_backward_2
// (src/module.cu:274-472; 16x16 CUDA-core tiles + float atomics) and, for dense feature
// matrices (reddit), sparse_matmul_kernel_forward/backward (:108-163).
//
// All use v_mfma_f32_16x16x4_f32 (exact fp32 inputs, fp32 accumulate). Fragment maps
// (cdna_hip_programming.md §3): A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
// C/D[row=4*(l>>4)+r][col=l&15].
//
//  k_gemm_nn : C[M,N] = drop(A)[M,K] * B   -- A streamed once from HBM straight into
//              registers (a wave owns 16 rows and ALL output columns, so A has no reuse
//              and needs no LDS); B (the small weight) is staged in LDS in K chunks and
//              shared by the block's waves.  The K index inside a 16-wide step is permuted
//              so every lane issues one 16-byte load per step (A[row][k0+4g .. k0+4g+3]).
//  k_gemm_tn : C[K,N] = drop(A)[M,K]^T * G[M,N] -- the long M reduction is split into row
//              slabs; each block writes its slab's partial [K,N] and k_gemm_tn_reduce adds
//              the slabs in slab order => deterministic (no float atomics).
#include "common.hpp"
#include "kernels.hpp"

namespace pgcn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// 4 dropout bits for elements idx..idx+3 (may straddle a 64-bit word)
__device__ __forceinline__ uint32_t mask4(const uint64_t *__restrict__ mask, long long idx) {
  const long long w = idx >> 6;
  const int sh = (int)(idx & 63);
  uint64_t v = mask[w] >> sh;
  if (sh > 60) v |= mask[w + 1] << (64 - sh);
  return (uint32_t)v & 0xfu;
}

// ------------------------------------------------------------------------------------------
// NN: block = 4 waves x 16 rows = 64 rows; NT output tiles of 16 columns per wave.
// ------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void k_gemm_nn(int M, int N, int K,
                                                 const float *__restrict__ A, int lda,
                                                 const float *__restrict__ B, int ldb,
                                                 int trans_b, float *__restrict__ C, int ldc,
                                                 const uint64_t *__restrict__ a_mask,
                                                 long long mask_base, long long mask_ld,
                                                 float a_scale, int nst) {
  // nst: columns of C this launch writes (ldc, or a 128-column slab's share of it)
  constexpr int KC = 64;               // K rows of B per LDS chunk
  constexpr int S = 16 * NT + 4;       // LDS row stride (== 4 mod 8: conflict-free reads)
  __shared__ float bs[KC * S];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const long long row = (long long)blockIdx.x * 64 + w * 16 + i;  // A row this lane loads
  const bool row_ok = row < M;
  const float *arow = A + (row_ok ? row : 0) * (long long)lda;
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += KC) {
    __syncthreads();
    // stage B[k0:k0+KC, 0:16NT] (zero outside [K, N])
    for (int e = threadIdx.x; e < KC * 16 * NT; e += 256) {
      const int kk = e / (16 * NT), j = e - kk * (16 * NT);
      const int k = k0 + kk;
      float val = 0.0f;
      if (k < K && j < N) val = trans_b ? B[(long long)j * ldb + k] : B[(long long)k * ldb + j];
      bs[kk * S + j] = val;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KC / 16; s++) {
      const int kb = k0 + 16 * s + 4 * g;  // this lane's 4 consecutive k
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row_ok && kb < K) {
        a = *reinterpret_cast<const float4 *>(arow + kb);
        if (kb + 3 >= K) {
          if (kb + 1 >= K) a.y = 0.f;
          if (kb + 2 >= K) a.z = 0.f;
          if (kb + 3 >= K) a.w = 0.f;
        }
        if (a_mask) {
          const uint32_t bits = mask4(a_mask, mask_base + row * mask_ld + kb);
          a.x *= (bits & 1) ? a_scale : 0.0f;
          a.y *= (bits & 2) ? a_scale : 0.0f;
          a.z *= (bits & 4) ? a_scale : 0.0f;
          a.w *= (bits & 8) ? a_scale : 0.0f;
        }
      }
      const float *brow = bs + (16 * s + 4 * g) * S + i;
#pragma unroll
      for (int t = 0; t < NT; t++) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, brow[0 * S + 16 * t], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, brow[1 * S + 16 * t], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, brow[2 * S + 16 * t], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, brow[3 * S + 16 * t], acc[t], 0, 0, 0);
      }
    }
  }
  // store: lane holds C[row0 + 4g + r][16t + i]
  const long long crow0 = (long long)blockIdx.x * 64 + w * 16 + 4 * g;
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const int col = 16 * t + i;
    if (col >= nst) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const long long rr = crow0 + r;
      if (rr < M) C[rr * ldc + col] = acc[t][r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// X-stream kernels (N <= 16): the two contractions that read the whole dense feature matrix
// X [M][lda] every training epoch -- Z = drop(X) W (forward) and W.grad = drop(X)^T dZ
// (backward).  X is read once per launch and never reused, so the design goal is bytes in
// flight: operands go straight from HBM to VGPRs (no LDS round trip), many independent
// 16-B loads per wave are issued before the MFMAs that consume them, and the loop keeps
// the next steps' loads outstanding while the current step computes.
//
// Dropout bits come in the "nibble" layout built by k_mask_nibbles from the flat
// element-order bitmap (the order hpdga's xorshift stream draws them, rng.cpp):
//   maskT[m][j] (j = 0..15, uint64) nibble c = keep bits of X[m][64c + 4j .. 64c + 4j + 3]
// so the 4 bits a lane needs for one float4 of row m are one nibble of ONE word it loads
// with the row (K <= 1024).  128 B per row: +5 % over the X row's 2408 B on reddit.
// ------------------------------------------------------------------------------------------
constexpr int XS_MAX_KC = 10;  // K <= 640 (64-wide chunks) for the register-resident paths

__device__ __forceinline__ void apply4(float4 &a, uint32_t bits, float scale) {
  a.x *= (bits & 1) ? scale : 0.0f;
  a.y *= (bits & 2) ? scale : 0.0f;
  a.z *= (bits & 4) ? scale : 0.0f;
  a.w *= (bits & 8) ? scale : 0.0f;
}

// maskT[m][j] from the flat bitmap (bit mask_base + m*mask_ld + k).  A block covers 16 rows:
// their bit range (16 * mask_ld bits, contiguous) is copied to LDS with coalesced loads, then
// thread (row, j) assembles its word from LDS.
constexpr int NIB_ROWS = 16;
constexpr int NIB_WORDS = 16 * 1024 / 64 + 2;  // words of 16 rows of <= 1024 bits (+ edges)

__global__ __launch_bounds__(256) void k_mask_nibbles(const uint64_t *__restrict__ mask,
                                                      long long mask_base, long long mask_ld,
                                                      int M, int K, uint64_t *__restrict__ out) {
  __shared__ uint64_t bits[NIB_WORDS];
  const long long m0 = (long long)blockIdx.x * NIB_ROWS;
  const long long p_first = mask_base + m0 * mask_ld;
  const long long w_first = p_first >> 6;
  const int rows = (int)min((long long)NIB_ROWS, (long long)M - m0);
  const long long p_end = mask_base + (m0 + rows - 1) * mask_ld + K;  // one past the last bit
  // words holding bits [p_first, p_end); a straddling last nibble past K peeks one word
  // further (LDS, never loaded) into bits the K mask clears
  const int n_words = (int)(((p_end + 63) >> 6) - w_first);
  for (int i = threadIdx.x; i < n_words; i += 256) bits[i] = mask[w_first + i];
  __syncthreads();
  const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
  if (r >= rows) return;
  const long long p0 = mask_base + (m0 + r) * mask_ld + 4 * j - (w_first << 6);  // local bit
  // nibble c sits at bit p0 + 64 c: word w0 + c, the same shift sh for every c (r03 late:
  // one LDS word per nibble, the next nibble's low word reused as this one's high word)
  const int w0 = (int)(p0 >> 6), sh = (int)(p0 & 63);
  const int nc = (K - 4 * j + 63) >> 6;  // nibbles with kb = 64 c + 4 j < K
  uint64_t word = 0, lo = bits[w0];
#pragma unroll
  for (int c = 0; c < 16; c++) {
    if (c < nc) {
      const uint64_t hi = bits[w0 + c + 1];
      uint64_t nib = (lo >> sh) & 0xfu;
      if (sh > 60) nib = (nib | (hi << (64 - sh))) & 0xfu;
      const int kb = 64 * c + 4 * j;
      if (kb + 4 > K) nib &= (1ull << (K - kb)) - 1;  // keep bits of k >= K are 0
      word |= nib << (4 * c);
      lo = hi;
    }
  }
  out[(m0 + r) * 16 + j] = word;
}

// NN: Z[M][N<=16] = drop(X) W.  A wave owns a 16-row group at a time (grid-stride over
// groups) and issues all of the group's A loads (one float4 per lane per 16-wide k-step:
// lane (i, g) reads X[row i][16 s + 4 g ..]) before its first MFMA; 2 waves per SIMD keep one
// group's loads in flight while the other computes.  B^T lives in LDS for the block's life:
// bt[j][k], row stride S = 8 mod 16 dwords, so the per-step float4 B operand read
// bt[i][16 s + 4 g ..] is conflict-free.  MFMA t of step s reduces k = 16 s + 4 g + t.
// DUAL (with MASKED): C = X W and C2 = drop(X) W from one pass over X -- the eval forward and
// the next training forward of the first layer share their weights (no optimizer step between
// them), so the engine computes both while X streams by once.  C2's MFMAs see exactly the
// operands of the MASKED kernel, in the same order: bit-identical to it.
template <int KC, bool MASKED, bool DUAL = false>
__global__ __launch_bounds__(256, 2) void k_xstream_nn(int M, int N, int K, int S,
                                                       const float *__restrict__ A, int lda,
                                                       const float *__restrict__ B, int ldb,
                                                       int trans_b, float *__restrict__ C,
                                                       int ldc, const uint64_t *__restrict__ maskT,
                                                       float a_scale, float *__restrict__ C2,
                                                       XsEpilogue epi) {
  static_assert(!DUAL || MASKED, "dual: the second product is the masked one");
  constexpr int NS = 4 * KC;  // 16-wide k-steps (the last ones may be past K)
  extern __shared__ float bt[];
  for (int e = threadIdx.x; e < 16 * NS * 16; e += 256) {
    const int k = e >> 4, j = e & 15;
    float v = 0.0f;
    if (k < K && j < N) v = trans_b ? B[(long long)j * ldb + k] : B[(long long)k * ldb + j];
    bt[j * S + k] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16;
  const long long wstride = (long long)gridDim.x * 4;
  const float *bl = bt + i * S + 4 * g;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (long long rg = (long long)blockIdx.x * 4 + w; rg < n_rg; rg += wstride) {
    const long long row = rg * 16 + i;
    const bool row_ok = row < M;
    const float *arow = A + (row_ok ? row : 0) * (long long)lda + 4 * g;
    float4 a[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
      a[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row_ok && 16 * s + 4 * g < K) a[s] = *reinterpret_cast<const float4 *>(arow + 16 * s);
    }
    uint64_t mw[4] = {0, 0, 0, 0};
    if constexpr (MASKED) {
      if (row_ok) {
#pragma unroll
        for (int q = 0; q < 4; q++) mw[q] = maskT[row * 16 + 4 * q + g];
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the B reads out of the load phase (VGPRs)
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f}, acc2 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const int kb = 16 * s + 4 * g;
      if (16 * s + 16 > K) {  // k >= K lanes of the tail steps (A's ld padding, may be NaN)
        if (kb + 1 > K) a[s].x = 0.f;
        if (kb + 2 > K) a[s].y = 0.f;
        if (kb + 3 > K) a[s].z = 0.f;
        if (kb + 4 > K) a[s].w = 0.f;
      }
      const float4 b = *reinterpret_cast<const float4 *>(bl + 16 * s);
      if constexpr (DUAL) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].z, b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].w, b.w, acc, 0, 0, 0);
      }
      if constexpr (MASKED)
        apply4(a[s], (uint32_t)(mw[s & 3] >> (4 * (s >> 2))) & 0xfu, a_scale);
      floatx4 &am = DUAL ? acc2 : acc;
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].x, b.x, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].y, b.y, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].z, b.z, am, 0, 0, 0);
      am = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s].w, b.w, am, 0, 0, 0);
    }
    // lane holds C[16 rg + 4g + r][i]
    if (i < ldc) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const long long rr = rg * 16 + 4 * g + r;
        if (rr < M) {
          float c = acc[r];
          if constexpr (!DUAL) {
            if (epi.bwd_drop) {
              const long long b = epi.drop_base + rr * ldc + i;
              c *= ((epi.bwd_drop[b >> 6] >> (b & 63)) & 1) ? epi.drop_scale : 0.0f;
            }
            if (epi.bwd_relu && !epi.bwd_relu[rr * ldc + i]) c = 0.0f;
            if (epi.relu && !(c > 0.0f)) c = 0.0f;  // k_relu_fwd's test (NaN -> 0)
            if (epi.next_table) {  // k_ring_prescale of the stored value: s_r * C[r][i]
              const long long sr = epi.next_sr;
              float *t = reinterpret_cast<float *>(epi.next_table +
                                                   (rr / sr) * 4 * sr + (i >> 2) * sr + rr % sr);
              t[i & 3] = c * epi.next_scale[rr];
            }
          }
          C[rr * ldc + i] = c;
          if constexpr (DUAL) C2[rr * ldc + i] = acc2[r];
        }
      }
    }
  }
}

// TN: W.grad[K][N<=16] = drop(X)^T G.  A wave owns ALL K columns of 4 rows per step (one
// step = 4 whole rows, contiguous); lane (i, g) holds X[m+g][64c + 4i ..] for chunk c and
// feeds MFMA (c, t) with output row k = 64c + 4i + t, reduction index = row g; its keep bits
// are nibble c of maskT[m+g][i] and its B operand G[m+g][i].  Steps are dealt round-robin to
// the grid's waves; three register sets keep steps n+1 and n+2 loading while n computes.
// Each block sums its 4 waves in LDS in wave order and writes one [K][16] partial; the
// partials are reduced in block order (k_slab_reduce1 / k_gemm_tn_reduce): deterministic.
template <int KC, bool MASKED>
struct TnStep {
  float4 a[KC];
  uint64_t mw;
  float bj;
  // Unconditional loads (no exec branches): rows past M read row M-1 and get bj = 0; the
  // columns of a lane past K read inside the row (clamped) and are zeroed in tn_compute.
  __device__ __forceinline__ void load(long long m, long long M, int g, int i, int K,
                                       const float *__restrict__ A, int lda,
                                       const float *__restrict__ G, int ldg, int N,
                                       const uint64_t *__restrict__ maskT) {
    const long long mr = m + g;
    const bool ok = mr < M;
    const long long row = ok ? mr : M - 1;
    const float *ar = A + row * (long long)lda;
#pragma unroll
    for (int c = 0; c < KC; c++) {
      int kb = 64 * c + 4 * i;
      kb = kb < lda - 4 ? kb : lda - 4;
      a[c] = *reinterpret_cast<const float4 *>(ar + kb);
    }
    const float gv = G[row * ldg + (i < N ? i : 0)];
    bj = (ok && i < N) ? gv : 0.0f;
    if constexpr (MASKED) mw = maskT[row * 16 + i];
  }
};

template <int KC, bool MASKED>
__device__ __forceinline__ void tn_compute(TnStep<KC, MASKED> &st, floatx4 (&acc)[KC][4], int i,
                                           int K, float a_scale) {
#pragma unroll
  for (int c = 0; c < KC; c++) {
    float4 x = st.a[c];
    const int kb = 64 * c + 4 * i;
    if (64 * c + 64 > K) {
      if (kb + 1 > K) x.x = 0.f;
      if (kb + 2 > K) x.y = 0.f;
      if (kb + 3 > K) x.z = 0.f;
      if (kb + 4 > K) x.w = 0.f;
    }
    if constexpr (MASKED) apply4(x, (uint32_t)(st.mw >> (4 * c)) & 0xfu, a_scale);
    acc[c][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, st.bj, acc[c][0], 0, 0, 0);
    acc[c][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, st.bj, acc[c][1], 0, 0, 0);
    acc[c][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, st.bj, acc[c][2], 0, 0, 0);
    acc[c][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, st.bj, acc[c][3], 0, 0, 0);
  }
}

// register sets in flight per wave in k_xstream_tn: 3 = steps n+1 and n+2 load while step n
// computes (480 of the 512 registers at KC = 10, accumulators in AGPRs); 2 = one step ahead
#ifndef PGCN_TN_SETS
#define PGCN_TN_SETS 3
#endif
constexpr int XS_TN_BLOCKS = 256;  // one 4-wave block per CU (1 wave per SIMD, ~300 registers)
// small products (<= XS_TN_SMALL_ROWS rows: the small graphs' layers) take 32 blocks, whose
// partials one ordered pass reduces (r04 late: one launch fewer per call; the blocks' steps
// stay a few per wave; 64 blocks measured equal, 16 slower: profiles/r04/ab_tn_small_blocks.txt)
#ifndef PGCN_TN_SMALL_BLOCKS
#define PGCN_TN_SMALL_BLOCKS 32
#endif
constexpr int XS_TN_SMALL_ROWS = 16384, XS_TN_SMALL_BLOCKS = PGCN_TN_SMALL_BLOCKS,
              TN_ONE_PASS = XS_TN_SMALL_BLOCKS > 32 ? XS_TN_SMALL_BLOCKS : 32;

template <int KC, bool MASKED>
__global__ __launch_bounds__(256, 1) void k_xstream_tn(int M, int N, int K,
                                                       const float *__restrict__ A, int lda,
                                                       const float *__restrict__ G, int ldg,
                                                       const uint64_t *__restrict__ maskT,
                                                       float a_scale, float *__restrict__ partial) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, i = lane & 15;
  floatx4 acc[KC][4];
#pragma unroll
  for (int c = 0; c < KC; c++)
#pragma unroll
    for (int t = 0; t < 4; t++) acc[c][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  const long long stride = (long long)gridDim.x * 4 * 4;  // rows between a wave's steps
  const long long n_steps = (M + 3) / 4;
  const long long wid = (long long)blockIdx.x * 4 + w;
  const long long my_steps = wid < n_steps ? (n_steps - wid + gridDim.x * 4 - 1) / (gridDim.x * 4) : 0;
  long long m = wid * 4;
#if PGCN_TN_SETS == 3
  // three register sets: steps n+1 and n+2 load while step n computes
  TnStep<KC, MASKED> s0, s1, s2;
  s0.load(m, M, g, i, K, A, lda, G, ldg, N, maskT);
  s1.load(m + stride, M, g, i, K, A, lda, G, ldg, N, maskT);
  for (long long n = 0; n < my_steps; n += 3) {
    s2.load(m + 2 * stride, M, g, i, K, A, lda, G, ldg, N, maskT);
    __builtin_amdgcn_sched_barrier(0);
    tn_compute(s0, acc, i, K, a_scale);
    s0.load(m + 3 * stride, M, g, i, K, A, lda, G, ldg, N, maskT);
    __builtin_amdgcn_sched_barrier(0);
    tn_compute(s1, acc, i, K, a_scale);
    s1.load(m + 4 * stride, M, g, i, K, A, lda, G, ldg, N, maskT);
    __builtin_amdgcn_sched_barrier(0);
    tn_compute(s2, acc, i, K, a_scale);
    m += 3 * stride;
  }
#else
  // two register sets: step n+1 loads while step n computes
  TnStep<KC, MASKED> s0, s1;
  s0.load(m, M, g, i, K, A, lda, G, ldg, N, maskT);
  for (long long n = 0; n < my_steps; n += 2) {
    s1.load(m + stride, M, g, i, K, A, lda, G, ldg, N, maskT);
    __builtin_amdgcn_sched_barrier(0);
    tn_compute(s0, acc, i, K, a_scale);
    // (past the wave's last step s1 holds zeros: its MFMAs add nothing)
    s0.load(m + 2 * stride, M, g, i, K, A, lda, G, ldg, N, maskT);
    __builtin_amdgcn_sched_barrier(0);
    tn_compute(s1, acc, i, K, a_scale);
    m += 2 * stride;
  }
#endif
  // waves 1..3 hand their chunk tiles to wave 0 through LDS (fixed order)
  __shared__ float red[3 * 64 * 16];
  float *p = partial + (long long)blockIdx.x * K * 16;
#pragma unroll
  for (int c = 0; c < KC; c++) {
    if (w > 0) {
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) red[((w - 1) * 64 + lane) * 16 + t * 4 + r] = acc[c][t][r];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        floatx4 v = acc[c][t];
#pragma unroll
        for (int q = 0; q < 3; q++)
#pragma unroll
          for (int r = 0; r < 4; r++) v[r] += red[(q * 64 + lane) * 16 + t * 4 + r];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int k = 64 * c + 4 * (4 * g + r) + t;
          if (k < K) p[(long long)k * 16 + i] = v[r];
        }
      }
    }
    __syncthreads();
  }
}


// ------------------------------------------------------------------------------------------
// TN split-M.  Block = 4 waves over a slab of rows; the K columns are cut into 64-wide chunks.
// Wave layout: WK waves along K x (4/WK) waves along rows.  Per step of 4 rows a lane
// (g = lane>>4, i = lane&15) loads ONE float4 A[m+g][kc*64 + 4i .. +3] (a wave reads 4 rows
// x 256 contiguous bytes) and feeds 4 MFMAs: MFMA t's A-operand row i is k = kc*64 + 4i + t,
// its reduction index is the row g.  Partials go to partial[slab][k][ldp].
// ------------------------------------------------------------------------------------------
constexpr int TN_U = 2;  // row steps whose loads are in flight together

template <int NJ, int KCW, int WK>
__global__ __launch_bounds__(256) void k_gemm_tn(int M, int N, int K, int slab,
                                                 const float *__restrict__ A, int lda,
                                                 const float *__restrict__ G, int ldg,
                                                 const uint64_t *__restrict__ a_mask,
                                                 long long mask_base, long long mask_ld,
                                                 float a_scale, float *__restrict__ partial,
                                                 int ldp) {
  constexpr int WR = 4 / WK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int wk = w % WK, wr = w / WK;
  const int c0 = (int)blockIdx.y * WK * KCW;  // first 64-wide K chunk of this block
  const long long m_begin = (long long)blockIdx.x * slab;
  long long m_end = m_begin + slab;
  if (m_end > M) m_end = M;
  floatx4 acc[KCW][4][NJ];
#pragma unroll
  for (int c = 0; c < KCW; c++)
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int j = 0; j < NJ; j++) acc[c][t][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // TN_U row steps per iteration: all their loads are issued before any MFMA consumes them
  for (long long m0 = m_begin + 4 * wr; m0 < m_end; m0 += 4 * WR * TN_U) {
    float b[TN_U][NJ];
    float4 a[TN_U][KCW];
#pragma unroll
    for (int u = 0; u < TN_U; u++) {
      const long long mr = m0 + 4 * WR * u + g;
      const bool ok = mr < m_end;
#pragma unroll
      for (int j = 0; j < NJ; j++) {
        const int col = 16 * j + i;
        b[u][j] = (ok && col < N) ? G[mr * ldg + col] : 0.0f;
      }
#pragma unroll
      for (int c = 0; c < KCW; c++) {
        const int kb = (c0 + wk + WK * c) * 64 + 4 * i;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok && kb < K) {
          x = *reinterpret_cast<const float4 *>(A + mr * lda + kb);
          if (kb + 1 >= K) x.y = 0.f;
          if (kb + 2 >= K) x.z = 0.f;
          if (kb + 3 >= K) x.w = 0.f;
          if (a_mask) {
            const uint32_t bits = mask4(a_mask, mask_base + mr * mask_ld + kb);
            x.x *= (bits & 1) ? a_scale : 0.0f;
            x.y *= (bits & 2) ? a_scale : 0.0f;
            x.z *= (bits & 4) ? a_scale : 0.0f;
            x.w *= (bits & 8) ? a_scale : 0.0f;
          }
        }
        a[u][c] = x;
      }
    }
#pragma unroll
    for (int u = 0; u < TN_U; u++)
#pragma unroll
      for (int c = 0; c < KCW; c++)
#pragma unroll
        for (int j = 0; j < NJ; j++) {
          acc[c][0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][c].x, b[u][j], acc[c][0][j], 0, 0, 0);
          acc[c][1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][c].y, b[u][j], acc[c][1][j], 0, 0, 0);
          acc[c][2][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][c].z, b[u][j], acc[c][2][j], 0, 0, 0);
          acc[c][3][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][c].w, b[u][j], acc[c][3][j], 0, 0, 0);
        }
  }
  // row-group partial sums of one block meet in LDS (fixed order), then one slab partial
  __shared__ float red[WR > 1 ? 4 * 64 * 16 : 1];
  float *p = partial + (long long)blockIdx.x * K * ldp;
#pragma unroll
  for (int c = 0; c < KCW; c++) {
#pragma unroll
    for (int j = 0; j < NJ; j++) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        floatx4 v = acc[c][t][j];
        if constexpr (WR > 1) {
          __syncthreads();
#pragma unroll
          for (int r = 0; r < 4; r++) red[(w * 64 + lane) * 4 + r] = v[r];
          __syncthreads();
          if (wr == 0) {
#pragma unroll
            for (int q = 1; q < WR; q++)
#pragma unroll
              for (int r = 0; r < 4; r++) v[r] += red[((wk + WK * q) * 64 + lane) * 4 + r];
          }
        }
        if (wr == 0) {
          const int col = 16 * j + i;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int k = (c0 + wk + WK * c) * 64 + 4 * (4 * g + r) + t;
            if (k < K && col < ldp) p[(long long)k * ldp + col] = v[r];
          }
        }
      }
    }
  }
}

// pass 1: part2[rg][e] = sum of slabs [rg*SPG, (rg+1)*SPG) of element e (slab order)
__global__ __launch_bounds__(256) void k_slab_reduce1(const float *__restrict__ partial,
                                                      int n_slabs, long long elems, int spg,
                                                      float *__restrict__ part2) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= elems) return;
  const int s0 = blockIdx.y * spg, s1 = min(n_slabs, s0 + spg);
  float s = 0.0f;
  // loads in batches of 16 before their (ordered) adds: one memory latency per batch
  for (int b0 = s0; b0 < s1; b0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = b0 + u < s1 ? partial[(long long)(b0 + u) * elems + e] : 0.0f;
#pragma unroll
    for (int u = 0; u < 16; u++)
      if (b0 + u < s1) s += v[u];
  }
  part2[(long long)blockIdx.y * elems + e] = s;
}

// pass 2: C[k][j] = sum over groups in order
__global__ __launch_bounds__(256) void k_gemm_tn_reduce(const float *__restrict__ part2,
                                                        int n_groups, int K, int N, int ldp,
                                                        float *__restrict__ C, int ldc, int nst) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)K * ldp) return;
  const int k = (int)(e / ldp), j = (int)(e - (long long)k * ldp);
  float s = 0.0f;
  // loads in batches of 16 before their (ordered) adds: one memory latency per batch
  const long long stride = (long long)K * ldp;
  for (int b0 = 0; b0 < n_groups; b0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = b0 + u < n_groups ? part2[(b0 + u) * stride + e] : 0.0f;
#pragma unroll
    for (int u = 0; u < 16; u++)
      if (b0 + u < n_groups) s += v[u];
  }
  if (j < nst) C[(long long)k * ldc + j] = j < N ? s : 0.0f;
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
bool xstream_ok(int N, int K) {
  return N >= 1 && N <= 16 && K >= 1 && (K + 63) / 64 <= XS_MAX_KC;
}

static int xs_stride(int K) {  // LDS row stride of B^T: >= 64*KC, = 8 mod 16 dwords
  int s = (K + 63) / 64 * 64;
  while (s % 16 != 8) s += 8;
  return s;
}

void launch_mask_nibbles(const uint64_t *mask, long long mask_base, long long mask_ld, int M,
                         int K, uint64_t *out, hipStream_t s) {
  PGCN_CHECK(K >= 1 && K <= 1024, PGCN_E_INVALID, "mask_nibbles: K must be in [1,1024]");
  if (M <= 0) return;
  PGCN_CHECK(mask_ld >= K && mask_ld <= 1024, PGCN_E_INVALID, "mask_nibbles: K <= mask_ld <= 1024");
  PGCN_LAUNCH(k_mask_nibbles, dim3((unsigned)ceil_div(M, NIB_ROWS)), dim3(256), 0, s, mask,
                     mask_base, mask_ld, M, K, out);
}

void launch_xstream_nn(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                       int trans_b, float *C, int ldc, const uint64_t *maskT, float a_scale,
                       hipStream_t s, float *C2, const XsEpilogue *epi, const XsMask *flat) {
  const XsEpilogue none{};
  const bool fl = flat && flat->bits;
  const XsEpilogue &e = epi ? *epi : none;
  PGCN_CHECK(!C2 || (!e.relu && !e.next_table && !e.bwd_drop && !e.bwd_relu), PGCN_E_INVALID,
             "xstream_nn: dual + epilogue");
  PGCN_CHECK(!e.next_table || (N <= 16 && ldc == 16), PGCN_E_INVALID,
             "xstream_nn: a staged table needs 16-column rows");
  PGCN_CHECK(xstream_ok(N, K), PGCN_E_INVALID, "xstream_nn: needs N <= 16, K <= 640");
  PGCN_CHECK(!C2 || maskT || fl, PGCN_E_INVALID, "xstream_nn: the dual product needs the mask");
  PGCN_CHECK(!fl || xstream_ring_ok(K, lda), PGCN_E_INVALID,
             "xstream_nn: a flat mask on the ring kernels' shapes only");
  PGCN_CHECK(lda % 4 == 0 && lda >= K, PGCN_E_INVALID, "gemm: lda must be a multiple of 4 >= K");
  if (M <= 0) return;
  if (xstream_ring_ok(K, lda)) {
    PGCN_CHECK(!e.bwd_drop && !e.bwd_relu, PGCN_E_INVALID, "xstream_nn: backward tails on the ring form");
    launch_xstream_nn_ring(M, N, K, A, lda, B, ldb, trans_b, C, ldc, maskT, a_scale, s, C2, e,
                           flat);
    return;
  }
  note_path(KP_XS_NN);
  const int kc = (K + 63) / 64, S = xs_stride(K);
  const long long n_rg = ceil_div(M, 16);
  const long long wgs = std::min<long long>(ceil_div(n_rg, 4), 2 * kCUs);
  const dim3 grid((unsigned)wgs), block(256);
  const size_t lds = (size_t)16 * S * sizeof(float);
#define XNN_CASE(KC)                                                                          \
  case KC:                                                                                    \
    if (C2)                                                                                   \
      PGCN_LAUNCH((k_xstream_nn<KC, true, true>), grid, block, lds, s, M, N, K, S, A,  \
                         lda, B, ldb, trans_b, C, ldc, maskT, a_scale, C2, e);                \
    else if (maskT)                                                                           \
      PGCN_LAUNCH((k_xstream_nn<KC, true>), grid, block, lds, s, M, N, K, S, A, lda, B, \
                         ldb, trans_b, C, ldc, maskT, a_scale, nullptr, e);                   \
    else                                                                                      \
      PGCN_LAUNCH((k_xstream_nn<KC, false>), grid, block, lds, s, M, N, K, S, A, lda,   \
                         B, ldb, trans_b, C, ldc, maskT, a_scale, nullptr, e);                \
    break;
  switch (kc) {
    XNN_CASE(1) XNN_CASE(2) XNN_CASE(3) XNN_CASE(4) XNN_CASE(5)
    XNN_CASE(6) XNN_CASE(7) XNN_CASE(8) XNN_CASE(9) XNN_CASE(10)
  }
#undef XNN_CASE
}

static void gemm_nn_slab(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                         int trans_b, float *C, int ldc, const uint64_t *a_mask,
                         long long mask_base, long long mask_ld, float a_scale, hipStream_t s,
                         int nst, const uint64_t *maskT);

void launch_gemm_nn(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                    int trans_b, float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                    long long mask_ld, float a_scale, hipStream_t s, const uint64_t *maskT) {
  PGCN_CHECK(lda % 4 == 0 && lda >= K, PGCN_E_INVALID, "gemm: lda must be a multiple of 4 >= K");
  PGCN_CHECK(N >= 1, PGCN_E_INVALID, "gemm: N must be >= 1");
  if (M <= 0) return;
  if (N > 128) {  // wide outputs (PART2 hidden 600): 128-column slabs of B and C, each slab
    // writing its own columns only (the last one also C's padding columns)
    for (int j0 = 0; j0 < N; j0 += 128)
      gemm_nn_slab(M, std::min(128, N - j0), K, A, lda,
                   trans_b ? B + (long long)j0 * ldb : B + j0, ldb, trans_b, C + j0, ldc, a_mask,
                   mask_base, mask_ld, a_scale, s, j0 + 128 >= N ? ldc - j0 : 128, maskT);
    return;
  }
  gemm_nn_slab(M, N, K, A, lda, B, ldb, trans_b, C, ldc, a_mask, mask_base, mask_ld, a_scale, s,
               ldc, maskT);
}

static void gemm_nn_slab(int M, int N, int K, const float *A, int lda, const float *B, int ldb,
                         int trans_b, float *C, int ldc, const uint64_t *a_mask,
                         long long mask_base, long long mask_ld, float a_scale, hipStream_t s,
                         int nst, const uint64_t *maskT) {
  if (!a_mask && xstream_ok(N, K) && nst == ldc) {
    launch_xstream_nn(M, N, K, A, lda, B, ldb, trans_b, C, ldc, nullptr, 1.0f, s, nullptr);
    return;
  }
  if (gemm_wide_ok(N)) {
    launch_gemm_nn_wide(M, N, K, A, lda, B, ldb, trans_b, C, ldc, a_mask, mask_base, mask_ld,
                        a_scale, s, nst, a_mask && K <= 1024 ? maskT : nullptr);
    return;
  }
  note_path(KP_GEMM_NN);
  const int nt = (N + 15) / 16;
  const dim3 grid((unsigned)ceil_div(M, 64)), block(256);
#define NN_CASE(T)                                                                            \
  case T:                                                                                     \
    PGCN_LAUNCH(k_gemm_nn<T>, grid, block, 0, s, M, N, K, A, lda, B, ldb, trans_b, C, \
                       ldc, a_mask, mask_base, mask_ld, a_scale, nst);                        \
    break;
  switch (nt) {
    NN_CASE(1) NN_CASE(2) NN_CASE(3) NN_CASE(4) NN_CASE(5) NN_CASE(6) NN_CASE(7) NN_CASE(8)
  }
#undef NN_CASE
}

struct TnPlan {
  int nj, nkc, wk, kcw, kgroups, slab, n_slabs, ldp, spg, n_groups;
};

static TnPlan tn_plan(int M, int N, int K) {
  TnPlan p;
  p.nj = (N + 15) / 16;
  p.ldp = p.nj * 16;
  p.nkc = (K + 63) / 64;
  p.wk = p.nkc >= 4 ? 4 : (p.nkc >= 2 ? 2 : 1);
  p.kcw = std::min(3, (p.nkc + p.wk - 1) / p.wk);
  if (p.nj > 4) p.kcw = 1;  // accumulators: 16 * kcw * nj registers (instantiated: kcw 1)
  p.kgroups = (p.nkc + p.wk * p.kcw - 1) / (p.wk * p.kcw);
  const int wr = 4 / p.wk;
  long long slab = ceil_div(M, 1024);  // ~4 blocks per CU: memory parallelism for the stream
  const int q = 4 * wr * TN_U;
  slab = (slab + q - 1) / q * q;
  if (slab < 64) slab = 64;
  p.slab = (int)slab;
  p.n_slabs = (int)std::max(1LL, ceil_div(M, slab));
  p.spg = 16;
  p.n_groups = (p.n_slabs + p.spg - 1) / p.spg;
  return p;
}

static int xs_tn_blocks(int M, int K, int lda) {
  return M <= XS_TN_SMALL_ROWS && !xstream_ring_ok(K, lda) ? XS_TN_SMALL_BLOCKS : XS_TN_BLOCKS;
}

static TnPlan xs_tn_plan(int K, int blocks) {  // k_xstream_tn: one [K][16] partial per block
  TnPlan p{};
  p.nj = 1;
  p.ldp = 16;
  p.nkc = (K + 63) / 64;
  p.n_slabs = blocks;
  p.spg = 16;
  p.n_groups = (p.n_slabs + p.spg - 1) / p.spg;
  return p;
}

static size_t plan_bytes(const TnPlan &p, int K) {
  return ((size_t)p.n_slabs + (size_t)p.n_groups) * (size_t)K * (size_t)p.ldp * sizeof(float);
}

size_t gemm_tn_workspace(int M, int N, int K) {
  N = std::min(N, 128);  // wider outputs run in 128-column slabs
  size_t ws = plan_bytes(tn_plan(M, N, K), K);  // either kernel family may run
  if (gemm_wide_ok(N)) ws = std::max(ws, gemm_tn_wide_workspace(M, N, K));
  if (N <= 16) ws = std::max(ws, plan_bytes(xs_tn_plan(K, XS_TN_BLOCKS), K));
  return ws;
}

static thread_local TnDeferList *g_tn_defer = nullptr;

void tn_defer(TnDeferList *list) { g_tn_defer = list; }

void tn_defer_flush(TnDeferList &list, hipStream_t s) {
  for (int i = 0; i < list.n; i++) {
    const TnDeferred &d = list.d[i];
    if (!d.src) continue;
    const long long elems = (long long)d.K * d.ldp;
    PGCN_LAUNCH(k_gemm_tn_reduce, dim3((unsigned)ceil_div(elems, 256)), dim3(256), 0, s, d.src,
                d.n_groups, d.K, d.N, d.ldp, d.C, d.N, d.N);
  }
  list.n = 0;
  list.used = 0;
}

// the deferred list's room for a first pass of `floats` outputs, or null (launch as usual)
static float *tn_defer_room(int N, int ldc, int nst, size_t floats) {
  TnDeferList *l = g_tn_defer;
  if (!l || l->n >= 4 || ldc != N || nst != N || !l->pool) return nullptr;
  const size_t at = (l->used + 63) / 64 * 64;
  if (at + floats > l->pool_floats) return nullptr;
  l->used = at + floats;
  return l->pool + at;
}

// ordered two-pass reduction of p.n_slabs partials [K][ldp] into C[K][ldc]
// One pass over the partials when they fit one first-pass group (the same sequential sum the
// two passes form), or up to `one_pass` partials (the small X-stream TN plan only: its 32 block
// partials in one sequential sum, r04 late -- another grouping than two passes of 16)
static void tn_reduce(const TnPlan &p, int M, int N, int K, float *partial, float *C, int ldc,
                      hipStream_t s, int nst = -1, int one_pass = 0) {
  if (nst < 0) nst = ldc;
  float *part2 = partial + (size_t)p.n_slabs * K * p.ldp;
  const long long elems = (long long)K * p.ldp;
  if (M > 0 && p.n_slabs <= std::max(one_pass, p.spg)) {  // one ordered pass over the partials
    PGCN_LAUNCH(k_gemm_tn_reduce, dim3((unsigned)ceil_div(elems, 256)), dim3(256), 0, s,
                partial, p.n_slabs, K, N, p.ldp, C, ldc, nst);
    return;
  }
  // tn_defer: the first pass's group sums into the deferred list's pool, the last pass left to
  // the Adam launch
  float *room = M > 0 ? tn_defer_room(N, ldc, nst, (size_t)p.n_groups * elems) : nullptr;
  if (room) part2 = room;
  if (M > 0)
    PGCN_LAUNCH(k_slab_reduce1, dim3((unsigned)ceil_div(elems, 256), (unsigned)p.n_groups),
                       dim3(256), 0, s, partial, p.n_slabs, elems, p.spg, part2);
  if (room) {
    TnDeferred &d = g_tn_defer->d[g_tn_defer->n++];
    d.src = part2;
    d.n_groups = p.n_groups;
    d.K = K;
    d.N = N;
    d.ldp = p.ldp;
    d.C = C;
    return;
  }
  PGCN_LAUNCH(k_gemm_tn_reduce, dim3((unsigned)ceil_div(elems, 256)), dim3(256), 0, s,
                     part2, M > 0 ? p.n_groups : 0, K, N, p.ldp, C, ldc, nst);
}

void launch_slab_reduce(float *partial, int n_slabs, int K, int N, int ldp, float *C, int ldc,
                        int nst, hipStream_t s) {
  TnPlan p{};
  p.n_slabs = n_slabs;
  p.ldp = ldp;
  p.spg = 16;
  p.n_groups = (n_slabs + p.spg - 1) / p.spg;
  tn_reduce(p, n_slabs, N, K, partial, C, ldc, s, nst);
}

static TnPlan blocks_plan(int n_blocks, int ldp) {
  TnPlan p{};
  p.n_slabs = n_blocks;
  p.ldp = ldp;
  // ~sqrt(n) partials per group in each pass (r03 late: 16 per group left the second pass
  // 228 serial loads per element for the loss kernel's 3,641 block partials, 8-11 us)
  int spg = 16;
  while ((long long)spg * spg < n_blocks) spg += 16;
  p.spg = spg;
  p.n_groups = (n_blocks + p.spg - 1) / p.spg;
  return p;
}

void launch_tn_reduce_one_pass(const float *partial, int n, int K, int N, int ldp, float *C,
                               int ldc, hipStream_t s) {
  const long long elems = (long long)K * ldp;
  PGCN_LAUNCH(k_gemm_tn_reduce, dim3((unsigned)ceil_div(elems, 256)), dim3(256), 0, s, partial, n,
              K, N, ldp, C, ldc, ldc);
}

float *tn_defer_blocks(int n_blocks, int K, int N, int ldp, float *C, int ldc) {
  float *room = n_blocks > 0 ? tn_defer_room(N, ldc, ldc, (size_t)n_blocks * K * ldp) : nullptr;
  if (!room) return nullptr;
  TnDeferred &d = g_tn_defer->d[g_tn_defer->n++];
  d.src = room;
  d.n_groups = n_blocks;
  d.K = K;
  d.N = N;
  d.ldp = ldp;
  d.C = C;
  return room;
}

size_t tn_reduce_blocks_workspace(int n_blocks, int K, int ldp) {
  return plan_bytes(blocks_plan(n_blocks, ldp), K);
}

void launch_tn_reduce_blocks(float *partial, int n_blocks, int K, int N, int ldp, float *C, int ldc,
                             hipStream_t s) {
  tn_reduce(blocks_plan(n_blocks, ldp), n_blocks, N, K, partial, C, ldc, s);
}

void launch_xstream_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                       float *C, int ldc, const uint64_t *maskT, float a_scale, void *workspace,
                       hipStream_t s, const XsMask *flat) {
  PGCN_CHECK(xstream_ok(N, K), PGCN_E_INVALID, "xstream_tn: needs N <= 16, K <= 640");
  PGCN_CHECK(!(flat && flat->bits) || xstream_ring_ok(K, lda), PGCN_E_INVALID,
             "xstream_tn: a flat mask on the ring kernels' shapes only");
  PGCN_CHECK(lda % 4 == 0 && lda >= K, PGCN_E_INVALID, "gemm_tn: lda must be a multiple of 4 >= K");
  const int blocks = xs_tn_blocks(M, K, lda);
  const TnPlan p = xs_tn_plan(K, blocks);
  float *partial = static_cast<float *>(workspace);
  // one ordered pass over the block partials (the small graphs' 32 blocks): under tn_defer the
  // partials go to the deferred list's pool and the Adam launch makes that pass
  const int one_pass = blocks == XS_TN_SMALL_BLOCKS ? TN_ONE_PASS : 0;
  float *room = M > 0 && p.n_slabs <= std::max(one_pass, p.spg)
                    ? tn_defer_room(N, ldc, ldc, (size_t)p.n_slabs * K * p.ldp)
                    : nullptr;
  if (room) partial = room;
  if (M > 0 && xstream_ring_ok(K, lda)) {
    launch_xstream_tn_ring(M, N, K, A, lda, G, ldg, maskT, a_scale, partial, XS_TN_BLOCKS, s,
                           flat);
  } else if (M > 0) {
    note_path(KP_XS_TN);
#define XTN_CASE(KC)                                                                           \
  case KC:                                                                                     \
    if (maskT)                                                                                 \
      PGCN_LAUNCH((k_xstream_tn<KC, true>), dim3(blocks), dim3(256), 0, s, M, N, K,       \
                         A, lda, G, ldg, maskT, a_scale, partial);                             \
    else                                                                                       \
      PGCN_LAUNCH((k_xstream_tn<KC, false>), dim3(blocks), dim3(256), 0, s, M, N,        \
                         K, A, lda, G, ldg, maskT, a_scale, partial);                          \
    break;
    switch (p.nkc) {
      XTN_CASE(1) XTN_CASE(2) XTN_CASE(3) XTN_CASE(4) XTN_CASE(5)
      XTN_CASE(6) XTN_CASE(7) XTN_CASE(8) XTN_CASE(9) XTN_CASE(10)
    }
#undef XTN_CASE
  }
  if (room) {
    TnDeferred &d = g_tn_defer->d[g_tn_defer->n++];
    d.src = partial;
    d.n_groups = p.n_slabs;
    d.K = K;
    d.N = N;
    d.ldp = p.ldp;
    d.C = C;
    return;
  }
  tn_reduce(p, M, N, K, partial, C, ldc, s, -1, one_pass);
}

static void gemm_tn_slab(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                         long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                         int nst, const uint64_t *maskT);

void launch_gemm_tn(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                    float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                    long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                    const uint64_t *maskT) {
  PGCN_CHECK(N >= 1, PGCN_E_INVALID, "gemm_tn: N must be >= 1");
  PGCN_CHECK(lda % 4 == 0 && lda >= K, PGCN_E_INVALID, "gemm_tn: lda must be a multiple of 4 >= K");
  if (N > 128) {  // 128-column slabs of G and C, one after another through the workspace,
    // each writing its own columns only (the last one also C's padding columns)
    for (int j0 = 0; j0 < N; j0 += 128)
      gemm_tn_slab(M, std::min(128, N - j0), K, A, lda, G + j0, ldg, C + j0, ldc, a_mask,
                   mask_base, mask_ld, a_scale, workspace, s, j0 + 128 >= N ? ldc - j0 : 128,
                   maskT);
    return;
  }
  gemm_tn_slab(M, N, K, A, lda, G, ldg, C, ldc, a_mask, mask_base, mask_ld, a_scale, workspace, s,
               ldc, maskT);
}

static void gemm_tn_slab(int M, int N, int K, const float *A, int lda, const float *G, int ldg,
                         float *C, int ldc, const uint64_t *a_mask, long long mask_base,
                         long long mask_ld, float a_scale, void *workspace, hipStream_t s,
                         int nst, const uint64_t *maskT) {
  if (!a_mask && xstream_ok(N, K) && nst == ldc) {
    launch_xstream_tn(M, N, K, A, lda, G, ldg, C, ldc, nullptr, 1.0f, workspace, s);
    return;
  }
  if (gemm_wide_ok(N) && ldg % 4 == 0 &&
      (reinterpret_cast<size_t>(G) & 15) == 0) {
    launch_gemm_tn_wide(M, N, K, A, lda, G, ldg, C, ldc, a_mask, mask_base, mask_ld, a_scale,
                        workspace, s, nst, a_mask && K <= 1024 ? maskT : nullptr);
    return;
  }
  const TnPlan p = tn_plan(M, N, K);
  float *partial = static_cast<float *>(workspace);
  if (M > 0) {
    note_path(KP_GEMM_TN);
    const dim3 grid((unsigned)p.n_slabs, (unsigned)p.kgroups), block(256);
    bool done = false;
#define TN_CASE(NJ, KCW, WK)                                                                   \
  if (!done && p.nj == NJ && p.kcw == KCW && p.wk == WK) {                                    \
    PGCN_LAUNCH((k_gemm_tn<NJ, KCW, WK>), grid, block, 0, s, M, N, K, p.slab, A, lda, G, \
                       ldg, a_mask, mask_base, mask_ld, a_scale, partial, p.ldp);              \
    done = true;                                                                               \
  }
#define TN_NJ(NJ) TN_CASE(NJ, 1, 1) TN_CASE(NJ, 1, 2) TN_CASE(NJ, 1, 4) TN_CASE(NJ, 2, 4) \
                  TN_CASE(NJ, 3, 4)
    TN_NJ(1) TN_NJ(2) TN_NJ(3) TN_NJ(4)
    TN_CASE(5, 1, 1) TN_CASE(5, 1, 2) TN_CASE(5, 1, 4)
    TN_CASE(6, 1, 1) TN_CASE(6, 1, 2) TN_CASE(6, 1, 4)
    TN_CASE(7, 1, 1) TN_CASE(7, 1, 2) TN_CASE(7, 1, 4)
    TN_CASE(8, 1, 1) TN_CASE(8, 1, 2) TN_CASE(8, 1, 4)
#undef TN_NJ
#undef TN_CASE
    PGCN_CHECK(done, PGCN_E_INVALID,
               "gemm_tn: no kernel for N=" + std::to_string(N) + " K=" + std::to_string(K));
  }
  tn_reduce(p, M, N, K, partial, C, ldc, s, nst);
}

}  // namespace pgcn
