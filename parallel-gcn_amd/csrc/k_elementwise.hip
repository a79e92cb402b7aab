// parallel-gcn_amd/csrc/k_elementwise.hip -- dropout (bit-exact hpdga masks), ReLU,
// fused cross-entropy + accuracy, scalar finalisation and Adam, for gfx950.
//
// Reference kernels replaced: dropout_kernel_forward/backward (src/module.cu:16-99),
// relu_kernel_forward/backward (:222-265), cross_entropy_loss_kernel (:484-541),
// get_accuracy_kernel / get_l2_penalty_kernel (src/gcn.cu:230-289),
// adam_step_kernel (src/optim.cu:42-55).
//
// Float contraction is OFF in this file: every product/sum rounds where the sequential
// CPU reference (hpdga-spring23) rounds, so Adam and dropout are bit-exact.
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace pgcn {

// ------------------------------------------------------------------------------------------
// Dropout masks: one thread per 64-draw chunk.  The chunk state is the xorshift128+ state at
// the draw element 64*c consumes (hpdga module.cpp:213-217 consumes one draw per element, in
// index order). After emitting the 64 mask bits the state is advanced by one epoch's worth
// of draws (`period`) with 32 nibble-table lookups.  The nibble tables (32 x 16 x 16 B = 8 KB
// in LDS) are read out of the byte tables M^period (16 x 256 entries): by linearity over
// GF(2), nibble p = v of the state maps to byte entry (p/2, v << 4(p%2)).  8 KB instead of
// the 64-KB byte tables keeps 8 workgroups per CU resident: each draw is a serial chain of
// 64-bit xor/shift ops, so the kernel needs the waves to hide it.
// ------------------------------------------------------------------------------------------
// 64 draws from xorshift128+ state (s0, s1) -> 64 keep bits (bit j: draw j >= threshold)
struct Xs64 {
  uint64_t s0, s1;
  uint32_t lo = 0, hi = 0;  // mask bits 0-31 / 32-63 (constant shifts: the loop is unrolled)
  __device__ __forceinline__ void step(int j, int threshold) {
    uint64_t t = s0;
    const uint64_t u = s1;
    s0 = u;
    t ^= t << 23;
    t ^= t >> 17;
    t ^= u ^ (u >> 26);
    s1 = t;
    const int r = (int)((uint32_t)(t + u) & 0x7fffffffu);
    const uint32_t bit = r >= threshold ? 1u : 0u;
    if (j < 32)
      lo |= bit << j;
    else
      hi |= bit << (j - 32);
  }
};

__global__ __launch_bounds__(256) void k_dropout_mask(uint64_t *__restrict__ states,
                                                      long long n_chunks, long long elem0,
                                                      long long elem_end, int threshold,
                                                      uint64_t *__restrict__ mask,
                                                      const uint4 *__restrict__ table) {
  __shared__ uint4 lut[32 * 16];
  for (int i = threadIdx.x; i < 32 * 16; i += blockDim.x) {
    const int p = i >> 4, v = i & 15;
    lut[i] = table[(p >> 1) * 256 + (v << (4 * (p & 1)))];
  }
  __syncthreads();
  // mask word of chunk c, then its state advanced by `period` draws: M^period * (a0, a1)
  auto emit = [&](long long c, uint64_t a0, uint64_t a1, uint64_t word) {
    const long long e = elem0 + 64 * c;  // first element of this chunk
    if (e + 64 > elem_end) {
      const long long valid = elem_end - e;
      word = valid <= 0 ? 0 : (word & ((valid >= 64) ? ~0ull : ((1ull << valid) - 1)));
    }
    mask[c] = word;
    uint64_t n0 = 0, n1 = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const uint4 v = lut[q * 16 + ((a0 >> (4 * q)) & 0xf)];
      n0 ^= ((uint64_t)v.y << 32) | v.x;
      n1 ^= ((uint64_t)v.w << 32) | v.z;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const uint4 v = lut[(16 + q) * 16 + ((a1 >> (4 * q)) & 0xf)];
      n0 ^= ((uint64_t)v.y << 32) | v.x;
      n1 ^= ((uint64_t)v.w << 32) | v.z;
    }
    states[2 * c] = n0;
    states[2 * c + 1] = n1;
  };
  // two chunks per thread and iteration: two independent xorshift chains interleaved (each
  // draw is a serial chain of 64-bit ops; the pair hides their latency at low occupancy)
  const long long G = (long long)gridDim.x * blockDim.x;
  for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < n_chunks; c += 2 * G) {
    const long long c2 = c + G;
    const bool two = c2 < n_chunks;
    const long long cb = two ? c2 : c;
    const uint64_t a0 = states[2 * c], a1 = states[2 * c + 1];
    const uint64_t b0 = states[2 * cb], b1 = states[2 * cb + 1];
    Xs64 x{a0, a1}, y{b0, b1};
#pragma unroll
    for (int j = 0; j < 64; j++) {
      x.step(j, threshold);
      y.step(j, threshold);
    }
    emit(c, a0, a1, ((uint64_t)x.hi << 32) | x.lo);
    if (two) emit(c2, b0, b1, ((uint64_t)y.hi << 32) | y.lo);
  }
}

// x[i] *= bit(base + i) ? scale : 0   (Dropout::forward on a grad-carrying variable and
// Dropout::backward on its grad; hpdga module.cpp:215, :226).
__device__ __forceinline__ uint32_t mask_bits4(const uint64_t *__restrict__ mask, long long idx) {
  const long long w = idx >> 6;
  const int sh = (int)(idx & 63);
  uint64_t v = mask[w] >> sh;
  if (sh > 60) v |= mask[w + 1] << (64 - sh);
  return (uint32_t)v & 0xfu;
}

__global__ __launch_bounds__(256) void k_dropout_apply(float *__restrict__ x, long long n,
                                                       const uint64_t *__restrict__ mask,
                                                       long long base, float scale) {
  const long long n4 = n >> 2;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (long long)gridDim.x * blockDim.x) {
    const long long i = q << 2;
    const uint32_t bits = mask_bits4(mask, base + i);
    float4 v = reinterpret_cast<float4 *>(x)[q];
    v.x *= (bits & 1) ? scale : 0.0f;
    v.y *= (bits & 2) ? scale : 0.0f;
    v.z *= (bits & 4) ? scale : 0.0f;
    v.w *= (bits & 8) ? scale : 0.0f;
    reinterpret_cast<float4 *>(x)[q] = v;
  }
  if (blockIdx.x == 0) {
    for (long long i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
      const long long b = base + i;
      x[i] *= ((mask[b >> 6] >> (b & 63)) & 1) ? scale : 0.0f;
    }
  }
}

// Row scatter of the output layer's restricted GraphSum: out[rows[r]] = src[r] (float4s).
__global__ __launch_bounds__(256) void k_scatter_rows(const float4 *__restrict__ src,
                                                      const int *__restrict__ rows, int n, int ld4,
                                                      float4 *__restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * ld4) return;
  const long long r = t / ld4;
  const int q = (int)(t - r * ld4);
  out[(long long)rows[r] * ld4 + q] = src[t];
}

void launch_scatter_rows(const float *src, const int *rows, int n, int ld, float *out,
                         hipStream_t s) {
  PGCN_CHECK(ld % 4 == 0, PGCN_E_INVALID, "scatter_rows: ld % 4");
  if (n <= 0) return;
  const long long tot = (long long)n * (ld / 4);
  hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4 *>(src), rows, n, ld / 4,
                     reinterpret_cast<float4 *>(out));
}

// loopback reduce-scatter / all-reduce: one element per thread, peers summed in rank order
// (deterministic; RCCL's own order is unspecified)
__global__ __launch_bounds__(256) void k_loopback_sum(LoopbackSrcs srcs, float *__restrict__ dst,
                                                      size_t count) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  float acc = srcs.p[0][i];
  for (int q = 1; q < srcs.n; q++) acc += srcs.p[q][i];
  dst[i] = acc;
}

void launch_loopback_sum(const LoopbackSrcs &srcs, float *dst, size_t count, hipStream_t s) {
  PGCN_CHECK(srcs.n >= 1 && srcs.n <= kLoopbackMaxRanks, PGCN_E_INVALID, "loopback_sum: ranks");
  if (count == 0) return;
  hipLaunchKernelGGL(k_loopback_sum, dim3((unsigned)ceil_div((long long)count, 256)), dim3(256), 0,
                     s, srcs, dst, count);
}

// out[r] = src[rows[r]] (float4s): the input of a column-subset GraphSum on the plain path
__global__ __launch_bounds__(256) void k_gather_rows(const float4 *__restrict__ src,
                                                     const int *__restrict__ rows, int n, int ld4,
                                                     float4 *__restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * ld4) return;
  const long long r = t / ld4;
  const int q = (int)(t - r * ld4);
  out[t] = src[(long long)rows[r] * ld4 + q];
}

void launch_gather_rows(const float *src, const int *rows, int n, int ld, float *out,
                        hipStream_t s) {
  PGCN_CHECK(ld % 4 == 0, PGCN_E_INVALID, "gather_rows: ld % 4");
  if (n <= 0) return;
  const long long tot = (long long)n * (ld / 4);
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4 *>(src), rows, n, ld / 4,
                     reinterpret_cast<float4 *>(out));
}

// ReLU (hpdga module.cpp:173-188)
__global__ __launch_bounds__(256) void k_relu_fwd(float *__restrict__ x, long long n,
                                                  uint8_t *__restrict__ mask, int training) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    const bool keep = v > 0.0f;
    if (training) mask[i] = keep;
    if (!keep) x[i] = 0.0f;
  }
}

__global__ __launch_bounds__(256) void k_relu_bwd(float *__restrict__ g, long long n,
                                                  const uint8_t *__restrict__ mask) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    if (!mask[i]) g[i] = 0.0f;
}

// ------------------------------------------------------------------------------------------
// Block reductions (wave64 shuffles, fixed tree => deterministic)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int BLOCK>
__device__ __forceinline__ float block_sum(float v, float *smem) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) smem[w] = v;
  __syncthreads();
  float r = 0.0f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < BLOCK / 64; i++) r += smem[i];
  }
  return r;  // valid in thread 0
}

// ------------------------------------------------------------------------------------------
// Cross entropy (hpdga module.cpp:122-153) + accuracy (hpdga gcn.cpp:150-164), one thread
// per row, every thread of the block computing (XR = 256 rows).  Labelled rows are
// max-shifted in place like the reference; the grad is written divided by the labelled count
// (known per split on the host).  Rows go through ONE LDS tile [XR][ld+1] (row stride ld+1:
// conflict-free per-row reads) with coalesced copies: logits in, shifted logits out, then the
// grad computed in place and copied out.  Per-block partial sums (loss, wrong) go to
// partials[2*block].
// ------------------------------------------------------------------------------------------
constexpr int XR = 256;  // rows per cross-entropy block (= threads; 128 measured slower, r02)
typedef float floatx4e __attribute__((ext_vector_type(4)));

// FUSED: the logits are computed here from the output layer's input H [n][ldh] (kh <= 16
// columns) and W [kh][ldw] with k_gemm_nn's v_mfma_f32_16x16x4_f32 sequence, so the same bits
// as the separate Matmul -- and then go through the same tile as the loaded ones (the output layer's Matmul forward + CrossEntropyLoss forward,
// hpdga module.cpp:13-38, :122-153, in one pass: the logits are written once, not written
// and read back).
template <bool FUSED>
__global__ __launch_bounds__(XR) void k_xent_fwd(float *__restrict__ logits, int ld,
                                                  float *__restrict__ grad,
                                                  const int *__restrict__ truth, int n, int c,
                                                  int count, int training,
                                                  float *__restrict__ partials, int write_back,
                                                  const float *__restrict__ H, int ldh, int kh,
                                                  const float *__restrict__ W, int ldw,
                                                  float *__restrict__ dH, int lddh,
                                                  float *__restrict__ dWp) {
  // write_back 0: the shifted logits stay in LDS (the compact output layer's logits are read
  // by nobody after the loss; hpdga's in-place shift is kept where the variable is visible)
  extern __shared__ float smem[];
  __shared__ float red[XR / 64];
  const int S = ld + 1;
  float *L = smem;  // [XR][S]
  const long long row0 = (long long)blockIdx.x * XR;
  const int rows = (int)min((long long)XR, (long long)n - row0);
  const long long base = row0 * ld;
  const int tile = rows * ld;
  // The tile is rows*ld contiguous floats (ld % 4 == 0, 16-B aligned): float4 copies,
  // XU per thread in flight (all loads of a batch before its LDS stores); float4 q = row
  // q / (ld/4), column 4 (q % (ld/4)) -- one division per float4, not per float.
  const int ld4 = ld >> 2, tile4 = tile >> 2;
  constexpr int XU = 8;
  auto to_lds = [&](const float *src) {
    for (int q0 = threadIdx.x; q0 < tile4; q0 += XR * XU) {
      float4 v[XU];
#pragma unroll
      for (int u = 0; u < XU; u++) {
        const int q = q0 + XR * u;
        if (q < tile4) v[u] = reinterpret_cast<const float4 *>(src + base)[q];
      }
#pragma unroll
      for (int u = 0; u < XU; u++) {
        const int q = q0 + XR * u;
        if (q < tile4) {
          const int r = q / ld4, j = 4 * (q - r * ld4);
          float *d = L + r * S + j;
          d[0] = v[u].x;
          d[1] = v[u].y;
          d[2] = v[u].z;
          d[3] = v[u].w;
        }
      }
    }
  };
  auto from_lds = [&](float *dst) {
    for (int q = threadIdx.x; q < tile4; q += XR) {
      const int r = q / ld4, j = 4 * (q - r * ld4);
      const float *d = L + r * S + j;
      reinterpret_cast<float4 *>(dst + base)[q] = make_float4(d[0], d[1], d[2], d[3]);
    }
  };
  // FUSED: W [k][j] (16 x ld) in the dynamic LDS past the tile (and past the waves' weight-grad
  // partials, which reuse the tile): sized to the layer, not to the largest class count
  float *wt = smem + (FUSED ? max(XR * S, (XR / 64) * 3 * 4 * 64) : 0);
  // FUSED: the lane's H operands of all four 16-row groups, loaded before W is staged (one
  // HBM latency for the block instead of one per group)
  float ha[4][4];
  if constexpr (FUSED) {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      long long grow = row0 + wv * 64 + q * 16 + ii;
      grow = grow < n ? grow : n - 1;
      const float *hr = H + grow * (long long)ldh;
#pragma unroll
      for (int t4 = 0; t4 < 4; t4++) ha[q][t4] = 4 * gi + t4 < kh ? hr[4 * gi + t4] : 0.0f;
    }
  }
  if constexpr (FUSED) {
    for (int e = threadIdx.x; e < 16 * ld; e += XR) {
      const int k = e / ld, j = e - k * ld;
      wt[e] = (k < kh && j < c) ? W[(long long)k * ldw + j] : 0.0f;
    }
    __syncthreads();
    // logits of the block's XR rows on MFMA, as k_gemm_nn<3> computes them: wave w takes rows
    // 64 w .. 64 w + 63 in groups of 16; lane (i, g) feeds MFMA t with H[row i][4 g + t] and
    // W[4 g + t][16 tt + i]; lane holds logits[4 g + r][16 tt + i] -> the tile
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float *a = ha[q];
      for (int tt = 0; 16 * tt < ld; tt++) {
        const int col = 16 * tt + ii;
        floatx4e acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t4 = 0; t4 < 4; t4++)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
              a[t4], col < ld ? wt[(4 * gi + t4) * ld + col] : 0.0f, acc, 0, 0, 0);
        if (col < ld) {
#pragma unroll
          for (int r = 0; r < 4; r++) L[(wv * 64 + q * 16 + 4 * gi + r) * S + col] = acc[r];
        }
      }
    }
  } else {
    to_lds(logits);
  }
  __syncthreads();
  float loss = 0.0f, wrong = 0.0f, se = 0.0f;
  const int t = threadIdx.x < rows ? truth[row0 + threadIdx.x] : -1;
  float *l = L + threadIdx.x * S;
  if (t >= 0) {
    float mx = -1e30f;
#pragma unroll 4
    for (int j = 0; j < c; j++) mx = fmaxf(mx, l[j]);
#pragma unroll 4
    for (int j = 0; j < c; j++) {
      const float v = l[j] - mx;
      l[j] = v;
      se += expf(v);
    }
    const float lt = l[t];
    loss = logf(se) - lt;
    bool w = false;
#pragma unroll 4
    for (int j = 0; j < c; j++) w |= l[j] > lt;
    wrong = w ? 1.0f : 0.0f;
  }
  __syncthreads();
  if (write_back || FUSED) from_lds(logits);
  if (training) {
    // the weight-grad phase's H operands (row 4 st + gi of the wave, column ii), loaded now so
    // their latency hides behind the grad computation
    float hw[16];
    if (FUSED && dWp) {
      const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
#pragma unroll
      for (int st = 0; st < 16; st++) {
        const int rloc = wv * 64 + 4 * st + gi;
        hw[st] = (rloc < rows && ii < kh) ? H[(row0 + rloc) * (long long)ldh + ii] : 0.0f;
      }
    }
    __syncthreads();  // the shifted logits have left the tile
    if (threadIdx.x < rows) {
      if (t >= 0) {
#pragma unroll 4
        for (int j = 0; j < c; j++) {
          float prob = expf(l[j]) / se;
          if (j == t) prob = (float)((double)prob - 1.0);  // hpdga module.cpp:145 (double temp)
          l[j] = prob / (float)count;
        }
        for (int j = c; j < ld; j++) l[j] = 0.0f;
      } else {
        for (int j = 0; j < ld; j++) l[j] = 0.0f;
      }
    }
    if (FUSED && dH) {
      // the output layer's input grad dH = grad W^T (Matmul::backward's a.grad) on MFMA in
      // k_xstream_nn's sequence (N = 16 outputs, K = c classes: step s, MFMA t, lane group g:
      // class 16 s + 4 g + t), from the grad tile
      __syncthreads();
      const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int rl = wv * 64 + q * 16;  // local rows rl .. rl + 15
        floatx4e acc = {0.f, 0.f, 0.f, 0.f};
        for (int s0 = 0; s0 < c; s0 += 16) {
#pragma unroll
          for (int t4 = 0; t4 < 4; t4++) {
            const int j = s0 + 4 * gi + t4;
            const float av = j < c ? L[(rl + ii) * S + j] : 0.0f;
            const float bv = (j < c && ii < kh) ? wt[ii * ld + j] : 0.0f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
          }
        }
        if (ii < lddh) {
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int rr = rl + 4 * gi + r;
            if (rr < rows) dH[(row0 + rr) * (long long)lddh + ii] = acc[r];
          }
        }
      }
    }
    // the output layer's weight grad, this block's share: partial [kh][48] = H^T grad
    // over the block's rows (wave partials on MFMA, added in wave order), reduced over the
    // blocks in block order by launch_tn_reduce_blocks
    floatx4e pw[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (FUSED && dWp) {
      if (!dH) __syncthreads();  // the grad tile is complete
      const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
#pragma unroll
      for (int st = 0; st < 16; st++) {  // 4-row steps over the wave's 64 rows
        const int rloc = wv * 64 + 4 * st + gi;
        const bool ok = rloc < rows;
        const float av = hw[st];
#pragma unroll
        for (int tt = 0; tt < 3; tt++) {
          const int col = 16 * tt + ii;
          const float bv = (ok && col < ld) ? L[rloc * S + col] : 0.0f;
          pw[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, pw[tt], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    from_lds(grad);
    if (FUSED && dWp) {
      __syncthreads();  // the tile is free: wave partials through it
      const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
      float *rw = L + wv * (3 * 4 * 64);
#pragma unroll
      for (int tt = 0; tt < 3; tt++)
#pragma unroll
        for (int r = 0; r < 4; r++) rw[(tt * 4 + r) * 64 + ln] = pw[tt][r];
      __syncthreads();
      if (wv == 0) {
        float *pb = dWp + (long long)blockIdx.x * kh * 48;  // [kh][48] per block
#pragma unroll
        for (int tt = 0; tt < 3; tt++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            float v = pw[tt][r];
#pragma unroll
            for (int w2 = 1; w2 < XR / 64; w2++) v += L[w2 * (3 * 4 * 64) + (tt * 4 + r) * 64 + ln];
            if (4 * gi + r < kh) pb[(4 * gi + r) * 48 + 16 * tt + ii] = v;
          }
      }
    }
  }
  const float ls = block_sum<XR>(loss, red);
  const float ws = block_sum<XR>(wrong, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = ls;
    partials[2 * blockIdx.x + 1] = ws;
  }
}

// sums[0] = sum loss partials, sums[1] = sum wrong, sums[2] = sum w^2 (fixed order)
__global__ __launch_bounds__(1024) void k_reduce_scalars(const float *__restrict__ partials,
                                                         int n_blocks,
                                                         const float *__restrict__ w,
                                                         long long n_w, float *__restrict__ sums,
                                                         int count, float wd,
                                                         float *__restrict__ out2,
                                                         const int *__restrict__ ctr,
                                                         int ring_cap) {
  __shared__ float red[16];
  float l = 0.0f, wr = 0.0f, q = 0.0f;
  for (int b = threadIdx.x; b < n_blocks; b += blockDim.x) {
    l += partials[2 * b];
    wr += partials[2 * b + 1];
  }
  for (long long i = threadIdx.x; i < n_w; i += blockDim.x) {
    const float x = w[i];
    q += x * x;
  }
  l = block_sum<1024>(l, red);
  wr = block_sum<1024>(wr, red);
  q = block_sum<1024>(q, red);
  if (threadIdx.x == 0) {
    sums[0] = l;
    sums[1] = wr;
    sums[2] = q;
    if (out2) {  // one GPU: k_compose's arithmetic here, no second launch
      if (ctr) out2 += 4 * (ctr[1] % ring_cap);
      out2[0] = l / (float)count + wd * q / 2.0f;
      out2[1] = (float)(count - (int)wr) / (float)count;
    }
  }
}

// out2 = {loss_sum/count + wd*l2/2, (count-wrong)/count}   (hpdga gcn.cpp:167-198)
__global__ void k_compose(const float *__restrict__ sums, int count, float wd,
                          float *__restrict__ out2, const int *__restrict__ ctr, int ring_cap) {
  if (threadIdx.x == 0) {
    // epoch graphs: the results-ring slot from the device epoch counter (ctr[1])
    if (ctr) out2 += 4 * (ctr[1] % ring_cap);
    const float loss = sums[0] / (float)count;
    const float l2 = wd * sums[2] / 2.0f;
    out2[0] = loss + l2;
    const int wrong = (int)sums[1];
    out2[1] = (float)(count - wrong) / (float)count;
  }
}

// Adam (hpdga optim.cpp:25-33): double temporaries where the reference has them.
__device__ __forceinline__ void adam_range(float *__restrict__ w, const float *__restrict__ g,
                                           float *__restrict__ m, float *__restrict__ v,
                                           long long n, float step_size, float beta1,
                                           float beta2, float eps, float wd, int decay) {
  const double ob1 = 1.0 - (double)beta1, ob2 = 1.0 - (double)beta2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float grad = g[i];
    const float wi = w[i];
    if (decay) grad += wd * wi;
    const float mi = (float)((double)(beta1 * m[i]) + ob1 * (double)grad);
    const float vi = (float)((double)(beta2 * v[i]) + (ob2 * (double)grad) * (double)grad);
    m[i] = mi;
    v[i] = vi;
    w[i] = wi - step_size * mi / (sqrtf(vi) + eps);
  }
}

// every weight of the model in one launch: tensor blockIdx.y
__global__ __launch_bounds__(256) void k_adam_multi(AdamBatch b, float step_size, float beta1,
                                                    float beta2, float eps, float wd,
                                                    const float *__restrict__ step_table,
                                                    const int *__restrict__ ctr, int table_cap) {
  if (step_table) step_size = step_table[ctr[0] % table_cap];
  const int t = blockIdx.y;
  adam_range(b.w[t], b.g[t], b.m[t], b.v[t], b.n[t], step_size, beta1, beta2, eps, wd,
             b.decay[t]);
}

__global__ __launch_bounds__(256) void k_adam(float *__restrict__ w, const float *__restrict__ g,
                                              float *__restrict__ m, float *__restrict__ v,
                                              long long n, float step_size, float beta1,
                                              float beta2, float eps, float wd, int decay,
                                              const float *__restrict__ step_table,
                                              const int *__restrict__ ctr, int table_cap) {
  // epoch graphs: the step size of step ctr[0] + 1, computed on the host (optim.cpp:24)
  if (step_table) step_size = step_table[ctr[0] % table_cap];
  adam_range(w, g, m, v, n, step_size, beta1, beta2, eps, wd, decay);
}


// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static int grid_for(long long work, int block = 256, int cap = 2048) {
  long long g = ceil_div(work, block);
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

void launch_dropout_mask(uint64_t *states, long long n_chunks, long long elem0,
                         long long elem_end, float p, uint64_t *mask, const void *table,
                         hipStream_t s, int max_blocks) {
  if (n_chunks <= 0) return;
  // hpdga module.cpp:211: threshold = int(p * MY_RAND_MAX) evaluated in float
  const int threshold = (int)(p * (float)0x7fffffff);
  // 8 KB LDS: up to 8 workgroups per CU (a side-stream draw takes fewer: max_blocks)
  const int grid = grid_for(ceil_div(n_chunks, 2), 256, max_blocks > 0 ? max_blocks : 8 * kCUs);
  hipLaunchKernelGGL(k_dropout_mask, dim3(grid), dim3(256), 0, s, states, n_chunks, elem0,
                     elem_end, threshold, mask, static_cast<const uint4 *>(table));
}

void launch_dropout_apply_based(float *x, long long n, const uint64_t *mask, long long base,
                                float scale, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_dropout_apply, dim3(grid_for(ceil_div(n, 4))), dim3(256), 0, s, x, n,
                     mask, base, scale);
}

void launch_relu_fwd(float *x, long long n, uint8_t *mask, int training, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_relu_fwd, dim3(grid_for(n)), dim3(256), 0, s, x, n, mask, training);
}

void launch_relu_bwd(float *g, long long n, const uint8_t *mask, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_relu_bwd, dim3(grid_for(n)), dim3(256), 0, s, g, n, mask);
}

int xent_blocks(int n) { return (int)ceil_div(n, XR); }

void launch_xent_fwd(float *logits, int ld, float *grad, const int *truth, int n, int c,
                     int count, int training, float *partials, hipStream_t s, int write_back) {
  if (n <= 0) return;
  PGCN_CHECK(ld <= 124 && c <= ld && ld % 4 == 0, PGCN_E_INVALID,
             "xent: classes must be <= 124 (ld a multiple of 4)");
  const size_t lds = (size_t)XR * (ld + 1) * sizeof(float);  // <= 256*125*4 = 125 KB
  static bool attr = false;
  if (!attr) {
    PGCN_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(k_xent_fwd<false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 125 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(k_xent_fwd<false>, dim3(xent_blocks(n)), dim3(XR), lds, s, logits, ld, grad,
                     truth, n, c, count, training, partials, write_back, nullptr, 0, 0, nullptr, 0,
                     nullptr, 0, nullptr);
}

void launch_out_xent(const float *H, int ldh, int kh, const float *W, int ldw, float *logits,
                     int ld, float *grad, const int *truth, int n, int c, int count, int training,
                     float *partials, hipStream_t s, float *dH, int lddh, float *dWp) {
  note_path(KP_OUT_XENT);
  if (n <= 0) return;
  PGCN_CHECK(ld <= 116 && c <= ld && ld % 4 == 0 && kh >= 1 && kh <= 16, PGCN_E_INVALID,
             "out_xent: classes <= 116, hidden <= 16");
  PGCN_CHECK(!dWp || ld <= 48, PGCN_E_INVALID, "out_xent: the weight-grad partial needs <= 48 classes");
  // the tile, and (weight-grad partials) room for the waves' [3][4][64] partials in it
  const size_t tile = (size_t)XR * (ld + 1), wparts = (size_t)(XR / 64) * 3 * 4 * 64;
  const size_t lds = ((wparts > tile ? wparts : tile) + (size_t)16 * ld) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    PGCN_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(k_xent_fwd<true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(k_xent_fwd<true>, dim3(xent_blocks(n)), dim3(XR), lds, s, logits, ld, grad,
                     truth, n, c, count, training, partials, 1, H, ldh, kh, W, ldw,
                     training ? dH : nullptr, lddh, training ? dWp : nullptr);
}

void launch_reduce_scalars(const float *partials, int n_blocks, const float *w, long long n_w,
                           float *sums, hipStream_t s, int count, float wd, float *out2,
                           const int *ctr, int ring_cap) {
  hipLaunchKernelGGL(k_reduce_scalars, dim3(1), dim3(1024), 0, s, partials, n_blocks, w, n_w,
                     sums, count, wd, out2, ctr, ring_cap);
}

void launch_compose(const float *sums, int count, float wd, float *out2, hipStream_t s,
                    const int *ctr, int ring_cap) {
  hipLaunchKernelGGL(k_compose, dim3(1), dim3(64), 0, s, sums, count, wd, out2, ctr, ring_cap);
}

// epoch graphs: the device copy of the host's (Adam step, epoch) counters
__global__ void k_counters(int *ctr, int set, int step, int epoch) {
  if (threadIdx.x == 0) {
    if (set) {
      ctr[0] = step;
      ctr[1] = epoch;
    } else {
      ctr[0] += 1;
      ctr[1] += 1;
    }
  }
}

void launch_counters(int *ctr, int set, int step, int epoch, hipStream_t s) {
  hipLaunchKernelGGL(k_counters, dim3(1), dim3(64), 0, s, ctr, set, step, epoch);
}

void launch_adam_multi(const AdamBatch &b, float step_size, float beta1, float beta2, float eps,
                       float wd, hipStream_t s, const float *step_table, const int *ctr,
                       int table_cap) {
  if (b.count <= 0) return;
  long long nmax = 0;
  for (int t = 0; t < b.count; t++) nmax = std::max(nmax, b.n[t]);
  hipLaunchKernelGGL(k_adam_multi, dim3(grid_for(nmax), b.count), dim3(256), 0, s, b, step_size,
                     beta1, beta2, eps, wd, step_table, ctr, table_cap);
}

void launch_adam(float *w, const float *g, float *m, float *v, long long n, float step_size,
                 float beta1, float beta2, float eps, float wd, int decay, hipStream_t s,
                 const float *step_table, const int *ctr, int table_cap) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n)), dim3(256), 0, s, w, g, m, v, n, step_size,
                     beta1, beta2, eps, wd, decay, step_table, ctr, table_cap);
}

}  // namespace pgcn
