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
#include <numeric>

#include "common.hpp"
#include "kernels.hpp"
#include "mask_draw.hpp"
#include "peer_sync.hpp"

#pragma clang fp contract(off)

namespace pgcn {

__global__ __launch_bounds__(256) void k_dropout_mask(MaskSeg a, MaskSeg b, int blocks_a,
                                                      const uint4 *__restrict__ table) {
  __shared__ uint4 lut[32 * 16];
  for (int i = threadIdx.x; i < 32 * 16; i += blockDim.x) {
    const int p = i >> 4, v = i & 15;
    lut[i] = table[(p >> 1) * 256 + (v << (4 * (p & 1)))];
  }
  __syncthreads();
  const bool in_a = (int)blockIdx.x < blocks_a;
  const MaskSeg &sg = in_a ? a : b;
  const long long bid = in_a ? blockIdx.x : blockIdx.x - blocks_a;
  const long long nblk = in_a ? blocks_a : gridDim.x - blocks_a;
  if (sg.per == 2)
    dropout_mask_seg<2>(sg, lut, bid * blockDim.x + threadIdx.x, nblk * blockDim.x);
  else
    dropout_mask_seg<1>(sg, lut, bid * blockDim.x + threadIdx.x, nblk * blockDim.x);
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
  PGCN_LAUNCH(k_scatter_rows, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4 *>(src), rows, n, ld / 4,
                     reinterpret_cast<float4 *>(out));
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
  PGCN_LAUNCH(k_gather_rows, dim3((unsigned)ceil_div(tot, 256)), dim3(256), 0, s,
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
// Cross entropy (hpdga module.cpp:122-153) + accuracy (hpdga gcn.cpp:150-164).  A block of XR
// = 64 rows, 4 waves, each wave working alone on its 16 rows (no block barrier between the
// phases): a row's classes are split over a lane quad (lane q takes classes q, q + 4, ...;
// C = 41: 11 per lane), max and exp-sum combined across the quad by xor shuffles in a fixed
// order ((s0 + s1) + (s2 + s3): commutative adds, every lane holds the same bits), so a row's
// serial chain is 11 steps instead of 41 (r02: one thread per row, 256-row blocks at 3 per CU
// with a block barrier per phase, 73 us per training call).  Labelled rows are max-shifted in
// place like the reference; the grad is written divided by the labelled count (known per split
// on the host).  A wave's rows go through its part of ONE LDS tile [XR][ld+1] with coalesced
// copies: logits in (or computed, FUSED), shifted logits out, then the grad computed in place
// and copied out.  Per-block partial sums (loss, wrong) go to partials[2*block].
// ------------------------------------------------------------------------------------------
#ifndef PGCN_XENT_ROWS
#define PGCN_XENT_ROWS 64
#endif
constexpr int XR = PGCN_XENT_ROWS;  // rows per cross-entropy block
constexpr int XT = 4 * XR;    // threads: a lane quad per row; wave w holds rows 16 w .. 16 w + 15
// tile row stride: a multiple of 4 (rows 16-B aligned: the copies move float4s), S / 4 odd (a
// wave's quad-per-row walks and the MFMA's 4-row stores hit 64 distinct banks) and >= 48
__host__ __device__ inline int xent_stride(int ld) {
  const int s = ld > 48 ? (ld + 3) & ~3 : 48;
  return (s / 4) % 2 ? s : s + 4;
}
typedef float floatx4e __attribute__((ext_vector_type(4)));

// XentFinal (kernels.hpp): the pass's scalars finished by the loss kernel's last block.  Called
// by every thread at the end of a block whose thread 0 holds the block's (loss, wrong) in
// red[0], red[1] (xent_tile).  Write-through partials (sc1 stores, drained, then the ticket)
// and write-through loads in the last block: the hand-off needs no cache maintenance
// (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores + agent-scope atomic counter,
// the last adder's sc1 loads after a workgroup barrier)
__device__ __forceinline__ void xent_finish(const XentFinal &fin, int count, float *red) {
  __shared__ float fred[16];
  __shared__ int last;
  // this block's slice of sum w^2 (W1 split evenly over the blocks, in index order per thread)
  const long long per = (fin.n_w + gridDim.x - 1) / gridDim.x;
  const long long lo = (long long)blockIdx.x * per, hi = min(fin.n_w, lo + per);
  float q = 0.0f;
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float v = fin.w[i];
    q += v * v;
  }
  q = block_sum<XT>(q, fred);
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      fin.part4, 0, (int)(gridDim.x * 16), 0x00020000);
  const int G = fin.group;
  const unsigned n_top = G > 0 ? (gridDim.x + G - 1) / G : gridDim.x;  // arrivals on `ticket`
  if (threadIdx.x == 0) {
    const u4 d = {__float_as_uint(red[0]), __float_as_uint(red[1]), __float_as_uint(q), 0u};
    __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)(blockIdx.x * 16), 0, 16);  // sc1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned *tk = fin.ticket;
    unsigned n_arr = gridDim.x;
    if (G > 0) {
      const unsigned g = blockIdx.x / G;
      tk = fin.gticket + 16 * g;
      n_arr = min((unsigned)G, gridDim.x - g * G);
    }
    const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == n_arr - 1;
  }
  __syncthreads();
  if (!last) return;
  if (G > 0) {
    // the group's last block: the group's partials in block order (a fixed tree), its sum to
    // gpart4[g] (sc1), the group ticket reset, one arrival on the top ticket
    const unsigned g = blockIdx.x / G, b0 = g * G, nb = min((unsigned)G, gridDim.x - b0);
    float gl = 0.0f, gw = 0.0f, gq = 0.0f;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) {
      const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((b0 + b) * 16), 0, 16);  // sc1
      gl += __uint_as_float(v.x);
      gw += __uint_as_float(v.y);
      gq += __uint_as_float(v.z);
    }
    gl = block_sum<XT>(gl, fred);
    gw = block_sum<XT>(gw, fred);
    gq = block_sum<XT>(gq, fred);
    const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(
        fin.gpart4, 0, (int)(n_top * 16), 0x00020000);
    if (threadIdx.x == 0) {
      const u4 d = {__float_as_uint(gl), __float_as_uint(gw), __float_as_uint(gq), 0u};
      __builtin_amdgcn_raw_buffer_store_b128(d, gs, (int)(g * 16), 0, 16);  // sc1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(fin.gticket + 16 * g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned old =
          __hip_atomic_fetch_add(fin.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == n_top - 1;
    }
    __syncthreads();
    if (!last) return;
  }
  float l = 0.0f, wr = 0.0f, w2 = 0.0f;
  {
    const __amdgpu_buffer_rsrc_t ts =
        G > 0 ? __builtin_amdgcn_make_buffer_rsrc(fin.gpart4, 0, (int)(n_top * 16), 0x00020000) : rs;
    for (int b = threadIdx.x; b < (int)n_top; b += blockDim.x) {
      const u4 v = __builtin_amdgcn_raw_buffer_load_b128(ts, b * 16, 0, 16);  // sc1
      l += __uint_as_float(v.x);
      wr += __uint_as_float(v.y);
      w2 += __uint_as_float(v.z);
    }
  }
  l = block_sum<XT>(l, fred);
  wr = block_sum<XT>(wr, fred);
  w2 = block_sum<XT>(w2, fred);
  if (threadIdx.x == 0) {
    if (fin.sums) {
      fin.sums[0] = l;
      fin.sums[1] = wr;
    }
    float *o = fin.out2;
    if (fin.ctr) o += 4 * (fin.ctr[1] % fin.ring_cap);
    o[0] = l / (float)count + fin.wd * w2 / 2.0f;
    o[1] = (float)(count - (int)wr) / (float)count;
    __hip_atomic_store(fin.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// a wave's LDS writes are visible to its own later LDS reads (one wave: in-order LDS pipe);
// this keeps the compiler from moving the reads above the writes
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// expf for x <= 0 (a max-shifted logit): the device library's expf sequence without its
// overflow select, which cannot fire there -- the same operations in the same order, so the
// same bits (tests: the loss kernel against the oracle; `test_exp_nonpos_matches_expf`)
__device__ __forceinline__ float exp_nonpos(float x) {
  const float l2e = 0x1.715476p+0f, l2e_lo = 0x1.4ae0bep-26f;
  const float ph = x * l2e;
  const float e = __builtin_rintf(ph);
  const float pl = fmaf(x, l2e_lo, fmaf(x, l2e, -ph));
  const float r = __builtin_ldexpf(__builtin_amdgcn_exp2f((ph - e) + pl), (int)e);
  return x < -0x1.9d1da0p+6f ? 0.0f : r;
}

__global__ void k_exp_check(const float *__restrict__ x, long long n, float *__restrict__ mine,
                            float *__restrict__ lib) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    mine[i] = exp_nonpos(x[i]);
    lib[i] = expf(x[i]);
  }
}

// a / b rounded to nearest from rb = RN(1 / b) (Markstein: q within an ulp, the residual exact
// by fma, one correction step): the IEEE quotient's bits for normal operands and results.
// The residual r = a - q b is exact only while its lowest bit (ulp(q) ulp(b) = 2^(e_q - 46))
// is representable, i.e. q >= 2^-103: below 2^-100 (r03's form missed bits for quotients up to
// 3e-38, the advisor's case) the loss kernel takes the IEEE division itself;
// tests/test_gpu_kernels.py test_div_rn_matches_ieee checks the bits over dense a (subnormals
// included) and b in [1, 128]
__device__ __forceinline__ float div_rn(float a, float b, float rb) {
  const float q = a * rb;
  if (__builtin_expect(fabsf(q) < 0x1p-100f, 0)) return a / b;
  const float r = fmaf(-q, b, a);
  return fmaf(r, rb, q);
}

__global__ void k_div_check(const float *__restrict__ a, const float *__restrict__ b, long long n,
                            float *__restrict__ q) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) q[i] = div_rn(a[i], b[i], 1.0f / b[i]);
}

void launch_exp_check(const float *x, long long n, float *mine, float *lib, hipStream_t s) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_exp_check, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, x, n, mine, lib);
}

void launch_div_check(const float *a, const float *b, long long n, float *q, hipStream_t s) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_div_check, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, a, b, n, q);
}

// FUSED: the logits are computed here from the output layer's input H [n][ldh] (kh <= 16
// columns) and W [kh][ldw] with k_gemm_nn's v_mfma_f32_16x16x4_f32 sequence, so the same bits
// as the separate Matmul -- and then go through the same tile as the loaded ones (the output
// layer's Matmul forward + CrossEntropyLoss forward, hpdga module.cpp:13-38, :122-153, in one
// pass: the logits are written once, not written and read back).  Training: also the output
// layer's input grad dH = grad W^T and (dWp) this block's partial of W.grad = H^T grad.
#ifdef PGCN_XENT_STAMPS
// diagnostic build only (tools/xent_stamps.py): per wave, shader-clock stamps at the kernel's
// phase boundaries and the wall clock at its start and end
__device__ unsigned long long g_xent_stamps[16384 * 12];
#define XST(k) (st[k] = __builtin_amdgcn_s_memtime())
#else
#define XST(k) ((void)0)
#endif
// CC / LDC / KH > 0: the class count, the logits row stride and the hidden width as
// compile-time constants (the launcher's specialisations: the bounds tests of the class
// loops, the MFMA operand selects and the tile arithmetic fold away); 0: runtime values
template <bool FUSED, int CC = 0, int LDC = 0, int KH = 0>
__device__ __forceinline__ void xent_tile(float *__restrict__ logits, int ld_rt,
                                                  float *__restrict__ grad,
                                                  const int *__restrict__ truth, int n, int c_rt,
                                                  int count, int training,
                                                  float *__restrict__ partials, int write_back,
                                                  const float *__restrict__ H, int ldh, int kh_rt,
                                                  const float *__restrict__ W, int ldw,
                                                  float *__restrict__ dH, int lddh,
                                                  float *__restrict__ dWp, const XentTable &tb,
                                                  const XentFinal &fin) {
  // write_back 0: the shifted logits stay in LDS (the compact output layer's logits are read
  // by nobody after the loss; hpdga's in-place shift is kept where the variable is visible)
  extern __shared__ float smem[];
  __shared__ float red[2 * (XT / 64)];
#ifdef PGCN_XENT_STAMPS
  unsigned long long st[12] = {};
  st[10] = __builtin_amdgcn_s_memrealtime();
#endif
  const int c = CC > 0 ? CC : c_rt, ld = LDC > 0 ? LDC : ld_rt, kh = KH > 0 ? KH : kh_rt;
  XST(0);
  // tile row stride (xent_stride) >= 48, so a wave's 16 rows can take its [3][4][64]
  // weight-grad partial once the grad has left the tile (no extra LDS)
  const int S = xent_stride(ld);
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, gi = ln >> 4, ii = ln & 15;
  const long long row0 = (long long)blockIdx.x * XR, wrow0 = row0 + 16 * wv;
  const int rows = (int)min((long long)XR, (long long)n - row0);
  const int wrows = max(0, min(16, rows - 16 * wv));  // this wave's rows
  float *L = smem + wv * 16 * S;  // the wave's part of the tile [16][S]
  // the wave's rows: wrows*ld contiguous floats (ld % 4 == 0, 16-B aligned), copied as float4
  // q = lane + 64 u (1 KB contiguous per wave instruction; r03: a quad per row, 176-B strided
  // pieces, made the kernel 20 % slower); row q / (ld/4) by a 24-bit multiply-shift (exact for
  // q < 2^20 / (ld/4); here q < 512)
  const int ld4 = ld >> 2, tile4 = (wrows * ld) >> 2;
  const unsigned magic = (1u << 20) / (unsigned)ld4 + 1u;
  const long long base = wrow0 * ld;
  auto to_lds = [&](const float *src) {
    floatx4e v[8];  // ld <= 124: 16 * 31 float4 <= 64 * 8
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = ln + 64 * u;
      if (q < tile4) v[u] = reinterpret_cast<const floatx4e *>(src + base)[q];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = ln + 64 * u;
      if (q < tile4) {
        const int r = (int)(__umul24((unsigned)q, magic) >> 20), j = 4 * (q - r * ld4);
        *reinterpret_cast<floatx4e *>(L + r * S + j) = v[u];
      }
    }
  };
  auto from_lds = [&](float *dst) {
    for (int q = ln; q < tile4; q += 64) {
      const int r = (int)(__umul24((unsigned)q, magic) >> 20), j = 4 * (q - r * ld4);
      reinterpret_cast<float4 *>(dst + base)[q] = *reinterpret_cast<const float4 *>(L + r * S + j);
    }
  };
  // FUSED: W [k][j] (16 x ld) past the tile
  float *wt = smem + XR * S;
  // FUSED: the lane's H operands of its wave's 16-row group (MFMA t of lane (gi, ii):
  // H[row ii][4 gi + t]) and, training with dWp, of the weight-grad steps (row 4 st + gi,
  // column ii), both loaded before W is staged (one HBM latency for the block)
  float ha[4], hw[4];
  // the quad of the wave's row rq (lane q takes classes q + 4 k); its truth label, loaded
  // with the block's first loads
  const int rq = ln >> 2, q = ln & 3;
  const int t = rq < wrows ? truth[wrow0 + rq] : -1;
  // FUSED training with tb.table: the table row of the dH row this lane writes (row 4 gi + q of
  // the wave's group, q = ii & 3), loaded with the first loads, and its scale once W is staged
  int tb_p = -1;
  float tb_s = 0.0f;
  if (FUSED && tb.table) {
    const int rr = 4 * gi + (ii & 3);
    const long long row = wrow0 + rr;
    tb_p = rr >= wrows ? -1 : (tb.pos ? tb.pos[row] : (row < tb.rows ? (int)row : -1));
  }
  if constexpr (FUSED) {
    const long long grow = wrow0 + ii < n ? wrow0 + ii : n - 1;
    const float *hr = H + grow * (long long)ldh;
    if (4 * gi + 3 < kh && ldh % 4 == 0) {
      const float4 h4 = *reinterpret_cast<const float4 *>(hr + 4 * gi);
      ha[0] = h4.x;
      ha[1] = h4.y;
      ha[2] = h4.z;
      ha[3] = h4.w;
    } else {
#pragma unroll
      for (int t4 = 0; t4 < 4; t4++) ha[t4] = 4 * gi + t4 < kh ? hr[4 * gi + t4] : 0.0f;
    }
    if (training && dWp) {
#pragma unroll
      for (int st = 0; st < 4; st++) {
        const int rloc = 4 * st + gi;
        hw[st] = (rloc < wrows && ii < kh) ? H[(wrow0 + rloc) * (long long)ldh + ii] : 0.0f;
      }
    }
    // W's 16 rows staged by the waves in turn (rows wv, wv + XT/64, ...), a lane per column
    for (int k = wv; k < 16; k += XT / 64)
      for (int j = ln; j < ld; j += 64) wt[k * ld + j] = (k < kh && j < c) ? W[(long long)k * ldw + j] : 0.0f;
    __syncthreads();  // W staged (the only barrier before the block's final sums)
    if (tb_p >= 0) tb_s = tb.scale[tb_p];
    XST(1);
    // logits of the wave's 16 rows on MFMA, as k_gemm_nn<3> computes them; lane holds
    // logits[4 gi + r][16 tt + ii] -> the tile
    for (int tt = 0; 16 * tt < ld; tt++) {
      const int col = 16 * tt + ii;
      floatx4e acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t4 = 0; t4 < 4; t4++)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(
            ha[t4], col < ld ? wt[(4 * gi + t4) * ld + col] : 0.0f, acc, 0, 0, 0);
      if (col < ld) {
#pragma unroll
        for (int r = 0; r < 4; r++) L[(4 * gi + r) * S + col] = acc[r];
      }
    }
  } else {
    to_lds(logits);
  }
  wave_lds_fence();
  XST(2);
  float loss = 0.0f, wrong = 0.0f, se = 0.0f;
  float *l = L + rq * S;
  // up to 48 classes (reddit: 41) the lane's classes live in registers: every LDS read of the
  // row issued at once, the exps independent (the loops' LDS round trips were the kernel's
  // serial chain); wider rows take the same steps through the tile
  constexpr int NV = 12;
  const bool regs = c <= 4 * NV;
  float v[NV];
  if (regs) {
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = q + 4 * k < c ? l[q + 4 * k] : -1e30f;
  }
  if (t >= 0) {  // uniform over the quad
    float mx = -1e30f;
    if (regs) {
#pragma unroll
      for (int k = 0; k < NV; k++) mx = fmaxf(mx, v[k]);
    } else {
      for (int j = q; j < c; j += 4) mx = fmaxf(mx, l[j]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    // shifted logits to the tile, the true class's read back and compared, then (registers)
    // each exp computed once and kept for the grad in place of its logit
    bool w = false;
    float lt, s = 0.0f;
    if (regs) {
#pragma unroll
      for (int k = 0; k < NV; k++) {
        if (q + 4 * k < c) {
          v[k] -= mx;
          l[q + 4 * k] = v[k];
        }
      }
      wave_lds_fence();  // the quad's shifted logits are all in the tile
      lt = l[t];
#pragma unroll
      for (int k = 0; k < NV; k++) w |= q + 4 * k < c && v[k] > lt;
#pragma unroll
      for (int k = 0; k < NV; k++) {
        if (q + 4 * k < c) {
          v[k] = exp_nonpos(v[k]);
          s += v[k];
        }
      }
    } else {
      for (int j = q; j < c; j += 4) {
        const float x = l[j] - mx;
        l[j] = x;
        s += exp_nonpos(x);
      }
      wave_lds_fence();  // the quad's shifted logits are all in the tile
      lt = l[t];
      for (int j = q; j < c; j += 4) w |= l[j] > lt;
    }
    s += __shfl_xor(s, 1, 64);      // lanes 0, 1: s0 + s1; lanes 2, 3: s2 + s3
    se = s + __shfl_xor(s, 2, 64);  // (s0 + s1) + (s2 + s3) on every lane
    const int wq = (int)w | __shfl_xor((int)w, 1, 64);
    const int wall = wq | __shfl_xor(wq, 2, 64);
    if (q == 0) {
      loss = logf(se) - lt;
      wrong = wall ? 1.0f : 0.0f;
    }
  }
  wave_lds_fence();
  XST(3);
  if (write_back || FUSED) from_lds(logits);
  XST(4);
  if (training) {
    wave_lds_fence();  // the shifted logits have been read out
    if (rq < wrows) {
      if (t >= 0) {
        // prob = e / se and prob / count as correctly rounded quotients from the correctly
        // rounded reciprocals (div_rn: the IEEE division's bits, 3 VALU ops instead of ~10);
        // prob - 1 in float: the double temporary of hpdga module.cpp:145 rounds the same
        // exact difference once
        const float rse = 1.0f / se, cnt = (float)count, rcnt = 1.0f / cnt;
        if (regs) {
#pragma unroll
          for (int k = 0; k < NV; k++) {
            const int j = q + 4 * k;
            if (j < c) {
              float prob = div_rn(v[k], se, rse);
              if (j == t) prob -= 1.0f;
              l[j] = div_rn(prob, cnt, rcnt);
            }
          }
        } else {
          for (int j = q; j < c; j += 4) {
            float prob = div_rn(exp_nonpos(l[j]), se, rse);
            if (j == t) prob -= 1.0f;
            l[j] = div_rn(prob, cnt, rcnt);
          }
        }
        for (int j = c + q; j < ld; j += 4) l[j] = 0.0f;
      } else {
        for (int j = q; j < ld; j += 4) l[j] = 0.0f;
      }
    }
    wave_lds_fence();  // the wave's grad rows are complete
    XST(5);
    if (FUSED && dH) {
      // the output layer's input grad dH = grad W^T (Matmul::backward's a.grad) on MFMA in
      // k_xstream_nn's sequence (N = 16 outputs, K = c classes: step s, MFMA t, lane group g:
      // class 16 s + 4 g + t), from the grad tile
      floatx4e acc = {0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < c; s0 += 16) {
#pragma unroll
        for (int t4 = 0; t4 < 4; t4++) {
          const int j = s0 + 4 * gi + t4;
          const float av = j < c ? L[ii * S + j] : 0.0f;
          const float bv = (j < c && ii < kh) ? wt[ii * ld + j] : 0.0f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        }
      }
      if (ii < lddh) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int rr = 4 * gi + r;
          if (rr < wrows) dH[(wrow0 + rr) * (long long)lddh + ii] = acc[r];
        }
      }
      if (tb.table) {
        // k_ring_prescale's s_p * dH[i][4 v .. 4 v + 3] as one float4 at table row p = pos[i]:
        // lane (gi, 4 v + q) takes row 4 gi + q's plane v from its quad (a 4 x 4 transpose in
        // four shuffles: in round k lane s of the quad sends acc[(s - k) & 3] to lane (s - k) & 3)
        const int q = ii & 3, v = ii >> 2, p = tb_p;
        float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int out_r = (q - k) & 3, in_c = (q + k) & 3;
          const float send = out_r == 0 ? acc[0] : out_r == 1 ? acc[1] : out_r == 2 ? acc[2] : acc[3];
          const float got = __shfl(send, (ln & ~3) | in_c, 64);
#pragma unroll
          for (int m = 0; m < 4; m++) o[m] = in_c == m ? got : o[m];
        }
        if (p >= 0)
          reinterpret_cast<float4 *>(tb.table)[(long long)(p / RING_SR) * (4 * RING_SR) +
                                               v * RING_SR + p % RING_SR] =
              make_float4(o[0] * tb_s, o[1] * tb_s, o[2] * tb_s, o[3] * tb_s);
      }
    }
    XST(6);
    // the output layer's weight grad, this block's share: partial [kh][48] = H^T grad over
    // the block's rows (wave partials over their 16 rows on MFMA, added in wave order),
    // reduced over the blocks in block order by launch_tn_reduce_blocks
    if (FUSED && dWp) {
      floatx4e pw[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int st = 0; st < 4; st++) {  // 4-row steps over the wave's 16 rows
        const int rloc = 4 * st + gi;
        const bool ok = rloc < wrows;
#pragma unroll
        for (int tt = 0; tt < 3; tt++) {
          const int col = 16 * tt + ii;
          const float bv = (ok && col < ld) ? L[rloc * S + col] : 0.0f;
          pw[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(hw[st], bv, pw[tt], 0, 0, 0);
        }
      }
      from_lds(grad);
      XST(7);
      wave_lds_fence();  // the grad has been read out: the wave's tile takes its partial
#pragma unroll
      for (int tt = 0; tt < 3; tt++)
#pragma unroll
        for (int r = 0; r < 4; r++) L[(tt * 4 + r) * 64 + ln] = pw[tt][r];
      __syncthreads();  // every wave's partial is in LDS
      if (wv == 0) {
        float *pb = dWp + (long long)blockIdx.x * kh * 48;  // [kh][48] per block
#pragma unroll
        for (int tt = 0; tt < 3; tt++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            float v = pw[tt][r];
#pragma unroll
            for (int w2 = 1; w2 < XT / 64; w2++) v += smem[w2 * 16 * S + (tt * 4 + r) * 64 + ln];
            if (4 * gi + r < kh) pb[(4 * gi + r) * 48 + 16 * tt + ii] = v;
          }
      }
    } else {
      from_lds(grad);
    }
  }
  XST(8);
  // (loss, wrong) block sums in one pass: the wave sums (fixed xor tree), then thread 0 adds
  // the waves' in wave order
  loss = wave_sum(loss);
  wrong = wave_sum(wrong);
  if (ln == 0) {
    red[2 * wv] = loss;
    red[2 * wv + 1] = wrong;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ls = red[0], ws = red[1];
#pragma unroll
    for (int w2 = 1; w2 < XT / 64; w2++) {
      ls += red[2 * w2];
      ws += red[2 * w2 + 1];
    }
    partials[2 * blockIdx.x] = ls;
    partials[2 * blockIdx.x + 1] = ws;
    red[0] = ls;  // (this thread's own reads of red are done)
    red[1] = ws;
  }
  if (fin.ticket) xent_finish(fin, count, red);
  XST(9);
#ifdef PGCN_XENT_STAMPS
  st[11] = __builtin_amdgcn_s_memrealtime();
  const long long wslot = (long long)blockIdx.x * (XT / 64) + wv;
  if (ln < 12 && wslot < 16384) {
    unsigned long long x = st[0];
#pragma unroll
    for (int k = 1; k < 12; k++) x = ln == k ? st[k] : x;
    g_xent_stamps[wslot * 12 + ln] = x;
  }
#endif
}

#define PGCN_XENT_ARGS                                                                          \
  float *__restrict__ logits, int ld, float *__restrict__ grad, const int *__restrict__ truth,   \
      int n, int c, int count, int training, float *__restrict__ partials, int write_back,       \
      const float *__restrict__ H, int ldh, int kh, const float *__restrict__ W, int ldw,        \
      float *__restrict__ dH, int lddh, float *__restrict__ dWp, XentTable tb, XentFinal fin
// the loss over given logits (61 VGPRs at 8 waves per SIMD would spill its copy registers)
__global__ __launch_bounds__(XT) void k_xent_fwd(PGCN_XENT_ARGS) {
  xent_tile<false>(logits, ld, grad, truth, n, c, count, training, partials, write_back, H, ldh,
                   kh, W, ldw, dH, lddh, dWp, tb, fin);
}
// the fused output layer + loss at 8 waves per SIMD (<= 64 VGPRs, no spill; reddit training
// call 45.0 -> 43.2 us, r03)
template <int CC, int LDC, int KH>
__global__ __launch_bounds__(XT) __attribute__((amdgpu_waves_per_eu(8))) void k_out_xent(
    PGCN_XENT_ARGS) {
  xent_tile<true, CC, LDC, KH>(logits, ld, grad, truth, n, c, count, training, partials,
                               write_back, H, ldh, kh, W, ldw, dH, lddh, dWp, tb, fin);
}
#undef PGCN_XENT_ARGS

// sums[0] = sum loss partials, sums[1] = sum wrong, sums[2] = sum w^2 (fixed order)
__global__ __launch_bounds__(1024) void k_reduce_scalars(const float *__restrict__ partials,
                                                         int n_blocks,
                                                         const float *__restrict__ w,
                                                         long long n_w, float *__restrict__ sums,
                                                         int count, float wd,
                                                         float *__restrict__ out2,
                                                         const int *__restrict__ ctr,
                                                         int ring_cap, float *__restrict__ raw4,
                                                         PeerSmall peer) {
  __shared__ float red[16];
  float l = 0.0f, wr = 0.0f, q = 0.0f;
  // a thread's elements b = tid + 1024 u in u order, 8 loads in flight before their adds (r03
  // late: one dependent load per add made this single-block launch 8 us)
  constexpr int U = 8;
  for (int b0 = threadIdx.x; b0 < n_blocks; b0 += U * 1024) {
    float2 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 1024 < n_blocks) v[u] = reinterpret_cast<const float2 *>(partials)[b0 + u * 1024];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b0 + u * 1024 < n_blocks) {
        l += v[u].x;
        wr += v[u].y;
      }
  }
  // the weights: 32 loads in flight per thread (r04: citeseer's 59 k-float W1 took 7 rounds
  // of 8; a thread's elements are still added in index order, so the same bits)
  constexpr int UW = 32;
  for (long long i0 = threadIdx.x; i0 < n_w; i0 += UW * 1024) {
    float v[UW];
#pragma unroll
    for (int u = 0; u < UW; u++) v[u] = i0 + u * 1024 < n_w ? w[i0 + u * 1024] : 0.0f;
#pragma unroll
    for (int u = 0; u < UW; u++)
      if (i0 + u * 1024 < n_w) q += v[u] * v[u];
  }
  l = block_sum<1024>(l, red);
  wr = block_sum<1024>(wr, red);
  q = block_sum<1024>(q, red);
  if (threadIdx.x == 0) {
    if (sums) {
      sums[0] = l;
      sums[1] = wr;
    }
    if (raw4) {  // edge-cut: all-reduced in place, then composed by the host
      raw4[0] = l;
      raw4[1] = wr;
      raw4[2] = q;
      raw4[3] = (float)count;
    }
    if (out2) {  // one GPU: k_compose's arithmetic here, no second launch
      if (ctr) out2 += 4 * (ctr[1] % ring_cap);
      out2[0] = l / (float)count + wd * q / 2.0f;
      out2[1] = (float)(count - (int)wr) / (float)count;
    }
  }
  // edge-cut between processes: the loss / wrong pair all-reduced over the ranks in this
  // launch (one launch per pass fewer; the same pushes and rank-order sum as PeerComm's)
  if (raw4 && peer.k.world) {
    __syncthreads();
    (void)peer_allreduce_block(raw4, 2, peer);
  }
}

// Adam (hpdga optim.cpp:25-33): double temporaries where the reference has them.  red.src:
// the gradient's last reduction pass first (stored to g, as k_gemm_tn_reduce would); peer
// (edge-cut, the weight gradients' all-reduce between processes): the received slots summed
// in rank order at the tensor's arena offset first (k_peer_sum's sum, stored to g)
__device__ __forceinline__ void adam_range(float *__restrict__ w, const float *__restrict__ g,
                                           float *__restrict__ m, float *__restrict__ v,
                                           long long n, float step_size, float beta1,
                                           float beta2, float eps, float wd, int decay,
                                           const TnDeferred &red = TnDeferred{},
                                           const PeerRecv *peer = nullptr, long long off = 0,
                                           long long bid = -1, long long nblk = 0) {
  const double ob1 = 1.0 - (double)beta1, ob2 = 1.0 - (double)beta2;
  if (bid < 0) {
    bid = blockIdx.x;
    nblk = gridDim.x;
  }
  for (long long i = bid * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
    float grad;
    if (peer) {
      float p[kPeerMaxRanks];
#pragma unroll
      for (int q = 0; q < kPeerMaxRanks; q++)
        if (q < peer->world) p[q] = peer->slot[q][off + i];
      grad = p[0];
#pragma unroll
      for (int q = 1; q < kPeerMaxRanks; q++)
        if (q < peer->world) grad += p[q];
      const_cast<float *>(g)[i] = grad;
    } else if (red.src) {
      grad = tn_deferred_sum(red, i);
      const_cast<float *>(g)[i] = grad;
    } else {
      grad = g[i];
    }
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
  if (b.peer.world) {
    acquire_system_workgroup();  // the peers' pushes (peer_sync.hpp)
    adam_range(b.w[t], b.g[t], b.m[t], b.v[t], b.n[t], step_size, beta1, beta2, eps, wd,
               b.decay[t], TnDeferred{}, &b.peer, b.arena_off[t]);
    return;
  }
  adam_range(b.w[t], b.g[t], b.m[t], b.v[t], b.n[t], step_size, beta1, beta2, eps, wd,
             b.decay[t], b.red[t]);
}

// One launch for the optimizer step and the next training forward's masks (mask_adam, r06; one
// GPU): workgroups [0, ga + gb) draw the masks as k_dropout_mask does (segment a, then b), the
// rest are k_adam_multi's (tensor t = (block - ga - gb) / adam_blocks).  The two are
// independent: the masks are the next epoch's, drawn from the same stream positions whenever
// they are drawn (Dropout::ahead_descs).
__global__ __launch_bounds__(256) void k_adam_mask(AdamBatch b, float step_size, float beta1,
                                                   float beta2, float eps, float wd, MaskSeg ma,
                                                   MaskSeg mb, int ga, int gb, int adam_blocks,
                                                   const uint4 *__restrict__ table) {
  __shared__ uint4 lut[32 * 16];
  if ((int)blockIdx.x < ga + gb) {
    for (int i = threadIdx.x; i < 32 * 16; i += blockDim.x) {
      const int p = i >> 4, v = i & 15;
      lut[i] = table[(p >> 1) * 256 + (v << (4 * (p & 1)))];
    }
    __syncthreads();
    const bool in_a = (int)blockIdx.x < ga;
    const MaskSeg &sg = in_a ? ma : mb;
    const long long bid = in_a ? blockIdx.x : blockIdx.x - ga;
    const long long nblk = in_a ? ga : gb;
    if (sg.per == 2)
      dropout_mask_seg<2>(sg, lut, bid * blockDim.x + threadIdx.x, nblk * blockDim.x);
    else
      dropout_mask_seg<1>(sg, lut, bid * blockDim.x + threadIdx.x, nblk * blockDim.x);
    return;
  }
  const int k = (int)blockIdx.x - ga - gb, t = k / adam_blocks;
  adam_range(b.w[t], b.g[t], b.m[t], b.v[t], b.n[t], step_size, beta1, beta2, eps, wd,
             b.decay[t], b.red[t], nullptr, 0, k % adam_blocks, adam_blocks);
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

MaskSeg mask_seg_of(const MaskDraw &d) {
  MaskSeg g;
  g.states = d.states;
  g.n_chunks = d.n_chunks;
  g.elem0 = d.elem0;
  g.elem_end = d.elem_end;
  g.threshold = (int)(d.p * (float)0x7fffffff);  // as launch_dropout_mask
  g.mask = d.mask;
  g.per = d.per;
  return g;
}

__global__ void k_mask_lut(const uint4 *__restrict__ table, uint4 *__restrict__ lut) {
  const int i = threadIdx.x, p = i >> 4, v = i & 15;
  lut[i] = table[(p >> 1) * 256 + (v << (4 * (p & 1)))];
}

void launch_mask_lut(const void *table, void *lut, hipStream_t s) {
  PGCN_LAUNCH(k_mask_lut, dim3(1), dim3(32 * 16), 0, s, static_cast<const uint4 *>(table),
              static_cast<uint4 *>(lut));
}

void launch_dropout_mask(uint64_t *states, long long n_chunks, long long elem0,
                         long long elem_end, float p, uint64_t *mask, const void *table,
                         hipStream_t s, int max_blocks, int per) {
  if (n_chunks <= 0) return;
  PGCN_CHECK(per == 1 || per == 2, PGCN_E_INVALID, "dropout_mask: words per state");
  // hpdga module.cpp:211: threshold = int(p * MY_RAND_MAX) evaluated in float
  const int threshold = (int)(p * (float)0x7fffffff);
  // 8 KB LDS: up to 8 workgroups per CU (a side-stream draw takes fewer: max_blocks)
  const int grid = grid_for(ceil_div(ceil_div(n_chunks, per), 2), 256,
                            max_blocks > 0 ? max_blocks : 8 * kCUs);
  MaskSeg a;
  a.states = states;
  a.n_chunks = n_chunks;
  a.elem0 = elem0;
  a.elem_end = elem_end;
  a.threshold = threshold;
  a.mask = mask;
  a.per = per;
  PGCN_LAUNCH(k_dropout_mask, dim3(grid), dim3(256), 0, s, a, MaskSeg{}, grid,
              static_cast<const uint4 *>(table));
}

void launch_dropout_mask2(const MaskDraw &d0, const MaskDraw &d1, const void *table,
                          hipStream_t s) {
  MaskSeg sg[2];
  int g[2];
  const MaskDraw *d[2] = {&d0, &d1};
  for (int i = 0; i < 2; i++) {
    sg[i].states = d[i]->states;
    sg[i].n_chunks = d[i]->n_chunks;
    sg[i].elem0 = d[i]->elem0;
    sg[i].elem_end = d[i]->elem_end;
    sg[i].threshold = (int)(d[i]->p * (float)0x7fffffff);  // as launch_dropout_mask
    sg[i].mask = d[i]->mask;
    PGCN_CHECK(d[i]->per == 1 || d[i]->per == 2, PGCN_E_INVALID, "dropout_mask2: words per state");
    sg[i].per = d[i]->per;
    g[i] = sg[i].n_chunks > 0 ? grid_for(ceil_div(ceil_div(sg[i].n_chunks, d[i]->per), 2), 256,
                                         8 * kCUs)
                              : 0;
  }
  if (g[0] + g[1] == 0) return;
  PGCN_LAUNCH(k_dropout_mask, dim3(g[0] + g[1]), dim3(256), 0, s, sg[0], sg[1], g[0],
              static_cast<const uint4 *>(table));
}

void launch_dropout_apply_based(float *x, long long n, const uint64_t *mask, long long base,
                                float scale, hipStream_t s) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_dropout_apply, dim3(grid_for(ceil_div(n, 4))), dim3(256), 0, s, x, n,
                     mask, base, scale);
}

void launch_relu_fwd(float *x, long long n, uint8_t *mask, int training, hipStream_t s) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_relu_fwd, dim3(grid_for(n)), dim3(256), 0, s, x, n, mask, training);
}

void launch_relu_bwd(float *g, long long n, const uint8_t *mask, hipStream_t s) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_relu_bwd, dim3(grid_for(n)), dim3(256), 0, s, g, n, mask);
}

int xent_blocks(int n) { return (int)ceil_div(n, XR); }

__global__ void k_empty() {}

void launch_empty(int n, hipStream_t s) {
  for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
}

void launch_xent_fwd(float *logits, int ld, float *grad, const int *truth, int n, int c,
                     int count, int training, float *partials, hipStream_t s, int write_back,
                     const XentFinal *fin) {
  if (n <= 0) return;
  PGCN_CHECK(ld <= 124 && c <= ld && ld % 4 == 0, PGCN_E_INVALID,
             "xent: classes must be <= 124 (ld a multiple of 4)");
  PGCN_CHECK(!fin || (fin->ticket && fin->part4 && fin->out2 &&
                      (fin->group == 0 || (fin->group > 0 && fin->gticket && fin->gpart4))),
             PGCN_E_INVALID,
             "xent: the fused finish needs its ticket, partials and output");
  const size_t lds = (size_t)XR * xent_stride(ld) * sizeof(float);  // <= 64*124*4 = 31 KB
  PGCN_LAUNCH(k_xent_fwd, dim3(xent_blocks(n)), dim3(XT), lds, s, logits, ld, grad,
                     truth, n, c, count, training, partials, write_back, nullptr, 0, 0, nullptr, 0,
                     nullptr, 0, nullptr, XentTable{}, fin ? *fin : XentFinal{});
}

void launch_out_xent(const float *H, int ldh, int kh, const float *W, int ldw, float *logits,
                     int ld, float *grad, const int *truth, int n, int c, int count, int training,
                     float *partials, hipStream_t s, float *dH, int lddh, float *dWp,
                     const XentTable *tb, const XentFinal *fin) {
  note_path(KP_OUT_XENT);
  PGCN_CHECK(!fin || (fin->ticket && fin->part4 && fin->out2 &&
                      (fin->group == 0 || (fin->group > 0 && fin->gticket && fin->gpart4))),
             PGCN_E_INVALID,
             "out_xent: the fused finish needs its ticket, partials and output");
  const XentTable t = training && dH && tb ? *tb : XentTable{};
  PGCN_CHECK(!t.table || (kh == 16 && t.scale), PGCN_E_INVALID,
             "out_xent: a prescaled table of a 16-column dH");
  if (n <= 0) return;
  PGCN_CHECK(ld <= 116 && c <= ld && ld % 4 == 0 && kh >= 1 && kh <= 16, PGCN_E_INVALID,
             "out_xent: classes <= 116, hidden <= 16");
  PGCN_CHECK(!dWp || ld <= 48, PGCN_E_INVALID, "out_xent: the weight-grad partial needs <= 48 classes");
  // the tile, and (weight-grad partials) room for the waves' [3][4][64] partials in it
  // the tile (which also takes the waves' weight-grad partials) and W
  const size_t lds = ((size_t)XR * xent_stride(ld) + (size_t)16 * ld) * sizeof(float);
#define OUT_XENT(...)                                                                          \
  PGCN_LAUNCH((k_out_xent<__VA_ARGS__>), dim3(xent_blocks(n)), dim3(XT), lds, s, logits, ld, grad, \
              truth, n, c, count, training, partials, 1, H, ldh, kh, W, ldw,                     \
              training ? dH : nullptr, lddh, training ? dWp : nullptr, t, fin ? *fin : XentFinal{})
  if (c == 41 && ld == 44 && kh == 16)  // reddit (41 classes, hidden 16)
    OUT_XENT(41, 44, 16);
  else if (c == 7 && ld == 8 && kh == 16)  // cora (reassoc_small)
    OUT_XENT(7, 8, 16);
  else if (c == 6 && ld == 8 && kh == 16)  // citeseer
    OUT_XENT(6, 8, 16);
  else if (c == 3 && ld == 4 && kh == 16)  // pubmed
    OUT_XENT(3, 4, 16);
  else
    OUT_XENT(0, 0, 0);
#undef OUT_XENT
}

void launch_reduce_scalars(const float *partials, int n_blocks, const float *w, long long n_w,
                           float *sums, hipStream_t s, int count, float wd, float *out2,
                           const int *ctr, int ring_cap, float *raw4, const PeerSmall *peer) {
  PGCN_CHECK(!peer || (raw4 && peer->k.world >= 1 && peer->k.world <= kPeerMaxRanks),
             PGCN_E_INVALID, "reduce_scalars: peer all-reduce of the raw pair");
  PGCN_LAUNCH(k_reduce_scalars, dim3(1), dim3(1024), 0, s, partials, n_blocks, w, n_w,
                     sums, count, wd, out2, ctr, ring_cap, raw4, peer ? *peer : PeerSmall{});
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
  PGCN_LAUNCH(k_counters, dim3(1), dim3(64), 0, s, ctr, set, step, epoch);
}

void launch_adam_multi(const AdamBatch &b, float step_size, float beta1, float beta2, float eps,
                       float wd, hipStream_t s, const float *step_table, const int *ctr,
                       int table_cap, const MaskDraw *draws, int n_draws, const void *table) {
  if (b.count <= 0) return;
  long long nmax = 0;
  for (int t = 0; t < b.count; t++) nmax = std::max(nmax, b.n[t]);
  if (n_draws > 0) {
    PGCN_CHECK(!step_table && !b.peer.world && n_draws <= 2 && table, PGCN_E_INVALID,
               "adam_mask: eager one-GPU steps, at most two masks, the jump table");
    MaskSeg sg[2];
    int g[2] = {0, 0};
    for (int i = 0; i < n_draws; i++) {
      const MaskDraw &d = draws[i];
      PGCN_CHECK(d.per == 1 || d.per == 2, PGCN_E_INVALID, "adam_mask: words per state");
      sg[i].states = d.states;
      sg[i].n_chunks = d.n_chunks;
      sg[i].elem0 = d.elem0;
      sg[i].elem_end = d.elem_end;
      sg[i].threshold = (int)(d.p * (float)0x7fffffff);  // as launch_dropout_mask
      sg[i].mask = d.mask;
      sg[i].per = d.per;
      g[i] = d.n_chunks > 0 ? grid_for(ceil_div(ceil_div(d.n_chunks, d.per), 2), 256, 8 * kCUs) : 0;
    }
    const int ga = grid_for(nmax);
    PGCN_LAUNCH(k_adam_mask, dim3((unsigned)(g[0] + g[1] + ga * b.count)), dim3(256), 0, s, b,
                step_size, beta1, beta2, eps, wd, sg[0], sg[1], g[0], g[1], ga,
                static_cast<const uint4 *>(table));
    return;
  }
  PGCN_LAUNCH(k_adam_multi, dim3(grid_for(nmax), b.count), dim3(256), 0, s, b, step_size,
                     beta1, beta2, eps, wd, step_table, ctr, table_cap);
}

void launch_adam(float *w, const float *g, float *m, float *v, long long n, float step_size,
                 float beta1, float beta2, float eps, float wd, int decay, hipStream_t s,
                 const float *step_table, const int *ctr, int table_cap) {
  if (n <= 0) return;
  PGCN_LAUNCH(k_adam, dim3(grid_for(n)), dim3(256), 0, s, w, g, m, v, n, step_size,
                     beta1, beta2, eps, wd, decay, step_table, ctr, table_cap);
}

#ifdef PGCN_XENT_STAMPS
extern "C" int pgcn_debug_xent_stamps(unsigned long long *host, long long n) {
  if (n > 16384LL * 12) n = 16384LL * 12;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xent_stamps), (size_t)n * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
}  // namespace pgcn
