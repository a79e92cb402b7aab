// tools/xs_micro.hip -- streaming-read shapes for the X-stream GEMMs (diagnostic tool).
// Reads the reddit-shaped X [232965][604] fp32 (563 MB) once per launch with the access shape
// of a wave-instruction varied, no MFMA (plain adds), to separate the shape's cost from the
// kernels' compute: which load shape and occupancy reach the ~6 TB/s HBM read rate.
//   A  16 rows x 64 B per instruction  (k_xstream_nn's lane map: lane (i, g) -> row i, k 4g..)
//   B   4 rows x 256 B per instruction (lane l -> row l / 16, floats 4 (l % 16) ..)
//   C  1 KB contiguous per instruction (a wave's 16-row group read as one flat range)
//   M  k_xstream_nn's loop with its MFMAs (16x16x4 f32), unmasked, N = 16
//   L  loader waves (LDS-DMA ring of row groups) + MFMA consumer waves
//   P  M software-pipelined across a wave's row groups (next group's loads during the MFMAs)
// at 2 waves per SIMD (512 or 1024 workgroups), plain and nontemporal loads.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/xs_micro tools/xs_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../parallel-gcn_amd/csrc/lds_dma.hpp"

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

constexpr int M = 232965, LDA = 604, K = 602;
constexpr int NS = 40;  // 16-float steps of a row (640 >= K)

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ float4 ld4(const float *p) {
  if constexpr (NT) {
    const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const float4 *>(p);
  }
}

__global__ void fill(float *x, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    x[i] = (float)((i * 2654435761u) & 1023) * (1.0f / 1024);
}

// A: lane (i, g) reads X[row i][16 s + 4 g ..] for s < NS (all loads, then the adds)
template <int OCC, bool NT>
__global__ __launch_bounds__(256, OCC) void shape_a(const float *__restrict__ X,
                                                    float *__restrict__ out) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  float tot = 0.f;
  for (long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    const long long row = rg * 16 + i;
    const float *a = X + (row < M ? row : 0) * (long long)LDA + 4 * g;
    float4 v[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) v[s] = 16 * s + 4 * g < K ? ld4<NT>(a + 16 * s) : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < NS; s++) tot += v[s].x + v[s].y + v[s].z + v[s].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = tot;
}

// S: shape A with a stall of SLEEP x 64 cycles after each group's adds (a stand-in for the
// MFMA phase: the wave issues nothing meanwhile)
template <int SLEEP>
__global__ __launch_bounds__(256, 2) void shape_s(const float *__restrict__ X,
                                                  float *__restrict__ out) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  float tot = 0.f;
  for (long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    const long long row = rg * 16 + i;
    const float *a = X + (row < M ? row : 0) * (long long)LDA + 4 * g;
    float4 v[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) v[s] = 16 * s + 4 * g < K ? ld4<false>(a + 16 * s) : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < NS; s++) tot += v[s].x + v[s].y + v[s].z + v[s].w;
#pragma unroll
    for (int z = 0; z < SLEEP / 8; z++) __builtin_amdgcn_s_sleep(8);
  }
  out[blockIdx.x * 256 + threadIdx.x] = tot;
}

// B: lane l reads X[row 4q + l / 16][64 c + 4 (l % 16) ..] for q < 4, c < 10
template <int OCC, bool NT>
__global__ __launch_bounds__(256, OCC) void shape_b(const float *__restrict__ X,
                                                    float *__restrict__ out) {
  const int lane = threadIdx.x & 63, r = lane >> 4, c4 = 4 * (lane & 15);
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  float tot = 0.f;
  for (long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    float4 v[NS];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const long long row = rg * 16 + 4 * q + r;
      const float *a = X + (row < M ? row : 0) * (long long)LDA + c4;
#pragma unroll
      for (int c = 0; c < 10; c++)
        v[10 * q + c] = 64 * c + c4 < K ? ld4<NT>(a + 64 * c) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < NS; s++) tot += v[s].x + v[s].y + v[s].z + v[s].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = tot;
}

// C: the group's 16 x 604 floats as one flat range, 1 KB per instruction (38 instructions)
template <int OCC, bool NT>
__global__ __launch_bounds__(256, OCC) void shape_c(const float *__restrict__ X,
                                                    float *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  constexpr int GF = 16 * LDA;  // floats per group
  constexpr int NI = (GF + 255) / 256;
  float tot = 0.f;
  for (long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    const long long f0 = rg * GF;
    const long long lim = (long long)M * LDA;
    float4 v[NI];
#pragma unroll
    for (int s = 0; s < NI; s++) {
      const long long f = f0 + 256 * s + 4 * lane;
      v[s] = (256 * s + 4 * lane < GF && f < lim) ? ld4<NT>(X + f) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < NI; s++) tot += v[s].x + v[s].y + v[s].z + v[s].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = tot;
}

// M: shape A feeding the MFMAs of k_xstream_nn (B = W^T staged in LDS); VAR 1: the B reads
// from LDS but plain adds instead of MFMAs; VAR 2: the MFMAs with B from registers (no LDS);
// VAR 3: as VAR 0 without the per-group stores (one store per lane at the end); VAR 4: as
// VAR 3 with the X loads replaced by register values (the MFMA chain alone); VAR 5: VAR 4 with
// B from registers; ACC: independent
// accumulators the steps rotate through (summed at the end of the group)
template <int OCC, bool NT, int VAR = 0, int ACC = 1>
__global__ __launch_bounds__(256, OCC) void shape_m(const float *__restrict__ X,
                                                    const float *__restrict__ W,
                                                    float *__restrict__ out) {
  constexpr int S = 648;  // 8 mod 16 dwords
  __shared__ float bt[16 * S];
  for (int e = threadIdx.x; e < 16 * 640; e += 256) {
    const int k = e >> 4, j = e & 15;
    bt[j * S + k] = k < K ? W[k * 16 + j] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  const float *bl = bt + i * S + 4 * g;
  float keep = 0.f;
  for (long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    const long long row = rg * 16 + i;
    const float *a = X + (row < M ? row : 0) * (long long)LDA + 4 * g;
    float4 v[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if constexpr (VAR >= 4) {
        const float f = (float)(rg + s);
        v[s] = make_float4(f, f + 1.f, f + 2.f, keep);
      } else {
        v[s] = 16 * s + 4 * g < K ? ld4<NT>(a + 16 * s) : make_float4(0, 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    floatx4 accs[ACC];
#pragma unroll
    for (int q = 0; q < ACC; q++) accs[q] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (ACC > 1 && 16 * s >= K) break;  // steps wholly past K add nothing
      floatx4 &acc = accs[s % ACC];
      const float4 b = (VAR == 2 || VAR == 5) ? make_float4(bl[0], bl[1], bl[2], bl[3])
                                : *reinterpret_cast<const float4 *>(bl + 16 * s);
      if constexpr (VAR == 1) {
        acc[0] += v[s].x * b.x;
        acc[1] += v[s].y * b.y;
        acc[2] += v[s].z * b.z;
        acc[3] += v[s].w * b.w;
      } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].z, b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].w, b.w, acc, 0, 0, 0);
      }
    }
    floatx4 acc = accs[0];
#pragma unroll
    for (int q = 1; q < ACC; q++) acc += accs[q];
    if constexpr (VAR >= 3) {
      keep += acc[0] + acc[1] + acc[2] + acc[3];
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const long long rr = rg * 16 + 4 * g + r;
        if (rr < M) out[rr * 16 + i] = acc[r];
      }
    }
  }
  if constexpr (VAR >= 3) out[blockIdx.x * 256 + threadIdx.x] = keep;
}

// P: shape M software-pipelined across groups: step s's registers are refilled with the next
// group's step s right after its MFMAs, so a wave's loads stay in flight while it computes
template <int OCC, bool NT>
__global__ __launch_bounds__(256, OCC) void shape_p(const float *__restrict__ X,
                                                    const float *__restrict__ W,
                                                    float *__restrict__ out) {
  constexpr int S = 648;
  __shared__ float bt[16 * S];
  for (int e = threadIdx.x; e < 16 * 640; e += 256) {
    const int k = e >> 4, j = e & 15;
    bt[j * S + k] = k < K ? W[k * 16 + j] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * 4;
  const float *bl = bt + i * S + 4 * g;
  long long rg = blockIdx.x * 4LL + (threadIdx.x >> 6);
  if (rg >= n_rg) return;
  float4 v[NS];
  {
    const long long row = min(rg * 16 + i, (long long)M - 1);
    const float *a = X + row * (long long)LDA + 4 * g;
#pragma unroll
    for (int s = 0; s < NS; s++) v[s] = 16 * s + 4 * g < K ? ld4<NT>(a + 16 * s) : make_float4(0, 0, 0, 0);
  }
  for (; rg < n_rg; rg += wstride) {
    const long long nrg = rg + wstride < n_rg ? rg + wstride : rg;
    const long long nrow = min(nrg * 16 + i, (long long)M - 1);
    const float *na = X + nrow * (long long)LDA + 4 * g;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const float4 b = *reinterpret_cast<const float4 *>(bl + 16 * s);
      if (16 * s + 16 > K) {
        const int kb = 16 * s + 4 * g;
        if (kb + 1 > K) v[s].x = 0.f;
        if (kb + 2 > K) v[s].y = 0.f;
        if (kb + 3 > K) v[s].z = 0.f;
        if (kb + 4 > K) v[s].w = 0.f;
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s].w, b.w, acc, 0, 0, 0);
      if (16 * s + 4 * g < K) v[s] = ld4<NT>(na + 16 * s);  // lanes past K: zeroed on use
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const long long rr = rg * 16 + 4 * g + r;
      if (rr < M) out[rr * 16 + i] = acc[r];
    }
  }
}

// H: shape M with each group's steps in PH phases of NS / PH loads + their MFMAs (same MFMA
// order as M), so fewer registers and OCC waves per SIMD
template <int THREADS, int MINB, int PH>
__global__ __launch_bounds__(THREADS, MINB) void shape_h(const float *__restrict__ X,
                                                    const float *__restrict__ W,
                                                    float *__restrict__ out) {
  constexpr int S = 648;
  constexpr int NP = NS / PH;
  __shared__ float bt[16 * S];
  for (int e = threadIdx.x; e < 16 * 640; e += THREADS) {
    const int k = e >> 4, j = e & 15;
    bt[j * S + k] = k < K ? W[k * 16 + j] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const long long n_rg = (M + 15) / 16, wstride = (long long)gridDim.x * (THREADS / 64);
  const float *bl = bt + i * S + 4 * g;
  for (long long rg = blockIdx.x * (THREADS / 64LL) + (threadIdx.x >> 6); rg < n_rg; rg += wstride) {
    const long long row = rg * 16 + i;
    const float *a = X + (row < M ? row : 0) * (long long)LDA + 4 * g;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ph = 0; ph < PH; ph++) {
      float4 v[NP];
#pragma unroll
      for (int q = 0; q < NP; q++) {
        const int s = ph * NP + q;
        v[q] = 16 * s + 4 * g < K ? ld4<false>(a + 16 * s) : make_float4(0, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NP; q++) {
        const int s = ph * NP + q;
        const float4 b = *reinterpret_cast<const float4 *>(bl + 16 * s);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q].x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q].y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q].z, b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v[q].w, b.w, acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const long long rr = rg * 16 + 4 * g + r;
      if (rr < M) out[rr * 16 + i] = acc[r];
    }
  }
}

// L: loader / consumer split.  Waves 0..NL-1 stream whole 16-row groups into an LDS ring by
// LDS-DMA (1 KB per instruction, no VGPRs; each loader one group at a time, vmcnt(0) then
// publish); waves NL.. (consumers) read the A fragments from LDS and run the MFMAs with B
// held in registers.  Row stride ST chunks of 16 B (== 2 mod 4: conflict-free ds_read_b128).
constexpr int L_NCH = (K + 3) / 4;                      // 16-B chunks of a row
constexpr int L_ST = (L_NCH + 1) / 4 * 4 + 2 >= L_NCH ? (L_NCH + 1) / 4 * 4 + 2 : L_NCH + 4;
constexpr int L_NI = (16 * L_ST + 63) / 64;             // DMA instructions per group
constexpr int L_SLOT = L_NI * 1024;                     // bytes per slot (1 KB multiple)
constexpr int L_NSLOT = (160 * 1024 - 64) / L_SLOT < 4 ? (160 * 1024 - 64) / L_SLOT : 4;

__device__ __forceinline__ void glds16_nt(const void *gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// NOMMA: the consumers only hand the slots back (the loaders' streaming rate alone)
// CF: consumers copy the group's fragments to registers and hand the slot back before the MFMAs
// PRIO: loaders at s_setprio 3; RT: slot geometry from kernel arguments (st, ni: runtime)
template <int NL, int NC, bool NTL = false, bool NOMMA = false, bool CF = false, bool PRIO = false,
          bool RT = false>
__global__ __launch_bounds__(64 * (NL + NC), 1) void shape_l(const float *__restrict__ X,
                                                             const float *__restrict__ W,
                                                             float *__restrict__ out, int rt_st = L_ST,
                                                             int rt_ni = L_NI) {
  const int ST = RT ? rt_st : L_ST, NI = RT ? rt_ni : L_NI;
  __shared__ __attribute__((aligned(1024))) char lds[L_NSLOT * L_SLOT + 64];
  unsigned *ready = reinterpret_cast<unsigned *>(lds + L_NSLOT * L_SLOT);
  unsigned *freed = ready + 8;
  if (threadIdx.x < 16) ready[threadIdx.x] = 0u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long n_rg = (M + 15) / 16;
  const int G = gridDim.x;
  const int T = (int)((n_rg - blockIdx.x + G - 1) / G);
  if (wave < NL) {  // loader
    if (PRIO) __builtin_amdgcn_s_setprio(3);
    const unsigned base = __builtin_amdgcn_readfirstlane(
        (unsigned)reinterpret_cast<size_t>((__attribute__((address_space(3))) char *)lds));
    for (int t = wave; t < T; t += NL) {
      const int slot = t % L_NSLOT;
      if (t >= L_NSLOT) pgcn::lds_wait_ge(freed + slot, (unsigned)(t - L_NSLOT + 1));
      const long long row0 = (blockIdx.x + (long long)t * G) * 16;
#pragma unroll 4
      for (int q = 0; q < NI; q++) {
        const int c = q * 64 + lane;
        int r = c / ST, ch = c - r * ST;
        r = r < 16 ? r : 15;
        ch = ch < L_NCH ? ch : L_NCH - 1;
        long long row = row0 + r;
        row = row < M ? row : M - 1;
        if constexpr (NTL)
          glds16_nt(X + row * LDA + 4 * ch, base + (unsigned)(slot * L_SLOT + q * 1024));
        else
          pgcn::glds16(X + row * LDA + 4 * ch, base + (unsigned)(slot * L_SLOT + q * 1024));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __atomic_store_n(ready + slot, (unsigned)(t + 1), __ATOMIC_RELAXED);
      asm volatile("" ::: "memory");
    }
    return;
  }
  const int cid = wave - NL, g = lane >> 4, i = lane & 15;
  float4 b[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) {
    const int k = 16 * s + 4 * g;
    b[s] = make_float4(k < K ? W[k * 16 + i] : 0.f, k + 1 < K ? W[(k + 1) * 16 + i] : 0.f,
                       k + 2 < K ? W[(k + 2) * 16 + i] : 0.f, k + 3 < K ? W[(k + 3) * 16 + i] : 0.f);
  }
  for (int t = cid; t < T; t += NC) {
    const int slot = t % L_NSLOT;
    pgcn::lds_wait_ge(ready + slot, (unsigned)(t + 1));
    const char *a = lds + slot * L_SLOT + i * L_ST * 16 + g * 16;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    float4 va[CF ? NS : 1];
    if constexpr (CF) {
#pragma unroll
      for (int s = 0; s < NS; s++)
        if (16 * s < K) va[s] = *reinterpret_cast<const float4 *>(a + 64 * s);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __atomic_store_n(freed + slot, (unsigned)(t + 1), __ATOMIC_RELAXED);
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
      if (NOMMA || 16 * s >= K) break;
      float4 v = CF ? va[CF ? s : 0] : *reinterpret_cast<const float4 *>(a + 64 * s);
      if (16 * s + 16 > K) {
        const int kb = 16 * s + 4 * g;
        if (kb + 1 > K) v.x = 0.f;
        if (kb + 2 > K) v.y = 0.f;
        if (kb + 3 > K) v.z = 0.f;
        if (kb + 4 > K) v.w = 0.f;
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, b[s].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, b[s].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.z, b[s].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(v.w, b[s].w, acc, 0, 0, 0);
    }
    if constexpr (!CF) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __atomic_store_n(freed + slot, (unsigned)(t + 1), __ATOMIC_RELAXED);
      asm volatile("" ::: "memory");
    }
    const long long rg = blockIdx.x + (long long)t * G;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const long long rr = rg * 16 + 4 * g + r;
      if (rr < M) out[rr * 16 + i] = acc[r];
    }
  }
}

static float *g_x, *g_w, *g_out;

template <typename F>
static void time_it(const char *name, int wgs, F launch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 3; r++) launch(wgs);
  CHECK(hipDeviceSynchronize());
  const int reps = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; r++) launch(wgs);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)M * K * 4;
  printf("{\"kernel\": \"%s\", \"wgs\": %d, \"us\": %.2f, \"GBs\": %.0f}\n", name, wgs, ms * 1e3,
         bytes / ms / 1e6);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

#define RUN(KER, OCC, NT, WGS)                                                                  \
  time_it(#KER "<" #OCC "," #NT ">", WGS, [](int w) {                                          \
    hipLaunchKernelGGL((KER<OCC, NT>), dim3(w), dim3(256), 0, 0, g_x, g_out);                  \
  })
#define RUNM(OCC, NT, WGS)                                                                      \
  time_it("shape_m<" #OCC "," #NT ">", WGS, [](int w) {                                        \
    hipLaunchKernelGGL((shape_m<OCC, NT>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);         \
  })
#define RUNP(OCC, NT, WGS)                                                                      \
  time_it("shape_p<" #OCC "," #NT ">", WGS, [](int w) {                                        \
    hipLaunchKernelGGL((shape_p<OCC, NT>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);         \
  })

int main() {
  const long long n = (long long)M * LDA;
  CHECK(hipMalloc(&g_x, n * 4));
  CHECK(hipMalloc(&g_w, 640 * 16 * 4));
  CHECK(hipMalloc(&g_out, (long long)M * 16 * 4 + 4096 * 256 * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, g_x, n);
  hipLaunchKernelGGL(fill, dim3(40), dim3(256), 0, 0, g_w, 640LL * 16);
  CHECK(hipDeviceSynchronize());
  RUN(shape_a, 2, false, 512);
  RUN(shape_a, 2, true, 512);
  RUN(shape_a, 2, false, 1024);
  RUN(shape_b, 2, false, 512);
  RUN(shape_b, 2, true, 512);
  RUN(shape_b, 2, false, 1024);
  RUN(shape_c, 2, false, 512);
  RUN(shape_c, 2, true, 512);
  RUN(shape_c, 2, false, 1024);
  RUNM(2, false, 512);
  RUNM(2, true, 512);
  RUNM(2, false, 1024);
  RUNP(2, false, 512);
  RUNP(1, false, 256);
  time_it("shape_s<40>", 512, [](int w) {
    hipLaunchKernelGGL((shape_s<40>), dim3(w), dim3(256), 0, 0, g_x, g_out);
  });
  time_it("shape_s<80>", 512, [](int w) {
    hipLaunchKernelGGL((shape_s<80>), dim3(w), dim3(256), 0, 0, g_x, g_out);
  });
  time_it("shape_s<160>", 512, [](int w) {
    hipLaunchKernelGGL((shape_s<160>), dim3(w), dim3(256), 0, 0, g_x, g_out);
  });
  time_it("shape_m_lds_adds", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 1>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_no_stores", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 3>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_h<256,2,2>", 512, [](int w) {
    hipLaunchKernelGGL((shape_h<256, 2, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_h<256,3,2>", 768, [](int w) {
    hipLaunchKernelGGL((shape_h<256, 3, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_h<512,2,2>", 512, [](int w) {
    hipLaunchKernelGGL((shape_h<512, 2, 2>), dim3(w), dim3(512), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_h<512,2,4>", 512, [](int w) {
    hipLaunchKernelGGL((shape_h<512, 2, 4>), dim3(w), dim3(512), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_h<1024,2,4>", 512, [](int w) {
    hipLaunchKernelGGL((shape_h<1024, 2, 4>), dim3(w), dim3(1024), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_mfma_only", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 4>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_acc2", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 0, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_acc4", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 0, 4>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_acc4_no_stores", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 3, 4>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_mfma_only_acc4", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 4, 4>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_mfma_only_acc2", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 4, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_mfma_only_regb_acc4", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 5, 4>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_mfma_only_regb_acc1", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 5, 1>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,3>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 3>), dim3(w), dim3(320), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2,nt>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2,nomma>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, false, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2,nt,nomma>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2,nt,cf>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true, false, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<3,2,nt,cf>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<3, 2, true, false, true>), dim3(w), dim3(320), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<4,2,nt,cf>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<4, 2, true, false, true>), dim3(w), dim3(384), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<3,3,nt,cf>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<3, 3, true, false, true>), dim3(w), dim3(384), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<4,2,nt,nomma>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<4, 2, true, true>), dim3(w), dim3(384), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2,nt,prio>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true, false, false, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out, L_ST, L_NI);
  });
  time_it("shape_l<2,2,nt,rt>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true, false, false, false, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out, L_ST, L_NI);
  });
  time_it("shape_l<2,2,nt,prio,rt>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2, true, false, false, true, true>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out, L_ST, L_NI);
  });
  time_it("shape_l<3,2,nt>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<3, 2, true>), dim3(w), dim3(320), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<1,3>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<1, 3>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<2,2>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<2, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_l<3,3>", 256, [](int w) {
    hipLaunchKernelGGL((shape_l<3, 3>), dim3(w), dim3(384), 0, 0, g_x, g_w, g_out);
  });
  time_it("shape_m_reg_b", 512, [](int w) {
    hipLaunchKernelGGL((shape_m<2, false, 2>), dim3(w), dim3(256), 0, 0, g_x, g_w, g_out);
  });
  CHECK(hipFree(g_x));
  CHECK(hipFree(g_w));
  CHECK(hipFree(g_out));
  return 0;
}
