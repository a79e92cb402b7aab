// parallel-gcn_amd/csrc/k_graphsum.hip -- GraphSum: CSR adjacency (Â, with self loops) x
// dense node features, for gfx950.
//
// Replaces graphsum_kernel (src/module.cu:172-210: one thread per (row, col), a sequential
// walk over the row) and hpdga GraphSum::forward/backward (module.cpp:82-111).
//
// Layout: node features are row-major [n][ld] fp32 with ld a multiple of 4 (16-B rows of
// float4; padding columns are kept zero by every producer).  A wavefront owns one work item
// = (row, slot range <= chunk); its 64 lanes are split into NB = 64/VEC neighbour groups of
// VEC lanes, each lane holding one float4 of the row: one wave instruction gathers NB full
// neighbour rows (NB*VEC*16 bytes, e.g. 16 rows x 64 B at dim 16) with coalesced 16-B lanes.
// Neighbour groups are summed in a fixed tree (xor-shuffles when VEC is a power of two, LDS
// otherwise), so the result is deterministic run to run.  Rows longer than one chunk are
// split over several waves that write partial rows; a second kernel adds the partials in
// slot order.  The schedule (items, combine list) is built once per (graph, VEC) on the host.
#include "common.hpp"
#include "kernels.hpp"

namespace pgcn {

__device__ __forceinline__ float4 f4_fma(float w, float4 x, float4 a) {
  a.x = fmaf(w, x.x, a.x);
  a.y = fmaf(w, x.y, a.y);
  a.z = fmaf(w, x.z, a.z);
  a.w = fmaf(w, x.w, a.w);
  return a;
}
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4_shfl_xor(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64), __shfl_xor(v.z, m, 64),
                     __shfl_xor(v.w, m, 64));
}

template <int VEC>
__global__ __launch_bounds__(256) void k_graphsum(const int4 *__restrict__ items, int n_items,
                                                  const int *__restrict__ indices,
                                                  const float *__restrict__ vals,
                                                  const float4 *__restrict__ in, int ld4_in,
                                                  float4 *__restrict__ out, int ld4_out,
                                                  float4 *__restrict__ partial) {
  constexpr int NB = 64 / VEC;
  constexpr bool POW2 = (VEC & (VEC - 1)) == 0;
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const int nb = lane / VEC, v = lane - nb * VEC;
  const bool active = nb < NB;
  for (long long it = (long long)blockIdx.x * 4 + wib; it < n_items;
       it += (long long)gridDim.x * 4) {
    const int4 item = items[it];  // {row, begin, end, slot}
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
      int j = item.y + nb;
      const int end = item.z;
      for (; j + 3 * NB < end; j += 4 * NB) {
        const int c0 = indices[j], c1 = indices[j + NB], c2 = indices[j + 2 * NB],
                  c3 = indices[j + 3 * NB];
        const float w0 = vals[j], w1 = vals[j + NB], w2 = vals[j + 2 * NB], w3 = vals[j + 3 * NB];
        const float4 x0 = in[(long long)c0 * ld4_in + v];
        const float4 x1 = in[(long long)c1 * ld4_in + v];
        const float4 x2 = in[(long long)c2 * ld4_in + v];
        const float4 x3 = in[(long long)c3 * ld4_in + v];
        acc = f4_fma(w0, x0, acc);
        acc = f4_fma(w1, x1, acc);
        acc = f4_fma(w2, x2, acc);
        acc = f4_fma(w3, x3, acc);
      }
      for (; j < end; j += NB) acc = f4_fma(vals[j], in[(long long)indices[j] * ld4_in + v], acc);
    }
    if constexpr (POW2) {
#pragma unroll
      for (int m = VEC; m < 64; m <<= 1) acc = f4_add(acc, f4_shfl_xor(acc, m));
    } else {
      // every lane gathers the NB partial float4s of its column v in group order
      float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < NB; k++) {
        const int src = k * VEC + (v < VEC ? v : 0);
        tot = f4_add(tot, make_float4(__shfl(acc.x, src, 64), __shfl(acc.y, src, 64),
                                      __shfl(acc.z, src, 64), __shfl(acc.w, src, 64)));
      }
      acc = tot;
    }
    if (nb == 0) {
      if (item.w < 0)
        out[(long long)item.x * ld4_out + v] = acc;
      else
        partial[(long long)item.w * VEC + v] = acc;
    }
  }
}

// out[row] = sum of partial slots [first, first+count) in slot order
template <int VEC>
__global__ __launch_bounds__(256) void k_graphsum_combine(const int4 *__restrict__ comb,
                                                          int n_comb,
                                                          const float4 *__restrict__ partial,
                                                          float4 *__restrict__ out, int ld4_out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ci = t / VEC;
  const int v = (int)(t - ci * VEC);
  if (ci >= n_comb) return;
  const int4 c = comb[ci];  // {row, first_slot, count, -}
  float4 acc = partial[(long long)c.y * VEC + v];
  for (int s = 1; s < c.z; s++) acc = f4_add(acc, partial[(long long)(c.y + s) * VEC + v]);
  out[(long long)c.x * ld4_out + v] = acc;
}

template <int VEC>
static void launch_vec(const GraphSchedule &s, const int *indices, const float *vals,
                       const float *in, int ld_in, float *out, int ld_out, float *partial,
                       hipStream_t st) {
  if (s.n_items > 0) {
    long long blocks = ceil_div(s.n_items, 4);
    if (blocks > 65535 * 16) blocks = 65535 * 16;
    hipLaunchKernelGGL(k_graphsum<VEC>, dim3((unsigned)blocks), dim3(256), 0, st, s.items,
                       s.n_items, indices, vals, reinterpret_cast<const float4 *>(in), ld_in / 4,
                       reinterpret_cast<float4 *>(out), ld_out / 4,
                       reinterpret_cast<float4 *>(partial));
  }
  if (s.n_comb > 0) {
    const long long threads = (long long)s.n_comb * VEC;
    hipLaunchKernelGGL(k_graphsum_combine<VEC>, dim3((unsigned)ceil_div(threads, 256)),
                       dim3(256), 0, st, s.comb, s.n_comb,
                       reinterpret_cast<const float4 *>(partial), reinterpret_cast<float4 *>(out),
                       ld_out / 4);
  }
}

void launch_graphsum(const GraphSchedule &s, const int *indices, const float *vals,
                     const float *in, int ld_in, float *out, int ld_out, float *partial,
                     hipStream_t st) {
  switch (s.vec) {
#define PGCN_VEC_CASE(V) \
  case V:                \
    launch_vec<V>(s, indices, vals, in, ld_in, out, ld_out, partial, st); break;
    PGCN_VEC_CASE(1) PGCN_VEC_CASE(2) PGCN_VEC_CASE(3) PGCN_VEC_CASE(4) PGCN_VEC_CASE(5)
    PGCN_VEC_CASE(6) PGCN_VEC_CASE(7) PGCN_VEC_CASE(8) PGCN_VEC_CASE(9) PGCN_VEC_CASE(10)
    PGCN_VEC_CASE(11) PGCN_VEC_CASE(12) PGCN_VEC_CASE(16) PGCN_VEC_CASE(32)
#undef PGCN_VEC_CASE
    default:
      throw Error(PGCN_E_INVALID, "graphsum: unsupported row width (float4 count " +
                                      std::to_string(s.vec) + ")");
  }
}

bool graphsum_vec_supported(int vec) {
  return (vec >= 1 && vec <= 12) || vec == 16 || vec == 32;
}

}  // namespace pgcn
