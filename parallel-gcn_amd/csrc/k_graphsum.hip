// parallel-gcn_amd/csrc/k_graphsum.hip -- GraphSum: CSR adjacency (Â, with self loops) x
// dense node features, for gfx950.
//
// Replaces graphsum_kernel (src/module.cu:172-210: one thread per (row, col), a sequential
// walk over the row) and hpdga GraphSum::forward/backward (module.cpp:82-111).
//
// Layout: node features are row-major [n][ld] fp32 with ld a multiple of 4 (16-B rows of
// float4; padding columns are kept zero by every producer).
//
// Work items.  The adjacency is cut into NBC column blocks (NBC = 8 on large graphs:
// one per XCD) and every (row, column block) segment into items of <= `chunk` slots
// (host-built schedule, sorted longest first inside a block).  Workgroup w serves column
// block w % NBC: consecutive workgroup ids are dealt round-robin to the 8 XCDs, so every
// workgroup of one column block runs on the same XCD and that XCD's 4 MB L2 holds the
// block's 1/8 slice of the gathered feature table (a speed property only -- results do not
// depend on placement).  A group of G lanes owns one item: its lanes are NB = G/VEC
// neighbour sub-groups of VEC lanes, each lane one float4 of a neighbour row, so one wave
// instruction gathers 64/VEC whole neighbour rows with 16-B lanes.  Sub-groups are summed in
// a fixed xor-tree => deterministic.  Each item writes its partial row to a slot; a combine
// kernel adds a row's slots in slot order (skipped for rows that are one whole item).
#include "common.hpp"
#include "gs_epilogue.hpp"
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

// One row by a whole workgroup (g_gs_split 3: the small graphs' hub rows): sub-group s of
// VEC lanes walks slots begin + s, + 256 / VEC, ...; the sub-groups are summed in a fixed
// xor-tree per wave, then the four waves in wave order through LDS.
template <int VEC>
__device__ __forceinline__ void wide_item(const int4 item, const int *__restrict__ indices,
                                          const float *__restrict__ vals,
                                          const float4 *__restrict__ in, int ld4_in,
                                          float4 *__restrict__ out, int ld4_out,
                                          const GsEpilogue &epi) {
  constexpr int NS = 256 / VEC;
  __shared__ float4 red[4][VEC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sg = threadIdx.x / VEC, v = threadIdx.x - sg * VEC;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int j = item.y + sg;
  const int end = item.z;
  for (; j + 3 * NS < end; j += 4 * NS) {
    int c[4];
    float wv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      c[u] = indices[j + u * NS];
      wv[u] = vals[j + u * NS];
    }
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = in[(long long)c[u] * ld4_in + v];
#pragma unroll
    for (int u = 0; u < 4; u++) acc = f4_fma(wv[u], x[u], acc);
  }
  if (j < end) {  // the last (at most 3) neighbours: clamped loads, guarded adds
    int c[3];
    float wv[3];
#pragma unroll
    for (int u = 0; u < 3; u++) {
      const int jj = min(j + u * NS, end - 1);
      c[u] = indices[jj];
      wv[u] = vals[jj];
    }
    float4 x[3];
#pragma unroll
    for (int u = 0; u < 3; u++) x[u] = in[(long long)c[u] * ld4_in + v];
#pragma unroll
    for (int u = 0; u < 3; u++)
      if (j + u * NS < end) acc = f4_fma(wv[u], x[u], acc);
  }
#pragma unroll
  for (int m = VEC; m < 64; m <<= 1) acc = f4_add(acc, f4_shfl_xor(acc, m));
  if (lane < VEC) red[w][lane] = acc;
  __syncthreads();
  if (threadIdx.x < VEC) {
    float4 tot = f4_add(f4_add(f4_add(red[0][v], red[1][v]), red[2][v]), red[3][v]);
    gs_epilogue(tot, item.x, 4 * v, epi);
    out[(long long)item.x * ld4_out + v] = tot;
  }
}

// G lanes per item (G | 64); VEC float4 per row.
template <int VEC, int G>
__global__ __launch_bounds__(256) void k_graphsum(const int4 *__restrict__ items,
                                                  const int *__restrict__ block_items,
                                                  int nbc, const int *__restrict__ indices,
                                                  const float *__restrict__ vals,
                                                  const float4 *__restrict__ in, int ld4_in,
                                                  float4 *__restrict__ out, int ld4_out,
                                                  float4 *__restrict__ partial, GsEpilogue epi,
                                                  const int *__restrict__ slot_comb,
                                                  int *__restrict__ comb_ctr,
                                                  const int4 *__restrict__ comb,
                                                  const int4 *__restrict__ wide, int n_wide) {
  constexpr int NB = G / VEC;  // neighbours per group per iteration
  constexpr int IPW = 64 / G;  // items per wave
  constexpr bool POW2 = (VEC & (VEC - 1)) == 0;
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  if constexpr (POW2) {
    if ((int)blockIdx.x < n_wide) {  // a workgroup item: 256 / VEC neighbour sub-groups
      wide_item<VEC>(wide[blockIdx.x], indices, vals, in, ld4_in, out, ld4_out, epi);
      return;
    }
  }
  const int q = lane / G, r = lane - q * G;
  const int nb = r / VEC, v = r - nb * VEC;
  const bool active = nb < NB;
  const int bid = blockIdx.x - n_wide, nblk = gridDim.x - n_wide;
  const int b = bid % nbc;
  const int wg = bid / nbc, nwg = nblk / nbc;
  const int first = block_items[b], last = block_items[b + 1];
  for (int it = first + (wg * 4 + wib) * IPW + q; it < last; it += nwg * 4 * IPW) {
    const int4 item = items[it];  // {row, begin, end, slot}
    // in-kernel combine: this split row's {row, first slot, count}, loaded beside the walk
    const bool arrive = slot_comb && item.w >= 0;
    int4 cm = make_int4(0, 0, 0, 0);
    if (arrive) cm = comb[slot_comb[item.w]];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
      int j = item.y + nb;
      const int end = item.z;
      for (; j + 3 * NB < end; j += 4 * NB) {
        int c0 = indices[j], c1 = indices[j + NB], c2 = indices[j + 2 * NB],
            c3 = indices[j + 3 * NB];
        const float w0 = vals[j], w1 = vals[j + NB], w2 = vals[j + 2 * NB], w3 = vals[j + 3 * NB];
        const float4 x0 = in[(long long)c0 * ld4_in + v], x1 = in[(long long)c1 * ld4_in + v],
                     x2 = in[(long long)c2 * ld4_in + v], x3 = in[(long long)c3 * ld4_in + v];
        acc = f4_fma(w0, x0, acc);
        acc = f4_fma(w1, x1, acc);
        acc = f4_fma(w2, x2, acc);
        acc = f4_fma(w3, x3, acc);
      }
      // the last (at most 3) neighbours of this lane: predicated, their index / value loads
      // together and then their gathers (r04: one dependent load pair per neighbour made a
      // low-degree row -- cora's are 4-5 -- several round trips long); same adds, same order
      if (j < end) {
        int cc[3];
        float ww[3];
#pragma unroll
        for (int u = 0; u < 3; u++) {  // (clamped, unpredicated: a missing neighbour re-reads
          const int jj = min(j + u * NB, end - 1);  // the last one and is not added)
          cc[u] = indices[jj];
          ww[u] = vals[jj];
        }
        float4 xx[3];
#pragma unroll
        for (int u = 0; u < 3; u++) xx[u] = in[(long long)cc[u] * ld4_in + v];
#pragma unroll
        for (int u = 0; u < 3; u++)
          if (j + u * NB < end) acc = f4_fma(ww[u], xx[u], acc);
      }
    }
    if constexpr (POW2) {
#pragma unroll
      for (int m = VEC; m < G; m <<= 1) acc = f4_add(acc, f4_shfl_xor(acc, m));
    } else {
      static_assert(POW2 || G == 64, "non power-of-two rows use whole-wave items");
      float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < NB; k++) {
        const int src = k * VEC + v;
        tot = f4_add(tot, make_float4(__shfl(acc.x, src, 64), __shfl(acc.y, src, 64),
                                      __shfl(acc.z, src, 64), __shfl(acc.w, src, 64)));
      }
      acc = tot;
    }
    if (nb == 0) {
      if (item.w < 0) {
        gs_epilogue(acc, item.x, 4 * v, epi);
        out[(long long)item.x * ld4_out + v] = acc;
      } else {
        partial[(long long)item.w * VEC + v] = acc;
      }
    }
    if (arrive) {  // (uniform over the item's G lanes)
      // release this slot, count the arrival; the row's last arrival acquires the others' and
      // adds the slots in slot order from zero, as k_graphsum_combine does: the same bits
      const int ci = slot_comb[item.w];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      int old = 0;
      if (r == 0)
        old = __hip_atomic_fetch_add(comb_ctr + ci, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = __shfl(old, q * G, 64);
      if (old == cm.z - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (nb == 0) {
          float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int k = 0; k < cm.z; k++)
            tot = f4_add(tot, partial[(long long)(cm.y + k) * VEC + v]);
          gs_epilogue(tot, cm.x, 4 * v, epi);
          out[(long long)cm.x * ld4_out + v] = tot;
        }
        if (r == 0) comb_ctr[ci] = 0;  // (no other item of the row is left: ready for the next call)
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// d = 16 on the XCD-blocked, 4-padded layout (the reddit hot path).  Cost model measured on
// gfx950 (tools/ta_micro.hip, L2-resident table): a float4 wave load touching 16 random 64-B
// rows costs ~37 CU-cycles, a dword load ~6; the previous per-item loop spent more time in
// serialized index -> gather round trips than in the gathers themselves.  Here a 16-lane
// group owns an item and walks it in 64-slot sub-chunks:
//   1. lane r loads slots 4r..4r+3 of the sub-chunk: ONE int4 (indices) + ONE float4
//      (coefficients) per lane -- the whole sub-chunk's edge list in two 16-B loads;
//   2. 16 steps s: neighbour sub-group nb takes slot 16*nb + s, fetched from lane
//      4*nb + (s>>2), component s&3 (ds_bpermute; the component is uniform per step), and
//      all 16 row gathers are independent loads issued back to back.
// Per-lane accumulation is sequential over s, sub-groups are combined by a fixed xor tree
// => deterministic.  Slots past the item end are skipped (exec-masked), padding slots carry
// coefficient 0.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int int4_comp(const int4 &v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ float float4_comp(const float4 &v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

__global__ __launch_bounds__(256) void k_graphsum16(const int4 *__restrict__ items,
                                                    const int *__restrict__ block_items, int nbc,
                                                    const int *__restrict__ indices,
                                                    const float *__restrict__ vals,
                                                    const float4 *__restrict__ in, int ld4_in,
                                                    float4 *__restrict__ out, int ld4_out,
                                                    float4 *__restrict__ partial,
                                                    GsEpilogue epi) {
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int q = lane >> 4, r = lane & 15;
  const int nb = r >> 2, v = r & 3;
  const int gbase = lane & ~15;
  const int b = blockIdx.x % nbc;
  const int wg = blockIdx.x / nbc, nwg = gridDim.x / nbc;
  const int first = block_items[b], last = block_items[b + 1];
  for (int it = first + (wg * 4 + wib) * 4 + q; it < last; it += nwg * 16) {
    const int4 item = items[it];  // {row, begin, end (4-aligned), slot}
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int base = item.y; base < item.z; base += 64) {
      const int e = base + 4 * r;
      int4 ci = make_int4(0, 0, 0, 0);
      float4 cw = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < item.z) {
        ci = *reinterpret_cast<const int4 *>(indices + e);
        cw = *reinterpret_cast<const float4 *>(vals + e);
      }
      const int lim = item.z - base - 16 * nb;  // slots of this sub-group in the sub-chunk
#pragma unroll
      for (int h = 0; h < 2; h++) {  // two batches of 8 independent gathers
        float4 x[8];
        float w[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
          const int s = 8 * h + t;
          const int src = gbase + 4 * nb + (s >> 2);
          const int c = __shfl(int4_comp(ci, s & 3), src, 64);
          w[t] = __shfl(float4_comp(cw, s & 3), src, 64);
          x[t] = s < lim ? in[(long long)c * ld4_in + v] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int t = 0; t < 8; t++) acc = f4_fma(w[t], x[t], acc);
      }
    }
    acc = f4_add(acc, f4_shfl_xor(acc, 4));
    acc = f4_add(acc, f4_shfl_xor(acc, 8));
    if (nb == 0) {
      if (item.w < 0) {
        gs_epilogue(acc, item.x, 4 * v, epi);
        out[(long long)item.x * ld4_out + v] = acc;
      } else {
        partial[(long long)item.w * 4 + v] = acc;
      }
    }
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void k_graphsum_combine(const int4 *__restrict__ comb,
                                                          int n_comb,
                                                          const float4 *__restrict__ partial,
                                                          float4 *__restrict__ out, int ld4_out,
                                                          GsEpilogue epi) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ci = t / VEC;
  const int v = (int)(t - ci * VEC);
  if (ci >= n_comb) return;
  const int4 c = comb[ci];  // {row, first_slot, count, -}
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < c.z; s++) acc = f4_add(acc, partial[(long long)(c.y + s) * VEC + v]);
  gs_epilogue(acc, c.x, 4 * v, epi);
  out[(long long)c.x * ld4_out + v] = acc;
}

template <int VEC, int G>
static void launch_vec(const GraphSchedule &s, const int *indices, const float *vals,
                       const float *in, int ld_in, float *out, int ld_out, float *partial,
                       hipStream_t st, const GsEpilogue &epi) {
  if (s.n_items > 0 || s.n_wide > 0) {
    constexpr int per_wg = 4 * (64 / G);  // items one workgroup takes per sweep
    long long per_block = ceil_div(s.max_block_items, per_wg);
    // enough workgroups per column block to fill the block's XCD several times over
    const long long cap = 4096 / s.nbc;
    if (per_block > cap) per_block = cap;
    if (per_block < 1) per_block = 1;
    const dim3 grid((unsigned)(per_block * s.nbc + s.n_wide)), block(256);
    // (measured and removed, r01: a software-pipelined k_graphsum16, 132 VGPRs at 3 waves per
    // SIMD, slower)
    if (VEC == 4 && s.nbc > 1 && s.gather16 == 0)
      PGCN_LAUNCH(k_graphsum16, grid, block, 0, st, s.items, s.block_items, s.nbc, indices,
                         vals, reinterpret_cast<const float4 *>(in), ld_in / 4,
                         reinterpret_cast<float4 *>(out), ld_out / 4,
                         reinterpret_cast<float4 *>(partial), epi);
    else
      PGCN_LAUNCH((k_graphsum<VEC, G>), grid, block, 0, st, s.items, s.block_items, s.nbc,
                         indices, vals, reinterpret_cast<const float4 *>(in), ld_in / 4,
                         reinterpret_cast<float4 *>(out), ld_out / 4,
                         reinterpret_cast<float4 *>(partial), epi, s.slot_comb, s.comb_ctr,
                         s.comb, s.wide, s.n_wide);
  }
  if (s.n_comb > 0 && !s.slot_comb) {
    const long long threads = (long long)s.n_comb * VEC;
    PGCN_LAUNCH(k_graphsum_combine<VEC>, dim3((unsigned)ceil_div(threads, 256)),
                       dim3(256), 0, st, s.comb, s.n_comb,
                       reinterpret_cast<const float4 *>(partial), reinterpret_cast<float4 *>(out),
                       ld_out / 4, epi);
  }
}

int graphsum_group_lanes(int vec) {
  if (vec <= 4 && (vec & (vec - 1)) == 0) return 16;  // 1, 2, 4 float4 per row
  if (vec == 8) return 32;
  return 64;
}

void launch_graphsum(const GraphSchedule &s, const int *indices, const float *vals,
                     const float *in, int ld_in, float *out, int ld_out, float *partial,
                     hipStream_t st, const GsEpilogue *epi) {
  note_path(KP_GS_GATHER);
  const GsEpilogue none{};
  const GsEpilogue &e = epi ? *epi : none;
  switch (s.vec) {
#define PGCN_VEC_CASE(V, G) \
  case V:                   \
    launch_vec<V, G>(s, indices, vals, in, ld_in, out, ld_out, partial, st, e); break;
    PGCN_VEC_CASE(1, 16) PGCN_VEC_CASE(2, 16) PGCN_VEC_CASE(3, 64) PGCN_VEC_CASE(4, 16)
    PGCN_VEC_CASE(5, 64) PGCN_VEC_CASE(6, 64) PGCN_VEC_CASE(7, 64) PGCN_VEC_CASE(8, 32)
    PGCN_VEC_CASE(9, 64) PGCN_VEC_CASE(10, 64) PGCN_VEC_CASE(11, 64) PGCN_VEC_CASE(12, 64)
    PGCN_VEC_CASE(16, 64) PGCN_VEC_CASE(32, 64)
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
