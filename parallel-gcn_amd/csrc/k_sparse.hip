// parallel-gcn_amd/csrc/k_sparse.hip -- SparseMatmul for sparse (svmlight) feature matrices.
//
// Replaces sparse_matmul_kernel_forward / _backward (src/module.cu:108-163) and hpdga
// SparseMatmul::forward/backward (module.cpp:49-72).
//  * forward: one lane per output (row, column); the row's nonzeros are walked in CSR order
//    with separate multiply and add (contraction off) => bit-identical to the CPU reference.
//    The input dropout is applied on the fly from the mask bits (the reference rewrites X in
//    place and restores it with set_input every pass; here X is never written).
//  * backward: W.grad = drop(X)^T * G via the transposed index (built once on the host):
//    per (feature, column) the contributions are summed in row order => bit-identical to
//    the CPU's scatter order and free of the reference's float atomics; the gathers of a
//    column's chain are done in parallel through LDS (k_spmm_csc_bwd).
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace pgcn {

__device__ __forceinline__ float drop_val(float a, const uint64_t *__restrict__ mask,
                                          long long bit, float scale) {
  if (!mask) return a;
  return a * (((mask[bit >> 6] >> (bit & 63)) & 1) ? scale : 0.0f);
}

// DUAL: c2 = drop(X) B beside c = X B from the same index / value / B loads (the eval forward
// and the next training forward share B: no optimizer step between them); each sum keeps its
// own products in CSR order, so c2 has the masked kernel's bits and c the unmasked one's.
template <bool DUAL>
__global__ __launch_bounds__(256) void k_spmm_csr(int m, int p, int ldc,
                                                  const int *__restrict__ indptr,
                                                  const int *__restrict__ indices,
                                                  const float *__restrict__ a,
                                                  const uint64_t *__restrict__ mask,
                                                  long long mask_base, float scale,
                                                  const float *__restrict__ b,
                                                  float *__restrict__ c, float *__restrict__ c2) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long i = t / p;
  const int k = (int)(t - i * p);
  if (i >= m) return;
  float sum = 0.0f, sum2 = 0.0f;
  int jj = indptr[i];
  const int je = indptr[i + 1];
  const uint64_t *m1 = DUAL ? nullptr : mask;  // c's mask (DUAL: c is the unmasked product)
  // r04: 8 nonzeros' index / value / mask loads issued together, then their B gathers, then
  // the adds in CSR order (one dependent load chain per 8 nonzeros instead of per nonzero;
  // the same products and the same order: the same bits)
  for (; jj + 8 <= je; jj += 8) {
    int ix[8];
    float av[8], aw[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      ix[u] = indices[jj + u];
      const float ar = a[jj + u];
      av[u] = drop_val(ar, m1, mask_base + jj + u, scale);
      if constexpr (DUAL) aw[u] = drop_val(ar, mask, mask_base + jj + u, scale);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) bv[u] = b[(long long)ix[u] * p + k];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      sum += av[u] * bv[u];
      if constexpr (DUAL) sum2 += aw[u] * bv[u];
    }
  }
  if (jj < je) {
    // the last (at most 7) nonzeros the same way: clamped, unpredicated loads (r04 late: one
    // dependent load pair per nonzero made cora's rows -- 18 nonzeros on average -- up to 7
    // round trips longer); the adds guarded, in CSR order
    int ix[7];
    float av[7], aw[7], bv[7];
#pragma unroll
    for (int u = 0; u < 7; u++) {
      const int j = min(jj + u, je - 1);
      ix[u] = indices[j];
      const float ar = a[j];
      av[u] = drop_val(ar, m1, mask_base + j, scale);
      if constexpr (DUAL) aw[u] = drop_val(ar, mask, mask_base + j, scale);
    }
#pragma unroll
    for (int u = 0; u < 7; u++) bv[u] = b[(long long)ix[u] * p + k];
#pragma unroll
    for (int u = 0; u < 7; u++)
      if (jj + u < je) {
        sum += av[u] * bv[u];
        if constexpr (DUAL) sum2 += aw[u] * bv[u];
      }
  }
  c[i * ldc + k] = sum;
  if constexpr (DUAL) c2[i * ldc + k] = sum2;
}

// One workgroup per (feature f, 16 gradient columns).  The serial chain of a column's
// contributions (row order, the CPU's scatter order) is latency-free: all CH threads gather a
// chunk of CH entries' products into LDS at once (one 64-B row of G per entry), then 16 lanes
// add them in entry order from LDS.  Same products, same order => the same bits as a lane
// walking the column alone (the r01 kernel, 1.9 ms on pubmed: 32 workgroups, one dependent
// gather per entry).  CH = 256, or 1024 when the features average more than 512 entries (r04:
// pubmed's ~2,000-entry columns took 8 chunks of 256, 38.9 us per call).  r04 late, PIPE (the
// 1024-thread form): the next chunk's loads are issued before this chunk's adds (its values,
// mask words and G rows, and the indices of the chunk after it): pubmed_synth 6.26-6.33k ->
// 6.77-6.79k epochs/s; in the 256-thread form cora lost 5 % with it (10.8k -> 10.2k,
// profiles/r04/ab_csc_pipe.txt), so that form loads each chunk after the last one's adds.
// Measured and dropped: U = 2 or 4 chunks' loads at once (U 4: 14.8 us on cora, 110 VGPRs
// halve the resident workgroups; U 2: no gain in the epoch, profiles/r04/ab_csc_u.txt).
template <int CH, bool PIPE = (CH >= 1024)>
__global__ __launch_bounds__(CH) void k_spmm_csc_bwd(int nf, int p, int ldg,
                                                     const int *__restrict__ csc_ptr,
                                                     const int *__restrict__ csc_row,
                                                     const int *__restrict__ csc_pos,
                                                     const float *__restrict__ a,
                                                     const uint64_t *__restrict__ mask,
                                                     long long mask_base, float scale,
                                                     const float *__restrict__ cgrad,
                                                     float *__restrict__ bgrad,
                                                     const int *__restrict__ order) {
  // products column-major (prod[c][entry], rows padded to CH + 4 floats): an adding lane
  // reads 4 consecutive entries of its column with one ds_read_b128 (16 lanes, 4 banks apart)
  __shared__ __attribute__((aligned(16))) float prod[16][CH + 4];
  // (order: the features by descending column length -- the longest chains start first)
  const int f = order ? order[blockIdx.x] : (int)blockIdx.x, k0 = blockIdx.y * 16,
            tid = threadIdx.x;
  const int e0 = csc_ptr[f], e1 = csc_ptr[f + 1];
  float sum = 0.0f;
  // the 16 lanes' ordered adds of the chunk at cb (its reads a batch ahead of the adds)
  auto add_chunk = [&](int cb) {
    const float *col = prod[tid];
    const int n = min(CH, e1 - cb);
    int j = 0;
    if (n >= 16) {
      float4 va[4], vb[4];
#pragma unroll
      for (int q = 0; q < 4; q++) va[q] = *reinterpret_cast<const float4 *>(col + 4 * q);
      for (;;) {
        bool more = j + 32 <= n;
        if (more) {
#pragma unroll
          for (int q = 0; q < 4; q++) vb[q] = *reinterpret_cast<const float4 *>(col + j + 16 + 4 * q);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          sum += va[q].x;
          sum += va[q].y;
          sum += va[q].z;
          sum += va[q].w;
        }
        j += 16;
        if (!more) break;
        more = j + 32 <= n;
        if (more) {
#pragma unroll
          for (int q = 0; q < 4; q++) va[q] = *reinterpret_cast<const float4 *>(col + j + 16 + 4 * q);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          sum += vb[q].x;
          sum += vb[q].y;
          sum += vb[q].z;
          sum += vb[q].w;
        }
        j += 16;
        if (!more) break;
      }
    }
    for (; j + 4 <= n; j += 4) {
      const float4 t = *reinterpret_cast<const float4 *>(col + j);
      sum += t.x;
      sum += t.y;
      sum += t.z;
      sum += t.w;
    }
    for (; j < n; j++) sum += col[j];
  };
  if ((ldg & 3) == 0 && e0 < e1) {  // engine layout: ld a multiple of 4, padding columns zero
    // clamped, unpredicated loads (entries past the column are never added)
    int pos, row;  // indices of the chunk after the current one
    auto idx = [&](int cb, int &ps, int &rw) {
      const int e = min(cb + tid, e1 - 1);
      ps = csc_pos[e];
      rw = csc_row[e];
    };
    float ar;
    uint64_t mw;
    float4 gv[4];
    auto vals = [&](int ps, int rw, float &av_, uint64_t &mw_, float4 *g4) {
      const float *g = cgrad + (long long)rw * ldg + k0;
      av_ = a[ps];
      mw_ = mask ? mask[(mask_base + ps) >> 6] : 0ull;
#pragma unroll
      for (int c4 = 0; c4 < 4; c4++)
        g4[c4] = k0 + 4 * c4 < ldg ? *reinterpret_cast<const float4 *>(g + 4 * c4)
                                   : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    };
    int cpos;  // the current chunk's value positions (its mask bits)
    idx(e0, cpos, row);
    vals(cpos, row, ar, mw, gv);
    if (PIPE && e0 + CH < e1) idx(e0 + CH, pos, row);
    for (int base = e0; base < e1; base += CH) {
      if (!PIPE && base != e0) {  // this chunk's loads, after the last chunk's adds
        idx(base, cpos, row);
        vals(cpos, row, ar, mw, gv);
      }
      const float av = mask ? ar * (((mw >> ((mask_base + cpos) & 63)) & 1) ? scale : 0.0f) : ar;
      if (base + tid < e1) {
#pragma unroll
        for (int c4 = 0; c4 < 4; c4++) {
          prod[4 * c4 + 0][tid] = gv[c4].x * av;
          prod[4 * c4 + 1][tid] = gv[c4].y * av;
          prod[4 * c4 + 2][tid] = gv[c4].z * av;
          prod[4 * c4 + 3][tid] = gv[c4].w * av;
        }
      }
      // the next chunk's values and the indices of the one after it, in flight over the adds
      const bool next = PIPE && base + CH < e1;  // (uniform)
      if (next) {
        cpos = pos;
        vals(pos, row, ar, mw, gv);
        if (base + 2 * CH < e1) idx(base + 2 * CH, pos, row);
      }
      __syncthreads();
      if (tid < 16) add_chunk(base);
      __syncthreads();
    }
  } else {
    for (int base = e0; base < e1; base += CH) {
      const int e = base + tid;
      if (e < e1) {
        const int ps = csc_pos[e];
        const float *g = cgrad + (long long)csc_row[e] * ldg + k0;
        const float v = drop_val(a[ps], mask, mask_base + ps, scale);
#pragma unroll
        for (int c = 0; c < 16; c++) prod[c][tid] = k0 + c < p ? g[c] * v : 0.0f;
      }
      __syncthreads();
      if (tid < 16) add_chunk(base);
      __syncthreads();
    }
  }
  if (tid < 16 && k0 + tid < p) bgrad[(long long)f * p + k0 + tid] = sum;
}

// W1.grad over sparse X as a fixed tree (knob "csc_tree", r06): thread t of the feature's
// workgroup sums the products of entries t, t + CH, ... in entry order (4 entries' index,
// value, mask and grad-row loads in flight together), then the CH partial rows are added in
// a fixed binary tree (through LDS, then lane shuffles in wave 0) over the smallest power of
// two of threads that holds the feature's entries -- deterministic, differing by the summation
// order only from the sequential chain k_spmm_csc_bwd keeps (hpdga's scatter order, bit-exact), whose longest
// column (cora: 1,083 entries) made that kernel the epoch's longest (14.8 us); 1,024 threads
// per feature on matrices of > 512 entries per feature, like k_spmm_csc_bwd
template <int CH>
__global__ __launch_bounds__(CH) void k_spmm_csc_tree(int nf, int p, int ldg,
                                                      const int *__restrict__ csc_ptr,
                                                      const int *__restrict__ csc_row,
                                                      const int *__restrict__ csc_pos,
                                                      const float *__restrict__ a,
                                                      const uint64_t *__restrict__ mask,
                                                      long long mask_base, float scale,
                                                      const float *__restrict__ cgrad,
                                                      float *__restrict__ bgrad,
                                                      const int *__restrict__ order) {
  __shared__ float red[CH / 2][17];  // [pair][column]: 17 keeps the rows' banks apart
  const int f = order ? order[blockIdx.x] : (int)blockIdx.x, k0 = blockIdx.y * 16,
            tid = threadIdx.x;
  const int e0 = csc_ptr[f], e1 = csc_ptr[f + 1];
  float acc[16];
#pragma unroll
  for (int c = 0; c < 16; c++) acc[c] = 0.0f;
  constexpr int U = 4;
  for (int b = e0 + tid; b < e1; b += U * CH) {
    int ps[U], rw[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = min(b + u * CH, e1 - 1);
      ps[u] = csc_pos[e];
      rw[u] = csc_row[e];
    }
    float av[U];
#pragma unroll
    for (int u = 0; u < U; u++) av[u] = drop_val(a[ps[u]], mask, mask_base + ps[u], scale);
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (b + u * CH >= e1) break;
      const float *g = cgrad + (long long)rw[u] * ldg + k0;
#pragma unroll
      for (int c = 0; c < 16; c++) acc[c] += (k0 + c < p ? g[c] : 0.0f) * av[u];
    }
  }
  // the tree, over the smallest power of two of threads that holds every entry (the threads
  // past it hold zeros): at each level the upper half's rows are added into the lower half's,
  // through LDS down to one wave, then within wave 0 by lane shuffles
  int span = 1;
  while (span < min(e1 - e0, CH)) span <<= 1;
  for (int h = span / 2; h >= 64; h >>= 1) {
    if (tid >= h && tid < 2 * h)
#pragma unroll
      for (int c = 0; c < 16; c++) red[tid - h][c] = acc[c];
    __syncthreads();
    if (tid < h)
#pragma unroll
      for (int c = 0; c < 16; c++) acc[c] += red[tid][c];
    __syncthreads();
  }
  if (tid >= 64) return;
  for (int h = min(span, 64) / 2; h >= 1; h >>= 1) {
#pragma unroll
    for (int c = 0; c < 16; c++) {
      const float o = __shfl_down(acc[c], h, 64);
      if (tid < h) acc[c] += o;
    }
  }
  if (tid == 0)
    for (int c = 0; c < 16 && k0 + c < p; c++) bgrad[(long long)f * p + k0 + c] = acc[c];
}

void launch_spmm_csr(int m, int p, int ldc, const int *indptr, const int *indices,
                     const float *a, const uint64_t *mask, long long mask_base, float scale,
                     const float *b, float *c, hipStream_t s) {
  if (m <= 0) return;
  const long long threads = (long long)m * p;
  PGCN_LAUNCH(k_spmm_csr<false>, dim3((unsigned)ceil_div(threads, 256)), dim3(256), 0, s, m, p,
              ldc, indptr, indices, a, mask, mask_base, scale, b, c, nullptr);
}

void launch_spmm_csr_dual(int m, int p, int ldc, const int *indptr, const int *indices,
                          const float *a, const uint64_t *mask, long long mask_base, float scale,
                          const float *b, float *c, float *c2, hipStream_t s) {
  PGCN_CHECK(mask && c2, PGCN_E_INVALID, "spmm_csr_dual: needs the mask and the second output");
  if (m <= 0) return;
  const long long threads = (long long)m * p;
  PGCN_LAUNCH(k_spmm_csr<true>, dim3((unsigned)ceil_div(threads, 256)), dim3(256), 0, s, m, p,
              ldc, indptr, indices, a, mask, mask_base, scale, b, c, c2);
}

void launch_spmm_csc_bwd(int nf, int p, int ldg, const int *csc_ptr, const int *csc_row,
                         const int *csc_pos, const float *a, const uint64_t *mask,
                         long long mask_base, float scale, const float *cgrad, float *bgrad,
                         hipStream_t s, long long nnz, const int *order, bool tree) {
  if (nf <= 0 || p <= 0) return;
  const dim3 grid((unsigned)nf, (unsigned)ceil_div(p, 16));
  if (tree) {
    if (nnz > 512LL * nf)
      PGCN_LAUNCH(k_spmm_csc_tree<1024>, grid, dim3(1024), 0, s, nf, p, ldg, csc_ptr, csc_row,
                  csc_pos, a, mask, mask_base, scale, cgrad, bgrad, order);
    else
      PGCN_LAUNCH(k_spmm_csc_tree<256>, grid, dim3(256), 0, s, nf, p, ldg, csc_ptr, csc_row,
                  csc_pos, a, mask, mask_base, scale, cgrad, bgrad, order);
    return;
  }
  if (nnz > 512LL * nf)
    PGCN_LAUNCH(k_spmm_csc_bwd<1024>, grid, dim3(1024), 0, s, nf, p, ldg, csc_ptr, csc_row,
                csc_pos, a, mask, mask_base, scale, cgrad, bgrad, order);
  else
    PGCN_LAUNCH(k_spmm_csc_bwd<256>, grid, dim3(256), 0, s, nf, p, ldg, csc_ptr, csc_row,
                csc_pos, a, mask, mask_base, scale, cgrad, bgrad, order);
}

}  // namespace pgcn
