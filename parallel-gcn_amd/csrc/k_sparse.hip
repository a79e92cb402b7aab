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

#ifndef PGCN_CSC_U
#define PGCN_CSC_U 4  // entries per thread per round of the 256-thread backward (A/B builds)
#endif

namespace pgcn {

__device__ __forceinline__ float drop_val(float a, const uint64_t *__restrict__ mask,
                                          long long bit, float scale) {
  if (!mask) return a;
  return a * (((mask[bit >> 6] >> (bit & 63)) & 1) ? scale : 0.0f);
}

__global__ __launch_bounds__(256) void k_spmm_csr(int m, int p, int ldc,
                                                  const int *__restrict__ indptr,
                                                  const int *__restrict__ indices,
                                                  const float *__restrict__ a,
                                                  const uint64_t *__restrict__ mask,
                                                  long long mask_base, float scale,
                                                  const float *__restrict__ b,
                                                  float *__restrict__ c) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long i = t / p;
  const int k = (int)(t - i * p);
  if (i >= m) return;
  float sum = 0.0f;
  int jj = indptr[i];
  const int je = indptr[i + 1];
  // r04: 8 nonzeros' index / value / mask loads issued together, then their B gathers, then
  // the adds in CSR order (one dependent load chain per 8 nonzeros instead of per nonzero;
  // the same products and the same order: the same bits)
  for (; jj + 8 <= je; jj += 8) {
    int ix[8];
    float av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      ix[u] = indices[jj + u];
      av[u] = drop_val(a[jj + u], mask, mask_base + jj + u, scale);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) bv[u] = b[(long long)ix[u] * p + k];
#pragma unroll
    for (int u = 0; u < 8; u++) sum += av[u] * bv[u];
  }
  if (jj < je) {
    // the last (at most 7) nonzeros the same way: clamped, unpredicated loads (r04 late: one
    // dependent load pair per nonzero made cora's rows -- 18 nonzeros on average -- up to 7
    // round trips longer); the adds guarded, in CSR order
    int ix[7];
    float av[7], bv[7];
#pragma unroll
    for (int u = 0; u < 7; u++) {
      const int j = min(jj + u, je - 1);
      ix[u] = indices[j];
      av[u] = drop_val(a[j], mask, mask_base + j, scale);
    }
#pragma unroll
    for (int u = 0; u < 7; u++) bv[u] = b[(long long)ix[u] * p + k];
#pragma unroll
    for (int u = 0; u < 7; u++)
      if (jj + u < je) sum += av[u] * bv[u];
  }
  c[i * ldc + k] = sum;
}

// One workgroup per (feature f, 16 gradient columns).  The serial chain of a column's
// contributions (row order, the CPU's scatter order) is latency-free: the CH threads gather
// U chunks of CH entries' products at once (U entries per thread: one round trip for the
// indices, one for the values, mask words and 64-B rows of G), then, chunk by chunk, stage
// them in LDS where 16 lanes add them in entry order.  Same products, same order => the same
// bits as a lane walking the column alone (the r01 kernel, 1.9 ms on pubmed: 32 workgroups,
// one dependent gather per entry).  <256, 4> (r04 late: cora's 1,083-entry column took five
// 256-entry rounds of two dependent loads each, 12.7 us per call), or <1024, 1> when the
// features average more than 512 entries (pubmed: 8 chunks of 256 took 38.9 us per call).
template <int CH, int U>
__global__ __launch_bounds__(CH) void k_spmm_csc_bwd(int nf, int p, int ldg,
                                                     const int *__restrict__ csc_ptr,
                                                     const int *__restrict__ csc_row,
                                                     const int *__restrict__ csc_pos,
                                                     const float *__restrict__ a,
                                                     const uint64_t *__restrict__ mask,
                                                     long long mask_base, float scale,
                                                     const float *__restrict__ cgrad,
                                                     float *__restrict__ bgrad) {
  __shared__ float prod[CH][17];
  const int f = blockIdx.x, k0 = blockIdx.y * 16, tid = threadIdx.x;
  const int e0 = csc_ptr[f], e1 = csc_ptr[f + 1];
  float sum = 0.0f;
  for (int base = e0; base < e1; base += CH * U) {
    float4 gv[U][4];
    float av[U];
    if ((ldg & 3) == 0) {  // engine layout: ld a multiple of 4, padding columns zero
      // every entry's index pair, then every value / mask word / G row: two round trips for
      // U * CH entries (clamped, unpredicated loads; entries past the column get 0)
      int pos[U], row[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int e = min(base + u * CH + tid, e1 - 1);
        pos[u] = csc_pos[e];
        row[u] = csc_row[e];
      }
      float ar[U];
      uint64_t mw[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const float *g = cgrad + (long long)row[u] * ldg + k0;
        ar[u] = a[pos[u]];
        mw[u] = mask ? mask[(mask_base + pos[u]) >> 6] : 0ull;
#pragma unroll
        for (int c4 = 0; c4 < 4; c4++)
          gv[u][c4] = k0 + 4 * c4 < ldg ? *reinterpret_cast<const float4 *>(g + 4 * c4)
                                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        av[u] = mask ? ar[u] * (((mw[u] >> ((mask_base + pos[u]) & 63)) & 1) ? scale : 0.0f)
                     : ar[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int cb = base + u * CH;  // this chunk's first entry (uniform)
      if (cb >= e1) break;
      const int e = cb + tid;
      if (e < e1) {
        if ((ldg & 3) == 0) {
#pragma unroll
          for (int c4 = 0; c4 < 4; c4++) {
            const float4 v = gv[u][c4];
            prod[tid][4 * c4 + 0] = v.x * av[u];
            prod[tid][4 * c4 + 1] = v.y * av[u];
            prod[tid][4 * c4 + 2] = v.z * av[u];
            prod[tid][4 * c4 + 3] = v.w * av[u];
          }
        } else {
          const int pos = csc_pos[e];
          const float *g = cgrad + (long long)csc_row[e] * ldg + k0;
          const float v = drop_val(a[pos], mask, mask_base + pos, scale);
#pragma unroll
          for (int c = 0; c < 16; c++) prod[tid][c] = k0 + c < p ? g[c] * v : 0.0f;
        }
      }
      __syncthreads();
      if (tid < 16) {
        // (r04: 32 LDS reads in flight per wait, was 8: the serial add chain of a long
        // column no longer waits on the LDS between every 8 adds)
        const int n = min(CH, e1 - cb);
        int j = 0;
        for (; j + 32 <= n; j += 32) {
          float v[32];
#pragma unroll
          for (int w = 0; w < 32; w++) v[w] = prod[j + w][tid];
#pragma unroll
          for (int w = 0; w < 32; w++) sum += v[w];
        }
        for (; j + 8 <= n; j += 8) {
          float v[8];
#pragma unroll
          for (int w = 0; w < 8; w++) v[w] = prod[j + w][tid];
#pragma unroll
          for (int w = 0; w < 8; w++) sum += v[w];
        }
        for (; j < n; j++) sum += prod[j][tid];
      }
      __syncthreads();
    }
  }
  if (tid < 16 && k0 + tid < p) bgrad[(long long)f * p + k0 + tid] = sum;
}

void launch_spmm_csr(int m, int p, int ldc, const int *indptr, const int *indices,
                     const float *a, const uint64_t *mask, long long mask_base, float scale,
                     const float *b, float *c, hipStream_t s) {
  if (m <= 0) return;
  const long long threads = (long long)m * p;
  PGCN_LAUNCH(k_spmm_csr, dim3((unsigned)ceil_div(threads, 256)), dim3(256), 0, s, m, p,
                     ldc, indptr, indices, a, mask, mask_base, scale, b, c);
}

void launch_spmm_csc_bwd(int nf, int p, int ldg, const int *csc_ptr, const int *csc_row,
                         const int *csc_pos, const float *a, const uint64_t *mask,
                         long long mask_base, float scale, const float *cgrad, float *bgrad,
                         hipStream_t s, long long nnz) {
  if (nf <= 0 || p <= 0) return;
  const dim3 grid((unsigned)nf, (unsigned)ceil_div(p, 16));
  if (nnz > 512LL * nf)
    PGCN_LAUNCH((k_spmm_csc_bwd<1024, 1>), grid, dim3(1024), 0, s, nf, p, ldg, csc_ptr, csc_row,
                csc_pos, a, mask, mask_base, scale, cgrad, bgrad);
  else
    PGCN_LAUNCH((k_spmm_csc_bwd<256, PGCN_CSC_U>), grid, dim3(256), 0, s, nf, p, ldg, csc_ptr, csc_row,
                csc_pos, a, mask, mask_base, scale, cgrad, bgrad);
}

}  // namespace pgcn
