// parallel-gcn_amd/csrc/k_sparse.hip -- SparseMatmul for sparse (svmlight) feature matrices.
//
// Replaces sparse_matmul_kernel_forward / _backward (src/module.cu:108-163) and hpdga
// SparseMatmul::forward/backward (module.cpp:49-72).
//  * forward: one lane per output (row, column); the row's nonzeros are walked in CSR order
//    with separate multiply and add (contraction off) => bit-identical to the CPU reference.
//    The input dropout is applied on the fly from the mask bits (the reference rewrites X in
//    place and restores it with set_input every pass; here X is never written).
//  * backward: W.grad = drop(X)^T * G via the transposed index (built once on the host):
//    one lane per (feature, column), contributions summed in row order => bit-identical to
//    the CPU's scatter order and free of the reference's float atomics.
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

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
  for (int jj = indptr[i]; jj < indptr[i + 1]; jj++) {
    const float av = drop_val(a[jj], mask, mask_base + jj, scale);
    sum += av * b[(long long)indices[jj] * p + k];
  }
  c[i * ldc + k] = sum;
}

__global__ __launch_bounds__(256) void k_spmm_csc_bwd(int nf, int p, int ldg,
                                                      const int *__restrict__ csc_ptr,
                                                      const int *__restrict__ csc_row,
                                                      const int *__restrict__ csc_pos,
                                                      const float *__restrict__ a,
                                                      const uint64_t *__restrict__ mask,
                                                      long long mask_base, float scale,
                                                      const float *__restrict__ cgrad,
                                                      float *__restrict__ bgrad) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long f = t / p;
  const int k = (int)(t - f * p);
  if (f >= nf) return;
  float sum = 0.0f;
  for (int e = csc_ptr[f]; e < csc_ptr[f + 1]; e++) {
    const int pos = csc_pos[e];
    const float av = drop_val(a[pos], mask, mask_base + pos, scale);
    sum += cgrad[(long long)csc_row[e] * ldg + k] * av;
  }
  bgrad[f * p + k] = sum;
}

void launch_spmm_csr(int m, int p, int ldc, const int *indptr, const int *indices,
                     const float *a, const uint64_t *mask, long long mask_base, float scale,
                     const float *b, float *c, hipStream_t s) {
  if (m <= 0) return;
  const long long threads = (long long)m * p;
  hipLaunchKernelGGL(k_spmm_csr, dim3((unsigned)ceil_div(threads, 256)), dim3(256), 0, s, m, p,
                     ldc, indptr, indices, a, mask, mask_base, scale, b, c);
}

void launch_spmm_csc_bwd(int nf, int p, int ldg, const int *csc_ptr, const int *csc_row,
                         const int *csc_pos, const float *a, const uint64_t *mask,
                         long long mask_base, float scale, const float *cgrad, float *bgrad,
                         hipStream_t s) {
  if (nf <= 0) return;
  const long long threads = (long long)nf * p;
  hipLaunchKernelGGL(k_spmm_csc_bwd, dim3((unsigned)ceil_div(threads, 256)), dim3(256), 0, s,
                     nf, p, ldg, csc_ptr, csc_row, csc_pos, a, mask, mask_base, scale, cgrad,
                     bgrad);
}

}  // namespace pgcn
