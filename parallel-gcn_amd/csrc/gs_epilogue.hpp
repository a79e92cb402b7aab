// parallel-gcn_amd/csrc/gs_epilogue.hpp -- the element-wise tail of a GraphSum, applied by
// whichever kernel forms a row's final sum (k_gs_lds_combine, the plain k_graphsum kernels and
// their combine), so the ReLU and Dropout modules around a GraphSum cost no launch of their own.
//
// Same operations, in the same order and with the same roundings, as the separate kernels
// (k_relu_fwd / k_dropout_apply / k_relu_bwd, k_elementwise.hip), so results are bit-identical:
//   forward  (hpdga gcn.cpp:91-97 module order GraphSum -> ReLU -> Dropout; module.cpp:173-228):
//     y = y > 0 ? y : 0            (relu_mask[i] = y > 0 when training)
//     y = y * (keep_i ? scale : 0) (training only: the hidden Dropout)
//   backward (reverse order: GraphSum.bwd -> Dropout.bwd -> ReLU.bwd):
//     g = g * (keep_i ? scale : 0)
//     g = relu_mask[i] ? g : 0
// Element i of row r, column c: relu_mask[r * relu_ld + c], dropout bit drop_base + r * drop_cols + c.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pgcn {

struct GsEpilogue {
  int mode = 0;                    // 0 none, 1 forward tail, 2 backward tail
  uint8_t *relu_mask = nullptr;    // mode 1: written (training), may be null; mode 2: read
  int relu_ld = 0;
  const uint64_t *drop_mask = nullptr;  // null: no dropout
  long long drop_base = 0;
  int drop_cols = 0;
  float drop_scale = 1.0f;
  int col0 = 0;  // column of the output pointer's first column (16-column passes)
  // the next GraphSum's prescaled input (ring schedule layout, k_ring_prescale): also write
  // next_scale[r] * y to float4 (r / sr) * 4 sr + (c / 4) sr + r % sr of next_table
  float4 *next_table = nullptr;
  const float *next_scale = nullptr;
  int next_sr = 0;
};

__device__ __forceinline__ uint32_t gs_epi_bits4(const uint64_t *__restrict__ mask, long long idx) {
  const long long w = idx >> 6;
  const int sh = (int)(idx & 63);
  uint64_t v = mask[w] >> sh;
  if (sh > 60) v |= mask[w + 1] << (64 - sh);
  return (uint32_t)v & 0xfu;
}

// The epilogue's loads (dropout words, ReLU mask bytes, the next table's row scale), issued
// together before the sums they apply to are formed: a kernel that loads them inside the
// epilogue waits for each behind the stores before it (hipcc cannot hoist a load over a store
// through a byte pointer), one HBM round trip apiece.
struct GsEpiIn {
  uint64_t w0 = 0, w1 = 0;  // dropout words (w1: a nibble that straddles two words)
  uint32_t rm = 0;          // mode 2: the forward's ReLU keep bytes
  float ns = 0.0f;          // next_scale[r]
};

__device__ __forceinline__ void gs_epi_load(GsEpiIn &in, long long r, int c0, const GsEpilogue &e) {
  if (e.mode == 0) return;
  c0 += e.col0;
  if (e.drop_mask) {
    const long long idx = e.drop_base + r * e.drop_cols + c0;
    in.w0 = e.drop_mask[idx >> 6];
    if ((idx & 63) > 60) in.w1 = e.drop_mask[(idx >> 6) + 1];
  }
  if (e.mode == 2) in.rm = *reinterpret_cast<const uint32_t *>(e.relu_mask + r * e.relu_ld + c0);
  if (e.next_table) in.ns = e.next_scale[r];
}

// a = the float4 of columns c0 .. c0+3 of row r (c0 % 4 == 0) of the output pointer, i.e.
// columns e.col0 + c0 .. of the variable; `in` from gs_epi_load(r, c0, e)
__device__ __forceinline__ void gs_epilogue(float4 &a, long long r, int c0, const GsEpilogue &e,
                                            const GsEpiIn &in) {
  if (e.mode == 0) return;
  c0 += e.col0;
  if (e.mode == 1) {
    const bool k0 = a.x > 0.0f, k1 = a.y > 0.0f, k2 = a.z > 0.0f, k3 = a.w > 0.0f;
    if (e.relu_mask) {
      const uint32_t m = (uint32_t)k0 | (uint32_t)k1 << 8 | (uint32_t)k2 << 16 | (uint32_t)k3 << 24;
      *reinterpret_cast<uint32_t *>(e.relu_mask + r * e.relu_ld + c0) = m;
    }
    if (!k0) a.x = 0.0f;
    if (!k1) a.y = 0.0f;
    if (!k2) a.z = 0.0f;
    if (!k3) a.w = 0.0f;
  }
  if (e.drop_mask) {
    const long long idx = e.drop_base + r * e.drop_cols + c0;
    const int sh = (int)(idx & 63);
    uint64_t v = in.w0 >> sh;
    if (sh > 60) v |= in.w1 << (64 - sh);
    const uint32_t bits = (uint32_t)v & 0xfu;
    const float s = e.drop_scale;
    a.x *= (bits & 1) ? s : 0.0f;
    a.y *= (bits & 2) ? s : 0.0f;
    a.z *= (bits & 4) ? s : 0.0f;
    a.w *= (bits & 8) ? s : 0.0f;
  }
  if (e.mode == 2) {
    const uint32_t m = in.rm;
    if (!(m & 0xffu)) a.x = 0.0f;
    if (!(m & 0xff00u)) a.y = 0.0f;
    if (!(m & 0xff0000u)) a.z = 0.0f;
    if (!(m & 0xff000000u)) a.w = 0.0f;
  }
  if (e.next_table) {  // as k_ring_prescale computes it from the stored output
    const float s = in.ns;
    const long long sr = e.next_sr;
    e.next_table[(r / sr) * 4 * sr + (c0 >> 2) * sr + r % sr] =
        make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
  }
}

// loads and application in one (kernels whose epilogue inputs cannot be loaded earlier)
__device__ __forceinline__ void gs_epilogue(float4 &a, long long r, int c0, const GsEpilogue &e) {
  GsEpiIn in;
  gs_epi_load(in, r, c0, e);
  gs_epilogue(a, r, c0, e, in);
}

}  // namespace pgcn
