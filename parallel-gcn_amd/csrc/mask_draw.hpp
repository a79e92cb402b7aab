// parallel-gcn_amd/csrc/mask_draw.hpp -- the dropout mask draw (bit-exact hpdga masks): the
// device side shared by k_dropout_mask / k_adam_mask (k_elementwise.hip) and the X-stream NN
// kernel's drawing waves (k_xstream_lds.hip, `mask_xstream`).
//
// Float contraction plays no part here (integer work only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

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
#ifndef PGCN_DROP_SHIFTIN
#define PGCN_DROP_SHIFTIN 1
#endif
struct Xs64 {
  uint64_t s0, s1;
  uint32_t lo = 0, hi = 0;  // mask bits 0-31 / 32-63 (constant shifts: the loop is unrolled)
  uint32_t thr2 = 0;          // threshold << 1 (PGCN_DROP_SHIFTIN)
  __device__ __forceinline__ void step(int j, int threshold) {
    uint64_t t = s0;
    const uint64_t u = s1;
    s0 = u;
    t ^= t << 23;
    {  // t ^ (t >> 17) ^ u ^ (u >> 26) per half: one three-input xor and one xor (r04: 14 ->
       // 12 VALU per draw; k_dropout_mask 111 -> 94 us alone on reddit's input mask)
      uint64_t y, z;  // full-rate 64-bit shifts (hipcc would split them into 32-bit pieces)
      asm("v_lshrrev_b64 %0, 17, %1" : "=v"(y) : "v"(t));
      asm("v_lshrrev_b64 %0, 26, %1" : "=v"(z) : "v"(u));
      uint32_t l = (uint32_t)t, h = (uint32_t)(t >> 32);
      asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(l) : "v"((uint32_t)y), "v"((uint32_t)z));
      asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
          : "+v"(h)
          : "v"((uint32_t)(y >> 32)), "v"((uint32_t)(z >> 32)));
      t = ((uint64_t)(h ^ (uint32_t)(u >> 32)) << 32) | (l ^ (uint32_t)u);
    }
    s1 = t;
#if PGCN_DROP_SHIFTIN
    // keep = ((t + u) & 0x7fffffff) >= threshold, compared as ((t + u) << 1) >= (threshold << 1)
    // (both < 2^32: the same order), shifted in at bit 0 (draw j ends at bit 31 - j of its
    // half; reversed once per half at the end)
    const uint32_t r2 = ((uint32_t)t + (uint32_t)u) << 1;
    uint32_t &w = j < 32 ? lo : hi;
    // w = 2 w + (thr2 <= r2): the compare's carry straight into the add (2 VALU ops)
    asm("v_cmp_le_u32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
        : "+v"(w)
        : "s"(thr2), "v"(r2)
        : "vcc");
#else
    const int r = (int)((uint32_t)(t + u) & 0x7fffffffu);
    const uint32_t bit = r >= threshold ? 1u : 0u;
    if (j < 32)
      lo |= bit << j;
    else
      hi |= bit << (j - 32);
#endif
  }
};

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
  return a;
}
// M^period (a0, a1) from the nibble tables: 32 lookups xor-ed, two per three-input xor
__device__ __forceinline__ uint64_t dmn_advance(const uint4 *lut, uint64_t a0, uint64_t a1,
                                                uint64_t &n1) {
  uint4 n = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int q = 0; q < 32; q += 2) {
    const uint64_t a = q < 16 ? a0 : a1;
    const int sh = 4 * (q & 15);
    const uint4 v = lut[q * 16 + ((a >> sh) & 0xf)];
    const uint4 w = lut[(q + 1) * 16 + ((a >> (sh + 4)) & 0xf)];
    n.x = xor3(n.x, v.x, w.x);
    n.y = xor3(n.y, v.y, w.y);
    n.z = xor3(n.z, v.z, w.z);
    n.w = xor3(n.w, v.w, w.w);
  }
  n1 = ((uint64_t)n.w << 32) | n.z;
  return ((uint64_t)n.y << 32) | n.x;
}

// One launch draws one or two variables' masks (MaskSeg b: the small graphs' hidden dropout
// drawn beside the input's, r04 late: one launch fewer per epoch); workgroups [0, blocks_a)
// take segment a, the rest segment b.  Every variable's chunk states advance by the same
// period (the whole epoch's draws), so one jump table serves both.
// (MaskSeg: kernels.hpp)

// PER = 2 (r06, the engine's layout): one state per 128 draws -- a thread draws two mask words
// from it and jumps it by the epoch's period once, where PER = 1 jumps per 64 draws (32 table
// lookups and 64 three-input xors: 2.5 of the ~14.5 VALU ops per draw) and reads and writes
// twice the states (35 MB per epoch on reddit's input mask)
// threads t0, t0 + G, ... of the G drawing threads (k_dropout_mask: every thread of the grid;
// the X-stream kernel: its drawing waves)
template <int PER>
__device__ __forceinline__ void dropout_mask_seg(const MaskSeg &sg, const uint4 *lut, long long t0,
                                                 long long G) {
  uint64_t *__restrict__ states = sg.states;
  uint64_t *__restrict__ mask = sg.mask;
  const long long n_chunks = sg.n_chunks, elem0 = sg.elem0, elem_end = sg.elem_end;
  const long long n_states = (n_chunks + PER - 1) / PER;
  const int threshold = sg.threshold;
  // mask word of 64-draw chunk c (trimmed past elem_end; no word past n_chunks)
  auto put = [&](long long c, uint64_t word) {
    if (c >= n_chunks) return;
    const long long e = elem0 + 64 * c;  // first element of this chunk
    if (e + 64 > elem_end) {
      const long long valid = elem_end - e;
      word = valid <= 0 ? 0 : (word & ((valid >= 64) ? ~0ull : ((1ull << valid) - 1)));
    }
    mask[c] = word;
  };
  // state k advanced by `period` draws: M^period * (a0, a1)
  auto advance = [&](long long k, uint64_t a0, uint64_t a1) {
    uint64_t n1;
    const uint64_t n0 = dmn_advance(lut, a0, a1, n1);
    states[2 * k] = n0;
    states[2 * k + 1] = n1;
  };
  // two chunks per thread and iteration: two independent xorshift chains interleaved (each
  // draw is a serial chain of 64-bit ops; the pair hides their latency at low occupancy)
  for (long long c = t0; c < n_states; c += 2 * G) {
    const long long c2 = c + G;
    const bool two = c2 < n_states;
    const long long cb = two ? c2 : c;
    const uint64_t a0 = states[2 * c], a1 = states[2 * c + 1];
    const uint64_t b0 = states[2 * cb], b1 = states[2 * cb + 1];
    Xs64 x{a0, a1}, y{b0, b1};
    x.thr2 = y.thr2 = (uint32_t)threshold << 1;
#pragma unroll
    for (int q = 0; q < PER; q++) {  // word q of each state's run
#pragma unroll
      for (int j = 0; j < 64; j++) {
        x.step(j, threshold);
        y.step(j, threshold);
      }
#if PGCN_DROP_SHIFTIN
      x.lo = __builtin_bitreverse32(x.lo);
      x.hi = __builtin_bitreverse32(x.hi);
      y.lo = __builtin_bitreverse32(y.lo);
      y.hi = __builtin_bitreverse32(y.hi);
#endif
      put(PER * c + q, ((uint64_t)x.hi << 32) | x.lo);
      if (two) put(PER * c2 + q, ((uint64_t)y.hi << 32) | y.lo);
      x.lo = x.hi = y.lo = y.hi = 0;
    }
    advance(c, a0, a1);
    if (two) advance(c2, b0, b1);
  }
}


}  // namespace pgcn
