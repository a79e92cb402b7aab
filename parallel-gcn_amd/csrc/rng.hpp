// parallel-gcn_amd/csrc/rng.hpp -- xorshift128+ (hpdga-spring23/src/rand.cpp:17-28).
#pragma once
#include <cstdint>

#include "../../include/pgcn.h"

namespace pgcn {

// One draw: advances s and returns the 31-bit output, exactly rand.cpp:17-28.
inline uint32_t xs_next(uint64_t s[2]) {
  uint64_t t = s[0];
  const uint64_t u = s[1];
  s[0] = u;
  t ^= t << 23;
  t ^= t >> 17;
  t ^= u ^ (u >> 26);
  s[1] = t;
  return (uint32_t)(t + u) & 0x7fffffffu;
}
inline void xs_advance(uint64_t s[2]) { (void)xs_next(s); }

struct BitMatrix {
  uint64_t col[128][2];
  void identity();
  void apply(const uint64_t in[2], uint64_t out[2]) const;
  BitMatrix mul(const BitMatrix &rhs) const;
};

BitMatrix xs_step_matrix();
BitMatrix xs_jump_matrix(uint64_t k);
void xs_jump(uint64_t s[2], uint64_t k);
void xs_byte_tables(const BitMatrix &m, uint64_t *table);  // 16*256*2 u64

constexpr int kDropChunk = 64;  // draws per chunk state == bits per mask word

}  // namespace pgcn
